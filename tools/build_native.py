#!/usr/bin/env python3
"""Build sparkmi's native extensions in-tree (no torch headers needed, so builds take seconds).

* ``sparkmi/_C*.so``        — HIP/CDNA4 kernels for gfx950 (hipcc --offload-arch=gfx950) +
                              pybind11 launch bindings (csrc/kernels/*.hip, csrc/bindings.cpp).
* ``sparkmi/_runtime*.so``  — host C++ runtime: libsvm parser, basic_english tokenizer and
                              vocab encoder, batch padding, shuffling (csrc/runtime/*.cpp), g++.
* ``sparkmi/_comm*.so``     — native communication layer: RCCL communicator + xGMI IPC one-shot
                              all-reduce (csrc/comm/*.hip, *.cpp), hipcc, linked against librccl.

Incremental: an object is rebuilt when its source or any header under csrc/include changes.
Usage: python tools/build_native.py [--force] [--jobs N] [--asan-runtime]
"""
import argparse
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
PKG = os.path.join(ROOT, "sparkmi")
ARCH = os.environ.get("SPARKMI_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


# per-kernel compiler flags: attention keeps its MFMA accumulators in VGPRs (the softmax works on
# them every chunk; the default AGPR form cost two accvgpr moves per element per chunk).
# -fno-honor-nans on the softmax kernels: fmaxf otherwise canonicalises both operands
# (v_max_f32 v, v, v) before every max of the online softmax; infinities keep their meaning.
KERNEL_FLAGS = {"attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form", "-fno-honor-nans"],
                "cross_entropy.hip": ["-fno-honor-nans"]}


def _ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _pybind_includes():
    import pybind11
    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _headers_mtime():
    t = 0.0
    for d in ("include",):
        p = os.path.join(CSRC, d)
        for f in os.listdir(p):
            t = max(t, os.path.getmtime(os.path.join(p, f)))
    return t


def _needs(src, obj, hdr_t, force):
    if force or not os.path.exists(obj):
        return True
    ot = os.path.getmtime(obj)
    return os.path.getmtime(src) > ot or hdr_t > ot


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build(force=False, jobs=8, verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    hdr_t = _headers_mtime()
    inc = ["-I" + os.path.join(CSRC, "include")]
    py_inc = ["-I" + p for p in _pybind_includes()]
    kern_dir = os.path.join(CSRC, "kernels")
    hip_srcs = sorted(os.path.join(kern_dir, f) for f in os.listdir(kern_dir) if f.endswith(".hip"))
    jobs_list = []
    objs = []
    for s in hip_srcs:
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        objs.append(o)
        if _needs(s, o, hdr_t, force):
            extra = KERNEL_FLAGS.get(os.path.basename(s), [])
            jobs_list.append([HIPCC, "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-c", s, "-o", o,
                              "-munsafe-fp-atomics"] + extra + inc)
    bind_src = os.path.join(CSRC, "bindings.cpp")
    bind_obj = os.path.join(OBJ, "bindings.o")
    objs.append(bind_obj)
    if _needs(bind_src, bind_obj, hdr_t, force):
        jobs_list.append(["g++", "-O2", "-std=c++17", "-fPIC", "-c", bind_src, "-o", bind_obj,
                          "-fvisibility=hidden", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"] + inc + py_inc)
    rt_dir = os.path.join(CSRC, "runtime")
    rt_srcs = sorted(os.path.join(rt_dir, f) for f in os.listdir(rt_dir) if f.endswith(".cpp"))
    rt_objs = []
    for s in rt_srcs:
        o = os.path.join(OBJ, "rt_" + os.path.basename(s) + ".o")
        rt_objs.append(o)
        if _needs(s, o, hdr_t, force):
            jobs_list.append(["g++", "-O3", "-std=c++17", "-fPIC", "-c", s, "-o", o, "-fvisibility=hidden",
                              "-pthread"] + inc + py_inc)
    comm_dir = os.path.join(CSRC, "comm")
    comm_objs = []
    for f in sorted(os.listdir(comm_dir)):
        s = os.path.join(comm_dir, f)
        o = os.path.join(OBJ, "comm_" + f + ".o")
        if f.endswith(".hip"):
            comm_objs.append(o)
            if _needs(s, o, hdr_t, force):
                jobs_list.append([HIPCC, "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-c", s, "-o", o] + inc)
        elif f.endswith(".cpp"):
            comm_objs.append(o)
            if _needs(s, o, hdr_t, force):
                jobs_list.append([HIPCC, "-O2", "-std=c++17", "-fPIC", "-c", s, "-o", o, "-fvisibility=hidden",
                                  "-I/opt/rocm/include"] + inc + py_inc)
    if jobs_list:
        with ThreadPoolExecutor(max_workers=jobs) as ex:
            for cmd, _ in zip(jobs_list, ex.map(_run, jobs_list)):
                if verbose:
                    print("[build]", os.path.basename(cmd[cmd.index("-c") + 1]), flush=True)
    suffix = _ext_suffix()
    c_so = os.path.join(PKG, "_C" + suffix)
    if force or not os.path.exists(c_so) or any(os.path.getmtime(o) > os.path.getmtime(c_so) for o in objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", c_so] + objs)
        if verbose:
            print("[link]", os.path.relpath(c_so, ROOT), flush=True)
    comm_so = os.path.join(PKG, "_comm" + suffix)
    if comm_objs and (force or not os.path.exists(comm_so) or
                      any(os.path.getmtime(o) > os.path.getmtime(comm_so) for o in comm_objs)):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", comm_so] + comm_objs +
             ["-L/opt/rocm/lib", "-lrccl"])
        if verbose:
            print("[link]", os.path.relpath(comm_so, ROOT), flush=True)
    rt_so = os.path.join(PKG, "_runtime" + suffix)
    if rt_objs and (force or not os.path.exists(rt_so) or
                    any(os.path.getmtime(o) > os.path.getmtime(rt_so) for o in rt_objs)):
        _run(["g++", "-shared", "-fPIC", "-pthread", "-o", rt_so] + rt_objs)
        if verbose:
            print("[link]", os.path.relpath(rt_so, ROOT), flush=True)
    return c_so, rt_so


SAN_FLAGS = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined", "-g",
             "-O1"]


def build_runtime_sanitized(out_dir=None, verbose=True):
    """Host-runtime extension built with AddressSanitizer + UBSan into
    build/asan/_runtime<suffix>; load it in a process started with libasan preloaded
    (tools/sanitize_runtime.py does both)."""
    out_dir = out_dir or os.path.join(ROOT, "build", "asan")
    os.makedirs(out_dir, exist_ok=True)
    inc = ["-I" + os.path.join(CSRC, "include")] + ["-I" + p for p in _pybind_includes()]
    rt_dir = os.path.join(CSRC, "runtime")
    srcs = sorted(os.path.join(rt_dir, f) for f in os.listdir(rt_dir) if f.endswith(".cpp"))
    so = os.path.join(out_dir, "_runtime" + _ext_suffix())
    _run(["g++", "-std=c++17", "-fPIC", "-shared", "-pthread", "-fvisibility=hidden", "-o", so] + SAN_FLAGS + inc +
         srcs)
    if verbose:
        print("[asan]", os.path.relpath(so, ROOT), flush=True)
    return so


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--asan-runtime", action="store_true", help="also build the sanitizer runtime extension")
    args = ap.parse_args()
    build(force=args.force, jobs=args.jobs)
    if args.asan_runtime:
        build_runtime_sanitized()


if __name__ == "__main__":
    sys.exit(main())
