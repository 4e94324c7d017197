#!/usr/bin/env python3
"""Build sparkmi's native extensions in-tree (no torch headers needed, so builds take seconds).

* ``sparkmi/_C*.so``        — HIP/CDNA4 kernels for gfx950 (hipcc --offload-arch=gfx950) +
                              pybind11 launch bindings (csrc/kernels/*.hip, csrc/bindings.cpp).
* ``sparkmi/_runtime*.so``  — host C++ runtime: libsvm parser, basic_english tokenizer and
                              vocab encoder, batch padding, shuffling (csrc/runtime/*.cpp), g++.
* ``sparkmi/_comm*.so``     — native communication layer: RCCL communicator + xGMI IPC one-shot
                              all-reduce (csrc/comm/*.hip, *.cpp), hipcc, linked against librccl.
* ``sparkmi/_io*.so``       — native input pipeline: pinned host ring, threaded row gather,
                              async H2D on a copy stream (csrc/io/*.cpp), hipcc.

Incremental by CONTENT, not mtime: every object carries a stamp (sha256 of its compile command,
its source and every header under csrc/include) and every library a stamp of its link command
and its objects' stamps; anything whose stamp differs is rebuilt.  Copied trees whose mtimes
say "up to date" while the sources changed (or the reverse) therefore build correctly.
Usage: python tools/build_native.py [--force] [--jobs N] [--asan-runtime]
"""
import argparse
import hashlib
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


_INC_RE = __import__("re").compile(r'^\s*#\s*include\s+"([^"]+)"', __import__("re").M)


def _headers_digest(src=None):
    """Digest of the csrc/include headers ``src`` includes (transitively), or of all of them: a
    header edit rebuilds only the translation units that see it."""
    inc_dir = os.path.join(CSRC, "include")
    if src is None:
        names = sorted(os.listdir(inc_dir))
    else:
        seen, todo = set(), [src]
        while todo:
            f = todo.pop()
            try:
                with open(f) as fh:
                    text = fh.read()
            except OSError:
                continue
            for name in _INC_RE.findall(text):
                path = os.path.join(inc_dir, name)
                if name not in seen and os.path.exists(path):
                    seen.add(name)
                    todo.append(path)
        names = sorted(seen)
    h = hashlib.sha256()
    for f in names:
        h.update(f.encode())
        with open(os.path.join(inc_dir, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _stamp_path(target):
    return os.path.join(OBJ, os.path.basename(target) + ".sha256")


def _read_stamp(target):
    try:
        with open(_stamp_path(target)) as f:
            return f.read().strip()
    except OSError:
        return None


def _write_stamp(target, digest):
    with open(_stamp_path(target), "w") as f:
        f.write(digest + "\n")


def _obj_digest(src, cmd, hdr):
    h = hashlib.sha256()
    h.update("\0".join(cmd).encode())
    h.update(hdr.encode())
    with open(src, "rb") as f:
        h.update(f.read())
    return h.hexdigest()


def _needs(target, digest, force):
    return force or not os.path.exists(target) or _read_stamp(target) != digest


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build(force=False, jobs=8, verbose=True):
    os.makedirs(OBJ, exist_ok=True)
    inc = ["-I" + os.path.join(CSRC, "include")]
    py_inc = ["-I" + p for p in _pybind_includes()]
    jobs_list = []  # (cmd, object, digest)

    def obj(src, o, cmd):
        d = _obj_digest(src, cmd, _headers_digest(src))
        if _needs(o, d, force):
            jobs_list.append((cmd, o, d))
        return o, d

    kern_dir = os.path.join(CSRC, "kernels")
    objs = []
    for s in sorted(os.path.join(kern_dir, f) for f in os.listdir(kern_dir) if f.endswith(".hip")):
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        extra = KERNEL_FLAGS.get(os.path.basename(s), [])
        objs.append(obj(s, o, [HIPCC, "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-c", s, "-o", o,
                               "-munsafe-fp-atomics"] + extra + inc))
    bind_src = os.path.join(CSRC, "bindings.cpp")
    bind_obj = os.path.join(OBJ, "bindings.o")
    objs.append(obj(bind_src, bind_obj, ["g++", "-O2", "-std=c++17", "-fPIC", "-c", bind_src, "-o", bind_obj,
                                         "-fvisibility=hidden", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"] +
                    inc + py_inc))
    rt_dir = os.path.join(CSRC, "runtime")
    rt_objs = []
    for s in sorted(os.path.join(rt_dir, f) for f in os.listdir(rt_dir) if f.endswith(".cpp")):
        o = os.path.join(OBJ, "rt_" + os.path.basename(s) + ".o")
        rt_objs.append(obj(s, o, ["g++", "-O3", "-std=c++17", "-fPIC", "-c", s, "-o", o, "-fvisibility=hidden",
                                  "-pthread"] + inc + py_inc))
    comm_dir = os.path.join(CSRC, "comm")
    comm_objs = []
    for f in sorted(os.listdir(comm_dir)):
        s = os.path.join(comm_dir, f)
        o = os.path.join(OBJ, "comm_" + f + ".o")
        if f.endswith(".hip"):
            comm_objs.append(obj(s, o, [HIPCC, "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-c", s, "-o",
                                        o] + inc))
        elif f.endswith(".cpp"):
            comm_objs.append(obj(s, o, [HIPCC, "-O2", "-std=c++17", "-fPIC", "-c", s, "-o", o, "-fvisibility=hidden",
                                        "-I/opt/rocm/include"] + inc + py_inc))
    io_dir = os.path.join(CSRC, "io")
    io_objs = []
    for f in sorted(os.listdir(io_dir)) if os.path.isdir(io_dir) else []:
        if f.endswith(".cpp"):
            s = os.path.join(io_dir, f)
            o = os.path.join(OBJ, "io_" + f + ".o")
            io_objs.append(obj(s, o, [HIPCC, "-O2", "-std=c++17", "-fPIC", "-c", s, "-o", o, "-fvisibility=hidden",
                                      "-I/opt/rocm/include"] + inc + py_inc))
    if jobs_list:
        with ThreadPoolExecutor(max_workers=jobs) as ex:
            for (cmd, o, d), _ in zip(jobs_list, ex.map(lambda j: _run(j[0]), jobs_list)):
                _write_stamp(o, d)
                if verbose:
                    print("[build]", os.path.basename(cmd[cmd.index("-c") + 1]), flush=True)

    def link(so, objs_, cmd):
        h = hashlib.sha256("\0".join(cmd).encode())
        for _, d in objs_:
            h.update(d.encode())
        d = h.hexdigest()
        if _needs(so, d, force):
            _run(cmd)
            _write_stamp(so, d)
            if verbose:
                print("[link]", os.path.relpath(so, ROOT), flush=True)

    suffix = _ext_suffix()
    c_so = os.path.join(PKG, "_C" + suffix)
    link(c_so, objs, [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", c_so] + [o for o, _ in objs])
    comm_so = os.path.join(PKG, "_comm" + suffix)
    if comm_objs:
        link(comm_so, comm_objs, [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", comm_so] +
             [o for o, _ in comm_objs] + ["-L/opt/rocm/lib", "-lrccl"])
    io_so = os.path.join(PKG, "_io" + suffix)
    if io_objs:
        link(io_so, io_objs, [HIPCC, "-shared", "-fPIC", "-o", io_so] + [o for o, _ in io_objs] + ["-pthread"])
    rt_so = os.path.join(PKG, "_runtime" + suffix)
    if rt_objs:
        link(rt_so, rt_objs, ["g++", "-shared", "-fPIC", "-pthread", "-o", rt_so] + [o for o, _ in rt_objs])
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
