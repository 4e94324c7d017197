#!/usr/bin/env python3
"""Compile every csrc/kernels/*.hip for gfx950 with the resource-usage remarks and list the
kernels that use scratch (private memory: spills or a non-inlined call's saved registers — a
__noinline__ tail once cost the LSTM forward 28 us and the CNN step 30 us) or run at 256 VGPRs.
Usage: python tools/check_scratch.py [files...]"""
import concurrent.futures as cf
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def scan(path):
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        f"-I{ROOT}/csrc/include", "-c", path, "-o", os.devnull,
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    out, name, res = r.stderr, None, []
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and int(m.group(1)) > 0:
            res.append((os.path.basename(path), name, int(m.group(1))))
    return res


def main():
    files = sys.argv[1:] or sorted(glob.glob(f"{ROOT}/csrc/kernels/*.hip"))
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        found = [x for r in ex.map(scan, files) for x in r]
    for f, n, s in found:
        print(f"{f}: {n}: scratch {s} B/lane")
    print(f"{len(found)} kernels with scratch")


if __name__ == "__main__":
    main()
