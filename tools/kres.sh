#!/bin/bash
# resource usage (VGPRs, scratch, LDS) of the kernels matching $2 in csrc/kernels/$1.hip, built
# with the same per-file flags as tools/build_native.py
f=$1; pat=$2; fl=""
[ "$f" = attention ] && fl="-mllvm -amdgpu-mfma-vgpr-form -fno-honor-nans"
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I/root/repo/csrc/include $fl -c /root/repo/csrc/kernels/$f.hip -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | grep -A12 "Function Name: .*$pat" | grep -E "Function Name|VGPRs:|Scratch" | sed 's/.*remark: *//; s/ \[-Rpass.*//' | paste - - -
