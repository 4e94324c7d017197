// Minibatch gather from HBM-resident datasets: out[i] = src[idx[i]] for rows of
// arbitrary byte width (16-B vector copies when aligned), and the uint8 -> float/bf16 gather
// with the ToTensor /255 scaling fused (distributed_cnn.py:90-106 transform=ToTensor()).
// One wave per output row; rows are independent so the grid simply covers the batch.
#include "smi_common.h"

__global__ void gather_rows_kernel(const unsigned char* __restrict__ src, const long long* __restrict__ idx,
                                   unsigned char* __restrict__ out, long n, long row_bytes) {
  const int lane = threadIdx.x & 63;
  for (long i = (long)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += (long)gridDim.x * 4) {
    const unsigned char* s = src + idx[i] * row_bytes;
    unsigned char* d = out + i * row_bytes;
    if ((row_bytes & 15) == 0 && (((uintptr_t)src | (uintptr_t)out) & 15) == 0) {
      for (long c = lane * 16; c < row_bytes; c += 64 * 16) *(uint4*)(d + c) = *(const uint4*)(s + c);
    } else {
      for (long c = lane; c < row_bytes; c += 64) d[c] = s[c];
    }
  }
}

__global__ void gather_u8_scale_kernel(const unsigned char* __restrict__ src, const long long* __restrict__ idx,
                                       void* __restrict__ out, long n, long row, float scale, int out_bf16) {
  const int lane = threadIdx.x & 63;
  for (long i = (long)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += (long)gridDim.x * 4) {
    const unsigned char* s = src + idx[i] * row;
    for (long c = lane; c < row; c += 64) {
      const float v = (float)s[c] * scale;
      if (out_bf16) ((unsigned short*)out)[i * row + c] = f2bf(v);
      else ((float*)out)[i * row + c] = v;
    }
  }
}

static unsigned gblocks(long n) {
  long b = (n + 3) / 4;
  return (unsigned)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

extern "C" int smi_gather_rows(const void* src, const long long* idx, void* out, long n, long row_bytes,
                               hipStream_t st) {
  hipLaunchKernelGGL(gather_rows_kernel, dim3(gblocks(n)), dim3(256), 0, st, (const unsigned char*)src, idx,
                     (unsigned char*)out, n, row_bytes);
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_gather_u8_scale(const void* src, const long long* idx, void* out, long n, long row, float scale,
                                   int out_bf16, hipStream_t st) {
  hipLaunchKernelGGL(gather_u8_scale_kernel, dim3(gblocks(n)), dim3(256), 0, st, (const unsigned char*)src, idx, out,
                     n, row, scale, out_bf16);
  SMI_CHECK_LAUNCH();
}
