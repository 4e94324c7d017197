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

// Graph-resident minibatch gather (sparkmi/data/dataset.py DeviceLoader(fixed=True)): the batch's
// row ids come from a device permutation at a DEVICE cursor, the rows of up to 4 arrays land in
// fixed output buffers, and the last block to finish advances the cursor — so a captured
// training-step graph (or a multi-step graph of several steps) draws its own next shuffled batch
// with no host involvement: out_a[i] = src_a[perm[cursor * B + i]], then cursor += 1.
// blockIdx.y = array; one wave per row (16-B copies when aligned).
#define GB_MAX 4
struct GatherBatchArgs {
  const unsigned char* src[GB_MAX]; unsigned char* out[GB_MAX]; long row_bytes[GB_MAX];
  const long long* perm; int* cursor; unsigned* done; int B; int count;
};
__global__ __launch_bounds__(256) void gather_batch_kernel(GatherBatchArgs a) {
  const int lane = threadIdx.x & 63, arr = blockIdx.y;
  const long base = (long)a.cursor[0] * a.B;
  const long rb = a.row_bytes[arr];
  const unsigned char* src = a.src[arr];
  unsigned char* out = a.out[arr];
  const bool v16 = (rb & 15) == 0 && (((uintptr_t)src | (uintptr_t)out) & 15) == 0;
  for (long i = (long)blockIdx.x * 4 + (threadIdx.x >> 6); i < a.B; i += (long)gridDim.x * 4) {
    const unsigned char* s = src + a.perm[base + i] * rb;
    unsigned char* d = out + i * rb;
    if (v16) {
      for (long c = lane * 16; c < rb; c += 64 * 16) *(uint4*)(d + c) = *(const uint4*)(s + c);
    } else {
      for (long c = lane; c < rb; c += 64) d[c] = s[c];
    }
  }
  // every block has read cursor[0] before its ticket (the read above precedes the barrier), so
  // the last block's bump is never seen early; the next launch sees it at the kernel boundary
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(a.done, 1u) == gridDim.x * gridDim.y - 1) {
    a.cursor[0] += 1;
    a.done[0] = 0u;
  }
}

extern "C" int smi_gather_batch(const void* const* src, void* const* out, const long* row_bytes, int count,
                                const long long* perm, int* cursor, unsigned* done, int B, hipStream_t st) {
  if (count < 1 || count > GB_MAX || B < 1 || !perm || !cursor || !done) return -1;
  GatherBatchArgs a{};
  for (int i = 0; i < count; ++i) {
    a.src[i] = (const unsigned char*)src[i]; a.out[i] = (unsigned char*)out[i]; a.row_bytes[i] = row_bytes[i];
  }
  a.perm = perm; a.cursor = cursor; a.done = done; a.B = B; a.count = count;
  hipLaunchKernelGGL(gather_batch_kernel, dim3(gblocks(B), (unsigned)count), dim3(256), 0, st, a);
  SMI_CHECK_LAUNCH();
}
