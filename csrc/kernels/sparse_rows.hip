// Row-sparse gradient exchange, device half (sparkmi/parallel/ddp.py DataParallel._sparse_exchange;
// the LSTM embedding of /root/reference/distributed_lstm.py:115, whose 12.3 MB
// dense gradient touches only the step's B*T rows).  After the all-gather every rank holds
// W lists of k (row id, gradient row) pairs — ids unique within a list, the dummy id nrow padding —
// and must leave g[v] = sum over ranks (in RANK ORDER, bit-identical on every rank) of v's rows,
// without touching the rest of the table:
//   1. sparse_pos:  pos[r][v] = j for every valid entry (r, j) (no conflicts: unique within a rank);
//   2. sparse_sum:  the entry of the LOWEST rank holding v owns it and writes
//                   g[v] = sum_{r' >= r, pos[r'][v] >= 0} rows[r'][pos[r'][v]] (rank order, one
//                   wave per owned row, lane = column);
//   3. sparse_clear: pos[r][v] = -1 again (the table starts and ends all -1: no per-step fill).
// Rows no rank touched keep their (zero) local gradient.  Three small launches, no atomics, no
// host sync: with a fixed list capacity the whole exchange is graph-capturable around the
// collective.
#include "smi_common.h"

__global__ __launch_bounds__(256) void sparse_pos_kernel(const long long* __restrict__ ids, int* __restrict__ pos,
                                                         int W, int k, long nrow) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)W * k) return;
  const long v = ids[e];
  if (v < 0 || v >= nrow) return;  // the dummy id
  const int r = (int)(e / k), j = (int)(e - (long)r * k);
  pos[(long)r * nrow + v] = j;
}

__global__ __launch_bounds__(256) void sparse_sum_kernel(const long long* __restrict__ ids,
                                                         const float* __restrict__ rows, const int* __restrict__ pos,
                                                         float* __restrict__ g, int W, int k, int d, long nrow) {
  const long e = (long)blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per list entry
  const int lane = threadIdx.x & 63;
  if (e >= (long)W * k) return;
  const long v = ids[e];
  if (v < 0 || v >= nrow) return;
  const int r = (int)(e / k);
  for (int q = 0; q < r; ++q)
    if (pos[(long)q * nrow + v] >= 0) return;  // a lower rank owns v
  for (int c = lane; c < d; c += 64) {
    float acc = 0.f;
    for (int q = r; q < W; ++q) {
      const int j = pos[(long)q * nrow + v];
      if (j >= 0) acc += rows[((long)q * k + j) * d + c];
    }
    g[v * d + c] = acc;
  }
}

__global__ __launch_bounds__(256) void sparse_clear_kernel(const long long* __restrict__ ids, int* __restrict__ pos,
                                                           int W, int k, long nrow) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long)W * k) return;
  const long v = ids[e];
  if (v < 0 || v >= nrow) return;
  pos[(long)(e / k) * nrow + v] = -1;
}

// ids [W][k] (int64), rows [W][k][d] fp32, pos [W][nrow] int32 (all -1 on entry and exit), g [nrow][d]
extern "C" int smi_sparse_rank_sum(const long long* ids, const float* rows, int* pos, float* g, int W, int k, int d,
                                   long nrow, hipStream_t st) {
  if (W < 1 || W > 64 || k < 1 || d < 1 || nrow < 1 || !ids || !rows || !pos || !g) return -1;
  const long n = (long)W * k;
  const unsigned b256 = (unsigned)((n + 255) / 256), bw = (unsigned)((n + 3) / 4);
  hipLaunchKernelGGL(sparse_pos_kernel, dim3(b256), dim3(256), 0, st, ids, pos, W, k, nrow);
  hipLaunchKernelGGL(sparse_sum_kernel, dim3(bw), dim3(256), 0, st, ids, rows, pos, g, W, k, d, nrow);
  hipLaunchKernelGGL(sparse_clear_kernel, dim3(b256), dim3(256), 0, st, ids, pos, W, k, nrow);
  SMI_CHECK_LAUNCH();
}
