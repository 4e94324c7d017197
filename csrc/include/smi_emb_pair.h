// The pair-compare ordering of the deterministic embedding backward (csrc/kernels/embedding.hip),
// shared with csrc/kernels/lstm.hip, whose forward launch runs it on the CUs its recurrence
// leaves idle.  For every token p: rank = # earlier tokens with its id, first = the id's first
// position (-1: padding, no gradient); then group sizes, exclusive scans, position-ordered member
// lists (list[off[first] + rank] = p) and chunks of at most EMB_CH members per group.  Integer
// results only: any thread count, any block order gives the same bits.
#pragma once
#include "smi_common.h"

#define EMB_PAIR_MAX 8192
#define EMB_CH 32
struct EmbPair {
  int* rank; int* first; int* list;
  int* ch_owner; int* ch_start; int* ch_len; int* ch_g0; int* ch_gn;  // per chunk
  unsigned* tick;   // per group (indexed by its first chunk), zeroed by the plan
  int* nchunks;
  float* part;      // [T][D] chunk partials of multi-chunk groups
};

__host__ __device__ inline EmbPair emb_pair_layout(void* ws, long T) {
  EmbPair e{};
  int* p = (int*)ws;
  e.rank = p; p += T;
  e.first = p; p += T;
  e.list = p; p += T;
  e.ch_owner = p; p += T;
  e.ch_start = p; p += T;
  e.ch_len = p; p += T;
  e.ch_g0 = p; p += T;
  e.ch_gn = p; p += T;
  e.tick = (unsigned*)p; p += T;
  e.nchunks = p; p += 4;
  e.part = (float*)p;
  return e;
}

// WT: the results are handed to another workgroup of the same launch (write-through stores,
// smi_common.h); the plan then reads them with device-scope loads (CC)
__device__ __forceinline__ void emb_st(int* p, int v, bool wt) {
  if (wt) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
__device__ __forceinline__ int emb_ld(const int* p, bool cc) {
  return cc ? __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
}

// rank / first of tokens [p0, p0 + 64) by NT threads: NT / 64 waves split the earlier positions.
// s_id: >= ((min(p0 + 64, T) + 3) & ~3) ints of LDS; s_cnt / s_min: [NT / 64][64]
template <int NT, bool WT>
__device__ __forceinline__ void emb_pair_rank_tile(const long long* __restrict__ ids, long T, long long pad,
                                                   const EmbPair& e, int p0, int* s_id, int (*s_cnt)[64],
                                                   int (*s_min)[64]) {
  constexpr int NW = NT / 64;
  const int n = (int)min((long)p0 + 64, T);  // positions 0 .. n - 1 compared
  const int n4 = (n + 3) & ~3;
  for (int i = threadIdx.x; i < n4; i += NT) s_id[i] = i < n ? (int)ids[i] : -2;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int p = p0 + lane;
  const int myid = p < n ? s_id[p] : -3;
  const bool live = p < n && (long long)myid != pad && myid >= 0;
  const int per = ((n4 / 4 + NW - 1) / NW) * 4;  // positions per wave (multiple of 4)
  const int q0 = w * per, q1 = min(q0 + per, n4);
  int cnt = 0, fmin = p;
  for (int q = q0; q < q1; q += 4) {
    const int4 v = *(const int4*)(s_id + q);  // same address on every lane: a broadcast read
    const int vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool eq = vv[k] == myid && q + k < p;
      cnt += eq ? 1 : 0;
      fmin = eq ? min(fmin, q + k) : fmin;
    }
  }
  s_cnt[w][lane] = cnt;
  s_min[w][lane] = fmin;
  __syncthreads();
  if (threadIdx.x < 64 && p < T) {
    int c = 0, f = p;
#pragma unroll
    for (int k = 0; k < NW; ++k) { c += s_cnt[k][lane]; f = min(f, s_min[k][lane]); }
    emb_st(e.rank + p, c, WT);
    emb_st(e.first + p, live ? f : -1, WT);
  }
}

// the plan, one workgroup of NT threads; s_f / s_off / s_coff: >= T ints of LDS each, s_wsum
// [2][NT / 64].  CC: rank / first come from other workgroups of this launch
template <int NT, bool CC>
__device__ __forceinline__ void emb_pair_plan_body(long T, const EmbPair& e, int* s_f, int* s_off, int* s_coff,
                                                   int (*s_wsum)[NT / 64]) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n = (int)T;
  for (int i = tid; i < n; i += NT) { s_f[i] = emb_ld(e.first + i, CC); s_off[i] = 0; }
  __syncthreads();
  for (int i = tid; i < n; i += NT)
    if (s_f[i] >= 0) atomicAdd(&s_off[s_f[i]], 1);  // group sizes (integer adds: order-free)
  __syncthreads();
  // chunks per group, then exclusive scans of sizes and chunk counts over the positions: thread
  // tid owns the contiguous range [tid * per, ...) — serial inside, wave / block prefix outside
  const int per = (n + NT - 1) / NT, a0 = min(n, tid * per), a1 = min(n, a0 + per);
  int ssum = 0, csum = 0;
  for (int i = a0; i < a1; ++i) {
    const int c = s_off[i];
    s_coff[i] = (c + EMB_CH - 1) / EMB_CH;
    ssum += c;
    csum += s_coff[i];
  }
  int sx = ssum, cx = csum;  // inclusive wave scans
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int ys = __shfl_up(sx, d, 64), yc = __shfl_up(cx, d, 64);
    if (lane >= d) { sx += ys; cx += yc; }
  }
  if (lane == 63) { s_wsum[0][w] = sx; s_wsum[1][w] = cx; }
  __syncthreads();
  int sb = 0, cb = 0;
  for (int k = 0; k < w; ++k) { sb += s_wsum[0][k]; cb += s_wsum[1][k]; }
  int so = sb + sx - ssum, co = cb + cx - csum;  // exclusive prefix of this thread's range
  for (int i = a0; i < a1; ++i) {
    const int c = s_off[i], nc = s_coff[i];
    s_off[i] = so;
    s_coff[i] = co;
    // chunk table of the group first at position i
    for (int k = 0; k < nc; ++k) {
      e.ch_owner[co + k] = i;
      e.ch_start[co + k] = so + k * EMB_CH;
      e.ch_len[co + k] = min(EMB_CH, c - k * EMB_CH);
      e.ch_g0[co + k] = co;
      e.ch_gn[co + k] = nc;
      e.tick[co + k] = 0u;
    }
    so += c;
    co += nc;
  }
  if (tid == NT - 1) *e.nchunks = co;
  __syncthreads();
  for (int i = tid; i < n; i += NT)
    if (s_f[i] >= 0) e.list[s_off[s_f[i]] + emb_ld(e.rank + i, CC)] = i;  // position order within the group
}
