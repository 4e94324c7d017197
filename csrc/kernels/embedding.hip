// Token embedding gather fused with the sinusoidal positional-encoding add and dropout, and
// its scatter-add backward.
//
// Reference: SentenceEmbedding.forward = dropout_{0.1}(Embedding(x) + PE) (transformer.py:57-62;
// PE table transformer.py:33-42, precomputed once here instead of per forward) and
// the LSTM's plain nn.Embedding with padding_idx (distributed_lstm.py:115,128).
// Forward: one thread per 8 contiguous features (16-B loads of the bf16 table copy), bf16 out.
// Backward (deterministic): ids are bucketed into position-ordered lists and each id's rows are
// summed in a fixed order (bit-reproducible, no float atomics; emb_det_* kernels).
// An fp32-atomic variant (runs of equal ids merged first) is kept for comparison.  Rows ==
// padding_idx are skipped (that row's gradient stays zero like torch's padding_idx).  Dense semantics are kept on
// purpose: the reference's Adam decays every row.
#include "smi_common.h"
#include "smi_split3.h"
#include "smi_emb_pair.h"

// T = storage of the table copy and the output: unsigned short (bf16 shadow) or float (fp32
// reference-precision path: the fp32 master table itself).
template <typename T>
__global__ void emb_fwd_kernel(const long long* __restrict__ ids, const T* __restrict__ table,
                               const float* __restrict__ pe, T* __restrict__ out, long Tn, int D, int S,
                               const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale,
                               unsigned short* __restrict__ P, long pps) {
  const uint32_t seed = smi_seed(seedp, salt);
  const int vpr = D / 8;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Tn * vpr) return;
  const long t = i / vpr;
  const int c = (int)(i % vpr) * 8;
  const long id = ids[t];
  V8<T> w;
  w.load(table + id * D + c);
  float o[8];
  const float* pr = pe ? pe + (long)(t % S) * D + c : nullptr;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float x = w[j] + (pr ? pr[j] : 0.f);
    if (thresh) x = smi_keep(seed, (uint32_t)(t * D + c + j), thresh) ? x * dscale : 0.f;
    o[j] = x;
  }
  V8<T>::store(out + t * D + c, o);
  if (P) {  // fp32 path: split planes [3][Tn][D] for the first layer's split-plane GEMMs
    uint32_t h[4], m[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) split3_pair(o[2 * e], o[2 * e + 1], h[e], m[e], l[e]);
    unsigned short* q = P + t * D + c;
    *(uint4*)q = make_uint4(h[0], h[1], h[2], h[3]);
    *(uint4*)(q + pps) = make_uint4(m[0], m[1], m[2], m[3]);
    *(uint4*)(q + 2 * pps) = make_uint4(l[0], l[1], l[2], l[3]);
  }
}

// One wave per run of EMB_RUN consecutive tokens, lane = column (a wave-instruction covers 64
// consecutive columns: 128-B coalesced loads, and 256-B contiguous float atomics — the shape the
// memory-side atomics run at full rate).  The wave loads all its rows first, then walks them in
// order and merges consecutive tokens with the same id in registers, so a run of equal ids (the
// padding tail of every sequence: ~25 % of the reference's tokens share one id) costs one atomic
// row per wave instead of one per token (same-address float atomics serialise at the L2).
#define EMB_RUN 8
__device__ __forceinline__ float emb_ld(const unsigned short* p) { return bf2f(*p); }
__device__ __forceinline__ float emb_ld(const float* p) { return *p; }
template <typename TS>
__global__ __launch_bounds__(256) void emb_bwd_kernel(const long long* __restrict__ ids,
                                                      const TS* __restrict__ dout,
                                                      float* __restrict__ dtable, long T, int D, long long padding_idx,
                                                      const uint32_t* seedp, uint32_t salt, uint32_t thresh,
                                                      float dscale) {
  const uint32_t seed = thresh ? smi_seed(seedp, salt) : 0u;
  const int lane = threadIdx.x & 63;
  const long t0 = ((long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * EMB_RUN;
  if (t0 >= T) return;
  const int nt = (int)min((long)EMB_RUN, T - t0);
  long long id[EMB_RUN];
#pragma unroll
  for (int i = 0; i < EMB_RUN; ++i) id[i] = i < nt ? ids[t0 + i] : padding_idx;
  for (int c0 = 0; c0 < D; c0 += 512) {
    float v[EMB_RUN][8];
#pragma unroll
    for (int i = 0; i < EMB_RUN; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j * 64 + lane;
        v[i][j] = (i < nt && c < D) ? emb_ld(dout + (t0 + i) * D + c) : 0.f;
      }
    float acc[8];
    long long cur = -1;
#pragma unroll
    for (int i = 0; i <= EMB_RUN; ++i) {
      const long long nid = (i < nt) ? id[i] : -2;
      if (nid != cur) {
        if (cur >= 0 && cur != padding_idx) {
          float* dst = dtable + cur * D + c0 + lane;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (c0 + j * 64 + lane < D) atomicAdd(dst + j * 64, acc[j]);
        }
        cur = nid;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = 0.f;
      }
      if (i < nt) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float g = v[i][j];
          if (thresh) g = smi_keep(seed, (uint32_t)((t0 + i) * D + c0 + j * 64 + lane), thresh) ? g * dscale : 0.f;
          acc[j] += g;
        }
      }
    }
  }
}

// ---- deterministic backward: id buckets, position-ordered lists, fixed-order sums -------------
// Bucket of id v = v % NB (NB chosen so a bucket holds <= EMB_SLOTS ids: slot = v / NB).
//  1. emb_det_count: per 256-token tile, the token count of every bucket (LDS int histogram);
//  2. emb_det_scan:  per bucket, exclusive offsets over tiles and the bucket's list start;
//  3. emb_det_place: every token writes its position to its bucket's list at (tile offset +
//     its rank among the tile's same-bucket tokens) — lists are in position order;
//  4. emb_det_sum:   workgroup (bucket, 64-column chunk): wave w sums the list entries
//     q = w (mod 8), 16 loads in flight, consecutive entries of one id in a register and other
//     ids per slot in LDS; the 8 wave partials are added in wave order, and rows that got tokens
//     are added into the table.  List entries carry the slot, so no id is loaded per token.
//     A bucket with >= EMB_HEAVY tokens (the padding id of padded batches: ~95 % of a Multi30k-
//     shaped batch) is cut into EMB_SPLIT fixed segments summed by separate workgroups into a
//     partial buffer, then emb_det_combine adds the segments in order (one workgroup per bucket
//     serialised ~1,000 rows per wave: 120 us of a 5.8 ms bf16 step).
// Every element is a fixed-order fp32 sum (independent of scheduling): bit-reproducible, no
// float atomics, and a long run of one id is spread over 8 x EMB_SPLIT waves.
#define EMB_TILE 256
#define EMB_SLOTS 24
#define EMB_CW 64
#define EMB_SW 8  // waves of the sum kernel
#define EMB_POS_BITS 26  // list entry: token position (< 2^26) | slot << 26
#define EMB_HEAVY 1024   // a bucket with >= this many tokens is summed by EMB_SPLIT workgroups
#define EMB_SPLIT 16

struct EmbDet {
  int tiles, NB;
  int* counts;  // [tiles][NB]
  int* offs;    // [tiles][NB]
  int* bstart;  // [NB + 1]
  int* list;    // [T]
  int hmax;          // capacity of the heavy-bucket list (T / EMB_HEAVY)
  int* heavy;        // [hmax + 1]: count, then the buckets with >= EMB_HEAVY tokens
  unsigned* pmask;   // [hmax][EMB_SPLIT] slots touched by each segment
  float* part;       // [hmax][EMB_SPLIT][EMB_SLOTS][D] segment partial sums
};

__device__ __forceinline__ int emb_bucket(long long id, long long pad, int NB) {
  return (id < 0 || id == pad) ? -1 : (int)(id % NB);
}

__global__ __launch_bounds__(EMB_TILE) void emb_det_count(const long long* __restrict__ ids, long T, long long pad,
                                                          EmbDet d) {
  extern __shared__ int hist[];
  for (int i = threadIdx.x; i < d.NB; i += EMB_TILE) hist[i] = 0;
  __syncthreads();
  const long t = (long)blockIdx.x * EMB_TILE + threadIdx.x;
  const int bk = t < T ? emb_bucket(ids[t], pad, d.NB) : -1;
  if (bk >= 0) atomicAdd(&hist[bk], 1);  // integer counts: order-independent
  __syncthreads();
  for (int i = threadIdx.x; i < d.NB; i += EMB_TILE) d.counts[(size_t)blockIdx.x * d.NB + i] = hist[i];
}

#define EMB_HBITS 2048  // LDS heavy-bucket bitmask words: NB <= 65,536 (V <= ~1.5M ids)
__global__ __launch_bounds__(1024) void emb_det_scan(EmbDet d) {
  __shared__ int wtot[16];
  __shared__ int carry;
  // heavy-bucket flags, set from the bucket totals this pass already holds in registers (the heavy
  // pass below re-read every bucket's start from global memory: a chain of dependent load
  // latencies per wave, ~60 % of this kernel)
  __shared__ unsigned hbits[EMB_HBITS];
  const bool lds_flags = d.NB <= 32 * EMB_HBITS;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry = 0;
  for (int i = threadIdx.x; i < EMB_HBITS; i += 1024) hbits[i] = 0u;
  __syncthreads();
  for (int b0 = 0; b0 < d.NB; b0 += 1024) {
    const int b = b0 + threadIdx.x;
    int run = 0;
    if (b < d.NB && d.tiles <= 32) {  // every tile's count in flight at once: one load latency
      int c[32];
#pragma unroll
      for (int t = 0; t < 32; ++t) c[t] = t < d.tiles ? d.counts[(size_t)t * d.NB + b] : 0;
#pragma unroll
      for (int t = 0; t < 32; ++t) {
        if (t < d.tiles) d.offs[(size_t)t * d.NB + b] = run;
        run += c[t];
      }
    } else if (b < d.NB) {
      int t = 0;
      for (; t + 8 <= d.tiles; t += 8) {  // 8 independent loads in flight
        int c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) c[u] = d.counts[(size_t)(t + u) * d.NB + b];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          d.offs[(size_t)(t + u) * d.NB + b] = run;
          run += c[u];
        }
      }
      for (; t < d.tiles; ++t) {
        d.offs[(size_t)t * d.NB + b] = run;
        run += d.counts[(size_t)t * d.NB + b];
      }
    }
    if (lds_flags && b < d.NB && run >= EMB_HEAVY) atomicOr(&hbits[b >> 5], 1u << (b & 31));  // LDS
    // block-wide exclusive scan of the bucket totals (wave shuffles, then the 16 wave totals)
    int inc = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    if (lane == 63) wtot[w] = inc;
    __syncthreads();
    int wbase = carry;
    for (int i = 0; i < w; ++i) wbase += wtot[i];
    if (b < d.NB) d.bstart[b] = wbase + inc - run;
    __syncthreads();
    if (threadIdx.x == 0) {
      int c = carry;
      for (int i = 0; i < 16; ++i) c += wtot[i];
      carry = c;
      if (b0 + 1024 >= d.NB) d.bstart[d.NB] = c;
    }
    __syncthreads();
  }
  // heavy buckets (>= EMB_HEAVY tokens), in bucket order; at most T / EMB_HEAVY of them.  All 16
  // waves: wave w counts its contiguous slice of buckets, the slices' counts are prefix-summed in
  // LDS, then every wave writes its heavy buckets at its offset (one wave walking 4096 buckets in
  // 64-bucket steps was a chain of 64 dependent global-load latencies)
  if (d.hmax > 0) {
    __shared__ int hcnt[16];
    const int per = ((d.NB + 15) / 16 + 63) / 64 * 64;
    const int lo = w * per, hi = min(d.NB, lo + per);
    auto heavy = [&](int b) {
      if (b >= hi) return false;
      if (lds_flags) return ((hbits[b >> 5] >> (b & 31)) & 1u) != 0u;
      return d.bstart[b + 1] - d.bstart[b] >= EMB_HEAVY;
    };
    int cnt = 0;
    for (int b0 = lo; b0 < hi; b0 += 64) cnt += __popcll(__ballot(heavy(b0 + lane)));
    if (lane == 0) hcnt[w] = cnt;
    __syncthreads();
    int base = 0, tot = 0;
    for (int i = 0; i < 16; ++i) {
      base += i < w ? hcnt[i] : 0;
      tot += hcnt[i];
    }
    for (int b0 = lo; b0 < hi; b0 += 64) {
      const int b = b0 + lane;
      const bool h = heavy(b);
      const unsigned long long bal = __ballot(h);
      if (h) {
        const int r = base + __popcll(bal & ((1ull << lane) - 1ull));
        if (r < d.hmax) d.heavy[1 + r] = b;
      }
      base += __popcll(bal);
    }
    if (threadIdx.x == 0) d.heavy[0] = min(tot, d.hmax);
  } else if (threadIdx.x == 0) {
    d.heavy[0] = 0;
  }
}

__global__ __launch_bounds__(EMB_TILE) void emb_det_place(const long long* __restrict__ ids, long T, long long pad,
                                                          EmbDet d) {
  __shared__ int sb[EMB_TILE];
  const long t = (long)blockIdx.x * EMB_TILE + threadIdx.x;
  const int bk = t < T ? emb_bucket(ids[t], pad, d.NB) : -1;
  sb[threadIdx.x] = bk;
  __syncthreads();
  if (bk < 0) return;
  int rank = 0;
  for (int i = 0; i < (int)threadIdx.x; ++i) rank += sb[i] == bk;
  // entry = position | slot << 26 (slot = id / NB < EMB_SLOTS): the sum kernel needs no id loads
  d.list[d.bstart[bk] + d.offs[(size_t)blockIdx.x * d.NB + bk] + rank] =
      (int)t | ((int)(ids[t] / d.NB) << EMB_POS_BITS);
}

template <typename TS, bool HEAVY>
__global__ __launch_bounds__(64 * EMB_SW) void emb_det_sum(const long long* __restrict__ ids,
                                                           const TS* __restrict__ dout, float* __restrict__ dtable,
                                                           int D, EmbDet d, const uint32_t* seedp, uint32_t salt,
                                                           uint32_t thresh, float dscale) {
  __shared__ float acc[EMB_SW][EMB_SLOTS][EMB_CW];
  __shared__ unsigned s_mask[EMB_SW];
  const int c0 = blockIdx.y * EMB_CW, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int bkt, beg, n, hb = 0;
  if (!HEAVY) {
    bkt = blockIdx.x;
    beg = d.bstart[bkt];
    n = d.bstart[bkt + 1] - beg;
    if (n == 0 || n >= EMB_HEAVY) return;  // uniform per workgroup; heavy buckets: split below
  } else {
    hb = blockIdx.x;
    if (hb >= d.heavy[0]) return;
    bkt = d.heavy[1 + hb];
    const int b0 = d.bstart[bkt], n0 = d.bstart[bkt + 1] - b0;
    const int seg = (n0 + EMB_SPLIT - 1) / EMB_SPLIT;  // segment z of the bucket's list
    beg = b0 + (int)blockIdx.z * seg;
    n = max(0, min(seg, n0 - (int)blockIdx.z * seg));
  }
  const uint32_t seed = thresh ? smi_seed(seedp, salt) : 0u;
  const int c = c0 + lane;
  const bool cok = c < D;
  unsigned mask = 0u;  // slots this wave touched (wave-uniform): rows are zeroed on first touch
  // a run of one slot accumulates in a register (a long run of one id — a padding tail — would
  // otherwise be a chain of dependent LDS read-modify-writes); flushed when the slot changes
  int rslot = -1;
  float racc = 0.f;
  auto flush = [&]() {
    if (rslot < 0) return;
    if (!((mask >> rslot) & 1u)) {
      mask |= 1u << rslot;
      acc[w][rslot][lane] = racc;
    } else {
      acc[w][rslot][lane] += racc;
    }
  };
  // this wave's entries q0, q0 + EMB_SW, ... (16 per round); the next round's list entries are
  // loaded while this round's rows are in flight
  int en[16], nx[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int q = w + u * EMB_SW;
    nx[u] = q < n ? d.list[beg + q] : -1;
  }
  for (int q0 = w; q0 < n; q0 += 16 * EMB_SW) {
    float g[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) en[u] = nx[u];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const long tt = en[u] >= 0 ? (long)(en[u] & ((1 << EMB_POS_BITS) - 1)) : 0;
      g[u] = (en[u] >= 0 && cok) ? emb_ld(dout + tt * D + c) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int q = q0 + 16 * EMB_SW + u * EMB_SW;
      nx[u] = q < n ? d.list[beg + q] : -1;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (en[u] < 0) break;
      const long tt = (long)(en[u] & ((1 << EMB_POS_BITS) - 1));
      float v = g[u];
      if (thresh) v = smi_keep(seed, (uint32_t)(tt * D + c), thresh) ? v * dscale : 0.f;
      const int slot = en[u] >> EMB_POS_BITS;
      if (slot != rslot) {
        flush();
        rslot = slot;
        racc = 0.f;
      }
      racc += v;
    }
  }
  flush();
  if (lane == 0) s_mask[w] = mask;
  __syncthreads();
  unsigned any = 0u;
#pragma unroll
  for (int ww = 0; ww < EMB_SW; ++ww) any |= s_mask[ww];
  if (HEAVY && threadIdx.x == 0 && blockIdx.y == 0) d.pmask[hb * EMB_SPLIT + blockIdx.z] = any;
  // wave w folds the touched slots w, w + 8, ... (partials in wave order): light buckets add
  // into the table, heavy-bucket segments write their partial for emb_det_combine
  for (int slot = w; slot < EMB_SLOTS; slot += EMB_SW) {
    if (!((any >> slot) & 1u) || !cok) continue;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < EMB_SW; ++ww)
      if ((s_mask[ww] >> slot) & 1u) s += acc[ww][slot][lane];
    if (HEAVY) d.part[(((long)hb * EMB_SPLIT + blockIdx.z) * EMB_SLOTS + slot) * D + c] = s;
    else dtable[((long)slot * d.NB + bkt) * D + c] += s;
  }
}

// heavy bucket hb, 64-column chunk: the EMB_SPLIT segment partials added in segment order
__global__ __launch_bounds__(256) void emb_det_combine(float* __restrict__ dtable, int D, EmbDet d) {
  const int hb = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (hb >= d.heavy[0]) return;
  const int bkt = d.heavy[1 + hb];
  const int c = blockIdx.y * EMB_CW + lane;
  unsigned m[EMB_SPLIT], any = 0u;
#pragma unroll
  for (int z = 0; z < EMB_SPLIT; ++z) {
    m[z] = d.pmask[hb * EMB_SPLIT + z];
    any |= m[z];
  }
  if (c >= D) return;
  for (int slot = w; slot < EMB_SLOTS; slot += 4) {
    if (!((any >> slot) & 1u)) continue;
    float s = 0.f;
#pragma unroll
    for (int z = 0; z < EMB_SPLIT; ++z)
      if ((m[z] >> slot) & 1u) s += d.part[(((long)hb * EMB_SPLIT + z) * EMB_SLOTS + slot) * D + c];
    dtable[((long)slot * d.NB + bkt) * D + c] += s;
  }
}

// ---- pair-compare backward for batches of up to EMB_PAIR_MAX tokens (3 launches) --------------
// The bucketed path above spends 5-6 launches (and a scan over every bucket of the vocabulary) on
// the ordering; for a step's few thousand tokens the ordering is cheaper as an all-pairs id
// comparison spread over the chip:
//  1. emb_pair_rank (one 1024-thread workgroup per 64 tokens, its 16 waves splitting the earlier
//     positions): for every token p, rank = # earlier tokens with its id and first = the id's first
//     position (-1: padding token, no gradient) — exact integer results, no atomics;
//  2. emb_pair_plan (one workgroup, all tokens in LDS): group sizes per first position (LDS integer
//     adds: order-independent), exclusive scans, member lists in position order
//     (list[off[first] + rank] = p), and chunks of at most EMB_CH members per group;
//  3. emb_pair_sum (one wave per chunk): the chunk's member rows summed in position order;
//     a one-chunk group adds its sum to its table row, a longer group's chunks write partials and
//     the group's last chunk to finish (ticket) adds them in chunk order.
// Every table row is one fixed-order fp32 sum: bit-reproducible, and long groups (a frequent word)
// are spread over several workgroups.
__global__ __launch_bounds__(1024) void emb_pair_rank(const long long* __restrict__ ids, long T, long long pad, EmbPair e) {
  __shared__ __attribute__((aligned(16))) int s_id[EMB_PAIR_MAX];
  __shared__ int s_cnt[16][64], s_min[16][64];
  emb_pair_rank_tile<1024, false>(ids, T, pad, e, blockIdx.x * 64, s_id, s_cnt, s_min);
}

__global__ __launch_bounds__(1024) void emb_pair_plan(long T, EmbPair e) {
  __shared__ int s_f[EMB_PAIR_MAX], s_off[EMB_PAIR_MAX], s_coff[EMB_PAIR_MAX];
  __shared__ int s_wsum[2][16];
  emb_pair_plan_body<1024, false>(T, e, s_f, s_off, s_coff, s_wsum);
}

template <typename TS>
__global__ __launch_bounds__(1024) void emb_pair_sum(const long long* __restrict__ ids, const TS* __restrict__ dout,
                                                     float* __restrict__ dtable, int D, EmbPair e,
                                                     const uint32_t* seedp, uint32_t salt, uint32_t thresh,
                                                     float dscale) {
  // one WAVE per chunk (16 per workgroup): a workgroup per chunk left the chip latency-bound on
  // thousands of one- or two-row chunks (transformer batch: 135 us per call); member positions
  // held one per lane and broadcast by __shfl — no LDS, no workgroup barrier
  const int lane = threadIdx.x & 63;
  const int k = blockIdx.x * 16 + (threadIdx.x >> 6);
  if (k >= *e.nchunks) return;  // wave-uniform
  const int start = e.ch_start[k], len = e.ch_len[k], g0 = e.ch_g0[k], gn = e.ch_gn[k];
  const int mine = lane < len ? e.list[start + lane] : 0;
  const long long id = ids[e.ch_owner[k]];
  const uint32_t seed = thresh ? smi_seed(seedp, salt) : 0u;
  for (int c = lane; c < D; c += 64) {
    float acc = 0.f;
    int m = 0;
    for (; m + 4 <= len; m += 4) {  // four rows in flight, added in position order
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long t = __shfl(mine, m + u, 64);
        v[u] = emb_ld(dout + t * D + c);
        if (thresh) v[u] = smi_keep(seed, (uint32_t)(t * D + c), thresh) ? v[u] * dscale : 0.f;
      }
      acc += v[0];
      acc += v[1];
      acc += v[2];
      acc += v[3];
    }
    for (; m < len; ++m) {
      const long t = __shfl(mine, m, 64);
      float v = emb_ld(dout + t * D + c);
      if (thresh) v = smi_keep(seed, (uint32_t)(t * D + c), thresh) ? v * dscale : 0.f;
      acc += v;
    }
    if (gn == 1) dtable[id * D + c] += acc;
    else smi_wt_store(e.part + (long)k * D + c, acc);  // write-through hand-off (smi_common.h)
  }
  if (gn == 1) return;
  smi_wt_drain();  // this wave's partial reached the coherence point
  int last = 0;
  if (lane == 0) last = atomicAdd(e.tick + g0, 1u) == (unsigned)gn - 1;
  if (!__shfl(last, 0, 64)) return;
  for (int c = lane; c < D; c += 64) {
    float acc = 0.f;
    for (int j = 0; j < gn; ++j) acc += smi_cc_load(e.part + (long)(g0 + j) * D + c);  // chunk order
    dtable[id * D + c] += acc;
  }
  if (lane == 0) e.tick[g0] = 0u;
}

static long emb_pair_ws_bytes(long T, long D) {
  return 4 * (9 * T + 4) + 4 * T * D + 64;
}

static int emb_det_nb(long V) {
  int NB = 1;
  while ((V + NB - 1) / NB > EMB_SLOTS) NB *= 2;
  return NB;
}

// scratch layout: counts, offs [tiles][NB]; bstart [NB + 1]; list [T]; heavy [hmax + 1];
// pmask [hmax][EMB_SPLIT]; (16-B aligned) part [hmax][EMB_SPLIT][EMB_SLOTS][D] fp32
static long emb_det_ints(long T, long NB, long hmax) {
  const long tiles = (T + EMB_TILE - 1) / EMB_TILE;
  return (2 * tiles * NB + NB + 1 + T + hmax + 1 + hmax * EMB_SPLIT + 3) / 4 * 4;
}
extern "C" long smi_emb_det_ws_bytes(long T, long V, long D) {
  const long hmax = T / EMB_HEAVY;
  const long det = 4 * emb_det_ints(T, emb_det_nb(V), hmax) + 4 * hmax * EMB_SPLIT * EMB_SLOTS * D + 64;
  const long pair = T <= EMB_PAIR_MAX ? emb_pair_ws_bytes(T, D) : 0;
  return det > pair ? det : pair;
}

// deterministic backward algorithm: 1 = pair-compare (<= EMB_PAIR_MAX tokens, default), 0 = the
// bucketed lists (emb_pair(0))
// batches the pair path takes by default: the all-pairs rank grows as T^2 — at the transformer's
// 8192 tokens it measured 40 us per call against the bucketed path's ~70 us for everything
// (profiles/r4e_fp32_step.txt); the LSTM's 4128 tokens gain (emb_pair_max overrides, <= 8192)
static long g_emb_pair_sel = -1;
extern "C" long smi_emb_pair_max(long set) {  // set < 0: query
  if (set >= 0) g_emb_pair_sel = set > EMB_PAIR_MAX ? EMB_PAIR_MAX : set;
  if (g_emb_pair_sel < 0) {
    g_emb_pair_sel = 4608;
    if (g_emb_pair_sel > EMB_PAIR_MAX) g_emb_pair_sel = EMB_PAIR_MAX;
  }
  return g_emb_pair_sel;
}
static long emb_pair_sel() { return smi_emb_pair_max(-1); }
static int g_emb_pair = -1;
extern "C" int smi_emb_pair(int set) {
  if (set == 0 || set == 1) g_emb_pair = set;
  if (g_emb_pair < 0) {
    g_emb_pair = 1;
  }
  return g_emb_pair;
}


static EmbDet emb_det_layout(void* ws, long T, long V) {
  EmbDet d{};
  d.tiles = (int)((T + EMB_TILE - 1) / EMB_TILE);
  d.NB = emb_det_nb(V);
  d.hmax = (int)(T / EMB_HEAVY);
  int* p = (int*)ws;
  d.counts = p; p += (size_t)d.tiles * d.NB;
  d.offs = p; p += (size_t)d.tiles * d.NB;
  d.bstart = p; p += d.NB + 1;
  d.list = p; p += T;
  d.heavy = p; p += d.hmax + 1;
  d.pmask = (unsigned*)p;
  d.part = (float*)ws + emb_det_ints(T, d.NB, d.hmax);
  return d;
}

// The ordering half of the deterministic backward depends on the ids alone, so a caller that
// knows them early (the forward) can run it beside other work: returns the algorithm the sum half
// must use (1 = pair-compare, 2 = bucketed lists, 0 = no scratch: fp32 atomics in the sum half).
static int emb_plan_launch(const long long* ids, long T, long long padding_idx, long V, void* ws, hipStream_t st) {
  if (!ws || V <= 0 || T <= 0) return 0;
  if (T <= emb_pair_sel() && smi_emb_pair(-1)) {
    EmbPair e = emb_pair_layout(ws, T);
    hipLaunchKernelGGL(emb_pair_rank, dim3((unsigned)((T + 63) / 64)), dim3(1024), 0, st, ids, T, padding_idx, e);
    hipLaunchKernelGGL(emb_pair_plan, dim3(1), dim3(1024), 0, st, T, e);
    return 1;
  }
  EmbDet d = emb_det_layout(ws, T, V);
  hipLaunchKernelGGL(emb_det_count, dim3(d.tiles), dim3(EMB_TILE), (size_t)d.NB * 4, st, ids, T, padding_idx, d);
  hipLaunchKernelGGL(emb_det_scan, dim3(1), dim3(1024), 0, st, d);
  hipLaunchKernelGGL(emb_det_place, dim3(d.tiles), dim3(EMB_TILE), 0, st, ids, T, padding_idx, d);
  return 2;
}

template <typename TS>
static int emb_sum_launch(int algo, const long long* ids, const void* dout, float* dtable, long T, int D,
                          long long padding_idx, const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale,
                          long V, void* ws, hipStream_t st) {
  if (algo == 1) {
    EmbPair e = emb_pair_layout(ws, T);
    hipLaunchKernelGGL(emb_pair_sum<TS>, dim3((unsigned)((T + 15) / 16)), dim3(1024), 0, st, ids, (const TS*)dout,
                       dtable, D, e, seedp, salt, thresh, dscale);
    return (int)hipGetLastError();
  }
  if (algo == 2) {
    EmbDet d = emb_det_layout(ws, T, V);
    const dim3 cg((D + EMB_CW - 1) / EMB_CW);
    hipLaunchKernelGGL((emb_det_sum<TS, false>), dim3(d.NB, cg.x), dim3(64 * EMB_SW), 0, st, ids, (const TS*)dout,
                       dtable, D, d, seedp, salt, thresh, dscale);
    if (d.hmax > 0) {
      hipLaunchKernelGGL((emb_det_sum<TS, true>), dim3(d.hmax, cg.x, EMB_SPLIT), dim3(64 * EMB_SW), 0, st, ids,
                         (const TS*)dout, dtable, D, d, seedp, salt, thresh, dscale);
      hipLaunchKernelGGL(emb_det_combine, dim3(d.hmax, cg.x), dim3(256), 0, st, dtable, D, d);
    }
    return (int)hipGetLastError();
  }
  const long waves = (T + EMB_RUN - 1) / EMB_RUN;
  hipLaunchKernelGGL(emb_bwd_kernel<TS>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, ids, (const TS*)dout,
                     dtable, T, D, padding_idx, seedp, salt, thresh, dscale);
  return (int)hipGetLastError();
}

template <typename TS>
static int emb_bwd_launch(const long long* ids, const void* dout, float* dtable, long T, int D, long long padding_idx,
                          const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, long V, void* ws,
                          hipStream_t st) {
  const int algo = emb_plan_launch(ids, T, padding_idx, V, ws, st);
  return emb_sum_launch<TS>(algo, ids, dout, dtable, T, D, padding_idx, seedp, salt, thresh, dscale, V, ws, st);
}

// the algorithm smi_emb_plan picks for T tokens over V rows (ws given)
extern "C" int smi_emb_plan_algo(long T, long V) {
  if (V <= 0 || T <= 0) return 0;
  return T <= emb_pair_sel() && smi_emb_pair(-1) ? 1 : 2;
}
extern "C" int smi_emb_plan(const long long* ids, long T, long long padding_idx, long V, void* ws, hipStream_t st) {
  return emb_plan_launch(ids, T, padding_idx, V, ws, st);
}
// the sum half after smi_emb_plan (algo = its return value); bf16: dout in bf16
extern "C" int smi_emb_sum(int algo, int bf16, const long long* ids, const void* dout, float* dtable, long T, int D,
                           long long padding_idx, const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale,
                           long V, void* ws, hipStream_t st) {
  if (bf16)
    return emb_sum_launch<unsigned short>(algo, ids, dout, dtable, T, D, padding_idx, seedp, salt, thresh, dscale, V,
                                          ws, st);
  return emb_sum_launch<float>(algo, ids, dout, dtable, T, D, padding_idx, seedp, salt, thresh, dscale, V, ws, st);
}

extern "C" int smi_emb_fwd(const long long* ids, const void* table, const float* pe, void* out, long T, int D, int S,
                           const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, hipStream_t st) {
  if (D % 8) return -1;
  const long n = T * (D / 8);
  hipLaunchKernelGGL(emb_fwd_kernel<unsigned short>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ids,
                     (const unsigned short*)table, pe, (unsigned short*)out, T, D, S, seedp, salt, thresh, dscale,
                     nullptr, 0L);
  SMI_CHECK_LAUNCH();
}
// planes / pps: optional split planes [3][T][D] of the output (0 for none)
extern "C" int smi_emb_fwd_f32(const long long* ids, const void* table, const float* pe, void* out, long T, int D, int S,
                               const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, void* planes,
                               long pps, hipStream_t st) {
  if (D % 8 || (planes && (((uintptr_t)planes & 15) || pps < T * D))) return -1;
  const long n = T * (D / 8);
  hipLaunchKernelGGL(emb_fwd_kernel<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ids,
                     (const float*)table, pe, (float*)out, T, D, S, seedp, salt, thresh, dscale,
                     (unsigned short*)planes, pps);
  SMI_CHECK_LAUNCH();
}

// V: table rows; ws: smi_emb_det_ws_bytes(T, V) bytes of scratch -> deterministic bucketed
// backward; null -> fp32 atomic adds
extern "C" int smi_emb_bwd(const long long* ids, const void* dout, float* dtable, long T, int D, long long padding_idx,
                           const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, long V, void* ws,
                           hipStream_t st) {
  return emb_bwd_launch<unsigned short>(ids, dout, dtable, T, D, padding_idx, seedp, salt, thresh, dscale, V, ws, st);
}
extern "C" int smi_emb_bwd_f32(const long long* ids, const void* dout, float* dtable, long T, int D, long long padding_idx,
                               const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, long V, void* ws,
                               hipStream_t st) {
  return emb_bwd_launch<float>(ids, dout, dtable, T, D, padding_idx, seedp, salt, thresh, dscale, V, ws, st);
}
