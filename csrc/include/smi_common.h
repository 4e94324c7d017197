// sparkmi common device helpers for gfx950 (CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SMI_WAVE 64

typedef __attribute__((ext_vector_type(8))) short bf16x8_t;   // MFMA A/B operand (16x16x32 / 32x32x16)
typedef __attribute__((ext_vector_type(4))) float f32x4_t;    // 16x16 accumulator
typedef __attribute__((ext_vector_type(16))) float f32x16_t;  // 32x32 accumulator
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4_t;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8_t;

// ---- bf16 <-> f32 (bit-level, round-to-nearest-even; NaN-preserving via quiet bit) ----
__device__ __forceinline__ float bf2f(unsigned short h) {
  return __uint_as_float(((unsigned int)h) << 16);
}
// f32 -> bf16 round-to-nearest-even through the hardware converter (v_cvt_pk_bf16_f32, NaN stays
// NaN): one instruction per PAIR of values instead of ~5 integer ops per value.
typedef __bf16 smi_bf16x2_t __attribute__((ext_vector_type(2)));
typedef float smi_f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned short f2bf(float f) {
  return __builtin_bit_cast(unsigned short, (__bf16)f);
}
__device__ __forceinline__ unsigned int pack2bf(float a, float b) {
  return __builtin_bit_cast(unsigned int, __builtin_convertvector(((smi_f32x2_t){a, b}), smi_bf16x2_t));
}

// ---- 8-element activation vectors, bf16 (16 B) or fp32 (32 B) storage, fp32 math ----
// Kernels that serve both the bf16 path and the fp32 reference-precision path are templated on
// the storage type T and load / store through V8<T>.
template <typename T> struct V8;
template <> struct V8<unsigned short> {
  u16x8_t v;
  __device__ __forceinline__ void load(const unsigned short* p) { v = *(const u16x8_t*)p; }
  __device__ __forceinline__ float operator[](int j) const { return bf2f(v[j]); }
  __device__ __forceinline__ static void store(unsigned short* p, const float (&x)[8]) {
    uint4 o;
    o.x = pack2bf(x[0], x[1]); o.y = pack2bf(x[2], x[3]); o.z = pack2bf(x[4], x[5]); o.w = pack2bf(x[6], x[7]);
    *(uint4*)p = o;
  }
};
template <> struct V8<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p) { a = *(const float4*)p; b = *(const float4*)(p + 4); }
  __device__ __forceinline__ float operator[](int j) const {
    return j < 4 ? (j == 0 ? a.x : j == 1 ? a.y : j == 2 ? a.z : a.w) : (j == 4 ? b.x : j == 5 ? b.y : j == 6 ? b.z : b.w);
  }
  __device__ __forceinline__ static void store(float* p, const float (&x)[8]) {
    *(float4*)p = make_float4(x[0], x[1], x[2], x[3]);
    *(float4*)(p + 4) = make_float4(x[4], x[5], x[6], x[7]);
  }
};

// ---- wave64 reductions ----
// All-lane butterfly on VALU cross-lane ops: DPP quad_perm [1,0,3,2] / [2,3,0,1] and the
// row_half_mirror / row_mirror patterns inside each 16-lane row, then the gfx950 row swaps
// v_permlane16_swap / v_permlane32_swap across rows.  (__shfl_xor lowers to ds_bpermute /
// ds_swizzle, an LDS-crossbar round trip per step: six dependent ~100-cycle steps per reduction.)
// Mirror patterns pair every lane with one from the other half of its group, so after the
// quad steps each step sums (or maxes) two disjoint, already-reduced halves.
#define SMI_DPP_QP1032 0xB1   // quad_perm [1,0,3,2]
#define SMI_DPP_QP2301 0x4E   // quad_perm [2,3,0,1]
#define SMI_DPP_HMIRROR 0x141 // row_half_mirror
#define SMI_DPP_MIRROR 0x140  // row_mirror
template <int CTRL>
__device__ __forceinline__ float smi_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float smi_row16_swap_sum(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(a[0]) + __uint_as_float(a[1]);
}
__device__ __forceinline__ float smi_row32_swap_sum(float v) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(a[0]) + __uint_as_float(a[1]);
}
__device__ __forceinline__ float smi_row16_swap_max(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
}
__device__ __forceinline__ float smi_row32_swap_max(float v) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
}
// reductions over each 32-lane half of the wave (quad / mirror DPP steps + the row16 swap)
__device__ __forceinline__ float half_wave_sum(float v) {
  v += smi_dpp<SMI_DPP_QP1032>(v);
  v += smi_dpp<SMI_DPP_QP2301>(v);
  v += smi_dpp<SMI_DPP_HMIRROR>(v);
  v += smi_dpp<SMI_DPP_MIRROR>(v);
  return smi_row16_swap_sum(v);
}
__device__ __forceinline__ float half_wave_max(float v) {
  v = fmaxf(v, smi_dpp<SMI_DPP_QP1032>(v));
  v = fmaxf(v, smi_dpp<SMI_DPP_QP2301>(v));
  v = fmaxf(v, smi_dpp<SMI_DPP_HMIRROR>(v));
  v = fmaxf(v, smi_dpp<SMI_DPP_MIRROR>(v));
  return smi_row16_swap_max(v);
}
__device__ __forceinline__ float wave_sum(float v) {
  v += smi_dpp<SMI_DPP_QP1032>(v);
  v += smi_dpp<SMI_DPP_QP2301>(v);
  v += smi_dpp<SMI_DPP_HMIRROR>(v);
  v += smi_dpp<SMI_DPP_MIRROR>(v);
  v = smi_row16_swap_sum(v);
  return smi_row32_swap_sum(v);
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, smi_dpp<SMI_DPP_QP1032>(v));
  v = fmaxf(v, smi_dpp<SMI_DPP_QP2301>(v));
  v = fmaxf(v, smi_dpp<SMI_DPP_HMIRROR>(v));
  v = fmaxf(v, smi_dpp<SMI_DPP_MIRROR>(v));
  v = smi_row16_swap_max(v);
  return smi_row32_swap_max(v);
}
// Transposing reduction of 64 per-lane values: lane L returns the wave-wide sum of t[L].
// Each exchange step halves the live values (a lane keeps the half selected by one bit of its
// lane id and receives the partner's copy of it), so 64 sums cost 63 exchanges + adds instead
// of 64 x 6 for independent wave_sum calls.  Partner sets: lane ^ 32, ^ 16 (permlane swaps),
// ^ 15 (row mirror), ^ 7 (half mirror), ^ 2, ^ 1 (quad perms) — independent over GF(2), so
// every lane's result covers all 64 lanes exactly once.  t is clobbered.
template <int W, int CTRL, int BIT>
__device__ __forceinline__ void smi_tsum_dpp_step(float (&t)[64], int lane) {
  const bool hi = (lane >> BIT) & 1;
#pragma unroll
  for (int j = 0; j < W; ++j) {
    const float keep = hi ? t[j + W] : t[j], send = hi ? t[j] : t[j + W];
    t[j] = keep + smi_dpp<CTRL>(send);
  }
}
__device__ __forceinline__ float wave_transpose_sum64(float (&t)[64]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < 32; ++j) {  // lanes < 32 keep t[j], lanes >= 32 keep t[j + 32]
    auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(t[j]), __float_as_uint(t[j + 32]), false, false);
    t[j] = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {  // even rows keep t[j], odd rows t[j + 16]
    auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(t[j]), __float_as_uint(t[j + 16]), false, false);
    t[j] = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  }
  smi_tsum_dpp_step<8, SMI_DPP_MIRROR, 3>(t, lane);
  smi_tsum_dpp_step<4, SMI_DPP_HMIRROR, 2>(t, lane);
  smi_tsum_dpp_step<2, SMI_DPP_QP2301, 1>(t, lane);
  smi_tsum_dpp_step<1, SMI_DPP_QP1032, 0>(t, lane);
  return t[0];
}
// sum over groups of `width` consecutive lanes (width power of two <= 64)
template <int W>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int W>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- counter-based dropout RNG ----
// keep(i) = hash(seed, i) >= p * 2^32. The same hash is implemented in
// sparkmi/ops/dropout.py (torch int64 arithmetic) so CPU and GPU masks are bit-identical.
__device__ __forceinline__ uint32_t smi_hash(uint32_t seed, uint32_t idx) {
  uint32_t h = idx * 0x9E3779B1u ^ (seed * 0x85EBCA77u + 0x165667B1u);
  h ^= h >> 16; h *= 0x7FEB352Du;
  h ^= h >> 15; h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}
// Per-call seed = device step seed (bumped by a captured kernel every step, so HIP-graph replays
// draw fresh masks) mixed with a static per-call-site salt.
__device__ __forceinline__ uint32_t smi_seed(const uint32_t* seedp, uint32_t salt) {
  return (seedp ? seedp[0] : 0u) * 0x9E3779B9u + salt;
}
__device__ __forceinline__ bool smi_keep(uint32_t seed, uint32_t idx, uint32_t thresh) {
  return smi_hash(seed, idx) >= thresh;
}

#define SMI_CHECK_LAUNCH() return (int)hipGetLastError()

// Workgroup barrier that orders LDS only: waits for this wave's LDS ops (lgkmcnt) but leaves its
// global loads / stores in flight (a plain __syncthreads() also drains vmcnt, which exposes the
// latency of prefetches and of stores nobody in the workgroup reads until much later).
__device__ __forceinline__ void smi_lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ---- hand-off between workgroups of ONE launch (ticketed last-workgroup reductions) ----
// Each XCD has its own L2, not coherent with the others, so an agent-scope fence is L2 maintenance
// of the whole XCD cache: release = buffer_wbl2 (write back every dirty line), acquire = buffer_inv
// (measured: the CNN step 52 -> 84 us with one fence pair per workgroup).  Instead
// (MI355X_MICROARCH "publish-large", "splitk-seam"): the producer writes what it hands off with
// device-scope (sc1) stores, which write through to the coherence point, drains them
// (smi_wt_drain, before the workgroup barrier that precedes the ticket; device atomics are
// coherent) and the consumer reads them with device-scope (sc1) loads.  No fences.
__device__ __forceinline__ void smi_wt_store(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float smi_cc_load(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// two floats as one 8-B granule (p 8-B aligned)
__device__ __forceinline__ void smi_wt_store2(float* p, float a, float b) {
  const unsigned long long v = (unsigned long long)__float_as_uint(a) | ((unsigned long long)__float_as_uint(b) << 32);
  __hip_atomic_store((unsigned long long*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 smi_cc_load2(const float* p) {
  const unsigned long long v = __hip_atomic_load((unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_float2(__uint_as_float((unsigned)v), __uint_as_float((unsigned)(v >> 32)));
}
// 16-B granules through a buffer resource (byte offset 16-B aligned), cache policy sc1 (aux bit
// 4), the same device-scope policy as the atomics above.  A device-scope access is one memory
// transaction per lane however wide it is (measured on the CNN tail: 4-B lanes ~17 GB/s per CU),
// so the widest granule moves 4x the bytes per transaction.
__device__ __forceinline__ float4 smi_cc_load4(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, 16));
}
__device__ __forceinline__ void smi_wt_store4(__amdgpu_buffer_rsrc_t rs, int byte_off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), rs,
                                         byte_off, 0, 16);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t smi_rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, bytes, 0x00020000);
}
__device__ __forceinline__ void smi_wt_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

