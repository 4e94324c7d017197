// All-reduce over IPC-mapped device memory, one node: every rank reads its
// peers' staging regions directly over xGMI (7 point-to-point links: all peers at once, one hop)
// instead of a ring's 2 (w - 1) latency-bound hops.
//  * ONE-SHOT (latency-bound buckets: the MLP's 256 B, the CNN's 31 KB gradients,
//    distributed_multilayer_perceptron.py:103-106, distributed_cnn.py:152-156): every rank reads
//    every peer's whole bucket and sums it — (w - 1) n floats over xGMI per rank, one signal round.
//  * TWO-SHOT (31 KB .. tens of MB, e.g. the LSTM's 12.3 MB dense embedding gradient): reduce-
//    scatter then all-gather — rank r sums chunk r of every peer's bucket (reading its 1/w slice
//    from all peers at once), publishes the sum in place, then every rank gathers the w reduced
//    chunks: 2 (w - 1) / w n floats per rank, two signal rounds.
//  * ZERO-COPY TWO-SHOT (algo 3; the transformer's bulk buckets when the start-up probe measures it
//    fastest): the same reduce-scatter + all-gather, but read straight out of every rank's
//    IPC-registered gradient buffer (a.data[q] = peer q's bucket) instead of a staged copy — no
//    copy of the bucket into staging and no reduced chunk written twice: 2 n fewer local HBM
//    bytes per call.  Three signal rounds: (1) every bucket is final (it was written by earlier
//    kernels on each rank: stream order, and their completion wrote their lines back), (2) every
//    rank's reduced chunk is published (system-scope release), (3) every rank finished reading its
//    peers' chunks — only then may a rank's next backward overwrite its bucket.
//
// Protocol (one launch per all-reduce, stream-ordered on every rank).  Device state ctr =
// {epoch, done ticket, signal value} advanced by each launch's last block (like the optimizers'
// step counter), so launches can sit in a captured HIP graph and replay — a small model's whole
// data-parallel step (forward, backward, this all-reduce, optimizer) is ONE graph replay.
//  1. block b copies its share of the local bucket into this rank's staging half (epoch & 1):
//     double-buffered, so a fast rank's next call never overwrites data a slow peer still reads
//     (a rank only starts call e + 1 after every peer signalled call e's first round, i.e.
//     finished call e - 1);
//  2. drain the stores (vmcnt(0)), barrier, thread q stores the round's signal value into slot
//     [b][my rank] of rank q (system-scope release) and polls slot [b][q] of its own region
//     (system-scope acquire, s_sleep back-off, BOUNDED: after `spins` polls (~4 s by default) the
//     block records a timeout in *err and gives up — a dead peer never hangs the GPU);
//  3. one-shot: block b sums its share of every rank's staging in rank order 0..w-1 (bit-identical
//     on every rank).  Two-shot: block b sums its share of chunk `rank` in rank order, writes it
//     back into its own staging (only this rank reads chunk `rank` there) and to the bucket,
//     signals round 2, then copies its share of every peer's reduced chunk into the bucket.
//  4. a timed-out wait poisons: the block writes NaN (and, two-shot, publishes NaN as its reduced
//     chunk) — a lost peer never becomes a finite, silently wrong gradient; *err stays set
//     (sticky) for the host-side check (sparkmi/parallel/ddp.py DataParallel.check).
// Signal values increase monotonically over all launches of both kernels (one per round), so the
// two kernels, any block counts and both rounds share one slot array.  Staging and signal regions
// are uncached (hipDeviceMallocUncached): peer reads over xGMI and polls never see stale lines.
// Only vector memory instructions are used.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "smi_ipc.h"

// signal round: publish `val` to every peer's slot [b][rank], wait for every peer's slot [b][q]
// to reach `val`; returns (block-uniform) whether some peer timed out.  A block that already knows
// of a loss (a sticky error from an earlier call, or this call's first round: `*timed_out` set
// before the round) still publishes its signal, so live peers are not kept waiting, but does not
// poll again: after a loss every later call poisons at once instead of spending the timeout.
__device__ __forceinline__ bool ipc_round(const IpcArgs& a, int b, unsigned val, int* timed_out) {
  const bool known = *timed_out != 0;  // block-uniform: written before the caller's last barrier
  __syncthreads();
  if ((int)threadIdx.x < a.world) {
    __atomic_thread_fence(__ATOMIC_RELEASE);  // system scope: this block's stores are visible first
    __hip_atomic_store(a.sig[threadIdx.x] + b * IPC_MAX_RANKS + a.rank, val, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* f = a.sig[a.rank] + b * IPC_MAX_RANKS + threadIdx.x;
    long spins = 0;
    while (!known && (int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - val) < 0) {
      if (++spins > a.spins) {  // a peer is gone
        __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        atomicOr(timed_out, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
  return *timed_out != 0;
}
// a loss recorded by an earlier call (sticky *err): this call poisons without polling
__device__ __forceinline__ void ipc_init_lost(const IpcArgs& a, int* timed_out) {
  if (threadIdx.x == 0)
    *timed_out = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0 ? 1 : 0;
  __syncthreads();
}

// the last block to finish advances the device state for the next launch (and, with the SGD
// epilogue, the optimizer's step counter and the dropout seed, as sgd_kernel's last block does)
__device__ __forceinline__ void ipc_advance(const IpcArgs& a, unsigned epoch, unsigned sval) {
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(a.done, 1u) == gridDim.x - 1) {
    a.ep[0] = epoch;
    a.sv[0] = sval;
    a.done[0] = 0u;
    if (a.p) {
      a.step[0] = a.step[0] + 1.f;
      if (a.seed) a.seed[0] += 1;
    }
  }
}
__device__ __forceinline__ unsigned short ipc_f2bf(float f) { return __builtin_bit_cast(unsigned short, (__bf16)f); }

__global__ __launch_bounds__(256) void ipc_allreduce_kernel(IpcArgs a) {
  const int b = blockIdx.x, nb = gridDim.x;
  const long n4 = a.n / 4;
  const long per = (n4 + nb - 1) / nb;
  const long lo = (long)b * per, hi = lo + per < n4 ? lo + per : n4;
  const unsigned epoch = a.ep[0] + 1u, sval = a.sv[0] + 1u;
  const long half = (long)(epoch & 1u) * a.cap;
  float4* mine = (float4*)(a.data[a.rank] + half);
  const float4* src = (const float4*)a.buf;
  for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = src[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __shared__ int timed_out;
  ipc_init_lost(a, &timed_out);
  const bool lost = ipc_round(a, b, sval, &timed_out);
  float4* out = (float4*)a.buf;
  if (lost) {  // poison: the bucket (and, with the SGD epilogue, the parameters) must not carry a finite partial sum
    const float nan = __builtin_nanf("");
    for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      out[i] = make_float4(nan, nan, nan, nan);
      if (a.p) ((float4*)a.p)[i] = make_float4(nan, nan, nan, nan);
    }
  } else {
    const float lr = a.p ? a.lr[0] : 0.f;
    for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      float4 acc = ((const float4*)(a.data[0] + half))[i];
      for (int r = 1; r < a.world; ++r) {
        const float4 v = ((const float4*)(a.data[r] + half))[i];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      if (!a.p) {
        out[i] = acc;
      } else {  // SGD epilogue: sgd_kernel's p -= lr * (g * gscale), zero_grad, shadow
        float4 pp = ((float4*)a.p)[i];
        pp.x -= lr * (acc.x * a.gscale); pp.y -= lr * (acc.y * a.gscale);
        pp.z -= lr * (acc.z * a.gscale); pp.w -= lr * (acc.w * a.gscale);
        ((float4*)a.p)[i] = pp;
        out[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a.pbf) {
          uint2 w;
          w.x = ipc_f2bf(pp.x) | ((unsigned)ipc_f2bf(pp.y) << 16);
          w.y = ipc_f2bf(pp.z) | ((unsigned)ipc_f2bf(pp.w) << 16);
          ((uint2*)a.pbf)[i] = w;
        }
      }
    }
  }
  ipc_advance(a, epoch, sval);
}

__global__ __launch_bounds__(256) void ipc_allreduce2_kernel(IpcArgs a) {
  const int b = blockIdx.x, nb = gridDim.x;
  const long n4 = a.n / 4;
  const long C = (n4 + a.world - 1) / a.world;  // float4 per chunk (the last one may be short)
  const long per = (C + nb - 1) / nb;           // float4 per block per chunk
  const unsigned epoch = a.ep[0] + 1u, s1 = a.sv[0] + 1u, s2 = s1 + 1u;
  const long half = (long)(epoch & 1u) * a.cap;
  float4* mine = (float4*)(a.data[a.rank] + half);
  float4* out = (float4*)a.buf;
  auto range = [&](int c, long& lo, long& hi) {  // block b's share of chunk c
    const long c0 = (long)c * C, c1 = c0 + C < n4 ? c0 + C : n4;
    lo = c0 + (long)b * per;
    hi = lo + per < c1 ? lo + per : c1;
  };
  // 1. stage block b's share of every chunk
  for (int c = 0; c < a.world; ++c) {
    long lo, hi;
    range(c, lo, hi);
    for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = out[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __shared__ int timed_out;
  ipc_init_lost(a, &timed_out);
  const float nan = __builtin_nanf("");
  // 2. reduce-scatter: sum this rank's chunk over all ranks (rank order), publish it in place
  bool lost = ipc_round(a, b, s1, &timed_out);
  {
    long lo, hi;
    range(a.rank, lo, hi);
    for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      float4 acc = make_float4(nan, nan, nan, nan);
      if (!lost) {
        acc = ((const float4*)(a.data[0] + half))[i];
        for (int r = 1; r < a.world; ++r) {
          const float4 v = ((const float4*)(a.data[r] + half))[i];
          acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
      }
      mine[i] = acc;
      out[i] = acc;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // 3. all-gather every peer's reduced chunk
  lost = ipc_round(a, b, s2, &timed_out);
  for (int q = 0; q < a.world; ++q) {
    if (q == a.rank) continue;
    long lo, hi;
    range(q, lo, hi);
    const float4* peer = (const float4*)(a.data[q] + half);
    for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) out[i] = lost ? make_float4(nan, nan, nan, nan) : peer[i];
  }
  if (lost) {  // this rank's own chunk too
    long lo, hi;
    range(a.rank, lo, hi);
    for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) out[i] = make_float4(nan, nan, nan, nan);
  }
  ipc_advance(a, epoch, s2);
}

// Zero-copy two-shot: a.data[q] is rank q's bucket itself (IPC-mapped; a.data[a.rank] == a.buf).
// Chunk c / block b ranges as in the staged two-shot, identical on every rank, so block b's
// signal covers exactly the ranges block b of every peer reads or overwrites.
__global__ __launch_bounds__(256) void ipc_allreduce_zc_kernel(IpcArgs a) {
  const int b = blockIdx.x, nb = gridDim.x;
  const long n4 = a.n / 4;
  const long C = (n4 + a.world - 1) / a.world;
  const long per = (C + nb - 1) / nb;
  const unsigned epoch = a.ep[0] + 1u, s1 = a.sv[0] + 1u, s2 = s1 + 1u, s3 = s2 + 1u;
  float4* out = (float4*)a.buf;
  auto range = [&](int c, long& lo, long& hi) {
    const long c0 = (long)c * C, c1 = c0 + C < n4 ? c0 + C : n4;
    lo = c0 + (long)b * per;
    hi = lo + per < c1 ? lo + per : c1;
  };
  __shared__ int timed_out;
  ipc_init_lost(a, &timed_out);
  const float nan = __builtin_nanf("");
  // 1. every rank's bucket is final: reduce chunk `rank` straight out of every bucket (rank
  //    order), in place — no peer reads chunk `rank` of this bucket (each reads its own chunk)
  bool lost = ipc_round(a, b, s1, &timed_out);
  {
    long lo, hi;
    range(a.rank, lo, hi);
    for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      float4 acc = make_float4(nan, nan, nan, nan);
      if (!lost) {
        acc = ((const float4*)a.data[0])[i];
        for (int r = 1; r < a.world; ++r) {
          const float4 v = ((const float4*)a.data[r])[i];
          acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
      }
      out[i] = acc;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // 2. every reduced chunk is published (the round's release): gather the peers' chunks over
  //    this bucket's raw ones (each peer finished reading them before it signalled this round)
  lost = ipc_round(a, b, s2, &timed_out);
  for (int q = 0; q < a.world; ++q) {
    if (q == a.rank) continue;
    long lo, hi;
    range(q, lo, hi);
    const float4* peer = (const float4*)a.data[q];
    for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) out[i] = lost ? make_float4(nan, nan, nan, nan) : peer[i];
  }
  if (lost) {
    long lo, hi;
    range(a.rank, lo, hi);
    for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) out[i] = make_float4(nan, nan, nan, nan);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // 3. every peer finished reading this rank's reduced chunk: the bucket is free again
  ipc_round(a, b, s3, &timed_out);
  ipc_advance(a, epoch, s3);
}

// algo 1: one-shot, 2: two-shot (staged), 3: zero-copy two-shot (a.data = the peers' buckets)
extern "C" int smi_ipc_allreduce(const IpcArgs* args, int blocks, int algo, hipStream_t st) {
  const IpcArgs& a = *args;
  if (a.world < 1 || a.world > IPC_MAX_RANKS || a.rank < 0 || a.rank >= a.world) return -1;
  if (a.n % 4 || (algo != 3 && a.n > a.cap) || ((uintptr_t)a.buf & 15)) return -1;
  if (args->spins < 1 || algo < 1 || algo > 3) return -1;
  if (algo == 3) {
    if (a.data[a.rank] != a.buf) return -1;
    for (int q = 0; q < a.world; ++q)
      if ((uintptr_t)a.data[q] & 15) return -1;
  }
  if (a.p && (algo != 1 || !a.lr || !a.step || ((uintptr_t)a.p & 15) || ((uintptr_t)a.pbf & 7))) return -1;
  if (blocks < 1) blocks = 1;
  if (blocks > IPC_MAX_BLOCKS) blocks = IPC_MAX_BLOCKS;
  if (algo == 1) hipLaunchKernelGGL(ipc_allreduce_kernel, dim3(blocks), dim3(256), 0, st, a);
  else if (algo == 2) hipLaunchKernelGGL(ipc_allreduce2_kernel, dim3(blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(ipc_allreduce_zc_kernel, dim3(blocks), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}
