// One-shot all-reduce over IPC-mapped device memory for latency-bound gradient buckets
// (SURVEY §5.8 item 3): the MLP's 256-B and the CNN's 31-KB gradients
// (distributed_multilayer_perceptron.py:103-106, distributed_cnn.py:152-156) cannot absorb a
// ring protocol's per-hop latency; here every rank reads every peer's bucket directly over xGMI
// (7 point-to-point links: all peers at once, one hop) and reduces locally.
//
// Protocol (one launch per all-reduce, stream-ordered on every rank).  The epoch lives in device
// memory (*ep, advanced by the launch's last block, like the optimizers' step counter), so the
// launch can be captured in a HIP graph and replayed — a small model's whole data-parallel step
// (forward, backward, this all-reduce, optimizer) is then ONE graph replay.
//  1. block b copies its chunk of the local bucket into this rank's staging region, half
//     (epoch & 1) — double-buffered so a fast rank's next call never overwrites data a slow
//     peer is still reading (a rank can only reach epoch+2 after every peer signalled epoch+1,
//     i.e. finished reading epoch);
//  2. every storing wave drains its stores (vmcnt(0)), the block barriers, and thread r stores
//     `epoch` into rank r's signal slot [b][my rank] with a system-scope release;
//  3. thread r polls this rank's signal slot [b][r] (system-scope acquire loads, s_sleep
//     back-off, BOUNDED: after `spins` polls (~4 s by default) it records a timeout in *err and
//     gives up, so a dead peer can never hang the GPU);
//  4. block b sums chunk b of all ranks' staging regions in rank order 0..world-1 — every rank
//     computes bit-identical results — and writes it back to the local bucket.  If any peer
//     timed out, the block writes NaN instead: a lost peer never turns into a finite, silently
//     wrong gradient; *err stays set (sticky) for the host-side health check
//     (sparkmi/parallel/ddp.py DataParallel.check) that fails the group.
// Staging and signal regions are allocated uncached (hipDeviceMallocUncached), so peer reads
// over xGMI and polls never see stale cache lines.  Only vector memory instructions are used.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "smi_ipc.h"

__global__ __launch_bounds__(256) void ipc_allreduce_kernel(IpcArgs a) {
  const int b = blockIdx.x, nb = gridDim.x;
  const long n4 = a.n / 4;
  const long per = (n4 + nb - 1) / nb;
  const long lo = (long)b * per, hi = lo + per < n4 ? lo + per : n4;
  const unsigned epoch = a.ep[0] + 1u;
  const long half = (long)(epoch & 1u) * a.cap;
  float4* mine = (float4*)(a.data[a.rank] + half);
  const float4* src = (const float4*)a.buf;
  for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = src[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __shared__ int timed_out;
  if (threadIdx.x == 0) timed_out = 0;
  __syncthreads();
  if ((int)threadIdx.x < a.world) {
    __atomic_thread_fence(__ATOMIC_RELEASE);  // system scope: the staging stores are visible first
    __hip_atomic_store(a.sig[threadIdx.x] + b * IPC_MAX_RANKS + a.rank, epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* f = a.sig[a.rank] + b * IPC_MAX_RANKS + threadIdx.x;
    long spins = 0;
    while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      if (++spins > a.spins) {  // a peer is gone
        __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        atomicOr(&timed_out, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
  }
  __syncthreads();
  float4* out = (float4*)a.buf;
  if (timed_out) {  // poison: the bucket must not carry a finite partial sum
    const float nan = __builtin_nanf("");
    for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) out[i] = make_float4(nan, nan, nan, nan);
  } else
  for (long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    float4 acc = ((const float4*)(a.data[0] + half))[i];
    for (int r = 1; r < a.world; ++r) {
      const float4 v = ((const float4*)(a.data[r] + half))[i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    out[i] = acc;
  }
  // advance the epoch: every block read ep[0] on entry; the last block to finish stores it
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(a.done, 1u) == gridDim.x - 1) {
    a.ep[0] = epoch;
    a.done[0] = 0u;
  }
}

extern "C" int smi_ipc_allreduce(const IpcArgs* args, int blocks, hipStream_t st) {
  const IpcArgs& a = *args;
  if (a.world < 1 || a.world > IPC_MAX_RANKS || a.rank < 0 || a.rank >= a.world) return -1;
  if (a.n % 4 || a.n > a.cap || ((uintptr_t)a.buf & 15)) return -1;
  if (args->spins < 1) return -1;
  if (blocks < 1) blocks = 1;
  if (blocks > IPC_MAX_BLOCKS) blocks = IPC_MAX_BLOCKS;
  hipLaunchKernelGGL(ipc_allreduce_kernel, dim3(blocks), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}
