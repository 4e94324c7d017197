// Argument block of the IPC one-shot / two-shot all-reduce (csrc/comm/ipc_allreduce.hip), shared
// with the host bindings (csrc/comm/comm.cpp).
#pragma once
#define IPC_MAX_RANKS 8
#define IPC_MAX_BLOCKS 128
#define IPC_DEFAULT_SPINS (1L << 24)  // ~4 s of s_sleep back-off before a peer counts as lost

struct IpcArgs {
  float* buf;                          // local bucket (in / out), 16-B aligned, n % 4 == 0
  long n;                              // floats
  float* data[IPC_MAX_RANKS];          // every rank's staging region: [2][cap] floats
  unsigned* sig[IPC_MAX_RANKS];        // every rank's signal region: [IPC_MAX_BLOCKS][IPC_MAX_RANKS]
  long cap;                            // floats per staging half
  int rank, world;
  unsigned* ep;                        // device epoch counter (read at entry, advanced at exit)
  unsigned* done;                      // zeroed ticket word of the exit advance
  unsigned* sv;                        // device signal value: the last value stored into signal slots
  int* err;                            // set to 1 on a poll timeout (sticky)
  long spins;                          // poll bound (s_sleep 8 back-off per poll)
  // optional plain-SGD epilogue of the one-shot kernel (the optimizer of a data-parallel small-model
  // step, sparkmi/parallel/ddp.py fuse_sgd): p -= lr * (sum * gscale), bf16 shadow refreshed, the
  // bucket zeroed instead of overwritten with the sum, the step counter (and dropout seed) advanced
  // by the last block — sgd_kernel's arithmetic (csrc/kernels/optim.hip), one launch fewer
  float* p;                            // master parameters at the bucket's offsets (null: no SGD)
  unsigned short* pbf;                 // their bf16 shadow or null
  const float* lr; float* step; int* seed; float gscale;
};
