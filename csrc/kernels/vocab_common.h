// Definitions shared by the decode-step vocabulary kernels (vocab.hip: tiled
// launch; vocab_rr.h: row-resident launch) and their combine.
#pragma once
#include "../common.h"

namespace cst {

struct VocabPartial {  // 32 bytes per (tile, row)
  float m;       // max logit in tile
  float s;       // sum exp(x - m)
  float zval;    // max of x/temp + gumbel
  float zlogit;  // logit at zidx
  int zidx;      // sampled token candidate
  int xidx;      // argmax token (first on ties)
  float xtgt;    // logit of the target token (-inf if not in tile)
  float pad;
};

// XCD-aware block order: blocks b and b+8 share an XCD (round-robin dispatch),
// so consecutive ids of the remapped index land on the same XCD's L2.  Vocab
// tiles are the outer index: the 8 XCDs each stream a contiguous 1/8 of W
// (~1.3 MB at V=10.5k, H=512) and every row tile re-reads it from their L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// 16-byte write-through stores / loads (buffer instructions with the sc1
// cache policy, bit 4 of the builtins' aux operand on gfx950): the hand-off
// form of data produced and consumed by different workgroups of ONE launch --
// the bytes bypass the consumer CU's L1 and are written through the producer
// XCD's L2, so no fence is needed on either side (the producer still drains
// its stores with s_waitcnt vmcnt(0) before it signals).
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
constexpr int CPOL_SC1 = 16;
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t r, int off, u32x4v v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, CPOL_SC1);
}
__device__ __forceinline__ u32x4v ld16_sc1(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, CPOL_SC1);
}
__device__ __forceinline__ int ld_sc1(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// VF_EXP: the saved copy is E = exp(x - eoff[r]) in bf16 instead of fp16 x
// (eoff = the row's LSE of the previous decode step), see vocab_grad.hip
enum VocabFlags : int {
  VF_SAMPLE = 1,
  VF_ARGMAX = 2,
  VF_BENCH_MAINLOOP = 4,
  VF_SAVE_F32 = 8,
  VF_EXP = 16
};

}  // namespace cst
