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

// VF_EXP: the saved copy is E = exp(x - eoff[r]) in bf16 instead of fp16 x
// (eoff = the row's LSE of the previous decode step), see vocab_grad.hip
constexpr int VF_TOPK_MAXK = 8;
__host__ __device__ constexpr int vf_topk_k(int flags) { return (flags >> 8) & 15; }
enum VocabFlags : int {
  VF_SAMPLE = 1,
  VF_ARGMAX = 2,
  VF_BENCH_MAINLOOP = 4,
  VF_SAVE_F32 = 8,
  VF_EXP = 16,
  // beam search: each (vocab tile, row) writes its TOPK_K(flags) best logits
  // (value, index) to logits16 as float2 [n_vt][R][K] instead of fp32 logits
  VF_TOPK = 32
};

}  // namespace cst
