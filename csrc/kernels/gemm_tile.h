// MFMA "NT" GEMM main loop for gfx950, shared by the fused decoder kernels.
//
//   C[m][n] = sum_k A[m][k] * B[n][k]     (A rows and B rows both K-contiguous)
//
// which is exactly the layout of every decoder product: activations (rows x K)
// times a PyTorch weight stored (out_features x in_features).  With both
// operands K-contiguous, one 16-byte load per lane feeds one
// v_mfma_f32_32x32x16_bf16 operand fragment (lane l: row l&31, k 8*(l>>5)..+7).
//
// Geometry: 256 threads = 4 wavefronts in a 2x2 grid; block tile BM x BN,
// K staged 64 at a time (one 128-byte row per tile row) through LDS, double
// buffered: the next K-tile's LDS-DMA loads are issued before the current
// tile's MFMAs, so HBM/L2 latency hides under the matrix work, and there is
// ONE barrier per K-tile.
// LDS rows are 16-byte-chunk XOR-swizzled (chunk ^ ((row >> 1) & 7)) so the
// 16-lane groups of ds_read_b128 hit 16 distinct bank slots.
//
// Row gathers are free: the A row pointer comes from a functor, so the LSTM
// kernel reads embedding rows by token id and h rows in the same pipeline.
#pragma once
#include "../common.h"

namespace cst {

template <int BM_, int BN_>
struct Tile {
  static constexpr int BM = BM_, BN = BN_, BK = 64, THREADS = 256;
  static constexpr int WM = BM / 2, WN = BN / 2;  // per-wave sub-tile
  static constexpr int TM = WM / 32, TN = WN / 32;
  static constexpr int A_CHUNKS = BM * 8 / THREADS;  // 16-byte chunks per thread
  static constexpr int B_CHUNKS = BN * 8 / THREADS;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  static constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int CSTRIDE = BN + 8;  // fp32 C tile row stride (bank-conflict free)
  static constexpr int C_BYTES = BM * CSTRIDE * 4;
  static constexpr int LDS_BYTES = (2 * STAGE_BYTES > C_BYTES) ? 2 * STAGE_BYTES : C_BYTES;
  static_assert(TM >= 1 && TN >= 1, "tile too small");
  static_assert(BM % 32 == 0 && BN % 32 == 0, "glds split: 8 rows per wave-instruction");
};

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) const void* gbl_ptr_t;

// One wave-instruction of LDS-DMA: each lane moves 16 bytes from its own
// global address to (wave-uniform base + 16 * lane).
__device__ __forceinline__ void glds16(const void* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)lds_base, 16, 0, 0);
}

// ARow(row, kt) / BRow(row, kt): pointer to the 64 bf16 of K-tile kt of that
// tile row (callers clamp out-of-range rows to a valid row).
//
// Staging is global -> LDS direct (global_load_lds_dwordx4): no staging
// registers at all.  One wave-instruction fills 1 KiB = 8 tile rows; lane l
// writes LDS byte 16*l of it, i.e. row 8j + l/8 and *physical* chunk l%8, so
// the XOR swizzle is applied to the SOURCE address (logical chunk =
// physical ^ ((row >> 1) & 7)) and undone by the same XOR on the ds_read.
template <class TL, class ARow, class BRow>
__device__ __forceinline__ void gemm_nt_mainloop(int nk, ARow arow, BRow brow, char* lds,
                                                 f32x16 (&acc)[TL::TM][TL::TN]) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;

#pragma unroll
  for (int i = 0; i < TL::TM; ++i)
#pragma unroll
    for (int j = 0; j < TL::TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto issue = [&](int buf, int kt) {
    char* A = lds + buf * TL::STAGE_BYTES;
    char* B = A + TL::A_BYTES;
#pragma unroll
    for (int i = 0; i < TL::BM / 32; ++i) {
      const int j = w + 4 * i, row = 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      glds16(arow(row, kt) + c * 8, A + 1024 * j);
    }
#pragma unroll
    for (int i = 0; i < TL::BN / 32; ++i) {
      const int j = w + 4 * i, row = 8 * j + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      glds16(brow(row, kt) + c * 8, B + 1024 * j);
    }
  };

  issue(0, 0);
  __syncthreads();  // vmcnt(0) + barrier: tile 0 landed
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) issue(cur ^ 1, kt + 1);  // in flight during this tile's MFMAs
    const char* A = lds + cur * TL::STAGE_BYTES;
    const char* B = A + TL::A_BYTES;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int c = 2 * s + (lane >> 5);
      bf16x8 af[TL::TM], bfr[TL::TN];
#pragma unroll
      for (int i = 0; i < TL::TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(A + swz(wr * TL::WM + i * 32 + (lane & 31), c));
#pragma unroll
      for (int j = 0; j < TL::TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(B + swz(wc * TL::WN + j * 32 + (lane & 31), c));
#pragma unroll
      for (int i = 0; i < TL::TM; ++i)
#pragma unroll
        for (int j = 0; j < TL::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();  // vmcnt(0) + barrier: next tile landed, this one free
  }
}

// Accumulators -> fp32 C tile in LDS (row stride TL::CSTRIDE), adding colbias(col).
template <class TL, class ColBias>
__device__ __forceinline__ void store_acc_to_lds(const f32x16 (&acc)[TL::TM][TL::TN],
                                                 float* C, ColBias colbias) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1;
#pragma unroll
  for (int j = 0; j < TL::TN; ++j) {
    const int col = wc * TL::WN + j * 32 + (lane & 31);
    const float b = colbias(col);
#pragma unroll
    for (int i = 0; i < TL::TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wr * TL::WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        C[row * TL::CSTRIDE + col] = acc[i][j][r] + b;
      }
    }
  }
}

}  // namespace cst
