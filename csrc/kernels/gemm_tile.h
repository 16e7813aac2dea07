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
// buffered: the next K-tile's global loads are issued before the current
// tile's MFMAs and written to the other LDS buffer after them, so HBM/L2
// latency hides under the matrix work and there is ONE barrier per K-tile.
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
  static_assert(BM * 8 % THREADS == 0 && BN * 8 % THREADS == 0, "chunk split");
};

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

// ARow(row, kt) / BRow(row, kt): pointer to the 64 bf16 of K-tile kt of that
// tile row (callers clamp out-of-range rows to a valid row).
template <class TL, class ARow, class BRow, class AHook>
__device__ __forceinline__ void gemm_nt_mainloop(int nk, ARow arow, BRow brow, AHook ahook,
                                                 char* lds, f32x16 (&acc)[TL::TM][TL::TN]) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  uint4 ra[TL::A_CHUNKS], rb[TL::B_CHUNKS];

#pragma unroll
  for (int i = 0; i < TL::TM; ++i)
#pragma unroll
    for (int j = 0; j < TL::TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < TL::A_CHUNKS; ++i) {
      const int idx = tid + i * TL::THREADS, row = idx >> 3, c = idx & 7;
      ra[i] = *reinterpret_cast<const uint4*>(arow(row, kt) + c * 8);
    }
#pragma unroll
    for (int i = 0; i < TL::B_CHUNKS; ++i) {
      const int idx = tid + i * TL::THREADS, row = idx >> 3, c = idx & 7;
      rb[i] = *reinterpret_cast<const uint4*>(brow(row, kt) + c * 8);
    }
  };
  auto lstore = [&](int buf, int kt) {
    char* A = lds + buf * TL::STAGE_BYTES;
    char* B = A + TL::A_BYTES;
#pragma unroll
    for (int i = 0; i < TL::A_CHUNKS; ++i) {
      const int idx = tid + i * TL::THREADS, row = idx >> 3, c = idx & 7;
      *reinterpret_cast<uint4*>(A + swz(row, c)) = ra[i];
      ahook(row, kt, c, ra[i]);
    }
#pragma unroll
    for (int i = 0; i < TL::B_CHUNKS; ++i) {
      const int idx = tid + i * TL::THREADS, row = idx >> 3, c = idx & 7;
      *reinterpret_cast<uint4*>(B + swz(row, c)) = rb[i];
    }
  };

  gload(0);
  lstore(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
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
    if (kt + 1 < nk) lstore(cur ^ 1, kt + 1);
    __syncthreads();
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
