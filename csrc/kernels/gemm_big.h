// 256 x 256 MFMA "NT" tile for the decode-step launch (vocab.hip big path):
//
//   C[m][n] = sum_k A[m][k] * B[n][k]      (A, B rows K-contiguous, bf16)
//
// 512 threads = 8 wavefronts in a 2 (M) x 4 (N) grid, each owning a 128 x 64
// sub-tile (4 x 2 v_mfma_f32_32x32x16_bf16 accumulators, 128 VGPRs); K staged
// 32 deep by LDS-DMA (buffer_load ... lds, 16 B per lane) into four 32 KB
// stages, three K-tiles in flight while one is multiplied, ONE raw barrier
// per K-tile.  (Two 64-deep stages, one K-tile in flight: 13.8 us for the
// main loop at the headline shape, 1.7 us per K-tile, latency-bound.)
//
// Why this tile for the decode step: the 128 x 64 tiles of gemm_tile.h
// (3 workgroups per CU, 1,660 tiles at R = 1,280, V = 10,509) pull 319 MB per
// step from L2 into the CUs, ~1.25 MB per CU -- the measured bound of that
// launch (~70 GB/s per CU).  256 x 256 tiles, one workgroup per CU and ONE
// round (205 vocabulary + 40 recurrent tiles on 256 CUs), pull 125 MB, and
// every tile's A and B operands are reused 256 times instead of 64 / 128.
#pragma once
#include "gemm_tile.h"

namespace cst {

struct BigTile {
  static constexpr int BM = 256, BN = 256, BK = 32, THREADS = 512, NW = 8;
  static constexpr int WAVES_N = 4, WM = 128, WN = 64, TM = WM / 32, TN = WN / 32;
  static constexpr int ROWB = BK * 2;  // bytes per staged row (64)
  static constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB;
  static constexpr int STAGE_BYTES = A_BYTES + B_BYTES;  // 32 KB
  static constexpr int STAGES = 4;                       // 3 K-tiles in flight
  static constexpr int LDS_BYTES = STAGES * STAGE_BYTES;  // 128 KB
  // one DMA wave-instruction = 64 lanes x 16 B = 16 rows of 64 B; 8 waves ->
  // 128 rows per round
  static constexpr int NA = BM / (16 * NW), NB = BN / (16 * NW);
  static constexpr int NI = NA + NB;  // DMA instructions per wave and K-tile
};

// 64-byte LDS rows (4 chunks of 16 B), chunk XOR-swizzled by (row >> 2) & 3:
// the 16-lane groups of a ds_read_b128 over 16 consecutive rows at one
// logical chunk then hit 16 distinct bank slots
__device__ __forceinline__ int big_swz(int row, int chunk) {
  return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4);
}
// tile row / physical chunk filled by lane `lane` of DMA instruction i of
// wave w (LDS bytes base + 16 lane); the SOURCE chunk is the logical one
__device__ __forceinline__ int big_dma_row(int w, int i, int lane) {
  return 16 * (w + BigTile::NW * i) + (lane >> 2);
}
__device__ __forceinline__ int big_dma_chunk(int row, int lane) {
  return (lane & 3) ^ ((row >> 2) & 3);
}

// Main loop: acc[i][j] (i < TM, j < TN) of wave (wr, wc) = (w / 4, w % 4)
// holds C rows wr * 128 + 32 i + .., columns wc * 64 + 32 j + ..
// (v_mfma_f32_32x32x16_bf16 output layout).  a / b: per-lane DMA byte
// offsets of the tile's rows (K-tile advance through the scalar offset).
// Pipeline: STAGES LDS buffers, STAGES - 1 K-tiles in flight; per K-tile a
// counted vmcnt (this wave's copy of tile kt landed, later ones stay in
// flight), ONE raw barrier (every wave's copy landed, every wave done with
// kt - 1), the refill of kt - 1's buffer with tile kt + STAGES - 1, then the
// MFMAs of tile kt.
__device__ __forceinline__ void big_mainloop(int nk, const DmaSrc<BigTile::NA>& a,
                                             const DmaSrc<BigTile::NB>& b, char* lds,
                                             f32x16 (&acc)[BigTile::TM][BigTile::TN]) {
  using T = BigTile;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wr = w / T::WAVES_N, wc = w % T::WAVES_N;
#pragma unroll
  for (int i = 0; i < T::TM; ++i)
#pragma unroll
    for (int j = 0; j < T::TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  auto issue = [&](int buf, int kt) {
    char* A = lds + buf * T::STAGE_BYTES;
    char* B = A + T::A_BYTES;
#pragma unroll
    for (int i = 0; i < T::NA; ++i)
      glds16(a.r0, a.voff0[i], kt * T::ROWB, A + 1024 * (w + T::NW * i));
#pragma unroll
    for (int i = 0; i < T::NB; ++i)
      glds16(b.r0, b.voff0[i], kt * T::ROWB, B + 1024 * (w + T::NW * i));
  };
#pragma unroll
  for (int p = 0; p < T::STAGES - 1; ++p)
    if (p < nk) issue(p, p);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 2 < nk) {
      wait_vmcnt<T::NI * 2>();
    } else if (kt + 1 < nk) {
      wait_vmcnt<T::NI>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (kt + T::STAGES - 1 < nk) issue((kt + T::STAGES - 1) % T::STAGES, kt + T::STAGES - 1);
    const char* A = lds + (kt % T::STAGES) * T::STAGE_BYTES;
    const char* B = A + T::A_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 2 * s + (lane >> 5);
      bf16x8 af[T::TM], bfr[T::TN];
#pragma unroll
      for (int i = 0; i < T::TM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(A + big_swz(wr * T::WM + i * 32 + (lane & 31), c));
#pragma unroll
      for (int j = 0; j < T::TN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(B + big_swz(wc * T::WN + j * 32 + (lane & 31), c));
#pragma unroll
      for (int i = 0; i < T::TM; ++i)
#pragma unroll
        for (int j = 0; j < T::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // every wave done with the stages (the epilogue reuses the LDS)
}

// DMA sources of a tile: rows [m0, m0 + 256) of A (clamped to rows_a - 1) and
// [n0, n0 + 256) of B (clamped to rows_b - 1), row strides lda / ldb elements
__device__ __forceinline__ void big_sources(const uint16_t* A, int rows_a, int lda, int m0,
                                            const uint16_t* B, int rows_b, int ldb, int n0, int nk,
                                            DmaSrc<BigTile::NA>& a, DmaSrc<BigTile::NB>& b) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  a.r0 = a.r1 = make_rsrc(A, (int64_t)rows_a * lda * 2);
  b.r0 = b.r1 = make_rsrc(B, (int64_t)rows_b * ldb * 2);
  a.ksplit = b.ksplit = nk;
#pragma unroll
  for (int i = 0; i < BigTile::NA; ++i) {
    const int row = big_dma_row(w, i, lane);
    a.voff0[i] = a.voff1[i] = min(m0 + row, rows_a - 1) * lda * 2 + big_dma_chunk(row, lane) * 16;
  }
#pragma unroll
  for (int i = 0; i < BigTile::NB; ++i) {
    const int row = big_dma_row(w, i, lane);
    b.voff0[i] = b.voff1[i] = min(n0 + row, rows_b - 1) * ldb * 2 + big_dma_chunk(row, lane) * 16;
  }
}

}  // namespace cst
