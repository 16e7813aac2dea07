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

template <int BM_, int BN_, int STAGES_ = 2>
struct Tile {
  static constexpr int BM = BM_, BN = BN_, BK = 64, THREADS = 256, STAGES = STAGES_;
  static constexpr int WM = BM / 2, WN = BN / 2;  // per-wave sub-tile
  static constexpr int TM = WM / 32, TN = WN / 32;
  static constexpr int A_CHUNKS = BM * 8 / THREADS;  // 16-byte chunks per thread
  static constexpr int B_CHUNKS = BN * 8 / THREADS;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  static constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int CSTRIDE = BN + 8;  // fp32 C tile row stride (bank-conflict free)
  static constexpr int C_BYTES = BM * CSTRIDE * 4;
  static constexpr int LDS_BYTES =
      (STAGES * STAGE_BYTES > C_BYTES) ? STAGES * STAGE_BYTES : C_BYTES;
  static constexpr int NI = (BM + BN) / 32;  // LDS-DMA wave-instructions per wave per tile
  static_assert(TM >= 1 && TN >= 1, "tile too small");
  static_assert(BM % 32 == 0 && BN % 32 == 0, "glds split: 8 rows per wave-instruction");
};

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// s_waitcnt vmcnt(N) with the other counters left alone (gfx9 encoding:
// vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14]).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, int64_t bytes) {
  const uint32_t n = bytes > 0x7fffffffLL ? 0x7fffffffu : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)n, 0x00020000);
}

// One wave-instruction of LDS-DMA (buffer_load_dwordx4 ... lds): lane l moves
// the 16 bytes at base + voff(l) + soff to LDS (wave-uniform dst) + 16 * l.
// The per-lane offset is computed once per kernel; the K-tile advance is the
// scalar soff, so the steady-state loop issues almost no VALU.
__device__ __forceinline__ void glds16(rsrc_t r, int voff, int soff, char* lds_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds_base, 16, voff, soff, 0, 0);
}

// Tile row / 16-byte chunk that lane `lane` of LDS-DMA instruction i of wave w
// fills.  One instruction fills 1 KiB = 8 tile rows; lane l writes LDS byte
// 16*l of it, i.e. row 8j + l/8 and *physical* chunk l%8, so the XOR swizzle
// is applied to the SOURCE (logical chunk = physical ^ ((row >> 1) & 7)) and
// undone by the same XOR on the ds_read.
__device__ __forceinline__ int dma_row(int w, int i, int lane) { return 8 * (w + 4 * i) + (lane >> 3); }
__device__ __forceinline__ int dma_chunk(int row, int lane) { return (lane & 7) ^ ((row >> 1) & 7); }

// Operand source of the main loop: K-tiles [0, ksplit) come from buffer 0,
// [ksplit, nk) from buffer 1 (the LSTM's [embedding rows ; h rows] operand);
// voff0/voff1 are per-lane byte offsets of each DMA instruction's row+chunk.
template <int NINS>
struct DmaSrc {
  rsrc_t r0, r1;
  int voff0[NINS], voff1[NINS];
  int ksplit;
};

// tid: thread index within the 256-thread group that owns this main loop
// (a block may run several groups on disjoint LDS, e.g. an in-block split-K;
// every group must run the same number of K-tiles: the barriers are
// block-wide).
template <class TL>
__device__ __forceinline__ void gemm_nt_mainloop_g(int tid, int nk, const DmaSrc<TL::BM / 32>& a,
                                                   const DmaSrc<TL::BN / 32>& b, char* lds,
                                                   f32x16 (&acc)[TL::TM][TL::TN]) {
  const int lane = tid & 63;
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
    if (kt < a.ksplit) {
#pragma unroll
      for (int i = 0; i < TL::BM / 32; ++i) glds16(a.r0, a.voff0[i], kt * 128, A + 1024 * (w + 4 * i));
    } else {
#pragma unroll
      for (int i = 0; i < TL::BM / 32; ++i)
        glds16(a.r1, a.voff1[i], (kt - a.ksplit) * 128, A + 1024 * (w + 4 * i));
    }
#pragma unroll
    for (int i = 0; i < TL::BN / 32; ++i) glds16(b.r0, b.voff0[i], kt * 128, B + 1024 * (w + 4 * i));
  };

  // Pipeline: STAGES LDS buffers, STAGES-1 tiles in flight.  Each iteration:
  //   wait for this wave's copy of tile kt (counted vmcnt: later tiles stay in
  //   flight), raw s_barrier (every wave's copy landed AND every wave is done
  //   with tile kt-1), refill tile kt-1's buffer with tile kt+STAGES-1, compute
  //   tile kt.  A raw barrier, not __syncthreads(): the latter's fence would
  //   drain vmcnt to 0 and serialise the pipeline.
#pragma unroll
  for (int p = 0; p < TL::STAGES - 1; ++p)
    if (p < nk) issue(p, p);
  for (int kt = 0; kt < nk; ++kt) {
    if (TL::STAGES > 2 && kt + 1 < nk) {
      wait_vmcnt<TL::NI * (TL::STAGES - 2)>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (kt + TL::STAGES - 1 < nk) issue((kt + TL::STAGES - 1) % TL::STAGES, kt + TL::STAGES - 1);
    const char* A = lds + (kt % TL::STAGES) * TL::STAGE_BYTES;
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
  }
  __syncthreads();  // all waves done with the staging buffers (epilogue reuses LDS)
}

template <class TL>
__device__ __forceinline__ void gemm_nt_mainloop(int nk, const DmaSrc<TL::BM / 32>& a,
                                                 const DmaSrc<TL::BN / 32>& b, char* lds,
                                                 f32x16 (&acc)[TL::TM][TL::TN]) {
  gemm_nt_mainloop_g<TL>((int)threadIdx.x, nk, a, b, lds, acc);
}

// Accumulators -> fp32 C tile in LDS (row stride TL::CSTRIDE), adding colbias(col).
template <class TL, class ColBias>
__device__ __forceinline__ void store_acc_to_lds(const f32x16 (&acc)[TL::TM][TL::TN],
                                                 float* C, ColBias colbias,
                                                 int tid = -1) {
  if (tid < 0) tid = (int)threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
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
