// Recurrent half of the LSTM step as a device function, so it can ride in
// the same launch as the vocabulary projection of the previous step:
//
//   pre_{t+1}[r][n] = sum_k h_t[r][k] W_hh[n][k] + vgate[r / vdiv][n]
//
// (packed gate order, fp32 accumulation; fp32 out, or fp16 with PH: the
// combine reads half the bytes -- pre-activations are O(1), fp16 keeps 11
// significant bits where the saved gates and h are bf16).  With temporal attention the weight operand
// carries NQ = A extra rows (W_q): those tiles write the attention query of
// step t+1, q_{t+1} = h_t W_q^T, to q_out instead, and vgate is nullptr (the
// attention kernel adds the per-row video term into pre afterwards).
//  It depends only on h_t, not on the token
// sampled at step t, so it runs CONCURRENTLY with vocab_t; the input-token
// term P[tok_{t+1}] and the cell nonlinearity are applied by the combine
// kernel once the token is known (vocab_combine_kernel's cell epilogue).
#pragma once
#include "gemm_tile.h"
#include "../launchers.h"

namespace cst {

__device__ __forceinline__ int xcd_remap_g(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

constexpr int LG_BM = 128, LG_BN = 64, LG_STAGES = 3;
using LGTile = Tile<LG_BM, LG_BN, LG_STAGES>;
using LGTile2 = Tile<LG_BM, LG_BN, 2>;

__host__ __device__ constexpr int lstm_gemm_blocks(int R, int H, int NQ = 0) {
  return ((4 * H + NQ) / LG_BN) * ((R + LG_BM - 1) / LG_BM);
}

template <class LT = LGTile, bool PH = false>
__device__ __forceinline__ void lstm_gemm_block(int bid, const uint16_t* __restrict__ h, int R,
                                                int H, const uint16_t* __restrict__ whh,
                                                const float* __restrict__ vgate, int vdiv,
                                                float* __restrict__ pre, char* lds,
                                                int NQ = 0, float* __restrict__ q_out = nullptr) {
  const int n_nt = (4 * H + NQ) / LG_BN, n_rt = (R + LG_BM - 1) / LG_BM;
  const int b = xcd_remap_g(bid, n_nt * n_rt);
  const int nt = b / n_rt, rt = b % n_rt;
  const int r0 = rt * LG_BM, n0 = nt * LG_BN;
  const int nk = H / 64;
  f32x16 acc[LT::TM][LT::TN];
  {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    DmaSrc<LG_BM / 32> a;
    DmaSrc<LG_BN / 32> bsrc;
    a.r0 = a.r1 = make_rsrc(h, (int64_t)R * H * 2);
    a.ksplit = nk;
#pragma unroll
    for (int i = 0; i < LG_BM / 32; ++i) {
      const int row = dma_row(w, i, lane);
      a.voff0[i] = min(r0 + row, R - 1) * H * 2 + dma_chunk(row, lane) * 16;
      a.voff1[i] = a.voff0[i];
    }
    bsrc.r0 = bsrc.r1 = make_rsrc(whh, (int64_t)(4 * H + NQ) * H * 2);
    bsrc.ksplit = nk;
#pragma unroll
    for (int i = 0; i < LG_BN / 32; ++i) {
      const int row = dma_row(w, i, lane);
      bsrc.voff0[i] = (n0 + row) * H * 2 + dma_chunk(row, lane) * 16;
      bsrc.voff1[i] = bsrc.voff0[i];
    }
    gemm_nt_mainloop<LT>(nk, a, bsrc, lds, acc);
  }
  float* C = reinterpret_cast<float*>(lds);
  store_acc_to_lds<LT>(acc, C, [](int) { return 0.f; });
  __syncthreads();
  // 16 lanes per row x 4 columns: 256-byte coalesced fp32 rows
  const int u = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const bool qtile = n0 >= 4 * H;
#pragma unroll 4
  for (int i = 0; i < LG_BM / 16; ++i) {
    const int row = rg + 16 * i, r = r0 + row;
    if (r < R) {
      const float4 x = *reinterpret_cast<const float4*>(C + row * LT::CSTRIDE + 4 * u);
      if (qtile) {
        *reinterpret_cast<float4*>(q_out + (int64_t)r * NQ + (n0 - 4 * H) + 4 * u) = x;
      } else if (vgate != nullptr) {
        const float4 vg =
            *reinterpret_cast<const float4*>(vgate + (int64_t)(r / vdiv) * (4 * H) + n0 + 4 * u);
        if (PH)
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(pre) + (int64_t)r * (4 * H) + n0 +
                                    4 * u) = pack_h4(x.x + vg.x, x.y + vg.y, x.z + vg.z, x.w + vg.w);
        else
          *reinterpret_cast<float4*>(pre + (int64_t)r * (4 * H) + n0 + 4 * u) =
              make_float4(x.x + vg.x, x.y + vg.y, x.z + vg.z, x.w + vg.w);
      } else if (PH) {
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(pre) + (int64_t)r * (4 * H) + n0 +
                                  4 * u) = pack_h4(x.x, x.y, x.z, x.w);
      } else {
        *reinterpret_cast<float4*>(pre + (int64_t)r * (4 * H) + n0 + 4 * u) = x;
      }
    }
  }
}

// The whole LSTM step of one tile (recurrent GEMM + the cell), for the XE
// all-rows forward (engine.cpp): with teacher forcing the input token of step
// t+1 is its label, known before the vocabulary projection of step t, so the
// cell needs no combine and the step rides in the decode launch of the
// previous step's vocabulary tiles.  gates = h_t W_hh^T + vgate + P[tok] ->
// cell -> c, h, dropout(h), saved gates: the epilogue of lstm.hip
// lstm_step_fwd_kernel on the lstm_gemm_block tiles (its operands gathered
// before the main loop, so their latency hides under the GEMM).
// (XeCell: launchers.h)
template <class LT>
__device__ __forceinline__ void lstm_cell_block(int bid, const uint16_t* __restrict__ h, int R,
                                                int H, const uint16_t* __restrict__ whh,
                                                const float* __restrict__ vgate, int vdiv,
                                                const XeCell& xc, const uint32_t* __restrict__ rng,
                                                char* lds) {
  const int n_nt = (4 * H) / LG_BN, n_rt = (R + LG_BM - 1) / LG_BM;
  const int b = xcd_remap_g(bid, n_nt * n_rt);
  const int nt = b / n_rt, rt = b % n_rt;
  const int r0 = rt * LG_BM, n0 = nt * LG_BN;
  const int nk = H / 64;
  const int u = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int hu = nt * 16 + u;  // hidden unit of the lane's 4 packed gates
  constexpr int RPT = LG_BM / 16;
  float4 px[RPT], vg[RPT];
  float cp[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = min(r0 + rg + 16 * i, R - 1);
    const int tk = (int)xc.tok[(int64_t)r * xc.tok_stride];
    px[i] = ld_h4(xc.ptab + (int64_t)tk * (4 * H) + n0 + 4 * u);
    vg[i] = *reinterpret_cast<const float4*>(vgate + (int64_t)(r / vdiv) * (4 * H) + n0 + 4 * u);
    cp[i] = xc.c_prev[(int64_t)r * H + hu];
  }
  f32x16 acc[LT::TM][LT::TN];
  {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    DmaSrc<LG_BM / 32> a;
    DmaSrc<LG_BN / 32> bsrc;
    a.r0 = a.r1 = make_rsrc(h, (int64_t)R * H * 2);
    a.ksplit = nk;
#pragma unroll
    for (int i = 0; i < LG_BM / 32; ++i) {
      const int row = dma_row(w, i, lane);
      a.voff0[i] = min(r0 + row, R - 1) * H * 2 + dma_chunk(row, lane) * 16;
      a.voff1[i] = a.voff0[i];
    }
    bsrc.r0 = bsrc.r1 = make_rsrc(whh, (int64_t)4 * H * H * 2);
    bsrc.ksplit = nk;
#pragma unroll
    for (int i = 0; i < LG_BN / 32; ++i) {
      const int row = dma_row(w, i, lane);
      bsrc.voff0[i] = (n0 + row) * H * 2 + dma_chunk(row, lane) * 16;
      bsrc.voff1[i] = bsrc.voff0[i];
    }
    gemm_nt_mainloop<LT>(nk, a, bsrc, lds, acc);
  }
  float* C = reinterpret_cast<float*>(lds);
  store_acc_to_lds<LT>(acc, C, [](int) { return 0.f; });
  __syncthreads();
  const float inv_keep = xc.drop_p > 0.f ? 1.f / (1.f - xc.drop_p) : 1.f;
  const uint32_t seed = rng_seed(rng, RNG_SLOT_DROPOUT);
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int row = rg + 16 * i, r = r0 + row;
    if (r < R) {
      const float4 x = *reinterpret_cast<const float4*>(C + row * LT::CSTRIDE + 4 * u);
      const CellFwd cf = cell_fwd(xc.cell, x.x + vg[i].x + px[i].x, x.y + vg[i].y + px[i].y,
                                  x.z + vg[i].z + px[i].z, x.w + vg[i].w + px[i].w, cp[i]);
      const int64_t o = (int64_t)r * H + hu;
      xc.c_out[o] = cf.c;
      xc.h_out[o] = f2bf(cf.h);
      const bool keep = xc.drop_p <= 0.f || dropout_keep(seed, xc.key, r, hu, xc.drop_p);
      xc.hd_out[o] = f2bf(keep ? cf.h * inv_keep : 0.f);
      uint2 pk;
      pk.x = (uint32_t)f2bf(cf.s0) | ((uint32_t)f2bf(cf.s1) << 16);
      pk.y = (uint32_t)f2bf(cf.s2) | ((uint32_t)f2bf(cf.s3) << 16);
      *reinterpret_cast<uint2*>(xc.gates_out + (int64_t)r * 4 * H + n0 + 4 * u) = pk;
    }
  }
}

}  // namespace cst
