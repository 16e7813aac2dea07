// K1/K9: fused LSTM decode step (embedding gather + gate GEMM + cell) and
// the per-step cell backward.
//
// Reference per decode step (/root/reference/model.py:271-278, 93-116):
// embed(it) -> cat([x, fc_feats]) -> cuDNN LSTM (bias=False, gate order
// i,f,g,o) with input size E + F*H = 2560.
//
// MI355X design:
//   * the video part W_ih[:, E:] . v is constant over time and identical for
//     the seq_per_img rows of a video, so it is computed ONCE per video by the
//     caller (vgate, B x 4H) and added in the epilogue, and the 20x row
//     duplication of FeatExpander (model.py:84-86) disappears;
//   * gate rows are packed so that one 64-column tile holds 16 hidden units x
//     4 gates (packed row 4u+g <- original row g*H+u): the whole cell update
//     happens in the GEMM epilogue, nothing but h/c leaves the kernel;
//   * the input-token term W_ie . emb[tok] is a row of the table
//     P = emb . W_ie^T (V x 4H, refreshed once per optimizer step by one
//     hipBLASLt GEMM), gathered in the epilogue, so the per-step GEMM is only
//     h_{t-1} . W_hh^T (K = H);
//   * training mode also emits, for the backward: post-activation gates, c_t,
//     h_t, and h after dropout (the input of the vocabulary projection; mask
//     from the mix32 counter hash dropout_keep(), regenerated in backward).
#include "gemm_tile.h"
#include "../launchers.h"

namespace cst {

constexpr int LB_M = 128, LB_N = 64;
// backward step pipeline depth per K group (48 KB of LDS each; 6 stages
// measured no faster)
constexpr int LSTM_BWD_STAGES = 3;

__device__ __forceinline__ int xcd_remap_l(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

template <int BM, int STAGES>
__global__ __launch_bounds__(256, 2) void lstm_step_fwd_kernel(
    const int64_t* __restrict__ tok, int64_t tok_stride, const uint16_t* __restrict__ ptab,
    const uint16_t* __restrict__ h_prev, const float* __restrict__ c_prev,
    const float* __restrict__ vgate, int vgate_div, int R, int H,
    const uint16_t* __restrict__ whh, uint16_t* __restrict__ h_out, float* __restrict__ c_out,
    uint16_t* __restrict__ hdrop_out, int ldh, float drop_p, const uint32_t* __restrict__ rng,
    int step, uint16_t* __restrict__ gates_out, const int* __restrict__ row_map, int cell) {
  using LTile = Tile<BM, LB_N, STAGES>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int n_nt = (4 * H) / LB_N, n_rt = (R + BM - 1) / BM;
  const int b = xcd_remap_l(blockIdx.x, n_nt * n_rt);
  const int nt = b / n_rt, rt = b % n_rt;
  const int r0 = rt * BM, n0 = nt * LB_N;
  const int nk = H / 64;

  // token ids of this row tile (used by the epilogue's table gather; upper
  // layers of a stacked decoder have no token term: tok = ptab = null)
  int* s_tok = reinterpret_cast<int*>(lds + LTile::LDS_BYTES);
  if (threadIdx.x < BM)
    s_tok[threadIdx.x] = tok ? (int)tok[(int64_t)min(r0 + (int)threadIdx.x, R - 1) * tok_stride] : 0;
  __syncthreads();

  // Epilogue operands are gathered BEFORE the main loop, so their latency
  // (random rows of an 86 MB table, video gates, c_{t-1}) hides under the GEMM.
  const int tid = threadIdx.x, u = tid & 15, rg = tid >> 4;
  const int hu = nt * 16 + u;  // global hidden unit
  constexpr int RPT = BM / 16;  // rows per thread
  float4 pre_px[RPT], pre_vg[RPT];
  float pre_c[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int row = rg + 16 * i, r = min(r0 + row, R - 1);
    pre_px[i] = ptab ? ld_h4(ptab + (int64_t)s_tok[row] * (4 * H) + n0 + 4 * u)
                     : make_float4(0.f, 0.f, 0.f, 0.f);
    pre_vg[i] = *reinterpret_cast<const float4*>(vgate + (int64_t)(r / vgate_div) * (4 * H) + n0 + 4 * u);
    pre_c[i] = c_prev ? c_prev[(int64_t)(row_map ? row_map[r] : r) * H + hu] : 0.f;
    CST_DCHECK(s_tok[row] >= 0);
    CST_DCHECK(row_map == nullptr || (row_map[r] >= 0 && row_map[r] < R));
  }

  // h_prev == nullptr: zero initial state (step 0 without an initial state),
  // no recurrent GEMM -- the step is the table gather and the cell
  const bool zero_h = h_prev == nullptr;
  f32x16 acc[LTile::TM][LTile::TN];
  if (!zero_h) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    DmaSrc<BM / 32> a;
    DmaSrc<LB_N / 32> bsrc;
    a.r0 = a.r1 = make_rsrc(h_prev, (int64_t)R * H * 2);
    a.ksplit = nk;
#pragma unroll
    for (int i = 0; i < BM / 32; ++i) {
      const int row = dma_row(w, i, lane);
      const int src = min(r0 + row, R - 1);  // beam search: h of the parent beam
      a.voff0[i] = (row_map ? row_map[src] : src) * H * 2 + dma_chunk(row, lane) * 16;
      a.voff1[i] = a.voff0[i];
    }
    bsrc.r0 = bsrc.r1 = make_rsrc(whh, (int64_t)4 * H * H * 2);
    bsrc.ksplit = nk;
#pragma unroll
    for (int i = 0; i < LB_N / 32; ++i) {
      const int row = dma_row(w, i, lane);
      bsrc.voff0[i] = (n0 + row) * H * 2 + dma_chunk(row, lane) * 16;
      bsrc.voff1[i] = bsrc.voff0[i];
    }
    gemm_nt_mainloop<LTile>(nk, a, bsrc, lds, acc);  // ends with a barrier (s_tok visible)
  }

  float* C = reinterpret_cast<float*>(lds);
  if (!zero_h) {
    store_acc_to_lds<LTile>(acc, C, [](int) { return 0.f; });
    __syncthreads();
  }

  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  const uint32_t seed = rng_seed(rng, RNG_SLOT_DROPOUT);
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int row = rg + 16 * i, r = r0 + row;
    if (r < R) {
      const float4 pre = zero_h ? make_float4(0.f, 0.f, 0.f, 0.f)
                                : *reinterpret_cast<const float4*>(C + row * LTile::CSTRIDE + 4 * u);
      const float4 vg = pre_vg[i], px = pre_px[i];
      const CellFwd cf = cell_fwd(cell, pre.x + vg.x + px.x, pre.y + vg.y + px.y,
                                  pre.z + vg.z + px.z, pre.w + vg.w + px.w, pre_c[i]);
      const int64_t o = (int64_t)r * H + hu;
      const float hv = cf.h;
      c_out[o] = cf.c;
      h_out[o] = f2bf(hv);
      if (hdrop_out) {
        const bool keep = drop_p <= 0.f || dropout_keep(seed, step, r, hu, drop_p);
        hdrop_out[(int64_t)r * ldh + hu] = f2bf(keep ? hv * inv_keep : 0.f);
      }
      if (gates_out) {
        uint2 pk;
        pk.x = (uint32_t)f2bf(cf.s0) | ((uint32_t)f2bf(cf.s1) << 16);
        pk.y = (uint32_t)f2bf(cf.s2) | ((uint32_t)f2bf(cf.s3) << 16);
        *reinterpret_cast<uint2*>(gates_out + (int64_t)r * 4 * H + n0 + 4 * u) = pk;
      }
    }
  }
}

// Fused backward step (replaces cell backward + a separate recurrent GEMM):
//   dh_rec = dG_{t+1} . W_hh            (MFMA, K = 4H, B operand W_hh^T)
//   dh     = dh_rec + mask * dh_logit / (1 - p)
//   cell backward of step t in the epilogue -> dG_t (bf16, packed gates),
//   dc_carry <- dc * f.
// One tile = BM rows x 64 hidden units: only (R/BM) x (H/64) = 160 tiles at
// R = 1280, H = 512 -- fewer than the 256 CUs, each a 32-deep K loop (the
// reverse loop is latency-bound).  So each block runs GROUPS = 2 groups of 4
// waves that split the tile's K range (in-block split-K): both groups stream
// their half of K through their own LDS pipeline, leave their fp32 partial
// tiles in LDS, and all 8 waves run the cell epilogue on the sum.  No global
// workspace, no atomics, and every epilogue operand is prefetched before the
// main loop.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// butterfly all-reduce of N per-lane values over 64 lanes: N - 1 shuffles,
// afterwards lane l holds the total of value index l (N = 64) in v[0]
template <int N, int M>
struct Bfly2 {
  static __device__ __forceinline__ void run(float* v, int lane) {
    constexpr int Hh = N / 2;
    const bool up = (lane & M) != 0;
#pragma unroll
    for (int i = 0; i < Hh; ++i) {
      const float send = up ? v[i] : v[i + Hh];
      const float keep = up ? v[i + Hh] : v[i];
      v[i] = keep + __shfl_xor(send, M, WAVE);
    }
    Bfly2<Hh, M / 2>::run(v, lane);
  }
};
template <>
struct Bfly2<1, 0> {
  static __device__ __forceinline__ void run(float*, int) {}
};

template <int BM, int GROUPS>
__device__ __forceinline__ void lstm_bwd_load_epi(int r0, int R, int H, int rg, int hu,
                                                  const uint16_t* __restrict__ gates,
                                                  const float* __restrict__ c_t,
                                                  const float* __restrict__ c_prev,
                                                  const float* __restrict__ dc_carry,
                                                  const float* __restrict__ dh_logit,
                                                  const float* __restrict__ dh_scale,
                                                  const DhOneHot& oh, uint2* pg, float* pc,
                                                  float* pcp, float* pdc, float* pdl) {
  constexpr int RG = 4 * GROUPS, RPT = BM / RG;
  // Branch-free: every load of the batch is issued back to back (a load under
  // a per-element null test becomes a branch with its own vmcnt(0) wait, one
  // dependent round trip per element); absent operands read a stand-in
  // pointer and are replaced afterwards (wave-uniform selects)
  const float* cpv = c_prev != nullptr ? c_prev : c_t;
  const float* dsv = dh_scale != nullptr ? dh_scale : dh_logit;
  float psc[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = min(r0 + rg + RG * i, R - 1);
    const int64_t o = (int64_t)r * H + hu;
    pg[i] = *reinterpret_cast<const uint2*>(gates + (int64_t)r * 4 * H + 4 * hu);
    pc[i] = c_t[o];
    pcp[i] = cpv[o];
    pdc[i] = dc_carry[o];
    pdl[i] = dh_logit[o];
    psc[i] = dsv[r];
  }
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    pcp[i] = c_prev != nullptr ? pcp[i] : 0.f;
    pdl[i] *= dh_scale != nullptr ? psc[i] : 1.f;
  }
  // forward-computed X = E W: the one-hot terms a W[ys] + b W[yx] of the row
  // (uniform branches; the token rows are gathered with the other operands)
  if (oh.a != nullptr) {
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = min(r0 + rg + RG * i, R - 1);
      const int y = oh.ys[r];
      pdl[i] = fmaf(oh.a[r], bf2f(oh.W[(int64_t)max(y, 0) * H + hu]), pdl[i]);
    }
  }
  if (oh.b != nullptr) {
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = min(r0 + rg + RG * i, R - 1);
      const int y = oh.yx[r];
      pdl[i] = fmaf(oh.b[r], bf2f(oh.W[(int64_t)max(y, 0) * H + hu]), pdl[i]);
    }
  }
}

// Attention epilogue (ATT): the tile's rows span the videos
// [r0 / vdiv, (r0 + BM - 1) / vdiv]; their gate-table slices for the tile's
// 64 hidden units (64 units x CP frames x 4 gates, bf16, 4 KB per video at
// CP = 8, layout gvb16[v][u][c][g]) are requested before the main loop and
// parked in LDS behind the C tiles; each thread forms
// sum_g dG[r][4u + g] Gv[v][u][c][g] for its rows with two v_dot2c_f32_bf16
// per frame on the bf16 gate-gradient pairs it has just packed, and a
// butterfly over the 64 units of the wave finishes the tile's partial.
constexpr int ATT_EPI_PF = 5;  // 16-byte slice chunks per thread
__host__ __device__ constexpr int att_epi_videos(int vdiv) { return (62 + vdiv) / vdiv + 1; }

bool att_bwd_epi_ok(int vdiv, int C, int H) {
  const int CP = C <= 8 ? 8 : 16;
  const int nv = att_epi_videos(vdiv);
  // slice chunks (16 B) of the block: nv x 64 units x 4 gates x CP x 2 B
  return C <= 16 && vdiv >= 2 && H % 64 == 0 && nv * 64 * 4 * CP * 2 <= ATT_EPI_PF * 512 * 16 &&
         2 * 64 * 72 * 4 + nv * 64 * 4 * CP * 2 <= 2 * LSTM_BWD_STAGES * 16384;
}

// Fused attention backward (AttBwdEpi::flags): one 512-thread workgroup per
// video, thread = (4 query units, row group of 4): A <= 512, rows <= 32.  The
// K-tiles of the launch's GEMM are reordered per group: group g streams its
// half of the dG_{t+1} tiles, then its half of the A / 64 tail tiles, so both
// groups reach the tail (dq_{t+1}, produced by the attention workgroups of the
// SAME launch) last.
constexpr int ATTF_MAXR = 32, ATTF_RG = 4;
bool att_bwd_fuse_ok(int vdiv, int C, int A, int H, int Bv, int R) {
  const int CP = C <= 8 ? 8 : 16;
  return att_bwd_epi_ok(vdiv, C, H) && vdiv <= ATTF_MAXR && vdiv * CP <= 512 && A % 128 == 0 &&
         A <= 512 && H % 128 == 0 && H / 64 <= 16 && Bv * vdiv == R;
}

typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// The attention workgroup (video b) of step t + 1 (see AttBwdEpi).  The scorer
// values u = tanh(P + q) come from the forward (one fp16 word each, common.h
// u_enc: accurate 1 - u^2 near saturation), so the backward has no
// transcendental:
//   dalpha[r][c] = the sum of the H/64 step-(t+1) partials; softmax backward
//   de = alpha (dalpha - sum_k alpha_k dalpha_k); thread (units 4 cq..4 cq+3,
//   rows rq, rq + 4, ...): dq[r][a] = w_a[a] sum_c de[r][c] (1 - u^2) (4 bf16
//   written through -- sc1 -- into dg_next's tail).  Hand-off to the GEMM
//   workgroups of the launch: every wave drains its stores (vmcnt(0)), a
//   workgroup barrier, then ONE agent-scope add on the video's flag; the
//   readers poll it and load the tail with sc1 loads (the no-fence form of
//   loss.hip / att_mfma.h).  Only then (off the critical path) dP[b][c][a] =
//   sum_r de (1 - u^2) w_a and dw_a = sum_{r, c} de u over the 4 row groups
//   (LDS), db_a by thread 0.  The u loads of the first 16 rows go out first:
//   they depend on nothing, so they overlap the dalpha loads and the softmax.
template <int CP>
__device__ __forceinline__ void att_bwd_fused_wg(const AttBwdEpi& f, int b, int R, int n_ut,
                                                 uint16_t* __restrict__ dgn, int ldg, char* lds) {
  float* s_da = reinterpret_cast<float*>(lds);
  float* s_de = s_da + ATTF_MAXR * CP;
  float* s_red = s_de + ATTF_MAXR * CP;  // (ATTF_RG - 1) x 128 x (8 frames x 4 + 4)
  const int tid = threadIdx.x, vdiv = f.vdiv, C = f.C, A = f.A;
  const int row0 = b * vdiv, nrc = vdiv * CP;
  const int cq = tid & 127, rq = tid >> 7;  // (rq is wave-uniform)
  const bool acol = 4 * cq < A;
  const int a = min(4 * cq, A - 4);
  constexpr int RB = 4;  // rows per batch and thread
  auto u_batch = [&](int i0, uint2 (&u)[RB][CP]) {
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int k = min(rq + ATTF_RG * (i0 + i), vdiv - 1);
#pragma unroll
      for (int c = 0; c < CP; ++c)
        u[i][c] = *reinterpret_cast<const uint2*>(f.u + ((int64_t)(row0 + k) * C + min(c, C - 1)) * A + a);
    }
  };
  uint2 ub[RB][CP];
  u_batch(0, ub);
  float dsum = 0.f;
  {
    const int rc = min(tid, nrc - 1);
    const float* pp = f.dal_next + (int64_t)row0 * CP + rc;
    float x[16];
#pragma unroll
    for (int ut = 0; ut < 16; ++ut) x[ut] = pp[(int64_t)min(ut, n_ut - 1) * R * CP];
#pragma unroll
    for (int ut = 0; ut < 16; ++ut) dsum += ut < n_ut ? x[ut] : 0.f;
  }
  const float4 wa4 = *reinterpret_cast<const float4*>(f.wa + a);
  const f32x2_t wa01 = {wa4.x, wa4.y}, wa23 = {wa4.z, wa4.w};
  float alr[CP];
  {
    const int rr = min(tid, vdiv - 1);
#pragma unroll
    for (int c = 0; c < CP; ++c) alr[c] = f.alpha[(int64_t)(row0 + rr) * C + min(c, C - 1)];
#pragma unroll
    for (int c = 0; c < CP; ++c) alr[c] = c < C ? alr[c] : 0.f;
  }
  if (tid < nrc) s_da[tid] = dsum;
  __syncthreads();
  if (tid < vdiv) {
    float sa = 0.f;
#pragma unroll
    for (int c = 0; c < CP; ++c) sa += alr[c] * s_da[tid * CP + c];
#pragma unroll
    for (int c = 0; c < CP; ++c) s_de[tid * CP + c] = alr[c] * (s_da[tid * CP + c] - sa);
  }
  __syncthreads();
  // dq rows of this thread; dP / dw_a contributions kept in registers
  f32x2_t dp[CP][2], dw[2];
#pragma unroll
  for (int c = 0; c < CP; ++c) dp[c][0] = dp[c][1] = f32x2_t{0.f, 0.f};
  dw[0] = dw[1] = f32x2_t{0.f, 0.f};
  auto rows = [&](int i0, const uint2 (&u)[RB][CP]) {
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int k = rq + ATTF_RG * (i0 + i);
      if (k < vdiv) {  // (wave-uniform)
        f32x2_t dq01 = {0.f, 0.f}, dq23 = {0.f, 0.f};
#pragma unroll
        for (int c = 0; c < CP; ++c) {
          if (c < C) {
            const float de = s_de[k * CP + c];
            const UDec e0 = u_dec(u[i][c].x & 0xffff), e1 = u_dec(u[i][c].x >> 16);
            const UDec e2 = u_dec(u[i][c].y & 0xffff), e3 = u_dec(u[i][c].y >> 16);
            const f32x2_t u01 = {e0.u, e1.u}, u23 = {e2.u, e3.u};
            const f32x2_t de2 = {de, de};
            const f32x2_t g01 = de2 * f32x2_t{e0.d, e1.d}, g23 = de2 * f32x2_t{e2.d, e3.d};
            dq01 += g01;
            dq23 += g23;
            dp[c][0] += g01;
            dp[c][1] += g23;
            dw[0] += de2 * u01;
            dw[1] += de2 * u23;
          }
        }
        dq01 *= wa01;
        dq23 *= wa23;
        if (acol) {
          const uint64_t pk = (uint64_t)((uint32_t)f2bf(dq01.x) | ((uint32_t)f2bf(dq01.y) << 16)) |
                              ((uint64_t)((uint32_t)f2bf(dq23.x) | ((uint32_t)f2bf(dq23.y) << 16))
                               << 32);
          __hip_atomic_store(reinterpret_cast<uint64_t*>(dgn + (int64_t)(row0 + k) * ldg + f.G4 + a),
                             pk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  };
  rows(0, ub);
  if (vdiv > ATTF_RG * RB) {  // rows 16..31
    u_batch(RB, ub);
    rows(RB, ub);
  }
  wait_vmcnt<0>();  // this wave's dq stores are done
  __syncthreads();
  if (tid == 0)
    __hip_atomic_fetch_add(f.flags + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // off the critical path: db_a, then dP / dw_a over the 4 row groups, 8
  // frames per LDS round
  if (tid == 0) {
    float sb = 0.f;
    for (int r = 0; r < vdiv; ++r)
      for (int c = 0; c < C; ++c) sb += s_de[r * CP + c];
    f.dba_part[b] += sb;
  }
  constexpr int RS = 8 * 4 + 4;  // LDS floats per (group, unit quad)
#pragma unroll
  for (int c0 = 0; c0 < CP; c0 += 8) {
    if (rq > 0) {
      float* sr = s_red + ((rq - 1) * 128 + cq) * RS;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        sr[4 * c] = dp[c0 + c][0].x;
        sr[4 * c + 1] = dp[c0 + c][0].y;
        sr[4 * c + 2] = dp[c0 + c][1].x;
        sr[4 * c + 3] = dp[c0 + c][1].y;
      }
      if (c0 == 0) {
        sr[32] = dw[0].x;
        sr[33] = dw[0].y;
        sr[34] = dw[1].x;
        sr[35] = dw[1].y;
      }
    }
    __syncthreads();
    if (rq == 0 && acol) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        if (c0 + c < C) {
          float4 v = make_float4(dp[c0 + c][0].x, dp[c0 + c][0].y, dp[c0 + c][1].x, dp[c0 + c][1].y);
#pragma unroll
          for (int g = 0; g < ATTF_RG - 1; ++g) {
            const float* sr = s_red + (g * 128 + cq) * RS + 4 * c;
            v.x += sr[0];
            v.y += sr[1];
            v.z += sr[2];
            v.w += sr[3];
          }
          float4* dst = reinterpret_cast<float4*>(f.dP_acc + ((int64_t)b * C + c0 + c) * A + a);
          const float4 o = *dst;
          *dst = make_float4(o.x + wa4.x * v.x, o.y + wa4.y * v.y, o.z + wa4.z * v.z,
                             o.w + wa4.w * v.w);
        }
      }
      if (c0 == 0) {
        float4 v = make_float4(dw[0].x, dw[0].y, dw[1].x, dw[1].y);
#pragma unroll
        for (int g = 0; g < ATTF_RG - 1; ++g) {
          const float* sr = s_red + (g * 128 + cq) * RS + 32;
          v.x += sr[0];
          v.y += sr[1];
          v.z += sr[2];
          v.w += sr[3];
        }
        float4* dst = reinterpret_cast<float4*>(f.dwa_part + (int64_t)b * A + a);
        const float4 o = *dst;
        *dst = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
      }
    }
    if (c0 + 8 < CP) __syncthreads();
  }
}

// glds16 with a cache policy (aux 16 = sc1: the load bypasses the non-coherent
// caches -- data written through by another workgroup of the launch)
template <int AUX>
__device__ __forceinline__ void glds16_aux(rsrc_t r, int voff, int soff, char* lds_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds_base, 16, voff, soff, 0, AUX);
}

// Wait (one poll per wave) until the attention workgroups of videos
// [v0, v0 + nv) released their dq rows.  They precede this workgroup in
// dispatch order (lower blockIdx), so they are resident or done; the bound
// only guarantees that every wave exits.
// A wait that runs out of polls counts itself in the device error word
// (poll_err, read by the host after the step: engine.device_errors); the
// gradient of that step is then not trusted (the trainer raises).
__device__ __forceinline__ void att_fuse_wait(const int* flags, int v0, int nv, int bound,
                                              int* err) {
  const int lane = threadIdx.x & 63;
  bool ok = false;
  for (int it = 0; it < bound; ++it) {
    const int f = __hip_atomic_load(flags + v0 + min(lane, nv - 1), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
    if (__all(f > 0)) {
      ok = true;
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  if (!ok && lane == 0 && err != nullptr)
    __hip_atomic_fetch_add(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The step kernel's main loop with the fused attention's ordering: K-tiles
// [0, ksplit) of the group from the primary offsets (dG_{t+1} columns, plain
// loads), [ksplit, nk) from the tail offsets (dq_{t+1} columns) -- issued
// only after att_fuse_wait, with sc1 (write-through data of this launch's
// attention workgroups).  Otherwise as gemm_nt_mainloop_g.
template <class TL, bool GATE>
__device__ __forceinline__ void gemm_bwd_mainloop_tail(int tid, int nk, const DmaSrc<TL::BM / 32>& a,
                                                       const DmaSrc<TL::BN / 32>& b, char* lds,
                                                       f32x16 (&acc)[TL::TM][TL::TN],
                                                       const int* flags, int v0, int nv,
                                                       int bound, int* err) {
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
#pragma unroll
  for (int i = 0; i < TL::TM; ++i)
#pragma unroll
    for (int j = 0; j < TL::TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  bool waited = !GATE;
  auto issue = [&](int buf, int kt) {
    char* A = lds + buf * TL::STAGE_BYTES;
    char* B = A + TL::A_BYTES;
    if (kt < a.ksplit) {
#pragma unroll
      for (int i = 0; i < TL::BM / 32; ++i)
        glds16(a.r0, a.voff0[i], kt * 128, A + 1024 * (w + 4 * i));
#pragma unroll
      for (int i = 0; i < TL::BN / 32; ++i)
        glds16(b.r0, b.voff0[i], kt * 128, B + 1024 * (w + 4 * i));
    } else {
      if (!waited) {
        att_fuse_wait(flags, v0, nv, bound, err);
        waited = true;
      }
      const int ks = (kt - a.ksplit) * 128;
#pragma unroll
      for (int i = 0; i < TL::BM / 32; ++i)
        glds16_aux<GATE ? 16 : 0>(a.r1, a.voff1[i], ks, A + 1024 * (w + 4 * i));  // 16: sc1
#pragma unroll
      for (int i = 0; i < TL::BN / 32; ++i)
        glds16(b.r1, b.voff1[i], ks, B + 1024 * (w + 4 * i));
    }
  };
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
  __syncthreads();
}

template <int BM, int STAGES, int GROUPS, bool ATT, int CP, bool FUSE = false>
__global__ __launch_bounds__(256 * GROUPS) void lstm_step_bwd_kernel(
    const uint16_t* __restrict__ dg_next, const uint16_t* __restrict__ whhT,
    const float* __restrict__ dh_logit, float* __restrict__ dc_carry,
    const uint16_t* __restrict__ gates, const float* __restrict__ c_t,
    const float* __restrict__ c_prev, int R, int H, float drop_p,
    const uint32_t* __restrict__ rng, int step, uint16_t* __restrict__ dG, int KD, int cell,
    const float* __restrict__ dh_scale, AttBwdEpi att, DhOneHot oh, int map_rows) {
  using TL = Tile<BM, 64, STAGES>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int n_ut = H / 64, n_rt = (R + BM - 1) / BM, n_tiles = n_ut * n_rt;
  static_assert(!FUSE || ATT, "the fused attention backward extends the attention epilogue");
  if (FUSE && (int)blockIdx.x < att.Bv) {  // step t + 1's attention backward (AttBwdEpi)
    const int vb = map_rows ? xcd_remap_l(blockIdx.x, att.Bv) : (int)blockIdx.x;
    att_bwd_fused_wg<CP>(att, vb, R, n_ut, const_cast<uint16_t*>(dg_next), KD, lds);
    return;
  }
  const int b = xcd_remap_l((int)blockIdx.x - (FUSE ? att.Bv : 0), n_tiles);
  const int ut = map_rows ? b % n_ut : b / n_rt, rt = map_rows ? b / n_ut : b % n_rt;
  const int r0 = rt * BM, u0 = ut * 64;
  const int nk_all = dg_next != nullptr ? KD / 64 : 0;  // KD = 4H (+ A with attention)
  const int grp = threadIdx.x >> 8, gtid = threadIdx.x & 255;
  const int nkg = nk_all / GROUPS, k0 = grp * nkg;  // (launcher: nk_all % GROUPS == 0)
  const int tid = threadIdx.x, u = tid & 63, rg = tid >> 6;
  const int hu = u0 + u;
  constexpr int RG = 4 * GROUPS, RPT = BM / RG;

  uint2 pg[RPT];
  float pc[RPT], pcp[RPT], pdc[RPT], pdl[RPT];
  // the epilogue operands' latency hides under the GEMM
  lstm_bwd_load_epi<BM, GROUPS>(r0, R, H, rg, hu, gates, c_t, c_prev, dc_carry, dh_logit,
                                dh_scale, oh, pg, pc, pcp, pdc, pdl);
  static_assert(!ATT || (GROUPS == 2 && BM == 64), "attention epilogue: 2 groups of 64 rows");
  constexpr int SLICE = 64 * 4 * CP;  // bf16 per video slice
  int v0 = 0, nvs = 0;
  // (a native vector type: an array of HIP's uint4 struct stayed a stack
  // object -- scratch stores / loads around the main loop)
  u32x4_t gpf[ATT ? ATT_EPI_PF : 1];
  if (ATT) {
    v0 = r0 / att.vdiv;
    nvs = min(r0 + BM, R) - 1 >= r0 ? (min(r0 + BM, R) - 1) / att.vdiv - v0 + 1 : 0;
#pragma unroll
    for (int k = 0; k < ATT_EPI_PF; ++k) {  // (unconditional loads, clamped)
      const int ch = tid + k * 256 * GROUPS, vj = min(ch / (SLICE / 8), nvs - 1),
                o = ch % (SLICE / 8);
      gpf[k] = reinterpret_cast<const u32x4_t*>(
          att.gvb16 + ((int64_t)(v0 + vj) * H + u0) * CP * 4)[o];
    }
  }

  f32x16 acc[TL::TM][TL::TN];
  if (FUSE && nkg > 0) {
    // group g: dG_{t+1} tiles [g nkd / 2, (g + 1) nkd / 2), then dq_{t+1} tail
    // tiles [nkd + g nka / 2, nkd + (g + 1) nka / 2)
    const int lane = gtid & 63, w = gtid >> 6;
    const int nkd = (KD - att.A) / 64, nka = att.A / 64;
    DmaSrc<BM / 32> a;
    DmaSrc<64 / 32> bsrc;
    a.r0 = a.r1 = make_rsrc(dg_next, (int64_t)R * KD * 2);
    a.ksplit = bsrc.ksplit = nkd / 2;
#pragma unroll
    for (int i = 0; i < BM / 32; ++i) {
      const int row = dma_row(w, i, lane);
      const int base = min(r0 + row, R - 1) * KD * 2 + dma_chunk(row, lane) * 16;
      a.voff0[i] = base + grp * (nkd / 2) * 128;
      a.voff1[i] = base + (nkd + grp * (nka / 2)) * 128;
    }
    bsrc.r0 = bsrc.r1 = make_rsrc(whhT, (int64_t)H * KD * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = dma_row(w, i, lane);
      const int base = (u0 + row) * KD * 2 + dma_chunk(row, lane) * 16;
      bsrc.voff0[i] = base + grp * (nkd / 2) * 128;
      bsrc.voff1[i] = base + (nkd + grp * (nka / 2)) * 128;
    }
    gemm_bwd_mainloop_tail<TL, true>(gtid, nkd / 2 + nka / 2, a, bsrc,
                                     lds + grp * TL::STAGES * TL::STAGE_BYTES, acc, att.flags, v0,
                                     nvs, att.poll_bound, att.poll_err);
  } else if (nkg > 0) {
    const int lane = gtid & 63, w = gtid >> 6;
    DmaSrc<BM / 32> a;
    DmaSrc<64 / 32> bsrc;
    a.r0 = a.r1 = make_rsrc(dg_next, (int64_t)R * KD * 2);
    a.ksplit = nkg;
#pragma unroll
    for (int i = 0; i < BM / 32; ++i) {
      const int row = dma_row(w, i, lane);
      a.voff0[i] = min(r0 + row, R - 1) * KD * 2 + k0 * 128 + dma_chunk(row, lane) * 16;
      a.voff1[i] = a.voff0[i];
    }
    bsrc.r0 = bsrc.r1 = make_rsrc(whhT, (int64_t)H * KD * 2);
    bsrc.ksplit = nkg;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = dma_row(w, i, lane);
      bsrc.voff0[i] = (u0 + row) * KD * 2 + k0 * 128 + dma_chunk(row, lane) * 16;
      bsrc.voff1[i] = bsrc.voff0[i];
    }
    gemm_nt_mainloop_g<TL>(gtid, nkg, a, bsrc, lds + grp * TL::STAGES * TL::STAGE_BYTES, acc);
  } else {
#pragma unroll
    for (int i = 0; i < TL::TM; ++i)
#pragma unroll
      for (int j = 0; j < TL::TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  }
  float* C = reinterpret_cast<float*>(lds);  // GROUPS partial tiles of BM x CSTRIDE
  store_acc_to_lds<TL>(acc, C + grp * BM * TL::CSTRIDE, [](int) { return 0.f; }, gtid);
  uint16_t* s_gv = reinterpret_cast<uint16_t*>(C + GROUPS * BM * TL::CSTRIDE);
  // 16-byte chunks of a unit's slice (frame pairs) are XOR-swizzled by the unit
  // index, so the 16-lane groups of the epilogue's ds_read_b128 (lanes =
  // consecutive units, CP * 8 bytes apart) hit distinct bank slots
  constexpr int NCH = CP / 2, SWD = 16 / NCH;
  if (ATT) {
#pragma unroll
    for (int k = 0; k < ATT_EPI_PF; ++k) {
      const int ch = tid + k * 256 * GROUPS;
      if (ch < nvs * (SLICE / 8)) {
        const int uu = (ch % (SLICE / 8)) / NCH, c2 = ch % NCH;
        reinterpret_cast<u32x4_t*>(s_gv)[ch - c2 + (c2 ^ ((uu / SWD) & (NCH - 1)))] = gpf[k];
      }
    }
  }
  __syncthreads();
  float pd[ATT ? RPT : 1][ATT ? CP : 1];

  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  const uint32_t seed = rng_seed(rng, RNG_SLOT_DROPOUT);
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int row = rg + RG * i, r = r0 + row;
    if (r < R) {
      const int64_t o = (int64_t)r * H + hu;
      float dh = 0.f;
#pragma unroll
      for (int g = 0; g < GROUPS; ++g) dh += C[(g * BM + row) * TL::CSTRIDE + u];
      const bool keep = drop_p <= 0.f || dropout_keep(seed, step, r, hu, drop_p);
      if (keep) dh += pdl[i] * inv_keep;
      const uint2 gp = pg[i];
      const CellBwd cb = cell_bwd(cell, dh, pdc[i], bf2f(gp.x & 0xffff), bf2f(gp.x >> 16),
                                  bf2f(gp.y & 0xffff), bf2f(gp.y >> 16), pc[i], pcp[i]);
      dc_carry[o] = cb.carry;
      uint2 pk;
      pk.x = (uint32_t)f2bf(cb.d0) | ((uint32_t)f2bf(cb.d1) << 16);
      pk.y = (uint32_t)f2bf(cb.d2) | ((uint32_t)f2bf(cb.d3) << 16);
      *reinterpret_cast<uint2*>(dG + (int64_t)r * KD + 4 * hu) = pk;
      if (ATT) {  // the row's dalpha over this thread's 4 gate columns (bf16 dG, as stored)
        const uint4* gs =
            reinterpret_cast<const uint4*>(s_gv + (r / att.vdiv - v0) * SLICE + u * CP * 4);
        const bf16x2_t d01 = __builtin_bit_cast(bf16x2_t, pk.x);
        const bf16x2_t d23 = __builtin_bit_cast(bf16x2_t, pk.y);
#pragma unroll
        for (int c2 = 0; c2 < CP / 2; ++c2) {  // frames 2 c2, 2 c2 + 1
          const uint4 q = gs[c2 ^ ((u / SWD) & (NCH - 1))];
          pd[i][2 * c2] = __builtin_amdgcn_fdot2_f32_bf16(
              d01, __builtin_bit_cast(bf16x2_t, q.x),
              __builtin_amdgcn_fdot2_f32_bf16(d23, __builtin_bit_cast(bf16x2_t, q.y), 0.f, false),
              false);
          pd[i][2 * c2 + 1] = __builtin_amdgcn_fdot2_f32_bf16(
              d01, __builtin_bit_cast(bf16x2_t, q.z),
              __builtin_amdgcn_fdot2_f32_bf16(d23, __builtin_bit_cast(bf16x2_t, q.w), 0.f, false),
              false);
        }
      }
    } else if (ATT) {
#pragma unroll
      for (int c = 0; c < CP; ++c) pd[i][c] = 0.f;
    }
  }
  if (ATT) {
    // sum over the wave's 64 hidden units: after the butterfly lane l holds
    // value l of each 64-value chunk (row i = idx / CP, frame c = idx % CP)
    float* flat = &pd[0][0];
    const int lane = tid & 63;
#pragma unroll
    for (int c0 = 0; c0 < RPT * CP; c0 += 64) {
      Bfly2<64, 32>::run(flat + c0, lane);
      const int idx = c0 + lane, i = idx / CP, c = idx % CP;
      const int r = r0 + rg + RG * i;
      if (r < R) att.dal_part[((int64_t)ut * R + r) * CP + c] = flat[c0];
    }
  }
}

int lstm_bwd_tiles(int R, int H) { return (H / 64) * ((R + 63) / 64); }

template <int GROUPS, bool ATT = false, int CP = 8, bool FUSE = false,
          int STAGES = LSTM_BWD_STAGES>
static void launch_lstm_step_bwd_g(const uint16_t* dg_next, const uint16_t* whhT,
                                   const float* dh_logit, float* dc_carry, const uint16_t* gates,
                                   const float* c_t, const float* c_prev, int R, int H,
                                   float drop_p, const uint32_t* rng, int step, uint16_t* dG,
                                   int KD, hipStream_t stream, int cell, const float* dh_scale,
                                   const AttBwdEpi& att, const DhOneHot& oh) {
  constexpr int BM = 64;
  using TL = Tile<BM, 64, STAGES>;
  constexpr int LDS = GROUPS * TL::STAGES * TL::STAGE_BYTES > GROUPS * BM * TL::CSTRIDE * 4
                          ? GROUPS * TL::STAGES * TL::STAGE_BYTES
                          : GROUPS * BM * TL::CSTRIDE * 4;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)lstm_step_bwd_kernel<BM, STAGES, GROUPS, ATT, CP, FUSE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr_set = true;
  }
  // (fused: the attention workgroups first, blockIdx < Bv -- see att_fuse_wait)
  const int n = (H / 64) * ((R + BM - 1) / BM) + (FUSE ? att.Bv : 0);
  static const int map_rows = getenv("CSTCAP_BWD_MAP") ? atoi(getenv("CSTCAP_BWD_MAP")) : 1;
  hipLaunchKernelGGL((lstm_step_bwd_kernel<BM, STAGES, GROUPS, ATT, CP, FUSE>), dim3(n),
                     dim3(256 * GROUPS), LDS, stream, dg_next, whhT, dh_logit, dc_carry, gates,
                     c_t, c_prev, R, H, drop_p, rng, step, dG, KD, cell, dh_scale, att, oh,
                     map_rows);
  post_launch("lstm_step_bwd_kernel", stream);
}

void launch_lstm_step_bwd(const uint16_t* dg_next, const uint16_t* whhT, const float* dh_logit,
                          float* dc_carry, const uint16_t* gates, const float* c_t,
                          const float* c_prev, int R, int H, float drop_p, const uint32_t* rng,
                          int step, uint16_t* dG, int KD, hipStream_t stream, int cell,
                          const float* dh_scale, const AttBwdEpi* att, const DhOneHot* ohp) {
  const DhOneHot oh = ohp != nullptr ? *ohp : DhOneHot{};
  // two K groups per block when the K-tiles split evenly
  // (measured per step: 1 group 4.66 ms, 2 groups 4.54 ms, 4 groups with 2
  // LDS stages each 4.51 vs 4.47 ms for 2 groups on another box)
  if (att != nullptr) {
    if ((KD / 64) % 2 != 0 || !att_bwd_epi_ok(att->vdiv, att->C, H) ||
        att->CP != (att->C <= 8 ? 8 : 16))
      throw std::runtime_error("lstm_step_bwd: unsupported attention epilogue shape");
    if (att->flags != nullptr) {
      if (dg_next == nullptr || !att_bwd_fuse_ok(att->vdiv, att->C, att->A, H, att->Bv, R) ||
          KD != 4 * H + att->A || att->G4 != 4 * H || att->dal_next == nullptr ||
          att->dal_next == att->dal_part)
        throw std::runtime_error("lstm_step_bwd: unsupported fused attention backward");
      if (att->CP == 8)
        launch_lstm_step_bwd_g<2, true, 8, true>(dg_next, whhT, dh_logit, dc_carry, gates, c_t,
                                                 c_prev, R, H, drop_p, rng, step, dG, KD, stream,
                                                 cell, dh_scale, *att, oh);
      else
        launch_lstm_step_bwd_g<2, true, 16, true>(dg_next, whhT, dh_logit, dc_carry, gates, c_t,
                                                  c_prev, R, H, drop_p, rng, step, dG, KD, stream,
                                                  cell, dh_scale, *att, oh);
      return;
    }
    if (att->CP == 8)
      launch_lstm_step_bwd_g<2, true, 8>(dg_next, whhT, dh_logit, dc_carry, gates, c_t, c_prev,
                                         R, H, drop_p, rng, step, dG, KD, stream, cell, dh_scale,
                                         *att, oh);
    else
      launch_lstm_step_bwd_g<2, true, 16>(dg_next, whhT, dh_logit, dc_carry, gates, c_t, c_prev,
                                          R, H, drop_p, rng, step, dG, KD, stream, cell, dh_scale,
                                          *att, oh);
    return;
  }
  const AttBwdEpi none{};
  if ((KD / 64) % 2 == 0)
    launch_lstm_step_bwd_g<2>(dg_next, whhT, dh_logit, dc_carry, gates, c_t, c_prev, R, H,
                              drop_p, rng, step, dG, KD, stream, cell, dh_scale, none, oh);
  else
    launch_lstm_step_bwd_g<1>(dg_next, whhT, dh_logit, dc_carry, gates, c_t, c_prev, R, H,
                              drop_p, rng, step, dG, KD, stream, cell, dh_scale, none, oh);
}

// 128-row tiles x 64 packed gate columns, 3 LDS stages (72 KB, 2 blocks per CU)
void launch_lstm_step_fwd(const int64_t* tok, int64_t tok_stride, const uint16_t* ptab,
                          const uint16_t* h_prev, const float* c_prev, const float* vgate,
                          int vgate_div, int R, int H, const uint16_t* whh, uint16_t* h_out,
                          float* c_out, uint16_t* hdrop_out, int ldh, float drop_p,
                          const uint32_t* rng, int step, uint16_t* gates_out, hipStream_t stream,
                          const int* row_map, int cell) {
  constexpr int BM = 128, STAGES = 3;
  constexpr int LDS = Tile<BM, LB_N, STAGES>::LDS_BYTES + BM * 4;  // + staged token ids
  const int n_nt = (4 * H) / LB_N, n_rt = (R + BM - 1) / BM;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)lstm_step_fwd_kernel<BM, STAGES>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr_set = true;
  }
  hipLaunchKernelGGL((lstm_step_fwd_kernel<BM, STAGES>), dim3(n_nt * n_rt), dim3(256), LDS,
                     stream, tok, tok_stride, ptab, h_prev, c_prev, vgate, vgate_div, R, H, whh,
                     h_out, c_out, hdrop_out, ldh, drop_p, rng, step, gates_out, row_map, cell);
  post_launch("lstm_step_fwd_kernel", stream);
}

}  // namespace cst
