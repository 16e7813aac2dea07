// K2/K3/K4/K7: fused vocabulary projection + log-softmax statistics +
// Monte-Carlo / greedy token selection, and its backward.
//
// Reference per decode step (/root/reference/model.py:281, 251-258, 326,
// 331-337): logit Linear (cuBLAS) -> log_softmax over V (writes R x V) ->
// torch.multinomial(exp(logp)) (in sample(): on the CPU) or torch.max.
//
// Here one launch computes the logits tile by MFMA and reduces it in the
// epilogue, so no R x V log-prob tensor is ever formed:
//
// vocab_fwd_tr_kernel / vocab_lstm_fwd_kernel (grid: V/128 vocab tiles x
// R/128 row tiles, XCD-aware; the latter also carries the next step's
// recurrent GEMM tiles)
//   * C^T = W(V x H) . h_drop(R x H)^T + b  with v_mfma_f32_32x32x16_bf16;
//   * optional fp16 copy of the logits (the backward's softmax input, so
//     the backward never recomputes the 0.4 TFLOP projection);
//   * per (row, tile) partials: max, sum(exp(x - max)), a multinomial draw
//     from softmax(x / temp) done in two exact levels -- inverse CDF inside
//     the tile over the exp() weights kept in registers, and an exponential
//     race across tiles (key log(tile mass) - log(E), E ~ Exp(1)) --, both
//     driven by counter hashes of (seed, step, row, tile), so no per-element
//     random numbers (the seed is read from device memory, so a replayed
//     HIP graph draws fresh samples);
//     greedy argmax, and the logit of the row's target token.
// vocab_combine_kernel (one wavefront per row)
//   * merges the tile partials: LSE, sampled / greedy / target token and
//     their log-probs; applies the step's token-selection mode (teacher
//     forcing, MIXER sampling, scheduled sampling, greedy) and the
//     reference's end-of-sequence rules (forward(): "all rows emitted EOS ->
//     stop" through a device-side counter; sample(): per-row unfinished
//     mask) without any host synchronisation.
// vocab_exp_convert_kernel
//   * step 0 of the exp store (see VF_EXP): fp16 logits -> bf16
//     exp(x - lse) in place; the backward (vocab_grad.hip) never forms dS.
#include "gemm_tile.h"
#include "lstm_gemm.h"
#include "att_mfma.h"
#include "vocab_common.h"
#include "../launchers.h"

namespace cst {

// -------------------------------------------------------------------------------
// Transposed epilogue: the MFMA computes C^T = W . h_drop^T (vocab rows
// as the M operand, caption rows as N).  In the 32x32 MFMA output layout lane l
// then holds, for caption row (l & 31) of each 32-row sub-tile, 16 vocabulary
// entries per 32-vocab sub-tile: the lane's 32 (TM = 2) logits of one row sit
// in its own registers.  Every per-row statistic (max, sum exp, argmax, target
// logit, inverse-CDF draw) is a register loop with no LDS C tile and no
// shuffles; only the 4 lane groups that share a row (2 half-waves x 2 vocab
// waves) are merged, through 16 KB of LDS, once per block.
//
// Sampling stays exact: each group draws inside its own 32 weights by inverse
// CDF and enters an exponential race with key m/temp + log(mass) - log(E)
// (E ~ Exp(1)); the race continues across the 4 groups here and across vocab
// tiles in vocab_combine_kernel, and the union of independent races is the
// race over all of V.
constexpr int VT_V = 128;  // vocab entries per block
// exp-store staging tile in LDS: BN rows x (VT_V + 8) bf16 (16-byte aligned
// row starts), placed behind the GroupStat area (4 groups x BN rows x 32 B)
constexpr int EXP_STAGE_LD = VT_V + 8;
__host__ __device__ constexpr int exp_stage_off(int BN) { return 4 * BN * 32; }
__host__ __device__ constexpr int epilogue_lds_bytes(int BN) {
  return exp_stage_off(BN) + BN * EXP_STAGE_LD * 2;
}
struct GroupStat {  // 32 bytes, one per (lane group, row) in LDS (exp_stage_off)
  float m, s, zkey, zlogit;
  int zidx, xidx;
  float xt, pad;
};

#define VOCAB_TR_PARAMS                                                                     \
  const uint16_t *__restrict__ hd, int ldh, int R, int H, const uint16_t *__restrict__ W,    \
      const float *__restrict__ bias, int V, uint16_t *__restrict__ logits16, int64_t ldl,   \
      VocabPartial *__restrict__ part, const int64_t *__restrict__ tgt, int64_t tgt_stride, \
      int flags, float inv_temp, const uint32_t *__restrict__ rng, int step,                 \
      const float *__restrict__ eoff
#define VOCAB_TR_ARGS \
  hd, ldh, R, H, W, bias, V, logits16, ldl, part, tgt, tgt_stride, flags, inv_temp, rng, step, eoff

// TOPK (flags VF_TOPK, beam search only): the per-tile top-K candidates
template <int BN, int STAGES, bool TOPK = false>
__device__ __forceinline__ void vocab_tr_block(int bid, char* lds, VOCAB_TR_PARAMS) {
  using TL = Tile<VT_V, BN, STAGES>;  // M = vocab, N = caption rows
  constexpr int TM = TL::TM, TN = TL::TN;
  static_assert(TM == 2, "lane owns 32 vocab entries per row");
  const int n_vt = (V + VT_V - 1) / VT_V, n_rt = (R + BN - 1) / BN;
  const int b = xcd_remap(bid, n_vt * n_rt);
  const int vt = b / n_rt, rt = b % n_rt;
  const int v0 = vt * VT_V, r0 = rt * BN;
  const int nk = H / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wr = w >> 1, wc = w & 1;
  const int half = lane >> 5;
  // the lane's vocab entries: vb + 32 i + 8 q + e   (i < TM, q < 4, e < 4)
  const int vb = v0 + wr * TL::WM + 4 * half;

  // epilogue operands prefetched before the main loop; columns past V get a
  // -inf bias so they vanish from every statistic
  float pb[TM][16];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int v = vb + 32 * i + 8 * q;
      if (v + 4 <= V) {
        const float4 x = *reinterpret_cast<const float4*>(bias + v);
        pb[i][4 * q] = x.x, pb[i][4 * q + 1] = x.y, pb[i][4 * q + 2] = x.z, pb[i][4 * q + 3] = x.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) pb[i][4 * q + e] = v + e < V ? bias[v + e] : -INFINITY;
      }
    }
  int tg[TN];
  float ec[TN];  // exp-store offsets of the lane's rows
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int r = min(r0 + wc * TL::WN + 32 * j + (lane & 31), R - 1);
    tg[j] = tgt != nullptr ? (int)tgt[(int64_t)r * tgt_stride] : -1;
    ec[j] = eoff != nullptr ? eoff[r] : 0.f;
  }

  f32x16 acc[TM][TN];
  {
    DmaSrc<VT_V / 32> a;
    DmaSrc<BN / 32> bsrc;
    a.r0 = a.r1 = make_rsrc(W, (int64_t)V * H * 2);
    a.ksplit = nk;
#pragma unroll
    for (int i = 0; i < VT_V / 32; ++i) {
      const int row = dma_row(w, i, lane);
      a.voff0[i] = min(v0 + row, V - 1) * H * 2 + dma_chunk(row, lane) * 16;
      a.voff1[i] = a.voff0[i];
    }
    bsrc.r0 = bsrc.r1 = make_rsrc(hd, (int64_t)R * ldh * 2);
    bsrc.ksplit = nk;
#pragma unroll
    for (int i = 0; i < BN / 32; ++i) {
      const int row = dma_row(w, i, lane);
      bsrc.voff0[i] = min(r0 + row, R - 1) * ldh * 2 + dma_chunk(row, lane) * 16;
      bsrc.voff1[i] = bsrc.voff0[i];
    }
    gemm_nt_mainloop<TL>(nk, a, bsrc, lds, acc);
  }
  if (flags & VF_BENCH_MAINLOOP) {  // microbenchmark: main loop only
    if (acc[0][0][0] == 1234.5f) part[0].pad = acc[TM - 1][TN - 1][15];
    return;
  }

  GroupStat* gs = reinterpret_cast<GroupStat*>(lds);  // [4 groups][BN rows]
  const int g = wr * 2 + half;
  const bool temp1 = inv_temp == 1.f;
  constexpr float L2E = 1.4426950408889634f;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int row_l = wc * TL::WN + 32 * j + (lane & 31);
    const int r = r0 + row_l;
    float x[TM][16];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int k = 0; k < 16; ++k) x[i][k] = acc[i][j][k] + pb[i][k];

    if (TOPK && (flags & VF_TOPK)) {
      // beam search: the lane's K best of its 32 logits (sorted, ties -> the
      // smaller index), then the 4 lane groups of the row merged below
      const int K = vf_topk_k(flags);
      float tv[VF_TOPK_MAXK];
      int ti[VF_TOPK_MAXK];
#pragma unroll
      for (int p = 0; p < VF_TOPK_MAXK; ++p) tv[p] = -INFINITY, ti[p] = 0x7fffffff;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          float cv = x[i][k];
          int ci = vb + 32 * i + 8 * (k >> 2) + (k & 3);  // ascending in (i, k): ties keep the first
#pragma unroll
          for (int p = 0; p < VF_TOPK_MAXK; ++p) {
            if (p < K && cv > tv[p]) {
              const float a = tv[p];
              const int b = ti[p];
              tv[p] = cv, ti[p] = ci;
              cv = a, ci = b;
            }
          }
        }
      float2* tk = reinterpret_cast<float2*>(lds + exp_stage_off(BN));  // [4 groups][BN rows][MAXK]
#pragma unroll
      for (int p = 0; p < VF_TOPK_MAXK; ++p)
        tk[(g * BN + row_l) * VF_TOPK_MAXK + p] = make_float2(tv[p], __int_as_float(ti[p]));
    } else if ((flags & VF_SAVE_F32) && logits16 != nullptr && r < R) {  // fp32 logits (beam search)
      float* dst = reinterpret_cast<float*>(logits16) + (int64_t)r * ldl;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int v = vb + 32 * i + 8 * q;
          if (v + 4 <= V) {
            *reinterpret_cast<float4*>(dst + v) =
                make_float4(x[i][4 * q], x[i][4 * q + 1], x[i][4 * q + 2], x[i][4 * q + 3]);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (v + e < V) dst[v + e] = x[i][4 * q + e];
          }
        }
    } else if (logits16 != nullptr && r < R && !(flags & VF_EXP)) {
      // fp16 logits: staged through LDS like the exp store (written below);
      // entries past V hold -inf and stay inside the row stride ldl
      uint16_t* et = reinterpret_cast<uint16_t*>(lds + exp_stage_off(BN)) + row_l * EXP_STAGE_LD;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int vl = vb - v0 + 32 * i + 8 * q;
          uint2 pk;
          pk.x = (uint32_t)f2h(x[i][4 * q]) | ((uint32_t)f2h(x[i][4 * q + 1]) << 16);
          pk.y = (uint32_t)f2h(x[i][4 * q + 2]) | ((uint32_t)f2h(x[i][4 * q + 3]) << 16);
          *reinterpret_cast<uint2*>(et + vl) = pk;
        }
    }

    float m = -INFINITY;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int k = 0; k < 16; ++k) m = fmaxf(m, x[i][k]);
    const float msafe = m == -INFINITY ? 0.f : m;
    const float ml = msafe * L2E;
    // exp weights stay in registers for the sampler's inverse CDF (no second
    // exp pass at temperature 1)
    float ew[TM][16];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        ew[i][k] = __builtin_amdgcn_exp2f(fmaf(x[i][k], L2E, -ml));
        s += ew[i][k];
      }
    if ((flags & VF_EXP) && logits16 != nullptr && r < R) {
      // E = exp(x - c) = exp(x - m) * exp(m - c): one multiply per entry on
      // the weights already in registers (bf16: fp32's exponent range, so in
      // range unless the row's LSE moves by ~80 from the previous step's; the
      // backward recomputes such rows exactly, vocab_grad.hip vgrad_fix)
      const float f = __builtin_amdgcn_exp2f((msafe - ec[j]) * L2E);
      // staged through LDS (behind the row statistics' GroupStat area): the
      // MFMA layout gives each lane 8-byte pieces of 32 different rows; the
      // block then writes whole 256-byte row segments (see below)
      uint16_t* et = reinterpret_cast<uint16_t*>(lds + exp_stage_off(BN)) + row_l * EXP_STAGE_LD;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int vl = vb - v0 + 32 * i + 8 * q;  // entries past V: weight 0
          uint2 pk;
          pk.x = (uint32_t)f2bf(ew[i][4 * q] * f) | ((uint32_t)f2bf(ew[i][4 * q + 1] * f) << 16);
          pk.y = (uint32_t)f2bf(ew[i][4 * q + 2] * f) | ((uint32_t)f2bf(ew[i][4 * q + 3] * f) << 16);
          *reinterpret_cast<uint2*>(et + vl) = pk;
        }
    }

    GroupStat st;
    st.m = m;
    st.s = s;
    st.pad = 0.f;
    st.xidx = 0x7fffffff;
    if (flags & VF_ARGMAX) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int v = vb + 32 * i + 8 * (k >> 2) + (k & 3);
          st.xidx = min(st.xidx, x[i][k] == m ? v : 0x7fffffff);
        }
    }
    st.xt = -INFINITY;
    if (tgt != nullptr) {
      const int d = tg[j] - vb;
      const bool mine = d >= 0 && d < 32 * TM && (d & 4) == 0;
      const int kk = mine ? (d >> 5) * 16 + ((d >> 3) & 3) * 4 + (d & 3) : -1;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int k = 0; k < 16; ++k) st.xt = (i * 16 + k == kk) ? x[i][k] : st.xt;
    }
    st.zkey = -INFINITY;
    st.zlogit = 0.f;
    st.zidx = 0x7fffffff;
    if (flags & VF_SAMPLE) {
      const float wl = msafe * inv_temp * L2E, wsc = inv_temp * L2E;
      float sw = s;
      if (!temp1) {
        sw = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            ew[i][k] = __builtin_amdgcn_exp2f(fmaf(x[i][k], wsc, -wl));
            sw += ew[i][k];
          }
      }
      const uint32_t rr = (uint32_t)min(r, R - 1);
      const uint32_t seed = rng_seed(rng, RNG_SLOT_SAMPLE);
      const uint32_t key = mix32(seed ^ mix32(rr * 0x9E3779B1u + (uint32_t)step * 0x85EBCA77u) ^
                                 (uint32_t)(vt * 4 + g) * 0xC2B2AE3Du);
      const float u = ((float)(key >> 8) + 0.5f) * (1.0f / 16777216.0f);
      const float tm = u * sw;
      // inverse CDF in the same summation order as sw, so the last positive
      // weight always satisfies cum >= tm
      float cum = 0.f, cl = 0.f;
      int cand = -1;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const float wv = ew[i][k];
          cum += wv;
          const bool hit = cand < 0 && cum >= tm && wv > 0.f;
          cand = hit ? vb + 32 * i + 8 * (k >> 2) + (k & 3) : cand;
          cl = hit ? x[i][k] : cl;
        }
      if (sw > 0.f && cand >= 0) {
        const uint32_t key2 = mix32(key ^ 0x68E31DA4u);
        const float u2 = ((float)(key2 >> 8) + 0.5f) * (1.0f / 16777216.0f);
        st.zkey = msafe * inv_temp + __logf(sw) - __logf(-__logf(u2));
        st.zidx = cand;
        st.zlogit = cl;
      }
    }
    gs[g * BN + row_l] = st;
  }
  __syncthreads();
  // merge the 4 lane groups of each row -> one VocabPartial per (tile, row)
  if (threadIdx.x < BN) {
    const int row_l = threadIdx.x, r = r0 + row_l;
    if (r < R) {
      GroupStat a = gs[row_l];
#pragma unroll
      for (int q = 1; q < 4; ++q) {
        const GroupStat c = gs[q * BN + row_l];
        const float M = fmaxf(a.m, c.m);
        a.s = (a.m == -INFINITY ? 0.f : a.s * __expf(a.m - M)) +
              (c.m == -INFINITY ? 0.f : c.s * __expf(c.m - M));
        if (c.m > a.m || (c.m == a.m && c.xidx < a.xidx)) a.xidx = c.xidx;
        a.m = M;
        if (c.zkey > a.zkey || (c.zkey == a.zkey && c.zidx < a.zidx)) {
          a.zkey = c.zkey;
          a.zidx = c.zidx;
          a.zlogit = c.zlogit;
        }
        a.xt = fmaxf(a.xt, c.xt);
      }
      VocabPartial p;
      p.m = a.m;
      p.s = a.s;
      p.zval = a.zkey;
      p.zlogit = a.zlogit;
      p.zidx = a.zidx;
      p.xidx = a.xidx;
      p.xtgt = a.xt;
      p.pad = 0.f;
      part[(int64_t)vt * R + r] = p;
      if (TOPK && (flags & VF_TOPK)) {  // merge the row's 4 sorted group lists -> K candidates
        const int K = vf_topk_k(flags);
        const float2* tk = reinterpret_cast<const float2*>(lds + exp_stage_off(BN));
        int hd4[4] = {0, 0, 0, 0};
        float2* dst = reinterpret_cast<float2*>(logits16) + ((int64_t)vt * R + r) * K;
        for (int k = 0; k < K; ++k) {
          float bvv = -INFINITY;
          int bii = 0x7fffffff, bq = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float2 c = hd4[q] < K ? tk[(q * BN + row_l) * VF_TOPK_MAXK + hd4[q]]
                                        : make_float2(-INFINITY, __int_as_float(0x7fffffff));
            const int ci = __float_as_int(c.y);
            if (c.x > bvv || (c.x == bvv && ci < bii)) bvv = c.x, bii = ci, bq = q;
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) hd4[q] += q == bq ? 1 : 0;
          dst[k] = make_float2(bvv, __int_as_float(bii));
        }
      }
    }
  }
  if (logits16 != nullptr && !(flags & (VF_SAVE_F32 | VF_TOPK))) {
    // the staged 16-bit tile (exp store or fp16 logits, written before the
    // barrier above): 16 bytes
    // per thread and pass, 16 threads per 256-byte row segment; columns past
    // V hold 0 (bias -inf) and are written up to the row stride ldl
    const uint16_t* et = reinterpret_cast<const uint16_t*>(lds + exp_stage_off(BN));
#pragma unroll
    for (int idx = threadIdx.x; idx < BN * (VT_V / 8); idx += 256) {
      const int row = idx / (VT_V / 8), ch = idx % (VT_V / 8);
      const int r = r0 + row, v = v0 + 8 * ch;
      if (r < R && v + 8 <= ldl)
        *reinterpret_cast<uint4*>(logits16 + (int64_t)r * ldl + v) =
            *reinterpret_cast<const uint4*>(et + row * EXP_STAGE_LD + 8 * ch);
    }
  }
}

template <int BN, int STAGES, int OCC, bool TOPK = false>
__global__ __launch_bounds__(256, OCC) void vocab_fwd_tr_kernel(VOCAB_TR_PARAMS) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  vocab_tr_block<BN, STAGES, TOPK>(blockIdx.x, lds, VOCAB_TR_ARGS);
}

// the same attention workgroups as a launch of their own
template <int AV>
__global__ __launch_bounds__(256) void att_mfma_fwd_kernel(AttMfmaArgs att) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  att_mfma_fwd_any<AV>(blockIdx.x, att, lds);
}

// host dispatch over the attention variants (frames padded to 8 / 16)
#define ATT_VARIANTS(X) X(8) X(16)

bool att_mfma_fwd_ok(int vdiv, int C, int A, int H, int per_frame) {
  return !per_frame && vdiv >= 1 && vdiv <= 32 && C >= 1 && C <= 16 && A % ATT_SLICE == 0 &&
         A <= 16 * ATT_SLICE && H % 32 == 0 && H >= 64 && H <= 512 &&
         att_mfma_lds_bytes(C, C <= 8 ? 8 : 16, H) <= 48 * 1024;
}
// training (the saved forward feeds the fused attention backward, which needs
// two or more rows per video): 2..32 rows per video
bool att_mfma_ok(int vdiv, int C, int A, int H, int per_frame) {
  return vdiv >= 2 && att_mfma_fwd_ok(vdiv, C, A, H, per_frame);
}

static void check_att_mfma(const AttMfmaArgs& a) {
  if (!att_mfma_fwd_ok(a.vdiv, a.C, a.A, a.H, 0) || a.G4 != 4 * a.H || a.CP != (a.C <= 8 ? 8 : 16) ||
      (!a.whole && (a.e_part == nullptr || a.cnt == nullptr)) ||
      (a.whole && att_mfma_video_lds_bytes(a.C, a.CP, a.H) > 48 * 1024))
    throw std::runtime_error("att_mfma: unsupported attention shape");
}

// CSTCAP_ATT_WHOLE=1: the whole-video form where its LDS fits.  Opt-in: one
// workgroup running all A / 64 slices in sequence outlasts the vocabulary tiles
// of the decode launch (att8 launch 63.8 vs 48.9 us; step 4.841 / 4.875 vs
// 4.502 / 4.506 ms, interleaved, profiles/r6/s2/att_whole/)
int att_mfma_whole_default(int C, int H) {
  static const bool env = [] {
    const char* e = getenv("CSTCAP_ATT_WHOLE");
    return e != nullptr && atoi(e) != 0;
  }();
  return env && att_mfma_video_lds_bytes(C, C <= 8 ? 8 : 16, H) <= 48 * 1024 ? 1 : 0;
}

template <int AV>
static void launch_att_mfma_fwd_t(const AttMfmaArgs& a, hipStream_t stream) {
  const int lds = att_mfma_lds_bytes(a.C, a.CP, a.H);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)att_mfma_fwd_kernel<AV>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 48 * 1024);
    attr_set = true;
  }
  hipLaunchKernelGGL(att_mfma_fwd_kernel<AV>, dim3(att_mfma_nblocks(a)), dim3(256),
                     a.whole ? att_mfma_video_lds_bytes(a.C, a.CP, a.H) : lds,
                     stream, a);
  post_launch("att_mfma_fwd_kernel", stream);
}

void launch_att_mfma_fwd(const AttMfmaArgs& a, hipStream_t stream) {
  check_att_mfma(a);
  switch (att_variant(a.C)) {
#define X(V) case V: launch_att_mfma_fwd_t<V>(a, stream); break;
    ATT_VARIANTS(X)
#undef X
    default: throw std::runtime_error("att_mfma: no kernel variant");
  }
}

// token-selection modes of one decode step
enum SelMode : int { SEL_GT = 0, SEL_SAMPLE = 1, SEL_GREEDY = 2, SEL_SS = 3 };

// One wavefront per row (4 rows per 256-thread workgroup by default, see
// launch_vocab_combine; 320 workgroups at R = 1280): each lane
// merges 2 tiles (6-step shuffle tree) and owns 8 of the cell epilogue's
// hidden units, so the chain partials -> merge -> token -> table row -> cell
// runs with half the per-lane work of the earlier half-wave rows (3.331-3.345
// vs 3.367-3.380 ms per training step, interleaved on one box,
// profiles/r5/combine/ab_c64_*.json).  LANES stays a template parameter.
constexpr int CMB_LANES = 64, CMB_THREADS = 64;
// end-of-sequence flags: per decode step CMB_CNT_SLOTS slots, one 128-byte
// line apart (see vocab_combine_kernel)
constexpr int CMB_CNT_SLOTS = 64, CMB_CNT_STRIDE = 32;
int combine_count_ints_per_step() { return CMB_CNT_SLOTS * CMB_CNT_STRIDE; }

// Cell epilogue of the NEXT decode step, applied as soon as its input token
// is chosen (see lstm_gemm.h): gates = pre + P[tok] -> i, f, g, o -> c, h.
struct CellArgs {
  const void* pre;     // (R, 4H) h_t W_hh^T + vgate, packed gates, fp32 (fp16 with
                       // pre_half); nullptr = no cell
  const uint16_t* vg16;  // nullable (R, 4H) bf16 per-row video gates (MFMA attention)
  const uint16_t* ptab;  // (V, 4H) fp16 projected embedding table
  const float* c_prev;
  float* c_out;
  uint16_t* h_out;
  uint16_t* hdrop_out;  // nullable; row stride ldh
  int ldh;
  uint16_t* gates_out;  // nullable (training: saved for the backward)
  int H;
  float drop_p;
  int step;  // decode step of the cell (dropout mask index)
  int cell;  // CellType
  int pre_half;
};
// the 4 packed pre-activations of hidden unit u of a row (PH: fp16 pre)
template <bool PH>
__device__ __forceinline__ float4 load_pre(const CellArgs& c, int64_t row_off, int u) {
  return PH ? ld_h4(reinterpret_cast<const uint16_t*>(c.pre) + row_off + 4 * u)
            : *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(c.pre) + row_off +
                                               4 * u);
}

struct RowStat {
  float m, s, zv, zl, xm, xt;
  int zi, xi;
};

__device__ __forceinline__ void merge_stat(RowStat& a, float m2, float s2, float zv2, float zl2,
                                           int zi2, float xm2, int xi2, float xt2) {
  const float M = fmaxf(a.m, m2);
  a.s = (a.m == -INFINITY ? 0.f : a.s * __expf(a.m - M)) +
        (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - M));
  a.m = M;
  if (zv2 > a.zv || (zv2 == a.zv && zi2 < a.zi)) {
    a.zv = zv2;
    a.zi = zi2;
    a.zl = zl2;
  }
  if (xm2 > a.xm || (xm2 == a.xm && xi2 < a.xi)) {
    a.xm = xm2;
    a.xi = xi2;
  }
  a.xt = fmaxf(a.xt, xt2);
}

// The row's outputs from its merged statistics (vocab_combine_kernel and the
// fused merge): LSE, target log-prob, and, when tok_out is set, the token
// chosen by the step's selection mode under the reference's end-of-sequence
// rules.  Returns the token (0 when no token is chosen).
struct RowSel {
  float* lse_out;
  float* g_xe;
  int64_t gxe_stride;
  int64_t* tok_out;
  int64_t tok_stride;
  float* g_sel;
  int64_t gsel_stride;
  int mode;
  float ss_prob;
  const uint32_t* rng;
  int step;
  uint8_t* unfinished;
  int V;  // (debug bound of the chosen token)
};
__device__ __forceinline__ int finish_row(const RowStat& a, int r, const RowSel& o, int64_t gt_tok,
                                          bool dead_pre, bool unf_pre) {
  const float lse = a.m + __logf(a.s);
  if (o.lse_out) o.lse_out[r] = lse;
  if (o.g_xe) o.g_xe[(int64_t)r * o.gxe_stride] = a.xt - lse;
  if (o.tok_out == nullptr) return 0;
  // (selects, not a switch over the fields: a mode-indexed field read made
  // the compiler spill the merged statistics to scratch)
  bool use_sample = o.mode == SEL_SAMPLE;
  if (o.mode == SEL_SS) {
    const u32x4 u = philox4x32({(uint32_t)r, RNG_SS, (uint32_t)o.step, 0u},
                               rng_seed(o.rng, RNG_SLOT_SAMPLE), 0x68E31DA4u);
    use_sample = u01(u.x) < o.ss_prob;
  }
  const bool greedy = o.mode == SEL_GREEDY;
  // (the empty asm pins the fields in registers: a select of two fields of the
  // same struct otherwise becomes a load through a selected address, which
  // puts the struct in scratch memory)
  float zl = a.zl, xm = a.xm, xt = a.xt;
  int zi = a.zi, xi = a.xi;
  asm volatile("" : "+v"(zl), "+v"(xm), "+v"(xt), "+v"(zi), "+v"(xi));
  int64_t tok = use_sample ? (int64_t)zi : greedy ? (int64_t)xi : gt_tok;
  const float tl = use_sample ? zl : greedy ? xm : xt;
  // reference forward(): once every row emitted EOS at one step, decoding
  // stops.  Sticky on the device: after such a step every token is forced
  // to 0, so the count of the previous step alone decides (one load, not a
  // dependent scan over all earlier steps)
  if (dead_pre) tok = 0;
  // per-row finished mask: reference sample(), or forward() with the
  // --mask_after_eos fix
  if (o.unfinished != nullptr) {
    const uint8_t u = unf_pre && (tok > 0);
    o.unfinished[r] = u;
    if (!u) tok = 0;
  }
  CST_DCHECK(tok >= 0 && tok < o.V);
  o.tok_out[(int64_t)r * o.tok_stride] = tok;
  if (o.g_sel) o.g_sel[(int64_t)r * o.gsel_stride] = tl - lse;
  return (int)tok;
}

template <int LANES, bool PH, int NT = CMB_THREADS>
__global__ __launch_bounds__(NT) void vocab_combine_kernel(
    const VocabPartial* __restrict__ part, int n_vt, int R, float* __restrict__ lse_out,
    int64_t* __restrict__ tok_out, int64_t tok_stride, float* __restrict__ g_sel,
    int64_t gsel_stride, float* __restrict__ g_xe, int64_t gxe_stride,
    const int64_t* __restrict__ gt, int64_t gt_stride, int mode, float ss_prob,
    const uint32_t* __restrict__ rng, int step, int* __restrict__ counts, int count_step,
    uint8_t* __restrict__ unfinished, CellArgs cell, int Rs) {
  __shared__ int s_nonzero;
  int tok_final = 0;
  const int sub = threadIdx.x & (LANES - 1);
  const int r = blockIdx.x * (NT / LANES) + (threadIdx.x / LANES);
  const bool valid = r < R;
  if (threadIdx.x == 0) s_nonzero = 0;
  // The row's tile partials are loaded unconditionally (clamped index,
  // neutralised in the merge) so they issue back to back: one memory round
  // trip instead of one per merge step.  The cell epilogue's token-independent
  // operands (pre-activations, c_t, video gates) are requested right AFTER
  // them: the vector-memory counter retires loads in order, so the merge
  // waits for the partials only while those are in flight (requested before
  // the partials, they delayed the merge; requested after the merge, their
  // latency added to the chain).  Only the token's table row waits for the
  // merge.
  constexpr int CMB_MAXP = 128 / LANES;  // n_vt <= 128: V <= 16384 at 128-wide tiles
  const bool fastp = n_vt <= CMB_MAXP * LANES;
  VocabPartial pp[CMB_MAXP];
  // the row's partials: tile t at prow[t * Rs] (Rs = R: one block of rows)
  const int rq = valid ? r : 0;
  const VocabPartial* prow = part + (int64_t)(rq / Rs) * n_vt * Rs + (rq % Rs);
  if (valid && fastp) {
#pragma unroll
    for (int k = 0; k < CMB_MAXP; ++k)
      pp[k] = prow[(int64_t)min(sub + k * LANES, n_vt - 1) * Rs];
  }
  const bool do_cell = cell.pre != nullptr && tok_out != nullptr;
  // one batch of CELL_U units per lane covers H <= 512 (every lane of the row
  // owns units sub, sub + 32, ...); larger H loads per batch after the merge
  constexpr int CELL_U = 512 / LANES;
  const bool pre_early = do_cell && valid && cell.H <= LANES * CELL_U;
  float4 pe[CELL_U];
  float ce[CELL_U];
  uint2 ve[CELL_U];
  if (pre_early) {
    const int H = cell.H;
    const int64_t prow = (int64_t)r * 4 * H;
#pragma unroll
    for (int k = 0; k < CELL_U; ++k) {
      const int u = min(sub + k * LANES, H - 1);  // (clamped: no branch)
      pe[k] = load_pre<PH>(cell, prow, u);
      ce[k] = cell.c_prev[(int64_t)r * H + u];
      if (cell.vg16 != nullptr)
        ve[k] = *reinterpret_cast<const uint2*>(cell.vg16 + (int64_t)r * 4 * H + 4 * u);
    }
  }
  // the selecting lane's other inputs, requested now (they do not depend on
  // the merge): ground-truth token, previous step's non-EOS count, row mask
  int64_t gt_pre = 0;
  bool unf_pre = true;
  if (valid && sub == 0 && tok_out != nullptr) {
    gt_pre = gt ? gt[(int64_t)r * gt_stride] : 0;
    unf_pre = unfinished == nullptr || unfinished[r] != 0;
  }
  // "some row emitted a non-EOS token at the previous step": CMB_CNT_SLOTS
  // cache-line-strided flag slots (written by the blocks of that step), read
  // by the row's lanes and OR-reduced across them
  int nz_prev = 1;
  if (counts != nullptr && count_step > 1 && tok_out != nullptr) {
    nz_prev = 0;
#pragma unroll
    for (int k = sub; k < CMB_CNT_SLOTS; k += LANES)
      nz_prev |= counts[((count_step - 1) * CMB_CNT_SLOTS + k) * CMB_CNT_STRIDE];
#pragma unroll
    for (int o = 1; o < LANES; o <<= 1) nz_prev |= __shfl_xor(nz_prev, o, 64);
  }
  const bool dead_pre = nz_prev == 0;
  RowStat a = {-INFINITY, 0.f, -INFINITY, 0.f, -INFINITY, -INFINITY, 0x7fffffff, 0x7fffffff};
  if (valid && fastp) {
#pragma unroll
    for (int k = 0; k < CMB_MAXP; ++k) {
      if (sub + k * LANES < n_vt) {
        const VocabPartial& p = pp[k];
        merge_stat(a, p.m, p.s, p.zval, p.zlogit, p.zidx, p.m, p.xidx, p.xtgt);
      }
    }
  } else if (valid) {
#pragma unroll 4
    for (int t = sub; t < n_vt; t += LANES) {
      const VocabPartial p = prow[(int64_t)t * Rs];
      merge_stat(a, p.m, p.s, p.zval, p.zlogit, p.zidx, p.m, p.xidx, p.xtgt);
    }
  }
#pragma unroll
  for (int o = 1; o < LANES; o <<= 1) {
    merge_stat(a, __shfl_xor(a.m, o, 64), __shfl_xor(a.s, o, 64), __shfl_xor(a.zv, o, 64),
               __shfl_xor(a.zl, o, 64), __shfl_xor(a.zi, o, 64), __shfl_xor(a.xm, o, 64),
               __shfl_xor(a.xi, o, 64), __shfl_xor(a.xt, o, 64));
  }
  __syncthreads();  // s_nonzero initialised
  if (valid && sub == 0) {
    const RowSel o{lse_out, g_xe, gxe_stride, tok_out, tok_stride, g_sel, gsel_stride,
                   mode, ss_prob, rng, step, unfinished, n_vt * VT_V};
    tok_final = finish_row(a, r, o, gt_pre, dead_pre, unf_pre);
    if (counts != nullptr && tok_out != nullptr && tok_final != 0) atomicAdd(&s_nonzero, 1);
  }
  if (do_cell) {
    // the row's 32 lanes: lane k owns hidden units k, k + 32, ... (coalesced)
    const int tk = __shfl(tok_final, (int)(threadIdx.x & 63) & ~(LANES - 1), 64);
    if (valid) {
      const int H = cell.H;
      const int64_t prow = (int64_t)r * 4 * H;
      const uint16_t* trow = cell.ptab + (int64_t)tk * 4 * H;
      const float inv_keep = cell.drop_p > 0.f ? 1.f / (1.f - cell.drop_p) : 1.f;
      const uint32_t dseed = rng_seed(rng, RNG_SLOT_DROPOUT);
      // batches of CELL_U units (all of H = 512 in one): every load of a
      // batch is issued before the first store (the stores could alias the
      // inputs as far as the compiler knows, which would serialise the loads)
      for (int u0 = sub; u0 < H; u0 += LANES * CELL_U) {
        float4 p[CELL_U], x[CELL_U];
        float cp[CELL_U];
        uint2 vq[CELL_U];
        if (pre_early) {
#pragma unroll
          for (int k = 0; k < CELL_U; ++k) {
            p[k] = pe[k];
            cp[k] = ce[k];
            vq[k] = ve[k];
            x[k] = ld_h4(trow + 4 * min(u0 + k * LANES, H - 1));
          }
        } else {
#pragma unroll
          for (int k = 0; k < CELL_U; ++k) {
            const int u = u0 + k * LANES;
            if (u < H) {
              p[k] = load_pre<PH>(cell, prow, u);
              x[k] = ld_h4(trow + 4 * u);
              cp[k] = cell.c_prev[(int64_t)r * H + u];
              if (cell.vg16 != nullptr)
                vq[k] = *reinterpret_cast<const uint2*>(cell.vg16 + (int64_t)r * 4 * H + 4 * u);
            }
          }
        }
        if (cell.vg16 != nullptr) {  // attention: the row's video gates (bf16)
#pragma unroll
          for (int k = 0; k < CELL_U; ++k) {
            p[k].x += bf2f(vq[k].x & 0xffff);
            p[k].y += bf2f(vq[k].x >> 16);
            p[k].z += bf2f(vq[k].y & 0xffff);
            p[k].w += bf2f(vq[k].y >> 16);
          }
        }
#pragma unroll
        for (int k = 0; k < CELL_U; ++k) {
          const int u = u0 + k * LANES;
          if (u < H) {
            const CellFwd cf = cell_fwd(cell.cell, p[k].x + x[k].x, p[k].y + x[k].y,
                                        p[k].z + x[k].z, p[k].w + x[k].w, cp[k]);
            const int64_t o = (int64_t)r * H + u;
            const float hv = cf.h;
            cell.c_out[o] = cf.c;
            cell.h_out[o] = f2bf(hv);
            if (cell.hdrop_out) {
              const bool keep =
                  cell.drop_p <= 0.f || dropout_keep(dseed, cell.step, r, u, cell.drop_p);
              cell.hdrop_out[(int64_t)r * cell.ldh + u] = f2bf(keep ? hv * inv_keep : 0.f);
            }
            if (cell.gates_out) {
              uint2 pk;
              pk.x = (uint32_t)f2bf(cf.s0) | ((uint32_t)f2bf(cf.s1) << 16);
              pk.y = (uint32_t)f2bf(cf.s2) | ((uint32_t)f2bf(cf.s3) << 16);
              *reinterpret_cast<uint2*>(cell.gates_out + (int64_t)r * 4 * H + 4 * u) = pk;
            }
          }
        }
      }
    }
  }
  if (counts != nullptr && tok_out != nullptr) {
    __syncthreads();
    // idempotent flag store into this block's slot: no same-address atomics
    // from all 640 blocks (those cost ~5 us per decode step)
    if (threadIdx.x == 0 && s_nonzero > 0)
      counts[(count_step * CMB_CNT_SLOTS + blockIdx.x % CMB_CNT_SLOTS) * CMB_CNT_STRIDE] = 1;
  }
}

// One launch = vocab projection of step t (rows hd_t) + the recurrent GEMM of
// step t+1 (pre_{t+1} = h_t W_hh^T + vgate, lstm_gemm.h).  The two are
// independent, so the LSTM's latency-bound GEMM fills the CUs the vocab
// tiles leave idle instead of running before it.  The first n_lstm_pad
// blocks (a multiple of 8, so both halves keep their XCD-aware mapping) are
// LSTM tiles.
// ATT: the first n_att workgroups (a multiple of 8, like the LSTM tiles) are
// the MFMA temporal attention of step t+1, one per video (att_mfma.h): they
// depend only on h_t too, and are dispatched first, so they finish under the
// vocabulary tiles.
template <int BN, int STAGES, int OCC, class LT, int AV, bool TOPK = false, bool PH = false>
__global__ __launch_bounds__(256, OCC) void vocab_lstm_fwd_kernel(
    VOCAB_TR_PARAMS, const uint16_t* __restrict__ h_t, const uint16_t* __restrict__ whh,
    const float* __restrict__ vgate, int vdiv, float* __restrict__ pre, int n_lstm_pad, int NQ,
    float* __restrict__ q_out, AttMfmaArgs att, int n_att) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int bid = blockIdx.x;
  if constexpr (AV != 0) {
    // (dispatched after the vocabulary tiles instead, into their drain:
    // att8 5.48-5.51 vs 5.19-5.22 ms per step, profiles/r3/ab_att_last.txt)
    if (bid < n_att) {
      if (bid < att_mfma_nblocks(att)) att_mfma_fwd_any<AV>(bid, att, lds);
      return;
    }
    bid -= n_att;
  }
  if (bid < n_lstm_pad) {
    if (bid < lstm_gemm_blocks(R, H, NQ))
      lstm_gemm_block<LT, PH>(bid, h_t, R, H, whh, vgate, vdiv, pre, lds, NQ, q_out);
    return;
  }
  vocab_tr_block<BN, STAGES, TOPK>(bid - n_lstm_pad, lds, VOCAB_TR_ARGS);
}

// XE all rows (engine.cpp): the first n_lstm_pad workgroups run the WHOLE
// LSTM step of the next rows (lstm_gemm.h lstm_cell_block: the input token is
// the label, so the cell needs no combine), the rest the vocabulary tiles of
// the current rows.  Either part may be empty.
template <int BN, int STAGES, int OCC>
__global__ __launch_bounds__(256, OCC) void vocab_lstm_xe_kernel(
    VOCAB_TR_PARAMS, const uint16_t* __restrict__ h_t, const uint16_t* __restrict__ whh,
    const float* __restrict__ vgate, int vdiv, XeCell xc, int n_lstm_pad) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int bid = blockIdx.x;
  if (bid < n_lstm_pad) {
    if (bid < lstm_gemm_blocks(R, H)) lstm_cell_block<LGTile2>(bid, h_t, R, H, whh, vgate, vdiv, xc, rng, lds);
    return;
  }
  vocab_tr_block<BN, STAGES>(bid - n_lstm_pad, lds, VOCAB_TR_ARGS);
}

// Exp-store conversion of one decode step's saved fp16 logits, in place:
// E = bf16(exp(x - lse_r)).  Used for step 0 only, whose rows have no
// previous-step LSE to offset by in the decode kernel (steps >= 1 write E
// directly, VF_EXP).  One block per row, 8 entries (16 bytes) per thread and
// iteration; the ragged tail (V % 8) scalar.
__global__ __launch_bounds__(256) void vocab_exp_convert_kernel(uint16_t* __restrict__ buf,
                                                                int64_t ldl, int V,
                                                                const float* __restrict__ lse) {
  const int r = blockIdx.x;
  uint16_t* row = buf + (int64_t)r * ldl;
  const float L = lse[r];
  const int nvec = V >> 3;
  for (int i = threadIdx.x; i < nvec; i += 256) {
    uint4 x = *reinterpret_cast<const uint4*>(row + 8 * i);
    uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      w[k] = (uint32_t)f2bf(__expf(h2f(w[k] & 0xffff) - L)) |
             ((uint32_t)f2bf(__expf(h2f(w[k] >> 16) - L)) << 16);
    *reinterpret_cast<uint4*>(row + 8 * i) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  const int v = 8 * nvec + (int)threadIdx.x;
  if (v < V) row[v] = f2bf(__expf(h2f(row[v]) - L));
}

// -------------------------------------------------------------------------------
// Launchers.  Tiles: 128 vocab x 64 caption rows, 2 LDS stages (48 KB, 3
// blocks per CU).
template <int BN, int STAGES, int OCC, bool TOPK = false>
static void launch_vocab_fwd_tr(const uint16_t* hd, int ldh, int R, int H, const uint16_t* W,
                                const float* bias, int V, uint16_t* logits16, int64_t ldl,
                                void* part, const int64_t* tgt, int64_t tgt_stride, int flags,
                                float inv_temp, const uint32_t* rng, int step,
                                hipStream_t stream, const float* eoff = nullptr) {
  using TL = Tile<VT_V, BN, STAGES>;
  constexpr int LDS = TL::STAGES * TL::STAGE_BYTES > epilogue_lds_bytes(BN)
                          ? TL::STAGES * TL::STAGE_BYTES
                          : epilogue_lds_bytes(BN);
  const int n_vt = (V + VT_V - 1) / VT_V, n_rt = (R + BN - 1) / BN;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)vocab_fwd_tr_kernel<BN, STAGES, OCC, TOPK>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr_set = true;
  }
  hipLaunchKernelGGL((vocab_fwd_tr_kernel<BN, STAGES, OCC, TOPK>), dim3(n_vt * n_rt), dim3(256), LDS,
                     stream, hd, ldh, R, H, W, bias, V, logits16, ldl, (VocabPartial*)part, tgt,
                     tgt_stride, flags, inv_temp, rng, step, eoff);
  post_launch("vocab_fwd_tr_kernel", stream);
}

void launch_vocab_fwd(const uint16_t* hd, int ldh, int R, int H, const uint16_t* W,
                      const float* bias, int V, uint16_t* logits16, int64_t ldl, void* part,
                      const int64_t* tgt, int64_t tgt_stride, int flags, float inv_temp,
                      const uint32_t* rng, int step, hipStream_t stream, const float* eoff) {
  // (microbenchmark at V = 10,509: 31.0 vs 33.5 us at R = 1280, 8.7 vs 12.4
  // us at R = 64 against 128-row tiles, 2 blocks per CU)
  if (flags & VF_TOPK) {
    if (vf_topk_k(flags) < 1 || vf_topk_k(flags) > VF_TOPK_MAXK)
      throw std::runtime_error("vocab_fwd: VF_TOPK needs 1 <= K <= 8");
    launch_vocab_fwd_tr<64, 2, 3, true>(hd, ldh, R, H, W, bias, V, logits16, ldl, part, tgt,
                                        tgt_stride, flags, inv_temp, rng, step, stream, eoff);
    return;
  }
  launch_vocab_fwd_tr<64, 2, 3>(hd, ldh, R, H, W, bias, V, logits16, ldl, part, tgt, tgt_stride,
                                flags, inv_temp, rng, step, stream, eoff);
}

// microbenchmark only (scripts/microbench_kernels.py): other tile / pipeline
// shapes of the vocab kernel, <BN, STAGES, OCC>
void launch_vocab_fwd_variant(int variant, const uint16_t* hd, int ldh, int R, int H,
                              const uint16_t* W, const float* bias, int V, uint16_t* logits16,
                              int64_t ldl, void* part, const int64_t* tgt, int64_t tgt_stride,
                              int flags, float inv_temp, const uint32_t* rng, int step,
                              hipStream_t stream) {
#define VV(BN, ST, OC)                                                                          \
  launch_vocab_fwd_tr<BN, ST, OC>(hd, ldh, R, H, W, bias, V, logits16, ldl, part, tgt, tgt_stride, \
                                  flags, inv_temp, rng, step, stream)
  switch (variant) {
    case 1: VV(128, 3, 1); break;
    case 2: VV(128, 4, 1); break;
    case 3: VV(64, 3, 2); break;
    case 5: VV(64, 4, 1); break;
    case 6: VV(128, 2, 2); break;
    default: VV(64, 2, 3); break;
  }
#undef VV
}

int vocab_num_tiles(int V) { return (V + VT_V - 1) / VT_V; }
int vocab_partial_bytes() { return (int)sizeof(VocabPartial); }

void launch_vocab_combine(const void* part, int n_vt, int R, float* lse_out, int64_t* tok_out,
                          int64_t tok_stride, float* g_sel, int64_t gsel_stride, float* g_xe,
                          int64_t gxe_stride, const int64_t* gt, int64_t gt_stride, int mode,
                          float ss_prob, const uint32_t* rng, int step, int* counts,
                          int count_step, uint8_t* unfinished, hipStream_t stream,
                          const CellLaunch* cl, int rows_per_step) {
  const int Rs = rows_per_step > 0 ? rows_per_step : R;
  if (R % Rs != 0) throw std::runtime_error("vocab_combine: R must be a multiple of rows_per_step");
  CellArgs cell{};
  if (cl != nullptr) {
    cell = CellArgs{cl->pre, cl->vg16, cl->ptab, cl->c_prev, cl->c_out, cl->h_out,
                    cl->hdrop_out, cl->ldh, cl->gates_out, cl->H, cl->drop_p, cl->step, cl->cell,
                    cl->pre_half};
  }
  // (fp16 pre as a template parameter: a runtime select between the two
  // load forms cost 1.6 us per combine, 14.3 vs 12.7 us in rocprofv3)
  // rows (wavefronts) per workgroup, CSTCAP_CMB_ROWS = 1 / 4 / 8: 4 by default
  // (headline 3.072-3.081 vs 3.095-3.119 ms per step with one row per
  // workgroup, three interleaved pairs, profiles/r6/s2/cmb_rows/)
  static const int rows_wg = [] {
    const char* e = getenv("CSTCAP_CMB_ROWS");
    const int v = e != nullptr ? atoi(e) : 4;
    return v == 1 || v == 8 ? v : 4;
  }();
  auto kern = rows_wg == 4   ? (cell.pre_half ? vocab_combine_kernel<CMB_LANES, true, 4 * CMB_LANES>
                                              : vocab_combine_kernel<CMB_LANES, false, 4 * CMB_LANES>)
              : rows_wg == 8 ? (cell.pre_half ? vocab_combine_kernel<CMB_LANES, true, 8 * CMB_LANES>
                                              : vocab_combine_kernel<CMB_LANES, false, 8 * CMB_LANES>)
                             : (cell.pre_half ? vocab_combine_kernel<CMB_LANES, true>
                                              : vocab_combine_kernel<CMB_LANES, false>);
  hipLaunchKernelGGL(kern, dim3((R + rows_wg - 1) / rows_wg),
                     dim3(rows_wg * CMB_LANES), 0, stream, (const VocabPartial*)part, n_vt, R, lse_out,
                     tok_out, tok_stride, g_sel, gsel_stride, g_xe, gxe_stride, gt, gt_stride, mode,
                     ss_prob, rng, step, counts, count_step, unfinished, cell, Rs);
  post_launch("vocab_combine_kernel", stream);
}

template <int BN, int STAGES, int OCC, class LT, int AV, bool TOPK = false, bool PH = false>
static void launch_vocab_lstm_t(const uint16_t* hd, int ldh, int R, int H, const uint16_t* W,
                                const float* bias, int V, uint16_t* logits16, int64_t ldl,
                                void* part, const int64_t* tgt, int64_t tgt_stride, int flags,
                                float inv_temp, const uint32_t* rng, int step, const uint16_t* h_t,
                                const uint16_t* whh, const float* vgate, int vdiv, float* pre,
                                int NQ, float* q_out, hipStream_t stream, const float* eoff,
                                const AttMfmaArgs* att) {
  using TL = Tile<VT_V, BN, STAGES>;
  constexpr int LV = TL::STAGES * TL::STAGE_BYTES > epilogue_lds_bytes(BN)
                         ? TL::STAGES * TL::STAGE_BYTES
                         : epilogue_lds_bytes(BN);
  constexpr int LDS = LV > LT::LDS_BYTES ? LV : LT::LDS_BYTES;
  static_assert(AV == 0 || LDS >= 48 * 1024, "attention workgroups assume 48 KB of LDS");
  const int n_vt = (V + VT_V - 1) / VT_V, n_rt = (R + BN - 1) / BN;
  AttMfmaArgs a{};
  int n_att = 0;
  if (AV != 0) {
    a = *att;
    n_att = (att_mfma_nblocks(a) + 7) / 8 * 8;
  }
  const int n_l = pre != nullptr ? (lstm_gemm_blocks(R, H, NQ) + 7) / 8 * 8 : 0;
  const int grid = n_att + n_l + n_vt * n_rt;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)vocab_lstm_fwd_kernel<BN, STAGES, OCC, LT, AV, TOPK, PH>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr_set = true;
  }
  hipLaunchKernelGGL((vocab_lstm_fwd_kernel<BN, STAGES, OCC, LT, AV, TOPK, PH>), dim3(grid), dim3(256),
                     LDS, stream, hd, ldh, R, H, W, bias, V, logits16, ldl, (VocabPartial*)part,
                     tgt, tgt_stride, flags, inv_temp, rng, step, eoff, h_t, whh, vgate, vdiv, pre,
                     n_l, NQ, q_out, a, n_att);
  post_launch("vocab_lstm_fwd_kernel", stream);
}

int vocab_part_slots(int V) { return (V + VT_V - 1) / VT_V; }


int launch_vocab_lstm_fwd(const uint16_t* hd, int ldh, int R, int H, const uint16_t* W,
                          const float* bias, int V, uint16_t* logits16, int64_t ldl, void* part,
                          const int64_t* tgt, int64_t tgt_stride, int flags, float inv_temp,
                          const uint32_t* rng, int step, const uint16_t* h_t, const uint16_t* whh,
                          const float* vgate, int vdiv, float* pre, hipStream_t stream, int NQ,
                          float* q_out, const float* eoff, const AttMfmaArgs* att, int pre_half) {
  // 64-row tiles, 3 blocks per CU (48 KB of LDS each; the recurrent tiles use
  // 2 stages to fit): one block's epilogue overlaps the others' main loops.
  // Measured 4.47 vs 4.54 ms per step against 128-row tiles at 2 blocks per
  // CU (3 interleaved rounds; profiles/r2/ab_vocab_tiles.txt)
  if ((flags & VF_TOPK) && pre_half) throw std::runtime_error("vocab_lstm_fwd: fp16 pre with VF_TOPK");
  if (flags & VF_TOPK) {  // beam search: per-tile top-K candidates
    if (vf_topk_k(flags) < 1 || vf_topk_k(flags) > VF_TOPK_MAXK)
      throw std::runtime_error("vocab_lstm_fwd: VF_TOPK needs 1 <= K <= 8");
    static const int beam_bn = [] {
      const char* e = getenv("CSTCAP_BEAM_BN");
      return e != nullptr && atoi(e) == 128 ? 128 : 64;
    }();
    if (att == nullptr && beam_bn == 128) {
      // 128-row tiles: the vocabulary matrix streamed ceil(R / 128) instead
      // of ceil(R / 64) times per step -- measured slower at the headline
      // beam shape (R = 320: 1.31 vs 1.09 ms per 64-video batch, 249
      // workgroups at 2 per CU against 415 at 3, profiles/r6/README_r6.md)
      launch_vocab_lstm_t<128, 2, 2, LGTile2, 0, true>(hd, ldh, R, H, W, bias, V, logits16, ldl,
                                                       part, tgt, tgt_stride, flags, inv_temp, rng,
                                                       step, h_t, whh, vgate, vdiv, pre, NQ, q_out,
                                                       stream, eoff, nullptr);
      return vocab_num_tiles(V);
    }
    if (att == nullptr) {
      launch_vocab_lstm_t<64, 2, 3, LGTile2, 0, true>(hd, ldh, R, H, W, bias, V, logits16, ldl,
                                                      part, tgt, tgt_stride, flags, inv_temp, rng,
                                                      step, h_t, whh, vgate, vdiv, pre, NQ, q_out,
                                                      stream, eoff, nullptr);
      return vocab_num_tiles(V);
    }
    // beam search with temporal attention: the attention workgroups compute
    // every current row's next video gates (vg16) from its own h_t; the fused
    // beam step then picks the parent's row, like pre
    check_att_mfma(*att);
#define VT(AVX)                                                                                 \
  case AVX:                                                                                      \
    launch_vocab_lstm_t<64, 2, 3, LGTile2, AVX, true>(hd, ldh, R, H, W, bias, V, logits16, ldl,   \
                                                      part, tgt, tgt_stride, flags, inv_temp, rng, \
                                                      step, h_t, whh, vgate, vdiv, pre, NQ, q_out, \
                                                      stream, eoff, att);                          \
    break;
    switch (att_variant(att->C)) {
      ATT_VARIANTS(VT)
      default: throw std::runtime_error("vocab_lstm_fwd: no attention variant");
    }
#undef VT
    return vocab_num_tiles(V);
  }
#define VL(AVX)                                                                                \
  if (pre_half)                                                                                \
    launch_vocab_lstm_t<64, 2, 3, LGTile2, AVX, false, true>(                                  \
        hd, ldh, R, H, W, bias, V, logits16, ldl, part, tgt, tgt_stride, flags, inv_temp, rng, \
        step, h_t, whh, vgate, vdiv, pre, NQ, q_out, stream, eoff, att);                       \
  else                                                                                         \
    launch_vocab_lstm_t<64, 2, 3, LGTile2, AVX>(hd, ldh, R, H, W, bias, V, logits16, ldl, part, \
                                                tgt, tgt_stride, flags, inv_temp, rng, step,  \
                                                h_t, whh, vgate, vdiv, pre, NQ, q_out, stream, \
                                                eoff, att)
  if (att == nullptr) {
    VL(0);
    return vocab_num_tiles(V);
  }
  check_att_mfma(*att);
  switch (att_variant(att->C)) {
#define X(AVX)  \
  case AVX:     \
    VL(AVX);    \
    break;
    ATT_VARIANTS(X)
#undef X
    default: throw std::runtime_error("vocab_lstm_fwd: no attention variant");
  }
#undef VL
  return vocab_num_tiles(V);
}

void launch_vocab_lstm_xe(const uint16_t* hd, int R, int H, const uint16_t* W, const float* bias,
                          int V, uint16_t* logits16, int64_t ldl, void* part, const int64_t* tgt,
                          const uint32_t* rng, const uint16_t* h_t, const uint16_t* whh,
                          const float* vgate, int vdiv, const XeCell* xc, hipStream_t stream) {
  constexpr int BN = 64, STAGES = 2, OCC = 3;
  using TL = Tile<VT_V, BN, STAGES>;
  constexpr int LV = TL::STAGES * TL::STAGE_BYTES > epilogue_lds_bytes(BN)
                         ? TL::STAGES * TL::STAGE_BYTES
                         : epilogue_lds_bytes(BN);
  constexpr int LDS = LV > LGTile2::LDS_BYTES ? LV : LGTile2::LDS_BYTES;
  if (H % 64 != 0 || (xc != nullptr && (h_t == nullptr || vgate == nullptr)))
    throw std::runtime_error("vocab_lstm_xe: unsupported operands");
  const int n_vt = (V + VT_V - 1) / VT_V, n_rt = (R + BN - 1) / BN;
  const int n_l = xc != nullptr ? (lstm_gemm_blocks(R, H) + 7) / 8 * 8 : 0;
  const int grid = n_l + (hd != nullptr ? n_vt * n_rt : 0);
  if (grid == 0) return;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)vocab_lstm_xe_kernel<BN, STAGES, OCC>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr_set = true;
  }
  const XeCell x = xc != nullptr ? *xc : XeCell{};
  hipLaunchKernelGGL((vocab_lstm_xe_kernel<BN, STAGES, OCC>), dim3(grid), dim3(256), LDS, stream,
                     hd, H, R, H, W, bias, V, logits16, ldl, (VocabPartial*)part, tgt, 1,
                     /*flags: VF_EXP*/ 16, 1.f, rng, 0, nullptr, h_t, whh, vgate, vdiv, x, n_l);
  post_launch("vocab_lstm_xe_kernel", stream);
}

void launch_vocab_exp_convert(uint16_t* buf, int64_t ldl, int V, int R, const float* lse,
                              hipStream_t stream) {
  hipLaunchKernelGGL(vocab_exp_convert_kernel, dim3(R), dim3(256), 0, stream, buf, ldl, V, lse);
  post_launch("vocab_exp_convert_kernel", stream);
}

}  // namespace cst
