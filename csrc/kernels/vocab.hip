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
// vocab_fwd_kernel  (grid: V/128 vocab tiles x R/128 row tiles, XCD-aware)
//   * C = h_drop(R x H) . W(V x H)^T + b  with v_mfma_f32_32x32x16_bf16;
//   * optional fp16 copy of the logits (the backward's softmax input, so
//     the backward never recomputes the 0.4 TFLOP projection);
//   * per (row, tile) partials: max, sum(exp(x - max)), Gumbel-max sample
//     argmax(x / temp - log(-log u)) with u from Philox(seed, step, row, v)
//     -- exact multinomial sampling from softmax(x / temp) in one pass --,
//     greedy argmax, and the logit of the row's target token.
// vocab_combine_kernel (one wavefront per row)
//   * merges the tile partials: LSE, sampled / greedy / target token and
//     their log-probs; applies the step's token-selection mode (teacher
//     forcing, MIXER sampling, scheduled sampling, greedy) and the
//     reference's end-of-sequence rules (forward(): "all rows emitted EOS ->
//     stop" through a device-side counter; sample(): per-row unfinished
//     mask) without any host synchronisation.
// vocab_bwd_ds_kernel
//   * dlogits = dG_sel (onehot(y_sel) - p) + dG_xe (onehot(y_xe) - p),
//     p = exp(x - lse), written as bf16 in place of the fp16 logits; the two
//     plain GEMMs dH = dS W and dW = dS^T H then run on hipBLASLt.
#include "gemm_tile.h"

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

constexpr int VB_M = 128, VB_N = 128;
using VTile = Tile<VB_M, VB_N>;

// XCD-aware block order: blocks b and b+8 share an XCD (round-robin dispatch),
// so consecutive ids of the remapped index land on the same XCD's L2.  Vocab
// tiles are the outer index: the 8 XCDs each stream a contiguous 1/8 of W
// (~1.3 MB at V=10.5k, H=512) and every row tile re-reads it from their L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

__global__ __launch_bounds__(256, 2) void vocab_fwd_kernel(
    const uint16_t* __restrict__ hd, int ldh, int R, int H, const uint16_t* __restrict__ W,
    const float* __restrict__ bias, int V, uint16_t* __restrict__ logits16, int64_t ldl,
    VocabPartial* __restrict__ part, const int64_t* __restrict__ tgt, int64_t tgt_stride,
    int do_sample, float inv_temp, uint32_t seed, int step) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int n_vt = (V + VB_N - 1) / VB_N, n_rt = (R + VB_M - 1) / VB_M;
  const int b = xcd_remap(blockIdx.x, n_vt * n_rt);
  const int vt = b / n_rt, rt = b % n_rt;
  const int r0 = rt * VB_M, v0 = vt * VB_N;
  const int nk = H / 64;

  f32x16 acc[VTile::TM][VTile::TN];
  auto arow = [&](int row, int kt) {
    const int r = min(r0 + row, R - 1);
    return hd + (int64_t)r * ldh + kt * 64;
  };
  auto brow = [&](int row, int kt) {
    const int v = min(v0 + row, V - 1);
    return W + (int64_t)v * H + kt * 64;
  };
  gemm_nt_mainloop<VTile>(nk, arow, brow, lds, acc);

  float* C = reinterpret_cast<float*>(lds);
  store_acc_to_lds<VTile>(acc, C, [&](int col) {
    const int v = v0 + col;
    return v < V ? bias[v] : 0.f;
  });
  __syncthreads();
  const int tid = threadIdx.x;

  // (a) fp16 logits, row-major coalesced 16-byte stores
  if (logits16 != nullptr) {
#pragma unroll
    for (int i = 0; i < (VB_M * VB_N / 8) / 256; ++i) {
      const int idx = tid + i * 256, row = idx >> 4, c8 = (idx & 15) * 8;
      const int r = r0 + row, v = v0 + c8;
      if (r < R && v < V) {
        const float* src = C + row * VTile::CSTRIDE + c8;
        uint16_t* dst = logits16 + (int64_t)r * ldl + v;
        if (v + 8 <= V) {
          uint4 pk;
          pk.x = (uint32_t)f2h(src[0]) | ((uint32_t)f2h(src[1]) << 16);
          pk.y = (uint32_t)f2h(src[2]) | ((uint32_t)f2h(src[3]) << 16);
          pk.z = (uint32_t)f2h(src[4]) | ((uint32_t)f2h(src[5]) << 16);
          pk.w = (uint32_t)f2h(src[6]) | ((uint32_t)f2h(src[7]) << 16);
          *reinterpret_cast<uint4*>(dst) = pk;
        } else {
          for (int e = 0; e < V - v; ++e) dst[e] = f2h(src[e]);
        }
      }
    }
  }

  // (b) per-row statistics: 2 threads per row, interleaved 4-column groups
  const int row = tid >> 1, h = tid & 1;
  const int r = r0 + row;
  const int rr = min(r, R - 1);
  const int target = tgt != nullptr ? (int)tgt[(int64_t)rr * tgt_stride] : -1;
  const float* Crow = C + row * VTile::CSTRIDE;
  float m = -INFINITY;
  int xidx = 0x7fffffff;
#pragma unroll 4
  for (int j = 0; j < 16; ++j) {
    const int c0 = 4 * (2 * j + h);
    const float4 x = *reinterpret_cast<const float4*>(Crow + c0);
    const int v = v0 + c0;
    const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (v + e < V && xs[e] > m) {
        m = xs[e];
        xidx = v + e;
      }
  }
  float s = 0.f, zval = -INFINITY, zlogit = 0.f, xtgt = -INFINITY;
  int zidx = 0x7fffffff;
#pragma unroll 2
  for (int j = 0; j < 16; ++j) {
    const int c0 = 4 * (2 * j + h);
    const float4 x = *reinterpret_cast<const float4*>(Crow + c0);
    const int v = v0 + c0;
    const float xs[4] = {x.x, x.y, x.z, x.w};
    u32x4 rnd = {0, 0, 0, 0};
    if (do_sample) rnd = philox4x32({(uint32_t)(v >> 2), (uint32_t)rr, RNG_GUMBEL, (uint32_t)step},
                                    seed, 0x2545F491u);
    const uint32_t rs[4] = {rnd.x, rnd.y, rnd.z, rnd.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (v + e >= V) continue;
      s += __expf(xs[e] - m);
      if (v + e == target) xtgt = xs[e];
      if (do_sample) {
        const float g = -__logf(-__logf(u01(rs[e])));
        const float z = xs[e] * inv_temp + g;
        if (z > zval) {
          zval = z;
          zidx = v + e;
          zlogit = xs[e];
        }
      }
    }
  }
  // merge the two threads of the row (adjacent lanes)
  {
    const float m2 = __shfl_xor(m, 1, 64), s2 = __shfl_xor(s, 1, 64);
    const int xi2 = __shfl_xor(xidx, 1, 64);
    const float M = fmaxf(m, m2);
    const float S = (m == -INFINITY ? 0.f : s * __expf(m - M)) +
                    (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - M));
    int xi = (m > m2 || (m == m2 && xidx < xi2)) ? xidx : xi2;
    const float zv2 = __shfl_xor(zval, 1, 64), zl2 = __shfl_xor(zlogit, 1, 64);
    const int zi2 = __shfl_xor(zidx, 1, 64);
    const bool mine = zval > zv2 || (zval == zv2 && zidx < zi2);
    const float xt2 = __shfl_xor(xtgt, 1, 64);
    if (h == 0 && r < R) {
      VocabPartial p;
      p.m = M;
      p.s = S;
      p.zval = mine ? zval : zv2;
      p.zlogit = mine ? zlogit : zl2;
      p.zidx = mine ? zidx : zi2;
      p.xidx = xi;
      p.xtgt = fmaxf(xtgt, xt2);
      p.pad = 0.f;
      part[(int64_t)vt * R + r] = p;
    }
  }
}

// token-selection modes of one decode step
enum SelMode : int { SEL_GT = 0, SEL_SAMPLE = 1, SEL_GREEDY = 2, SEL_SS = 3 };

// 8 lanes per row, 32 rows per 256-thread block: lanes with the same sub-index
// read 32 consecutive partial records (1 KiB) per tile -> coalesced.
constexpr int CMB_LANES = 8, CMB_ROWS = 256 / CMB_LANES;

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

__global__ __launch_bounds__(256) void vocab_combine_kernel(
    const VocabPartial* __restrict__ part, int n_vt, int R, float* __restrict__ lse_out,
    int64_t* __restrict__ tok_out, int64_t tok_stride, float* __restrict__ g_sel,
    int64_t gsel_stride, float* __restrict__ g_xe, int64_t gxe_stride,
    const int64_t* __restrict__ gt, int64_t gt_stride, int mode, float ss_prob,
    uint32_t seed, int step, int* __restrict__ counts, int count_step,
    uint8_t* __restrict__ unfinished) {
  __shared__ int s_nonzero;
  const int sub = threadIdx.x & (CMB_LANES - 1);
  const int r = blockIdx.x * CMB_ROWS + (threadIdx.x / CMB_LANES);
  const bool valid = r < R;
  if (threadIdx.x == 0) s_nonzero = 0;
  RowStat a = {-INFINITY, 0.f, -INFINITY, 0.f, -INFINITY, -INFINITY, 0x7fffffff, 0x7fffffff};
  if (valid) {
    for (int t = sub; t < n_vt; t += CMB_LANES) {
      const VocabPartial p = part[(int64_t)t * R + r];
      merge_stat(a, p.m, p.s, p.zval, p.zlogit, p.zidx, p.m, p.xidx, p.xtgt);
    }
  }
#pragma unroll
  for (int o = 1; o < CMB_LANES; o <<= 1) {
    merge_stat(a, __shfl_xor(a.m, o, 64), __shfl_xor(a.s, o, 64), __shfl_xor(a.zv, o, 64),
               __shfl_xor(a.zl, o, 64), __shfl_xor(a.zi, o, 64), __shfl_xor(a.xm, o, 64),
               __shfl_xor(a.xi, o, 64), __shfl_xor(a.xt, o, 64));
  }
  __syncthreads();  // s_nonzero initialised
  if (valid && sub == 0) {
    const float lse = a.m + __logf(a.s);
    if (lse_out) lse_out[r] = lse;
    if (g_xe) g_xe[(int64_t)r * gxe_stride] = a.xt - lse;
    if (tok_out != nullptr) {
      const int64_t gt_tok = gt ? gt[(int64_t)r * gt_stride] : 0;
      int64_t tok;
      float tl;
      switch (mode) {
        case SEL_SAMPLE: tok = a.zi; tl = a.zl; break;
        case SEL_GREEDY: tok = a.xi; tl = a.xm; break;
        case SEL_SS: {
          const u32x4 u = philox4x32({(uint32_t)r, RNG_SS, (uint32_t)step, 0u}, seed, 0x68E31DA4u);
          const bool use_sample = u01(u.x) < ss_prob;
          tok = use_sample ? (int64_t)a.zi : gt_tok;
          tl = use_sample ? a.zl : a.xt;
          break;
        }
        default: tok = gt_tok; tl = a.xt; break;
      }
      // reference forward(): once every row emitted EOS at one step, decoding stops
      if (counts != nullptr) {
        bool dead = false;
        for (int k = 1; k < count_step; ++k) dead |= (counts[k] == 0);
        if (dead) tok = 0;
      }
      // per-row finished mask: reference sample(), or forward() with the
      // --mask_after_eos fix
      if (unfinished != nullptr) {
        const uint8_t u = unfinished[r] && (tok > 0);
        unfinished[r] = u;
        if (!u) tok = 0;
      }
      tok_out[(int64_t)r * tok_stride] = tok;
      if (g_sel) g_sel[(int64_t)r * gsel_stride] = tl - lse;
      if (counts != nullptr && tok != 0) atomicAdd(&s_nonzero, 1);
    }
  }
  if (counts != nullptr && tok_out != nullptr) {
    __syncthreads();
    if (threadIdx.x == 0 && s_nonzero > 0) atomicAdd(&counts[count_step], s_nonzero);
  }
}

__global__ __launch_bounds__(256) void vocab_bwd_ds_kernel(
    uint16_t* __restrict__ buf, int64_t ldl, int V, int R, int T, int T_sel,
    const float* __restrict__ lse, const int64_t* __restrict__ y_sel, int64_t ysel_rs,
    const float* __restrict__ dg_sel, int64_t dgsel_rs, const int64_t* __restrict__ y_xe,
    int64_t yxe_rs, const float* __restrict__ dg_xe, int64_t dgxe_rs) {
  // one block per (t, r) row of the [T][R][ldl] buffer
  const int64_t rowid = blockIdx.x;
  const int t = (int)(rowid / R), r = (int)(rowid % R);
  const bool has_sel = dg_sel != nullptr && t < T_sel;
  const float a = has_sel ? dg_sel[(int64_t)r * dgsel_rs + t] : 0.f;
  const float bb = dg_xe ? dg_xe[(int64_t)r * dgxe_rs + t] : 0.f;
  const int ys = has_sel ? (int)y_sel[(int64_t)r * ysel_rs + t] : -1;
  const int yx = dg_xe ? (int)y_xe[(int64_t)r * yxe_rs + t] : -1;
  const float L = lse[rowid];
  const float ab = a + bb;
  uint16_t* row = buf + rowid * ldl;
  const int nvec = V >> 3;
  for (int i = threadIdx.x; i < nvec; i += 256) {
    uint4 x = *reinterpret_cast<const uint4*>(row + i * 8);
    uint32_t ws[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int v = i * 8 + 2 * k;
      float lo = -ab * __expf(h2f(ws[k] & 0xffff) - L);
      float hi = -ab * __expf(h2f(ws[k] >> 16) - L);
      lo += (v == ys ? a : 0.f) + (v == yx ? bb : 0.f);
      hi += (v + 1 == ys ? a : 0.f) + (v + 1 == yx ? bb : 0.f);
      ws[k] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
    }
    *reinterpret_cast<uint4*>(row + i * 8) = make_uint4(ws[0], ws[1], ws[2], ws[3]);
  }
  for (int v = (nvec << 3) + threadIdx.x; v < V; v += 256) {
    float d = -ab * __expf(h2f(row[v]) - L) + (v == ys ? a : 0.f) + (v == yx ? bb : 0.f);
    row[v] = f2bf(d);
  }
}

// -------------------------------------------------------------------------------
void launch_vocab_fwd(const uint16_t* hd, int ldh, int R, int H, const uint16_t* W,
                      const float* bias,
                      int V, uint16_t* logits16, int64_t ldl, void* part, const int64_t* tgt,
                      int64_t tgt_stride, int do_sample, float inv_temp, uint32_t seed, int step,
                      hipStream_t stream) {
  const int n_vt = (V + VB_N - 1) / VB_N, n_rt = (R + VB_M - 1) / VB_M;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)vocab_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        VTile::LDS_BYTES);
    attr_set = true;
  }
  hipLaunchKernelGGL(vocab_fwd_kernel, dim3(n_vt * n_rt), dim3(256), VTile::LDS_BYTES, stream,
                     hd, ldh, R, H, W, bias, V, logits16, ldl, (VocabPartial*)part, tgt, tgt_stride,
                     do_sample, inv_temp, seed, step);
}

int vocab_num_tiles(int V) { return (V + VB_N - 1) / VB_N; }
int vocab_partial_bytes() { return (int)sizeof(VocabPartial); }
int vocab_fwd_lds_bytes() { return VTile::LDS_BYTES; }

void launch_vocab_combine(const void* part, int n_vt, int R, float* lse_out, int64_t* tok_out,
                          int64_t tok_stride, float* g_sel, int64_t gsel_stride, float* g_xe,
                          int64_t gxe_stride, const int64_t* gt, int64_t gt_stride, int mode,
                          float ss_prob, uint32_t seed, int step, int* counts, int count_step,
                          uint8_t* unfinished, hipStream_t stream) {
  hipLaunchKernelGGL(vocab_combine_kernel, dim3((R + CMB_ROWS - 1) / CMB_ROWS), dim3(256), 0,
                     stream,
                     (const VocabPartial*)part, n_vt, R, lse_out, tok_out, tok_stride, g_sel,
                     gsel_stride, g_xe, gxe_stride, gt, gt_stride, mode, ss_prob, seed, step,
                     counts, count_step, unfinished);
}

void launch_vocab_bwd_ds(uint16_t* buf, int64_t ldl, int V, int R, int T, int T_sel,
                         const float* lse, const int64_t* y_sel, int64_t ysel_rs,
                         const float* dg_sel, int64_t dgsel_rs, const int64_t* y_xe,
                         int64_t yxe_rs, const float* dg_xe, int64_t dgxe_rs, hipStream_t stream) {
  hipLaunchKernelGGL(vocab_bwd_ds_kernel, dim3((unsigned)((int64_t)T * R)), dim3(256), 0, stream,
                     buf, ldl, V, R, T, T_sel, lse, y_sel, ysel_rs, dg_sel, dgsel_rs, y_xe,
                     yxe_rs, dg_xe, dgxe_rs);
}

}  // namespace cst
