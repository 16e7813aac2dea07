// P10 FeatPool, fused: per modality Linear -> ReLU -> Dropout, concatenated
// (reference /root/reference/model.py:46-69), forward and weight backward.
//
// The reference (and the plain PyTorch path) runs, per modality, one small
// GEMM (64 videos x 512 x d_f), a ReLU, a dropout and finally a concat -- ~15
// latency-bound launches forward and as many backward, ~0.2 ms per SCST step
// on MI355X.  Here:
//   * forward: ONE launch of 64 x 64 output tiles for every modality at once,
//     split over K (256-wide chunks) so ~240 workgroups fill the chip; fp32
//     operands (the module keeps the reference's fp32 precision -- plain bf16
//     operands would move ReLU decisions near zero and with them whole
//     gradient terms), split into bf16 hi + lo on the bf16 matrix cores (see
//     fp_mfma_step); partial tiles go to a workspace and
//     a second launch sums them, adds the bias, applies ReLU and the dropout
//     mask (counter hash of (seed, row, column), like the decoder's dropout)
//     and writes the concatenated (rows, F*H) output;
//   * backward: ONE launch computes dW_f = dz^T x_f for every modality, with
//     dz = dout * [out > 0] / (1 - p) formed while loading (ReLU and dropout
//     backward from the saved output alone: out > 0 iff the unit was kept and
//     its pre-activation was positive), and the bias gradient in the blocks
//     of the first K tile.  The features need no gradient.
#include "../common.h"
#include "../launchers.h"

namespace cst {

constexpr int FP_T = 64;     // output tile (rows x units, or units x k)
constexpr int FP_KS = 32;    // K step per LDS stage
constexpr int FP_KCH = 256;  // forward split-K chunk
constexpr int FP_LDA = FP_KS + 1;  // fp32 row stride in LDS (conflict-free column reads)
constexpr int FEATPOOL_DROP_KEY = 0x46504C;  // dropout_keep "step" key of FeatPool

// One 64x64 tile += A(64 x KS) B(64 x KS)^T from fp32 LDS tiles (row stride
// FP_LDA): wave w owns the 32x32 quarter (w >> 1, w & 1).  The fp32 operands
// are split in registers into hi = bf16(x) and lo = bf16(x - hi) (x = hi + lo
// to 2^-16 relative) and each 16-deep step is three bf16 MFMAs (hi hi + hi lo
// + lo hi, fp32 accumulate; the dropped lo lo term is below 2^-16): products
// within ~2^-16 of fp32 for 6 x 32 instead of 16 x 64 matrix-core cycles per
// 32-deep K step (v_mfma_f32_32x32x16_bf16 vs v_mfma_f32_32x32x2_f32, whose
// fp32 rate is 1/16 of bf16; the att8 frame FeatPool over 512 rows took 49 us
// forward and 55 us backward on the fp32 matrix cores).
// 32x32x16 bf16: lane l supplies row / column l % 32 at k = 8 (l / 32) + 0..7
// (the same LDS words the fp32 form read, conflict-free with stride FP_LDA).
__device__ __forceinline__ void fp_mfma_step(const float* As, const float* Bs, f32x16& acc) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1;
  const float* ar = As + (wr * 32 + (lane & 31)) * FP_LDA + 8 * (lane >> 5);
  const float* br = Bs + (wc * 32 + (lane & 31)) * FP_LDA + 8 * (lane >> 5);
#pragma unroll
  for (int s = 0; s < FP_KS / 16; ++s) {
    bf16x8 ah, al, bh, bl;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float a = ar[16 * s + e], b = br[16 * s + e];
      const __bf16 ha = (__bf16)a, hb = (__bf16)b;
      ah[e] = ha, al[e] = (__bf16)(a - (float)ha);
      bh[e] = hb, bl[e] = (__bf16)(b - (float)hb);
    }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  }
}

// (row, col) of accumulator element r of lane `lane` in the 64x64 tile
__device__ __forceinline__ int acc_row(int r, int lane, int wr) {
  return wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}

// ---- forward: partial tiles --------------------------------------------------
// block -> (modality f, row tile, unit tile, K chunk); partial 64x64 tile to ws
__global__ __launch_bounds__(256) void featpool_fwd_partial_kernel(FeatPoolArgs a, float* ws) {
  __shared__ float As[2][FP_T * FP_LDA];
  __shared__ float Bs[2][FP_T * FP_LDA];
  int f = 0;
  while (f + 1 < a.nf && (int)blockIdx.x >= a.s[f + 1].blk0) ++f;
  const FeatPoolSeg& g = a.s[f];
  int b = (int)blockIdx.x - g.blk0;
  const int nkc = (g.d + FP_KCH - 1) / FP_KCH, nut = a.H / FP_T;
  const int kc = b % nkc;
  b /= nkc;
  const int ut = b % nut, rt = b / nut;
  const int r0 = rt * FP_T, u0 = ut * FP_T, k0 = kc * FP_KCH;
  const int kend = min(g.d, k0 + FP_KCH);
  const int tid = threadIdx.x;
  // each thread stages 2 float4 of A and of B per K step: tile row tid/8 + 32 i,
  // columns 4 (tid % 8)
  float4 ra[2], rb[2];
  auto load = [&](int k) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (tid >> 3) + 32 * i, kk = k + 4 * (tid & 7);
      const bool kin = kk < kend;  // d % 4 == 0 (host check): a float4 is in or out
      const int r = r0 + row;
      ra[i] = (kin && r < a.rows) ? *reinterpret_cast<const float4*>(g.x + (int64_t)r * g.ld + kk)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
      rb[i] = kin ? *reinterpret_cast<const float4*>(g.w + (int64_t)(u0 + row) * g.d + kk)
                  : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto stage = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (tid >> 3) + 32 * i, kk = 4 * (tid & 7);
      float* pa = &As[buf][row * FP_LDA + kk];
      float* pb = &Bs[buf][row * FP_LDA + kk];
      pa[0] = ra[i].x, pa[1] = ra[i].y, pa[2] = ra[i].z, pa[3] = ra[i].w;
      pb[0] = rb[i].x, pb[1] = rb[i].y, pb[2] = rb[i].z, pb[3] = rb[i].w;
    }
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int nks = (kend - k0 + FP_KS - 1) / FP_KS;
  load(k0);
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    stage(buf);
    __syncthreads();
    if (ks + 1 < nks) load(k0 + (ks + 1) * FP_KS);  // in flight under the MFMAs
    fp_mfma_step(As[buf], Bs[buf], acc);
  }
  const int lane = tid & 63, w = tid >> 6, wr = w >> 1, wc = w & 1;
  float* out = ws + (int64_t)blockIdx.x * FP_T * FP_T;
#pragma unroll
  for (int r = 0; r < 16; ++r)
    out[acc_row(r, lane, wr) * FP_T + wc * 32 + (lane & 31)] = acc[r];
}

// ---- forward: sum of the K chunks + bias + ReLU + dropout -> (rows, F*H) ------
__global__ __launch_bounds__(256) void featpool_fwd_epilogue_kernel(FeatPoolArgs a, const float* ws,
                                                                    float* out, float drop_p,
                                                                    const uint32_t* rng) {
  const int FH = a.nf * a.H;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)a.rows * FH) return;
  const int r = (int)(i / FH), col = (int)(i % FH);
  const int f = col / a.H, u = col % a.H;
  const FeatPoolSeg& g = a.s[f];
  const int nkc = (g.d + FP_KCH - 1) / FP_KCH, nut = a.H / FP_T;
  const int rt = r / FP_T, ut = u / FP_T;
  const int base = g.blk0 + (rt * nut + ut) * nkc;
  // the K chunks' partials: 8 loads in flight per thread (4 independent sums)
  // instead of one dependent load per chunk (up to 16 chunks per modality)
  const float* src = ws + (int64_t)base * FP_T * FP_T + (r % FP_T) * FP_T + (u % FP_T);
  float zs[4] = {g.b[u], 0.f, 0.f, 0.f};
  int kc = 0;
  for (; kc + 8 <= nkc; kc += 8) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = src[(int64_t)(kc + e) * FP_T * FP_T];
#pragma unroll
    for (int e = 0; e < 8; ++e) zs[e & 3] += v[e];
  }
  for (; kc < nkc; ++kc) zs[kc & 3] += src[(int64_t)kc * FP_T * FP_T];
  const float z = (zs[0] + zs[1]) + (zs[2] + zs[3]);
  float y = fmaxf(z, 0.f);
  if (drop_p > 0.f) {
    const bool keep = dropout_keep(rng_seed(rng, RNG_SLOT_DROPOUT), FEATPOOL_DROP_KEY, r, col, drop_p);
    y = keep ? y * (1.f / (1.f - drop_p)) : 0.f;
  }
  out[i] = y;
}

// ---- backward: dW_f = dz^T x_f, db_f = sum_rows dz ----------------------------
// block -> (modality f, unit tile, k tile); K = rows in steps of FP_KS
__global__ __launch_bounds__(256) void featpool_bwd_kernel(FeatPoolArgs a, const float* dout,
                                                           const float* outp, float inv_keep,
                                                           FeatPoolGrads gr) {
  __shared__ float As[FP_T * FP_LDA];  // dz^T: units x rows
  __shared__ float Bs[FP_T * FP_LDA];  // x^T: k x rows
  int f = 0;
  while (f + 1 < a.nf && (int)blockIdx.x >= a.s[f + 1].bblk0) ++f;
  const FeatPoolSeg& g = a.s[f];
  int b = (int)blockIdx.x - g.bblk0;
  const int nkt = (g.d + FP_T - 1) / FP_T;
  const int kt = b % nkt, ut = b / nkt;
  const int u0 = ut * FP_T, k0 = kt * FP_T, FH = a.nf * a.H;
  const int tid = threadIdx.x;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float dbias = 0.f;  // kt == 0 blocks, thread tid < 64: unit u0 + tid
  // 32 rows x 64 columns of dz and of x per K step: 2 float4 of each per
  // thread.  The next step's rows are requested before this step's MFMAs, so
  // their latency hides under the math (a K loop of 16 steps at 512 rows).
  float4 dy[2], yv[2], xv[2];
  auto load = [&](int rs) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rr = (tid >> 4) + 16 * i, c4 = 4 * (tid & 15), r = rs + rr;
      dy[i] = yv[i] = xv[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < a.rows) {
        const int64_t o = (int64_t)r * FH + f * a.H + u0 + c4;
        dy[i] = *reinterpret_cast<const float4*>(dout + o);
        yv[i] = *reinterpret_cast<const float4*>(outp + o);
        if (k0 + c4 < g.d) xv[i] = *reinterpret_cast<const float4*>(g.x + (int64_t)r * g.ld + k0 + c4);
      }
    }
  };
  load(0);
  for (int rs = 0; rs < a.rows; rs += FP_KS) {
    // written transposed (column-major = K-contiguous per unit / k)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rr = (tid >> 4) + 16 * i, c4 = 4 * (tid & 15);
      const float4 d = dy[i], y = yv[i], x = xv[i];
      As[(c4 + 0) * FP_LDA + rr] = y.x > 0.f ? d.x * inv_keep : 0.f;
      As[(c4 + 1) * FP_LDA + rr] = y.y > 0.f ? d.y * inv_keep : 0.f;
      As[(c4 + 2) * FP_LDA + rr] = y.z > 0.f ? d.z * inv_keep : 0.f;
      As[(c4 + 3) * FP_LDA + rr] = y.w > 0.f ? d.w * inv_keep : 0.f;
      Bs[(c4 + 0) * FP_LDA + rr] = x.x;
      Bs[(c4 + 1) * FP_LDA + rr] = x.y;
      Bs[(c4 + 2) * FP_LDA + rr] = x.z;
      Bs[(c4 + 3) * FP_LDA + rr] = x.w;
    }
    __syncthreads();
    if (rs + FP_KS < a.rows) load(rs + FP_KS);
    fp_mfma_step(As, Bs, acc);
    if (kt == 0 && tid < FP_T) {  // bias gradient: this step's dz column of the unit (LDS)
#pragma unroll 8
      for (int rr = 0; rr < FP_KS; ++rr) dbias += As[tid * FP_LDA + rr];
    }
    __syncthreads();
  }
  const int lane = tid & 63, w = tid >> 6, wr = w >> 1, wc = w & 1;
  float* dw = gr.dw[f];
  const int k = k0 + wc * 32 + (lane & 31);
  if (k < g.d) {
#pragma unroll
    for (int r = 0; r < 16; ++r) dw[(int64_t)(u0 + acc_row(r, lane, wr)) * g.d + k] = acc[r];
  }
  if (kt == 0 && tid < FP_T) gr.db[f][u0 + tid] = dbias;
}

void featpool_layout(FeatPoolArgs& a) {
  int blk = 0, bblk = 0;
  const int nrt = (a.rows + FP_T - 1) / FP_T, nut = a.H / FP_T;
  for (int f = 0; f < a.nf; ++f) {
    a.s[f].blk0 = blk;
    a.s[f].bblk0 = bblk;
    blk += nrt * nut * ((a.s[f].d + FP_KCH - 1) / FP_KCH);
    bblk += nut * ((a.s[f].d + FP_T - 1) / FP_T);
  }
  a.fwd_blocks = blk;
  a.bwd_blocks = bblk;
}

void launch_featpool_fwd(const FeatPoolArgs& a, float* ws, float* out, float drop_p,
                         const uint32_t* rng, hipStream_t stream) {
  hipLaunchKernelGGL(featpool_fwd_partial_kernel, dim3(a.fwd_blocks), dim3(256), 0, stream, a, ws);
  post_launch("featpool_fwd_partial_kernel", stream);
  const int64_t n = (int64_t)a.rows * a.nf * a.H;
  hipLaunchKernelGGL(featpool_fwd_epilogue_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     stream, a, (const float*)ws, out, drop_p, rng);
  post_launch("featpool_fwd_epilogue_kernel", stream);
}

void launch_featpool_bwd(const FeatPoolArgs& a, const float* dout, const float* out, float drop_p,
                         const FeatPoolGrads& gr, hipStream_t stream) {
  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  hipLaunchKernelGGL(featpool_bwd_kernel, dim3(a.bwd_blocks), dim3(256), 0, stream, a, dout, out,
                     inv_keep, gr);
  post_launch("featpool_bwd_kernel", stream);
}

}  // namespace cst
