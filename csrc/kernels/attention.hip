// K11-ext: temporal attention over the num_chunks frame vectors of a video,
// per decode step, forward and backward.
//
// The reference only declares temporal attention (`--num_chunks`, "> 1:
// attention with num_chunks", /root/reference/opts.py:241-245; the loader
// allocates (B, C, dim), dataloader.py:87) and asserts C == 1 in FeatPool
// (model.py:61-66).  The model here (TemporalAttention in
// cst_captioning_amd/models/modules.py) is additive attention conditioned on
// h_{t-1}:
//     e_c   = w_a . tanh(P[b, c] + q_r) + b_a,  P = W_f v_c + b_f,  q_r = W_q h_{t-1, r}
//     alpha = softmax_c(e),  ctx_r = sum_c alpha_c v_c,  gates += W_iv ctx_r.
// The same kernels run the reference's modal attention MANet
// (/root/reference/model.py:119-142) with the F modality blocks of the video
// vector as the "frames": there the scorer weights differ per frame,
//     e_f = A_m[f] . tanh(p + W_hm h_{t-1}) + b_m[f],  p = W_fm v + b_fm + b_hm,
// i.e. per-frame rows w_a[c] (wa_ld = A) and biases b_a[c] (ba_ld = 1) over a
// P that is the same for every frame (the caller expands it).
//
// MI355X design:
//   * ctx only enters the LSTM through W_iv, which is linear, so the caller
//     precomputes the per-frame gate table Gv[b, c] = W_iv v_c (B x C x 4H,
//     packed gate order) ONCE per batch; per step the kernel forms
//     vgate_r = sum_c alpha_c Gv[b, c] (C x 4H FMAs per row) instead of a
//     (R x F*H) . (F*H x 4H) GEMM -- 4H/C times less work per step;
//   * one workgroup owns ATT_RPW rows of ONE video.  Thread t owns the
//     attention units a = t + 256 j: it reads its own columns of the video's
//     projected frame tile P[b] (C x A) and of the rows' queries (coalesced),
//     accumulates the partial scores of all RPW x C (row, frame) pairs in
//     registers, and a butterfly all-reduce (N - 1 shuffles for N values,
//     instead of 6 per value) plus a cross-wave LDS sum finishes every score
//     at once; the video's Gv[b] rows (L2-resident, shared by its row groups)
//     are prefetched into registers at kernel start, so their latency hides
//     under the scores;
//   * in the rollout the query q_{t+1} = W_q h_t comes from extra W_q tiles of
//     the merged decode launch's recurrent GEMM (lstm_gemm.h), and the kernel
//     adds each row's vgate straight into that GEMM's pre-activations
//     (accumulate = 1), which the combine kernel's cell epilogue consumes;
//   * backward (per reverse step, after the fused LSTM step backward has
//     produced dG_t): dalpha = dG_t . Gv[b]^T, softmax backward, and the
//     tanh-scorer backward.  dq_t is written as bf16 into the tail columns
//     [4H, 4H + A) of the dG_t row, so the next reverse step's fused GEMM
//     (K = 4H + A against [W_hh^T | W_q^T]) folds dh_{t-1} += dq_t W_q into
//     the recurrence and the batched weight-gradient GEMM yields dW_q for
//     free.  dP / dw_a / db_a accumulate in per-workgroup slots (the grid
//     shape is the same every step, so no atomics and a deterministic sum).
#include "att_fwd.h"
#include "att_mfma.h"
#include "../launchers.h"

namespace cst {

template <int MAXC, int RPW>
__global__ __launch_bounds__(ATT_THREADS) void att_fwd_kernel(AttFwdArgs args) {
  att_fwd_block<MAXC, RPW>(blockIdx.x, args);
}

// dG: (R, ldg) bf16 rows, gate gradients in columns [0, G4); dq_t is written
// as bf16 into columns [G4, G4 + A) when write_dq.  PERC: per-frame scorer
// weights (MANet): dw_a / db_a slots are (C, A) / (C) per workgroup.
template <int MAXC, bool PERC, int RPW>
__global__ __launch_bounds__(ATT_THREADS) void att_bwd_kernel(
    uint16_t* __restrict__ dG, int ldg, const float* __restrict__ gv,
    const float* __restrict__ pre, const float* __restrict__ q, const float* __restrict__ alpha,
    const float* __restrict__ wa, int vdiv, int ngroups, int C, int A, int G4, int write_dq,
    float* __restrict__ dpre_part, float* __restrict__ dwa_part, float* __restrict__ dba_part) {
  __shared__ float s_red[ATT_WAVES * RPW * MAXC];
  __shared__ float s_da[RPW * MAXC];
  const int b = blockIdx.x / ngroups, g = blockIdx.x % ngroups;
  const int r0 = b * vdiv + g * RPW, nr = min(RPW, vdiv - g * RPW);
  const int tid = threadIdx.x;
  // this block's accumulator slots of dP / dw_a (read-modify-write every
  // reverse step) and its columns of P / q: requested up front, so the loads
  // overlap phase 1
  constexpr int AJ = 2;  // attention units per thread held in registers (A <= 512)
  constexpr int NW = PERC ? MAXC : 1;  // scorer-weight rows
  const bool apf = MAXC <= 8 && A <= AJ * ATT_THREADS;  // (register budget)
  float acc_dp[AJ][MAXC], acc_dw[AJ][NW], pv[AJ][MAXC], qv[AJ][RPW], wap[AJ][NW];
  float* dpp = dpre_part + (int64_t)blockIdx.x * C * A;
  float* dwp = dwa_part + (int64_t)blockIdx.x * (PERC ? C : 1) * A;
  const float* P = pre + (int64_t)b * C * A;
  if (apf) {
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      const int a = tid + j * ATT_THREADS;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        acc_dw[j][w] = (a < A && w < C) ? dwp[w * A + a] : 0.f;
        wap[j][w] = (a < A && w < C) ? wa[PERC ? w * A + a : a] : 0.f;
      }
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        acc_dp[j][c] = (a < A && c < C) ? dpp[c * A + a] : 0.f;
        pv[j][c] = (a < A && c < C) ? P[c * A + a] : 0.f;
      }
#pragma unroll
      for (int s = 0; s < RPW; ++s)
        qv[j][s] = (a < A && q != nullptr && s < nr) ? q[(int64_t)(r0 + s) * A + a] : 0.f;
    }
  }

  // the softmax-backward thread's attention weights, requested now
  float avp[MAXC <= 8 ? MAXC : 1];
  if (MAXC <= 8 && tid < nr) {
#pragma unroll
    for (int c = 0; c < (MAXC <= 8 ? MAXC : 1); ++c)
      avp[c] = c < C ? alpha[(int64_t)(r0 + tid) * C + c] : 0.f;
  }
  // 1. dalpha[s][c] = dG_r . Gv[b, c]  (the first ATT_GPF column groups of the
  // rows' dG are requested up front with the partial slots)
  uint2 dgp[ATT_GPF][RPW];
#pragma unroll
  for (int j = 0; j < ATT_GPF; ++j)
#pragma unroll
    for (int s = 0; s < RPW; ++s) {
      const int cg = tid + j * ATT_THREADS;
      dgp[j][s] = (s < nr && cg < (G4 >> 2))
                      ? *reinterpret_cast<const uint2*>(dG + (int64_t)(r0 + s) * ldg + 4 * cg)
                      : make_uint2(0u, 0u);
    }
  float part[RPW][MAXC];
#pragma unroll
  for (int s = 0; s < RPW; ++s)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) part[s][c] = 0.f;
  const float4* G = reinterpret_cast<const float4*>(gv + (int64_t)b * C * G4);
  const int G44 = G4 >> 2;
  // C <= 8, 4H <= 2048: the video's frame gate rows are requested with the dG
  // rows (one memory round trip for the whole dalpha phase)
  const bool gpf = MAXC <= 8 && G44 <= ATT_GPF * ATT_THREADS;
  if (gpf) {
    float4 gvp[ATT_GPF][MAXC <= 8 ? MAXC : 1];
#pragma unroll
    for (int j = 0; j < ATT_GPF; ++j)
#pragma unroll
      for (int c = 0; c < (MAXC <= 8 ? MAXC : 1); ++c) {
        const int cg = tid + j * ATT_THREADS;
        gvp[j][c] = (c < C && cg < G44) ? G[(int64_t)c * G44 + cg] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
    for (int j = 0; j < ATT_GPF; ++j) {
#pragma unroll
      for (int s = 0; s < RPW; ++s) {
        const uint2 raw = dgp[j][s];  // zero for rows / columns outside
        const float4 d = make_float4(bf2f(raw.x & 0xffff), bf2f(raw.x >> 16),
                                     bf2f(raw.y & 0xffff), bf2f(raw.y >> 16));
#pragma unroll
        for (int c = 0; c < (MAXC <= 8 ? MAXC : 1); ++c) {
          const float4 v = gvp[j][c];
          part[s][c] += d.x * v.x + d.y * v.y + d.z * v.z + d.w * v.w;
        }
      }
    }
  }
  for (int cg = tid, j = 0; !gpf && cg < G44; cg += ATT_THREADS, ++j) {
    float4 d[RPW];
#pragma unroll
    for (int s = 0; s < RPW; ++s) {
      d[s] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (s < nr) {
        const uint2 raw = j < ATT_GPF ? dgp[j < ATT_GPF ? j : 0][s]
                                      : *reinterpret_cast<const uint2*>(dG + (int64_t)(r0 + s) * ldg + 4 * cg);
        d[s] = make_float4(bf2f(raw.x & 0xffff), bf2f(raw.x >> 16), bf2f(raw.y & 0xffff),
                           bf2f(raw.y >> 16));
      }
    }
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c < C) {
        const float4 v = G[(int64_t)c * G44 + cg];
#pragma unroll
        for (int s = 0; s < RPW; ++s)
          part[s][c] += d[s].x * v.x + d[s].y * v.y + d[s].z * v.z + d[s].w * v.w;
      }
    }
  }
  block_sum_partials<MAXC, RPW>(part, s_red, s_da);
  // 2. softmax backward: de_c = alpha_c (dalpha_c - sum_k alpha_k dalpha_k), in place
  if (tid < nr) {
    const float* al = alpha + (int64_t)(r0 + tid) * C;
    float* da = s_da + tid * MAXC;
    float av[MAXC], sa = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (MAXC <= 8)
        av[c] = avp[MAXC <= 8 ? c : 0];
      else
        av[c] = c < C ? al[c] : 0.f;
      sa += c < C ? av[c] * da[c] : 0.f;
    }
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
      if (c < C) da[c] = av[c] * (da[c] - sa);
  }
  __syncthreads();
  const float* s_de = s_da;
  if (PERC) {
    if (tid < C) {
      float sb = 0.f;
      for (int s = 0; s < nr; ++s) sb += s_de[s * MAXC + tid];
      dba_part[(int64_t)blockIdx.x * C + tid] += sb;
    }
  } else if (tid == 0) {
    float sb = 0.f;
    for (int s = 0; s < nr; ++s)
      for (int c = 0; c < C; ++c) sb += s_de[s * MAXC + c];
    dba_part[blockIdx.x] += sb;
  }
  // 3. scorer backward, thread per attention unit a:
  //    dz = de_c w_a (1 - u^2), u = tanh(P_c + q_s); dq_s = sum_c dz; dP_c = sum_s dz
  auto unit = [&](int a, const float* pa, const float* qa, float (&dp)[MAXC], float (&dwa)[NW],
                  const float* wv) {  // wv: the unit's scorer weights (prefetched) or nullptr
    float dq[RPW];
#pragma unroll
    for (int s = 0; s < RPW; ++s) dq[s] = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c < C) {
        const float wa_a = wv != nullptr ? wv[PERC ? c : 0] : wa[PERC ? c * A + a : a];
#pragma unroll
        for (int s = 0; s < RPW; ++s) {
          if (s < nr) {
            const float u = tanhf_(pa[c] + qa[s]);
            const float de = s_de[s * MAXC + c];
            dwa[PERC ? c : 0] += de * u;
            const float dz = de * wa_a * (1.f - u * u);
            dq[s] += dz;
            dp[c] += dz;
          }
        }
      }
    }
    if (write_dq) {
#pragma unroll
      for (int s = 0; s < RPW; ++s)
        if (s < nr) dG[(int64_t)(r0 + s) * ldg + G4 + a] = f2bf(dq[s]);
    }
  };
  if (apf) {
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      const int a = tid + j * ATT_THREADS;
      if (a < A) {
        unit(a, pv[j], qv[j], acc_dp[j], acc_dw[j], wap[j]);
#pragma unroll
        for (int w = 0; w < NW; ++w)
          if (w < C) dwp[w * A + a] = acc_dw[j][w];
#pragma unroll
        for (int c = 0; c < MAXC; ++c)
          if (c < C) dpp[c * A + a] = acc_dp[j][c];
      }
    }
  } else {
    for (int a = tid; a < A; a += ATT_THREADS) {
      float dp[MAXC], pa[MAXC], qa[RPW], dw[NW];
#pragma unroll
      for (int w = 0; w < NW; ++w) dw[w] = 0.f;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        dp[c] = 0.f;
        pa[c] = c < C ? P[c * A + a] : 0.f;
      }
#pragma unroll
      for (int s = 0; s < RPW; ++s)
        qa[s] = (q != nullptr && s < nr) ? q[(int64_t)(r0 + s) * A + a] : 0.f;
      unit(a, pa, qa, dp, dw, nullptr);
#pragma unroll
      for (int w = 0; w < NW; ++w)
        if (w < C) dwp[w * A + a] += dw[w];
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
        if (c < C) dpp[c * A + a] += dp[c];
    }
  }
}

int att_groups(int vdiv, int rpw) { return (vdiv + rpw - 1) / rpw; }

// MFMA attention path, backward of one reverse step (see launchers.h): block
// (video b, 64-unit slice of A; 4 row groups of the video's rows, so the
// tanh-scorer loop of a thread covers 8 rows, not 16: 512 blocks at A = 512
// spread it over every CU).  dalpha[r][c] = the sum of the backward step
// kernel's H/64 partials (lstm.hip attention epilogue: the dG . Gv^T
// contraction happened there, on the dG tile already in registers), so this
// kernel never reads the 4H-wide dG rows or the gate tables.  Softmax backward
// per row, then thread (unit a, row parity) runs the tanh-scorer backward over
// its rows: dq_t[r][a] as bf16 into the dG row's tail (the next reverse step's
// recurrent GEMM folds dq_t W_q into dh_{t-1}), dP[b][c][a] accumulated in
// place (this block owns it), dw_a / db_a into per-video slots.
constexpr int ATTB_UNITS = 64, ATTB_RG = 4, ATTB_MAXR = 8;  // rows per group (vdiv <= 32)
template <int CP>
__global__ __launch_bounds__(256) void att_bwd_mfma_kernel(
    const float* __restrict__ dal_part, int n_ut, int R, const float* __restrict__ alpha,
    const float* __restrict__ q, const float* __restrict__ P, const float* __restrict__ wa,
    int vdiv, int C, int A, int G4, uint16_t* __restrict__ dG, int ldg, int write_dq,
    float* __restrict__ dP_acc, float* __restrict__ dwa_part, float* __restrict__ dba_part) {
  __shared__ float s_da[32 * CP];
  __shared__ float s_de[32 * CP];
  __shared__ float s_red[(ATTB_RG - 1) * ATTB_UNITS * (CP + 1)];
  const int b = blockIdx.x, sl = blockIdx.y, tid = threadIdx.x;
  const int row0 = b * vdiv;
  const int a = sl * ATTB_UNITS + (tid & (ATTB_UNITS - 1)), par = tid / ATTB_UNITS;
  // 1. dalpha[r][c] = sum of the step kernel's H/64 partials, one (r, c) per
  // thread: its loads go out first (they gate the softmax backward)
  const int nrc = vdiv * CP;
  constexpr int MAXUT = 16;  // H <= 1024: every partial load goes out at once
  float dsum[2] = {0.f, 0.f};
#pragma unroll
  for (int h2 = 0; h2 < 2; ++h2) {
    // (no conditional loads: indices clamped, values masked)
    const int rc = min(tid + 256 * h2, nrc - 1);
    const float* pp = dal_part + (int64_t)row0 * CP + rc;
    float x[MAXUT];
#pragma unroll
    for (int ut = 0; ut < MAXUT; ++ut) x[ut] = pp[(int64_t)min(ut, n_ut - 1) * R * CP];
#pragma unroll
    for (int ut = 0; ut < MAXUT; ++ut) dsum[h2] += ut < n_ut ? x[ut] : 0.f;
  }
  // this thread's scorer operands and accumulators, requested meanwhile
  float pv[CP], qv[ATTB_MAXR];
#pragma unroll
  for (int c = 0; c < CP; ++c) pv[c] = P[((int64_t)b * C + min(c, C - 1)) * A + a];
  const float wav = wa[a];
  const float* qb = q != nullptr ? q : P;  // step 0: q = 0 (masked below)
#pragma unroll
  for (int k = 0; k < ATTB_MAXR; ++k) {
    const int rr = min(par + ATTB_RG * k, vdiv - 1);
    qv[k] = qb[(int64_t)(q != nullptr ? row0 + rr : 0) * A + a];
  }
  if (q == nullptr) {
#pragma unroll
    for (int k = 0; k < ATTB_MAXR; ++k) qv[k] = 0.f;
  }
  float dp_old[CP], dw_old;
#pragma unroll
  for (int c = 0; c < CP; ++c) dp_old[c] = dP_acc[((int64_t)b * C + min(c, C - 1)) * A + a];
  dw_old = dwa_part[(int64_t)b * A + a];
  float alr[CP];
  {
    const int rr = min(tid, vdiv - 1);
#pragma unroll
    for (int c = 0; c < CP; ++c) alr[c] = alpha[(int64_t)(row0 + rr) * C + min(c, C - 1)];
#pragma unroll
    for (int c = 0; c < CP; ++c) alr[c] = c < C ? alr[c] : 0.f;
  }
#pragma unroll
  for (int h2 = 0; h2 < 2; ++h2)
    if (tid + 256 * h2 < nrc) s_da[tid + 256 * h2] = dsum[h2];
  __syncthreads();
  // 2. softmax backward: de_c = alpha_c (dalpha_c - sum_k alpha_k dalpha_k)
  if (tid < vdiv) {
    float sa = 0.f;
#pragma unroll
    for (int c = 0; c < CP; ++c) sa += alr[c] * s_da[tid * CP + c];
#pragma unroll
    for (int c = 0; c < CP; ++c) s_de[tid * CP + c] = alr[c] * (s_da[tid * CP + c] - sa);
  }
  __syncthreads();
  if (sl == 0 && tid == 0) {
    float sb = 0.f;
    for (int r = 0; r < vdiv; ++r)
      for (int c = 0; c < C; ++c) sb += s_de[r * CP + c];
    dba_part[b] += sb;
  }
  // 3. tanh-scorer backward over this thread's rows
  float dp[CP], dw = 0.f;
#pragma unroll
  for (int c = 0; c < CP; ++c) dp[c] = 0.f;
#pragma unroll
  for (int k = 0; k < ATTB_MAXR; ++k) {
    const int rr = par + ATTB_RG * k;
    if (rr < vdiv) {
      float dq = 0.f;
#pragma unroll
      for (int c = 0; c < CP; ++c) {
        if (c < C) {
          const float u = tanh_fast(pv[c] + qv[k]);
          const float de = s_de[rr * CP + c];
          dw = fmaf(de, u, dw);
          const float dz = de * wav * fmaf(-u, u, 1.f);
          dq += dz;
          dp[c] += dz;
        }
      }
      if (write_dq) dG[(int64_t)(row0 + rr) * ldg + G4 + a] = f2bf(dq);
    }
  }
  const int ul = tid & (ATTB_UNITS - 1);
  if (par > 0) {
    float* sr = s_red + ((par - 1) * ATTB_UNITS + ul) * (CP + 1);
#pragma unroll
    for (int c = 0; c < CP; ++c) sr[c] = dp[c];
    sr[CP] = dw;
  }
  __syncthreads();
  if (par == 0) {
#pragma unroll
    for (int g = 0; g < ATTB_RG - 1; ++g) {
      const float* sr = s_red + (g * ATTB_UNITS + ul) * (CP + 1);
#pragma unroll
      for (int c = 0; c < CP; ++c) dp[c] += sr[c];
      dw += sr[CP];
    }
#pragma unroll
    for (int c = 0; c < CP; ++c)
      if (c < C) dP_acc[((int64_t)b * C + c) * A + a] = dp_old[c] + dp[c];
    dwa_part[(int64_t)b * A + a] = dw_old + dw;
  }
}

void launch_att_bwd_mfma(const float* dal_part, int n_ut, int R, const float* alpha,
                         const float* q, const float* P, const float* wa, int Bv, int vdiv, int C,
                         int CP, int A, int G4, uint16_t* dG, int ldg, int write_dq, float* dP_acc,
                         float* dwa_part, float* dba_part, hipStream_t stream) {
  if (vdiv > ATTB_RG * ATTB_MAXR || A % ATTB_UNITS != 0 || C > CP || (CP != 8 && CP != 16) ||
      Bv * vdiv != R || n_ut > 16)
    throw std::runtime_error("att_bwd_mfma: unsupported shape");
  const dim3 grid(Bv, A / ATTB_UNITS);
  if (CP == 8)
    hipLaunchKernelGGL(att_bwd_mfma_kernel<8>, grid, dim3(256), 0, stream, dal_part, n_ut, R, alpha,
                       q, P, wa, vdiv, C, A, G4, dG, ldg, write_dq, dP_acc, dwa_part, dba_part);
  else
    hipLaunchKernelGGL(att_bwd_mfma_kernel<16>, grid, dim3(256), 0, stream, dal_part, n_ut, R,
                       alpha, q, P, wa, vdiv, C, A, G4, dG, ldg, write_dq, dP_acc, dwa_part,
                       dba_part);
  post_launch("att_bwd_mfma_kernel", stream);
}

// Video-gate gradient of the per-frame gate tables (after the reverse loop):
//     dGv[b, c, :] = sum over steps t and rows r of video b of alpha[t, r, c] dG_t[r, 0:G4].
// A batched GEMM over (step, video) pairs has K = 20 rows and 1,792 batch
// entries (3 TFLOP/s, plus a 117 MB fp32 intermediate summed over steps);
// here block (b, step chunk) streams its rows' bf16 dG once (16 bytes per
// thread and row, coalesced), the row's C attention weights are uniform
// across the block, and each thread keeps C x 8 fp32 sums; one partial per
// step chunk (summed by the caller: deterministic, no atomics).
constexpr int DGV_TCHUNK = 4;
template <int MAXC>
__global__ __launch_bounds__(256) void att_dgv_kernel(const uint16_t* __restrict__ dG, int ldg,
                                                      const float* __restrict__ alpha, int n_steps,
                                                      int R, int Bv, int vdiv, int C, int G4,
                                                      float* __restrict__ part) {
  const int b = blockIdx.x, tc = blockIdx.y;
  const int t0 = tc * DGV_TCHUNK, t1 = min(n_steps, t0 + DGV_TCHUNK);
  for (int cg = threadIdx.x; 8 * cg < G4; cg += 256) {
    float acc[MAXC][8];
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[c][k] = 0.f;
    for (int t = t0; t < t1; ++t) {
#pragma unroll 4
      for (int rr = 0; rr < vdiv; ++rr) {
        const int64_t row = (int64_t)t * R + (int64_t)b * vdiv + rr;
        const uint4 g = *reinterpret_cast<const uint4*>(dG + row * ldg + 8 * cg);
        const uint32_t w[4] = {g.x, g.y, g.z, g.w};
        float d[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d[2 * k] = bf2f(w[k] & 0xffff);
          d[2 * k + 1] = bf2f(w[k] >> 16);
        }
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
          const float al = c < C ? alpha[row * C + c] : 0.f;
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[c][k] += al * d[k];
        }
      }
    }
    float* out = part + ((int64_t)tc * Bv + b) * C * G4 + 8 * cg;
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
      if (c < C) {
        reinterpret_cast<float4*>(out + (int64_t)c * G4)[0] =
            make_float4(acc[c][0], acc[c][1], acc[c][2], acc[c][3]);
        reinterpret_cast<float4*>(out + (int64_t)c * G4)[1] =
            make_float4(acc[c][4], acc[c][5], acc[c][6], acc[c][7]);
      }
  }
}

int att_dgv_chunks(int n_steps) { return (n_steps + DGV_TCHUNK - 1) / DGV_TCHUNK; }

void launch_att_dgv(const uint16_t* dG, int ldg, const float* alpha, int n_steps, int R, int Bv,
                    int vdiv, int C, int G4, float* part, hipStream_t stream) {
  if (C > 8 || G4 % 8 != 0 || ldg % 8 != 0 || Bv * vdiv != R)
    throw std::runtime_error("att_dgv: C <= 8, G4 and ldg multiples of 8, R = Bv * vdiv");
  hipLaunchKernelGGL(att_dgv_kernel<8>, dim3(Bv, att_dgv_chunks(n_steps)), dim3(256), 0, stream,
                     dG, ldg, alpha, n_steps, R, Bv, vdiv, C, G4, part);
  post_launch("att_dgv_kernel", stream);
}

template <int RPW>
static void launch_att_fwd_t(const float* gv, const float* pre, const float* q,
                             const int* q_rowmap, const float* wa, const float* ba, int Bv,
                             int vdiv, int C, int A, int G4, float* vg_out, float* alpha_out,
                             hipStream_t stream, int accumulate, int per_frame) {
  const int ng = (vdiv + RPW - 1) / RPW;
  const int wa_ld = per_frame ? A : 0, ba_ld = per_frame ? 1 : 0;
#define ATT_FWD(M)                                                                              \
  hipLaunchKernelGGL((att_fwd_kernel<M, RPW>), dim3(Bv * ng), dim3(ATT_THREADS), 0, stream, args)
  const AttFwdArgs args{gv, pre, q, q_rowmap, wa, ba, wa_ld, ba_ld, vdiv, ng, C, A, G4, vg_out,
                        alpha_out, accumulate};
  if (C <= 8)
    ATT_FWD(8);
  else if (C <= 16)
    ATT_FWD(16);
  else
    ATT_FWD(32);
#undef ATT_FWD
  post_launch("att_fwd_kernel", stream);
}

void launch_att_fwd(const float* gv, const float* pre, const float* q, const int* q_rowmap,
                    const float* wa, const float* ba, int Bv, int vdiv, int C, int A, int G4,
                    float* vg_out, float* alpha_out, hipStream_t stream, int accumulate,
                    int per_frame, int rpw) {
  if (rpw == 0) rpw = vdiv >= 4 ? 4 : vdiv >= 2 ? 2 : 1;
  switch (rpw) {
    case 1: launch_att_fwd_t<1>(gv, pre, q, q_rowmap, wa, ba, Bv, vdiv, C, A, G4, vg_out, alpha_out, stream, accumulate, per_frame); break;
    case 2: launch_att_fwd_t<2>(gv, pre, q, q_rowmap, wa, ba, Bv, vdiv, C, A, G4, vg_out, alpha_out, stream, accumulate, per_frame); break;
    default: launch_att_fwd_t<4>(gv, pre, q, q_rowmap, wa, ba, Bv, vdiv, C, A, G4, vg_out, alpha_out, stream, accumulate, per_frame); break;
  }
}

template <int MAXC, bool PERC, int RPW>
static void launch_att_bwd_t(uint16_t* dG, int ldg, const float* gv, const float* pre,
                             const float* q, const float* alpha, const float* wa, int Bv, int vdiv,
                             int C, int A, int G4, int write_dq, float* dpre_part, float* dwa_part,
                             float* dba_part, hipStream_t stream) {
  const int ng = att_groups(vdiv, RPW);
  hipLaunchKernelGGL((att_bwd_kernel<MAXC, PERC, RPW>), dim3(Bv * ng), dim3(ATT_THREADS), 0, stream, dG, ldg,
                     gv, pre, q, alpha, wa, vdiv, ng, C, A, G4, write_dq, dpre_part, dwa_part,
                     dba_part);
  post_launch("att_bwd_kernel", stream);
}

void launch_att_bwd(uint16_t* dG, int ldg, const float* gv, const float* pre, const float* q,
                    const float* alpha, const float* wa, int Bv, int vdiv, int C, int A, int G4,
                    int write_dq, float* dpre_part, float* dwa_part, float* dba_part,
                    hipStream_t stream, int per_frame, int rpw) {
#define ATT_BWD(M, PF, RP)                                                                   \
  launch_att_bwd_t<M, PF, RP>(dG, ldg, gv, pre, q, alpha, wa, Bv, vdiv, C, A, G4, write_dq,   \
                              dpre_part, dwa_part, dba_part, stream)
  if (per_frame) {  // MANet: C = number of modalities
    if (C > 8) throw std::runtime_error("per-frame attention weights: at most 8 frames");
    if (rpw == 2) ATT_BWD(8, true, 2); else ATT_BWD(8, true, 4);
  } else if (C <= 8) {
    if (rpw == 2) ATT_BWD(8, false, 2); else ATT_BWD(8, false, 4);
  } else if (C <= 16) {
    ATT_BWD(16, false, 4);
  } else {
    ATT_BWD(32, false, 4);
  }
#undef ATT_BWD
}

}  // namespace cst
