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
//
// MI355X design:
//   * ctx only enters the LSTM through W_iv, which is linear, so the caller
//     precomputes the per-frame gate table Gv[b, c] = W_iv v_c (B x C x 4H,
//     packed gate order) ONCE per batch; per step the kernel forms
//     vgate_r = sum_c alpha_c Gv[b, c] (C x 4H FMAs per row) instead of a
//     (R x F*H) . (F*H x 4H) GEMM -- 4H/C times less work per step;
//   * one workgroup owns ATT_RPW rows of ONE video: the video's projected
//     frame tile P[b] (C x A), the rows' queries and w_a are staged in LDS
//     once and every (row, frame) score is a wave-wide dot product out of
//     LDS; the Gv[b] rows stream from L2 (shared by the video's row groups)
//     as float4;
//   * backward (per reverse step, after the fused LSTM step backward has
//     produced dG_t): dalpha = dG_t . Gv[b]^T, softmax backward, and the
//     tanh-scorer backward.  dq_t is written as bf16 into the tail columns
//     [4H, 4H + A) of the dG_t row, so the next reverse step's fused GEMM
//     (K = 4H + A against [W_hh^T | W_q^T]) folds dh_{t-1} += dq_t W_q into
//     the recurrence and the batched weight-gradient GEMM yields dW_q for
//     free.  dP / dw_a / db_a accumulate in per-workgroup slots (the grid
//     shape is the same every step, so no atomics and a deterministic sum).
#include "../common.h"

namespace cst {

constexpr int ATT_THREADS = 256, ATT_RPW = 4;

__device__ __forceinline__ void att_stage(float* s_pre, float* s_q, float* s_wa,
                                          const float* __restrict__ pre,
                                          const float* __restrict__ q,
                                          const int* __restrict__ q_rowmap,
                                          const float* __restrict__ wa, int b, int r0, int nr,
                                          int C, int A) {
  const int tid = threadIdx.x, A4 = A >> 2;
  const float4* src = reinterpret_cast<const float4*>(pre + (int64_t)b * C * A);
  for (int i = tid; i < C * A4; i += ATT_THREADS) reinterpret_cast<float4*>(s_pre)[i] = src[i];
  for (int i = tid; i < ATT_RPW * A4; i += ATT_THREADS) {
    const int s = i / A4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (q != nullptr && s < nr) {
      const int r = r0 + s, qr = q_rowmap ? q_rowmap[r] : r;
      v = reinterpret_cast<const float4*>(q + (int64_t)qr * A)[i - s * A4];
    }
    reinterpret_cast<float4*>(s_q)[i] = v;
  }
  for (int i = tid; i < A; i += ATT_THREADS) s_wa[i] = wa[i];
}

// grid: Bv * ngroups blocks; block (b, g) owns rows b*vdiv + g*RPW ... (< (b+1)*vdiv)
__global__ __launch_bounds__(ATT_THREADS) void att_fwd_kernel(
    const float* __restrict__ gv, const float* __restrict__ pre, const float* __restrict__ q,
    const int* __restrict__ q_rowmap, const float* __restrict__ wa, const float* __restrict__ ba,
    int vdiv, int ngroups, int C, int A, int G4, float* __restrict__ vg_out,
    float* __restrict__ alpha_out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* s_pre = sm;
  float* s_q = s_pre + C * A;
  float* s_wa = s_q + ATT_RPW * A;
  float* s_e = s_wa + A;  // ATT_RPW x C
  const int b = blockIdx.x / ngroups, g = blockIdx.x % ngroups;
  const int r0 = b * vdiv + g * ATT_RPW, nr = min(ATT_RPW, vdiv - g * ATT_RPW);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  att_stage(s_pre, s_q, s_wa, pre, q, q_rowmap, wa, b, r0, nr, C, A);
  __syncthreads();
  // scores: one wave per (row, frame) pair, lanes stride the attention dim
  const float bias = ba[0];
  for (int p = w; p < nr * C; p += ATT_THREADS / WAVE) {
    const int s = p / C, c = p - s * C;
    const float* pc = s_pre + c * A;
    const float* qs = s_q + s * A;
    float acc = 0.f;
    for (int a = lane; a < A; a += WAVE) acc += s_wa[a] * tanhf_(pc[a] + qs[a]);
    acc = wave_sum(acc);
    if (lane == 0) s_e[s * C + c] = acc + bias;
  }
  __syncthreads();
  if (tid < nr) {  // softmax over frames, one thread per row
    float* e = s_e + tid * C;
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) m = fmaxf(m, e[c]);
    float sum = 0.f;
    for (int c = 0; c < C; ++c) {
      const float x = __expf(e[c] - m);
      e[c] = x;
      sum += x;
    }
    const float inv = 1.f / sum;
    for (int c = 0; c < C; ++c) {
      e[c] *= inv;
      if (alpha_out) alpha_out[(int64_t)(r0 + tid) * C + c] = e[c];
    }
  }
  __syncthreads();
  // vgate_r = sum_c alpha_rc Gv[b, c]: each thread owns float4 column groups
  const float4* G = reinterpret_cast<const float4*>(gv + (int64_t)b * C * G4);
  const int G44 = G4 >> 2;
  for (int cg = tid; cg < G44; cg += ATT_THREADS) {
    float4 acc[ATT_RPW];
#pragma unroll
    for (int s = 0; s < ATT_RPW; ++s) acc[s] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int c = 0; c < C; ++c) {
      const float4 v = G[(int64_t)c * G44 + cg];
#pragma unroll
      for (int s = 0; s < ATT_RPW; ++s) {
        const float al = s_e[min(s, nr - 1) * C + c];
        acc[s].x += al * v.x;
        acc[s].y += al * v.y;
        acc[s].z += al * v.z;
        acc[s].w += al * v.w;
      }
    }
#pragma unroll
    for (int s = 0; s < ATT_RPW; ++s)
      if (s < nr) reinterpret_cast<float4*>(vg_out + (int64_t)(r0 + s) * G4)[cg] = acc[s];
  }
}

// dG: (R, ldg) bf16 rows, gate gradients in columns [0, G4); dq_t is written
// as bf16 into columns [G4, G4 + A) when write_dq.
template <int MAXC>
__global__ __launch_bounds__(ATT_THREADS) void att_bwd_kernel(
    uint16_t* __restrict__ dG, int ldg, const float* __restrict__ gv,
    const float* __restrict__ pre, const float* __restrict__ q, const float* __restrict__ alpha,
    const float* __restrict__ wa, int vdiv, int ngroups, int C, int A, int G4, int write_dq,
    float* __restrict__ dpre_part, float* __restrict__ dwa_part, float* __restrict__ dba_part) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* s_pre = sm;
  float* s_q = s_pre + C * A;
  float* s_wa = s_q + ATT_RPW * A;
  float* s_red = s_wa + A;                                   // 4 waves x RPW x MAXC
  float* s_de = s_red + (ATT_THREADS / WAVE) * ATT_RPW * MAXC;  // RPW x MAXC
  const int b = blockIdx.x / ngroups, g = blockIdx.x % ngroups;
  const int r0 = b * vdiv + g * ATT_RPW, nr = min(ATT_RPW, vdiv - g * ATT_RPW);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  att_stage(s_pre, s_q, s_wa, pre, q, nullptr, wa, b, r0, nr, C, A);

  // 1. dalpha[s][c] = dG_r . Gv[b, c]
  float part[ATT_RPW][MAXC];
#pragma unroll
  for (int s = 0; s < ATT_RPW; ++s)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) part[s][c] = 0.f;
  const float4* G = reinterpret_cast<const float4*>(gv + (int64_t)b * C * G4);
  const int G44 = G4 >> 2;
  for (int cg = tid; cg < G44; cg += ATT_THREADS) {
    float4 d[ATT_RPW];
#pragma unroll
    for (int s = 0; s < ATT_RPW; ++s) {
      d[s] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (s < nr) {
        const uint2 raw = *reinterpret_cast<const uint2*>(dG + (int64_t)(r0 + s) * ldg + 4 * cg);
        d[s] = make_float4(bf2f(raw.x & 0xffff), bf2f(raw.x >> 16), bf2f(raw.y & 0xffff),
                           bf2f(raw.y >> 16));
      }
    }
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c < C) {
        const float4 v = G[(int64_t)c * G44 + cg];
#pragma unroll
        for (int s = 0; s < ATT_RPW; ++s)
          part[s][c] += d[s].x * v.x + d[s].y * v.y + d[s].z * v.z + d[s].w * v.w;
      }
    }
  }
#pragma unroll
  for (int s = 0; s < ATT_RPW; ++s)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c < C) {
        const float v = wave_sum(part[s][c]);
        if (lane == 0) s_red[(w * ATT_RPW + s) * MAXC + c] = v;
      }
    }
  __syncthreads();
  // 2. softmax backward: de_c = alpha_c (dalpha_c - sum_k alpha_k dalpha_k)
  if (tid < nr) {
    const float* al = alpha + (int64_t)(r0 + tid) * C;
    float da[MAXC], sa = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      da[c] = 0.f;
      if (c < C) {
#pragma unroll
        for (int k = 0; k < ATT_THREADS / WAVE; ++k) da[c] += s_red[(k * ATT_RPW + tid) * MAXC + c];
        sa += al[c] * da[c];
      }
    }
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
      if (c < C) s_de[tid * MAXC + c] = al[c] * (da[c] - sa);
  }
  __syncthreads();
  if (tid == 0) {
    float sb = 0.f;
    for (int s = 0; s < nr; ++s)
      for (int c = 0; c < C; ++c) sb += s_de[s * MAXC + c];
    dba_part[blockIdx.x] += sb;
  }
  // 3. scorer backward, thread per attention unit a:
  //    dz = de_c w_a (1 - u^2), u = tanh(P_c + q_s); dq_s = sum_c dz; dP_c = sum_s dz
  for (int a = tid; a < A; a += ATT_THREADS) {
    const float wa_a = s_wa[a];
    float dq[ATT_RPW];
#pragma unroll
    for (int s = 0; s < ATT_RPW; ++s) dq[s] = 0.f;
    float dwa = 0.f;
    for (int c = 0; c < C; ++c) {
      const float pc = s_pre[c * A + a];
      float dp = 0.f;
#pragma unroll
      for (int s = 0; s < ATT_RPW; ++s) {
        if (s < nr) {
          const float u = tanhf_(pc + s_q[s * A + a]);
          const float de = s_de[s * MAXC + c];
          dwa += de * u;
          const float dz = de * wa_a * (1.f - u * u);
          dq[s] += dz;
          dp += dz;
        }
      }
      dpre_part[((int64_t)blockIdx.x * C + c) * A + a] += dp;
    }
    dwa_part[(int64_t)blockIdx.x * A + a] += dwa;
    if (write_dq) {
#pragma unroll
      for (int s = 0; s < ATT_RPW; ++s)
        if (s < nr) dG[(int64_t)(r0 + s) * ldg + G4 + a] = f2bf(dq[s]);
    }
  }
}

int att_groups(int vdiv) { return (vdiv + ATT_RPW - 1) / ATT_RPW; }

static size_t att_lds_bytes(int C, int A, int maxc) {
  return sizeof(float) * ((size_t)C * A + ATT_RPW * A + A +
                          (size_t)(ATT_THREADS / WAVE + 1) * ATT_RPW * maxc);
}

size_t att_max_lds() { return 64 * 1024; }

size_t att_lds_need(int C, int A) { return att_lds_bytes(C, A, C <= 8 ? 8 : C <= 16 ? 16 : 32); }

void launch_att_fwd(const float* gv, const float* pre, const float* q, const int* q_rowmap,
                    const float* wa, const float* ba, int Bv, int vdiv, int C, int A, int G4,
                    float* vg_out, float* alpha_out, hipStream_t stream) {
  const int ng = att_groups(vdiv);
  const size_t lds = sizeof(float) * ((size_t)C * A + ATT_RPW * A + A + ATT_RPW * C);
  hipLaunchKernelGGL(att_fwd_kernel, dim3(Bv * ng), dim3(ATT_THREADS), lds, stream, gv, pre, q,
                     q_rowmap, wa, ba, vdiv, ng, C, A, G4, vg_out, alpha_out);
}

template <int MAXC>
static void launch_att_bwd_t(uint16_t* dG, int ldg, const float* gv, const float* pre,
                             const float* q, const float* alpha, const float* wa, int Bv, int vdiv,
                             int C, int A, int G4, int write_dq, float* dpre_part, float* dwa_part,
                             float* dba_part, hipStream_t stream) {
  const int ng = att_groups(vdiv);
  hipLaunchKernelGGL(att_bwd_kernel<MAXC>, dim3(Bv * ng), dim3(ATT_THREADS),
                     att_lds_bytes(C, A, MAXC), stream, dG, ldg, gv, pre, q, alpha, wa, vdiv, ng,
                     C, A, G4, write_dq, dpre_part, dwa_part, dba_part);
}

void launch_att_bwd(uint16_t* dG, int ldg, const float* gv, const float* pre, const float* q,
                    const float* alpha, const float* wa, int Bv, int vdiv, int C, int A, int G4,
                    int write_dq, float* dpre_part, float* dwa_part, float* dba_part,
                    hipStream_t stream) {
  if (C <= 8)
    launch_att_bwd_t<8>(dG, ldg, gv, pre, q, alpha, wa, Bv, vdiv, C, A, G4, write_dq, dpre_part,
                        dwa_part, dba_part, stream);
  else if (C <= 16)
    launch_att_bwd_t<16>(dG, ldg, gv, pre, q, alpha, wa, Bv, vdiv, C, A, G4, write_dq, dpre_part,
                         dwa_part, dba_part, stream);
  else
    launch_att_bwd_t<32>(dG, ldg, gv, pre, q, alpha, wa, Bv, vdiv, C, A, G4, write_dq, dpre_part,
                         dwa_part, dba_part, stream);
}

}  // namespace cst
