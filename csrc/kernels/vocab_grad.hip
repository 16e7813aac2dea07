// K7: vocab-head backward from the exp store, without ever forming dS.
//
// Reference (/root/reference/model.py:281 log_softmax of the logit Linear,
// criteria of /root/reference/train.py / utils.py): every loss of the
// recipes is a per-row weighted log-prob of one chosen token, so for row
// (t, r) with weights a (sampled / chosen token ys) and b (target token yx):
//     dS_rv = a [v = ys] + b [v = yx] - (a + b) p_rv.
// The decode kernel saved E_rv = exp(x_rv - c_r) (bf16, c_r = the row's LSE
// of the previous step; step 0: its own LSE), so p_rv = s_r E_rv with
// s_r = exp(c_r - lse_r).  With alpha_r = -(a + b) s_r the one-hot terms fold
// into the row's own entries of E (vgrad_onehot: E'_{r,ys} = E_{r,ys} + a /
// alpha_r, likewise yx; two scattered bf16 updates per row), so
//     dS = diag(alpha) E'
// exactly, and with plain hipBLASLt GEMMs over E':
//     dHd = alpha . (E' W)          (row scales applied by the reverse loop)
//     dW  = E'^T (alpha . Hd)       (vgrad_rows writes the scaled Hd rows)
//     db  = sum_r alpha_r E'_r      (vgrad_colsum)
// The former dS pass (read fp16 logits, write bf16 dS: 1.5 GB of HBM traffic,
// ~0.44 ms per step) disappears.  A row whose weights cancel on two different
// tokens (a + b = 0 with ys != yx, so dS_r = a (e_ys - e_yx)) keeps |alpha| >=
// 2^-10 (|a| + |b|) s: its softmax part is then off by at most 2^-10 (|a| +
// |b|) in total.
//
// (The XE all-rows forward, engine.cpp, writes E = exp(x) with c = 0 for every
// row: VGradRows::zero_off, s_r = exp(-lse_r), guarded for |lse_r| > 60.)
//
// Range of the exp store: E = exp(x - c) with c = the previous step's LSE
// stays inside bf16 (fp32's exponent range) while the row's LSE moves by
// less than ~80 between steps (overflow above, loss of the row's mass to
// underflow below).  vgrad_onehot lists every row whose LSE moved by more
// than EXP_SAFE_LSE_JUMP (60) and vgrad_fix recomputes those rows exactly
// from the saved vocab input (offset = the row's own LSE, so s = 1) before
// the GEMMs read them: no silent NaN / zero gradient, no skipped step, and a
// running count of recomputed rows for the log.
#include "../common.h"
#include "../launchers.h"

namespace cst {

struct RowW {
  float a, b, s, al;
  int ys, yx;
};

// unit_s: the row's E was written with its own LSE as offset (vgrad_fix)
__device__ __forceinline__ RowW row_weights(const VGradRows& g, int64_t row, bool unit_s = false) {
  RowW w;
  const int t = (int)(row / g.R), r = (int)(row % g.R);
  const bool sel = g.dg_sel != nullptr && t < g.T_sel;
  w.a = sel ? g.dg_sel[(int64_t)r * g.T_sel + t] : 0.f;
  w.ys = sel ? (int)g.y_sel[(int64_t)r * g.T_sel + t] : -1;
  w.b = g.dg_xe != nullptr ? g.dg_xe[(int64_t)r * g.dgxe_rs + t] : 0.f;
  w.yx = g.dg_xe != nullptr ? (int)g.y_xe[(int64_t)r * g.yxe_rs + t] : -1;
  w.s = unit_s       ? 1.f
        : g.zero_off ? __expf(-g.lse[row])
        : t > 0      ? __expf(g.lse[(int64_t)(t - 1) * g.R + r] - g.lse[row])
                     : 1.f;
  w.al = -(w.a + w.b) * w.s;
  // weights that (nearly) cancel on two different tokens: keep alpha away from
  // 0 so the one-hot terms stay representable (ys == yx cancels exactly)
  if (w.a != 0.f && w.b != 0.f && w.ys >= 0 && w.yx >= 0 && w.ys != w.yx) {
    const float floor_al = 0.0009765625f * (fabsf(w.a) + fabsf(w.b)) * w.s;
    if (fabsf(w.al) < floor_al) w.al = w.al < 0.f ? -floor_al : floor_al;
  }
  return w;
}

// the one-hot terms of row weights w folded into the row's E
__device__ __forceinline__ void fold_onehot(const VGradRows& g, const RowW& w, uint16_t* e) {
  if (w.al == 0.f) return;  // no gradient through this row
  const float inv = 1.f / w.al;
  const bool us = w.a != 0.f && w.ys >= 0, ux = w.b != 0.f && w.yx >= 0;
  CST_DCHECK(!us || w.ys < g.V);
  CST_DCHECK(!ux || w.yx < g.V);
  if (us && ux && w.ys == w.yx) {
    e[w.ys] = f2bf(bf2f(e[w.ys]) + (w.a + w.b) * inv);
  } else {
    if (us) e[w.ys] = f2bf(bf2f(e[w.ys]) + w.a * inv);
    if (ux) e[w.yx] = f2bf(bf2f(e[w.yx]) + w.b * inv);
  }
}

// one thread per row: alpha, and the one-hot terms folded into E
__global__ __launch_bounds__(256) void vgrad_onehot_kernel(VGradRows g, uint16_t* __restrict__ E,
                                                           int64_t ldl,
                                                           float* __restrict__ alpha) {
  const int64_t NR = (int64_t)g.n_steps * g.R;
  const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (row >= NR) return;
  const int t = (int)(row / g.R);
  if (g.oh_a != nullptr) {  // forward-computed X: the loop adds the one-hot terms itself
    const RowW w = row_weights(g, row);
    g.oh_a[row] = w.a;
    g.oh_ys[row] = w.ys;
    if (g.oh_b != nullptr) {
      g.oh_b[row] = w.b;
      g.oh_yx[row] = w.yx;
    }
  }
  if (g.fix != nullptr && (t > 0 || g.zero_off)) {
    const float d = g.zero_off ? g.lse[row] : g.lse[row] - g.lse[row - g.R];
    if (fabsf(d) > EXP_SAFE_LSE_JUMP) {  // E may be out of range: recomputed by vgrad_fix
      const int k = atomicAdd(g.fix, 1);
      g.fix[1 + k] = (int)row;
      return;
    }
  }
  const RowW w = row_weights(g, row);
  alpha[row] = w.al;
  fold_onehot(g, w, E + row * ldl);
}

void launch_vgrad_onehot(const VGradRows& g, uint16_t* E, int64_t ldl, float* alpha,
                         hipStream_t stream) {
  const int64_t NR = (int64_t)g.n_steps * g.R;
  hipLaunchKernelGGL(vgrad_onehot_kernel, dim3((unsigned)((NR + 255) / 256)), dim3(256), 0, stream,
                     g, E, ldl, alpha);
  post_launch("vgrad_onehot_kernel", stream);
}

// Exact recompute of the rows vgrad_onehot listed (rare: an LSE jump of more
// than 60 between consecutive steps).  One block per listed row at a time:
// the row's vocab input (H bf16) in LDS, x_v = hd . W_v + b_v by 16-byte W
// loads, E_v = exp(x_v - lse_row) (s = 1), then alpha and the one-hot fold.
constexpr int VFIX_BLOCKS = 256, VFIX_MAXH = 2048;
__global__ __launch_bounds__(256) void vgrad_fix_kernel(VGradRows g, const uint16_t* __restrict__ hd,
                                                        const uint16_t* __restrict__ W,
                                                        const float* __restrict__ bias,
                                                        uint16_t* __restrict__ E, int64_t ldl,
                                                        float* __restrict__ alpha,
                                                        int* __restrict__ fix_total) {
  __shared__ float s_h[VFIX_MAXH];
  const int n = g.fix[0];
  if (blockIdx.x == 0 && threadIdx.x == 0 && fix_total != nullptr && n > 0) fix_total[0] += n;
  const int H = g.H;
  for (int k = blockIdx.x; k < n; k += gridDim.x) {
    const int64_t row = g.fix[1 + k];
    __syncthreads();  // s_h of the previous row consumed
    for (int i = threadIdx.x; i < H; i += 256) s_h[i] = bf2f(hd[row * H + i]);
    __syncthreads();
    const float L = g.lse[row];
    uint16_t* e = E + row * ldl;
    for (int v = threadIdx.x; v < g.V; v += 256) {
      const uint4* wr = reinterpret_cast<const uint4*>(W + (int64_t)v * H);
      float x = 0.f;
      for (int c = 0; c < H / 8; ++c) {
        const uint4 q = wr[c];
        const uint32_t wv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x = fmaf(s_h[8 * c + 2 * j], bf2f(wv[j] & 0xffff), x);
          x = fmaf(s_h[8 * c + 2 * j + 1], bf2f(wv[j] >> 16), x);
        }
      }
      e[v] = f2bf(__expf(x + bias[v] - L));
    }
    __syncthreads();  // the row's E is complete before the one-hot fold
    if (g.X != nullptr) {  // forward-computed X = E W: this row's, from the exact E
      for (int hc = threadIdx.x; hc < H; hc += 256) {
        float x = 0.f;
        for (int v = 0; v < g.V; ++v) x = fmaf(bf2f(e[v]), bf2f(W[(int64_t)v * H + hc]), x);
        g.X[row * H + hc] = x;
      }
      __syncthreads();  // every thread read the unfolded row
    }
    if (threadIdx.x == 0) {
      const RowW w = row_weights(g, row, /*unit_s=*/true);
      alpha[row] = w.al;
      fold_onehot(g, w, e);
    }
  }
}

void launch_vgrad_fix(const VGradRows& g, const uint16_t* hd, const uint16_t* W, const float* bias,
                      uint16_t* E, int64_t ldl, float* alpha, int* fix_total, hipStream_t stream) {
  if (g.fix == nullptr) return;
  if (g.H % 8 != 0 || g.H > VFIX_MAXH)
    throw std::runtime_error("vgrad_fix: H must be a multiple of 8 and <= 2048");
  hipLaunchKernelGGL(vgrad_fix_kernel, dim3(VFIX_BLOCKS), dim3(256), 0, stream, g, hd, W, bias, E,
                     ldl, alpha, fix_total);
  post_launch("vgrad_fix_kernel", stream);
}

constexpr int VG_THREADS = 256, VG_ROWS = VG_THREADS / WAVE;

// One wavefront per rollout row, 8-column chunks per lane: hs = bf16(alpha
// Hd) (and dHd = alpha X in place when dhd is given; the engine instead lets
// the reverse loop scale the rows it reads, so this pass leaves the critical
// path).
// ldhs > H (augmented rows, ldhs = H + 8k): columns H, H + 1 of the row also
// get alpha as two bf16 words (hi, lo = alpha - hi) and the rest zeros, so the
// dW GEMM over these rows also yields the bias gradient E'^T alpha
__global__ __launch_bounds__(VG_THREADS) void vgrad_rows_kernel(
    const float* __restrict__ alpha, int64_t NR, int H, const uint16_t* __restrict__ hd,
    float* __restrict__ dhd, uint16_t* __restrict__ hs, int ldhs) {
  const int64_t row = (int64_t)blockIdx.x * VG_ROWS + (threadIdx.x >> 6);
  if (row >= NR) return;
  const int lane = threadIdx.x & 63;
  const float al = alpha[row];
  if (8 * lane < ldhs - H) {
    const uint16_t hi = f2bf(al), lo = f2bf(al - bf2f(hi));
    *reinterpret_cast<uint4*>(hs + row * ldhs + H + 8 * lane) =
        make_uint4(lane == 0 ? ((uint32_t)hi | ((uint32_t)lo << 16)) : 0u, 0u, 0u, 0u);
  }
  for (int c = lane; 8 * c < H; c += WAVE) {
    if (dhd != nullptr) {
      float4* xp = reinterpret_cast<float4*>(dhd + row * H + 8 * c);
      float4 x0 = xp[0], x1 = xp[1];
      x0.x *= al, x0.y *= al, x0.z *= al, x0.w *= al;
      x1.x *= al, x1.y *= al, x1.z *= al, x1.w *= al;
      xp[0] = x0;
      xp[1] = x1;
    }
    const uint4 h = *reinterpret_cast<const uint4*>(hd + row * H + 8 * c);
    const uint32_t hw[4] = {h.x, h.y, h.z, h.w};
    uint32_t ho[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      ho[k] = (uint32_t)f2bf(al * bf2f(hw[k] & 0xffff)) |
              ((uint32_t)f2bf(al * bf2f(hw[k] >> 16)) << 16);
    *reinterpret_cast<uint4*>(hs + row * ldhs + 8 * c) = make_uint4(ho[0], ho[1], ho[2], ho[3]);
  }
}

void launch_vgrad_rows(const float* alpha, int64_t NR, int H, const uint16_t* hd, float* dhd,
                       uint16_t* hs, hipStream_t stream, int ldhs) {
  if (ldhs <= 0) ldhs = H;
  if (H % 8 != 0) throw std::runtime_error("vgrad_rows: H must be a multiple of 8");
  if (ldhs < H || (ldhs - H) % 8 != 0 || ldhs - H > 8 * WAVE)
    throw std::runtime_error("vgrad_rows: ldhs must be H + 8k (k <= 64)");
  hipLaunchKernelGGL(vgrad_rows_kernel, dim3((unsigned)((NR + VG_ROWS - 1) / VG_ROWS)),
                     dim3(VG_THREADS), 0, stream, alpha, NR, H, hd, dhd, hs, ldhs);
  post_launch("vgrad_rows_kernel", stream);
}

// Bias gradient, softmax part: db_v = sum_r alpha_r E_rv.  Block (i, j) owns
// CS_ROWS rows and the 8-column chunks [256 j, 256 j + 256); each thread keeps
// its chunk's 8 sums in registers over the rows (CS_UNROLL row loads in
// flight) and writes one partial row per block; a second launch sums the
// partials per column (deterministic, no atomics).
// Rows per block: 128 fills the chip (1,680 workgroups at the headline shape,
// ~160 us at HBM rate) and delays the reverse loop the sums run under; 1024
// (210 workgroups) leaves most CU slots to the loop: interleaved A/B
// 3.559-3.579 vs 3.602-3.611 ms per step, 4096 3.659-3.676, 768 3.465-3.486
// vs 1024 3.477-3.479 (profiles/r4/README_r4.md).
constexpr int CS_ROWS = 128, CS_UNROLL = 8;

static int colsum_rows() { return 1024; }

int vgrad_colsum_blocks(int64_t NR) {
  const int rows = colsum_rows();
  return (int)((NR + rows - 1) / rows);
}

__global__ __launch_bounds__(256) void vgrad_colsum_kernel(const uint16_t* __restrict__ E,
                                                           int64_t ldl, int V, int64_t NR,
                                                           const float* __restrict__ alpha,
                                                           float* __restrict__ part, int rows) {
  __shared__ float s_al[CS_ROWS];
  const int ci = blockIdx.y * 256 + threadIdx.x;  // chunk
  const int v0 = 8 * ci;
  const int nv = min(8, V - v0);  // ragged last chunk: lanes >= nv are masked
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  const int64_t rb = (int64_t)blockIdx.x * rows;
  for (int64_t r0 = rb; r0 < min(rb + rows, NR); r0 += CS_ROWS) {
    const int nr = (int)min((int64_t)CS_ROWS, NR - r0);
    __syncthreads();  // previous chunk's weights read
    if ((int)threadIdx.x < nr) s_al[threadIdx.x] = alpha[r0 + threadIdx.x];
    __syncthreads();
    if (v0 >= V) continue;
    const uint16_t* base = E + r0 * ldl + v0;
    for (int i = 0; i < nr; i += CS_UNROLL) {
      uint4 x[CS_UNROLL];
#pragma unroll
      for (int u = 0; u < CS_UNROLL; ++u)
        x[u] = i + u < nr ? *reinterpret_cast<const uint4*>(base + (int64_t)(i + u) * ldl)
                          : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int u = 0; u < CS_UNROLL; ++u) {
        const float al = i + u < nr ? s_al[i + u] : 0.f;
        const uint32_t w[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          acc[2 * k] += al * bf2f(w[k] & 0xffff);
          acc[2 * k + 1] += al * bf2f(w[k] >> 16);
        }
      }
    }
  }
  if (v0 >= V) return;
  float* out = part + (int64_t)blockIdx.x * V + v0;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (k < nv) out[k] = acc[k];
}

// 64 columns per block, 4 groups of 64 threads splitting the partial rows
// (8 loads in flight each), summed through LDS
__global__ __launch_bounds__(256) void vgrad_colsum_reduce_kernel(const float* __restrict__ part,
                                                                  int nb, int V,
                                                                  float* __restrict__ db) {
  __shared__ float s_p[4][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int v = blockIdx.x * 64 + c;
  float s = 0.f;
  if (v < V) {
    int b = g;
    for (; b + 28 < nb; b += 32) {
      float x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = part[(int64_t)(b + 4 * u) * V + v];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += x[u];
    }
    for (; b < nb; b += 4) s += part[(int64_t)b * V + v];
  }
  s_p[g][c] = s;
  __syncthreads();
  if (g == 0 && v < V) db[v] = s_p[0][c] + s_p[1][c] + s_p[2][c] + s_p[3][c];
}

void launch_vgrad_colsum(const uint16_t* E, int64_t ldl, int V, int64_t NR, const float* alpha,
                         float* part, float* dblog, hipStream_t stream) {
  // the ragged last chunk reads a whole 16-byte chunk: it must stay inside the row
  if (ldl < (V + 7) / 8 * 8 || ldl % 8 != 0)
    throw std::runtime_error("vgrad_colsum: row stride must cover V rounded up to 8");
  const int nb = vgrad_colsum_blocks(NR);
  const int nch = (V + 7) / 8;
  hipLaunchKernelGGL(vgrad_colsum_kernel, dim3(nb, (nch + 255) / 256), dim3(256), 0, stream, E, ldl,
                     V, NR, alpha, part, colsum_rows());
  post_launch("vgrad_colsum_kernel", stream);
  hipLaunchKernelGGL(vgrad_colsum_reduce_kernel, dim3((V + 63) / 64), dim3(256), 0, stream, part,
                     nb, V, dblog);
  post_launch("vgrad_colsum_reduce_kernel", stream);
}

}  // namespace cst
