// K12: fused global-norm gradient clipping + Adam over ONE flat fp32 buffer.
//
// Reference: clip_grad_norm_(params, 0.25) + optim.Adam(lr) (default betas
// 0.9/0.999, eps 1e-8) at /root/reference/train.py:217-218,492 -- per-tensor
// kernels plus a host-side norm.  Here the whole model (~20 M fp32 params) is
// one contiguous buffer (the same buffer the DP all-reduce moves), so:
//   pass 1  adam_sumsq_kernel: grid-stride float4 sum of squares ->
//           one partial per block (deterministic tree, no atomics);
//   pass 2  adam_update_kernel: every block re-reduces the <=1024 partials
//           (4 KB, L2-resident) to the global norm, computes
//           coef = min(1, clip / (norm + 1e-6)) on device and applies
//           PyTorch's Adam update with the clipped gradient; an optional
//           device-side skip flag (non-finite loss) turns the step into a
//           no-op without a host round trip.
// Learning rate and step count live in device memory, so the bias
// corrections of a replayed HIP graph follow the live step count and an LR
// decay between replays needs no re-capture.  hyper = [lr, step at the start
// of the update, skipped updates, step after the update]: the update pass
// reads hyper[1] (every block) and block 0 writes hyper[3] (the step advances
// only when the update is applied, as torch.optim.Adam's step does); the
// next sum-of-squares pass commits hyper[3] -> hyper[1].
//
// NaN guard: the update is skipped when the caller's flag is set (non-finite
// loss, possibly on another DP rank) OR when the global gradient norm is not
// finite (an overflowing gradient with a finite loss, e.g. an exp-store
// entry out of bf16 range: clip / inf = 0 and inf * 0 = NaN would otherwise
// poison p, m, v for good).  Every DP rank reduces the same gradient, so they
// skip together.  Skips are counted in hyper[2] (reported in the log line).
//
// gscale: the gradient buffer holds gscale^-1 times the gradient (the DP
// all-reduce SUMS over N ranks; gscale = 1/N folds the average in here
// instead of a separate pass over the buffer).
//
// The update pass also refreshes the bf16 shadow copies of the decoder
// weights that the MFMA kernels read (ShadowSegs: vocab head, embedding, and
// the LSTM weights re-packed into the gate-interleaved [W_ie | W_hh] layout),
// so no separate conversion / cat / gather pass runs after the optimizer.
// Memory-bound: 5 x 4 B read + 3 x 4 B write per parameter (+ 2 B per
// shadowed parameter).
#include "../common.h"
#include "../launchers.h"

namespace cst {

constexpr int ADAM_THREADS = 256;
constexpr int ADAM_MAX_PARTIALS = 1024;

__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x < ADAM_THREADS / 64) r = sh[threadIdx.x];
  if (w == 0) r = wave_sum(r);
  return r;  // valid in wave 0
}

__global__ __launch_bounds__(ADAM_THREADS) void adam_sumsq_kernel(const float* __restrict__ g,
                                                                   int64_t n,
                                                                   float* __restrict__ partials,
                                                                   float* __restrict__ hyper) {
  __shared__ float sh[ADAM_THREADS / 64];
  // commit the previous update's step count (no block of this pass reads it)
  if (blockIdx.x == 0 && threadIdx.x == 0) hyper[1] = hyper[3];
  float acc = 0.f;
  const int64_t n4 = n >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = blockIdx.x * (int64_t)ADAM_THREADS + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * ADAM_THREADS) {
    const float4 x = g4[i];
    acc += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += ADAM_THREADS) acc += g[i] * g[i];
  }
  const float s = block_sum(acc, sh);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// packed gate row of source weight row g*H + u: 4u + slot(g), slot(g) = bits
// [2g, 2g + 2) of the segment's slot map (LSTM 0xE4: i,f,g,o -> 0,1,2,3; GRU
// W_ih 0x24: r,z,n -> 0,1,2; GRU W_hh 0x34: r,z,n -> 0,1,3; RNN 0x0)
__device__ __forceinline__ int64_t packed_gate_row(int64_t row, int H, int slots) {
  const int g = (int)(row / H);
  return (row - (int64_t)g * H) * 4 + ((slots >> (2 * g)) & 3);
}

__device__ __forceinline__ void shadow_store(const ShadowSegs& ss, int64_t e, float val) {
#pragma unroll
  for (int k = 0; k < SHADOW_MAX_SEGS; ++k) {
    if (k >= ss.n) break;
    const ShadowSeg& g = ss.s[k];
    const int64_t j = e - g.off;
    if (j < 0 || j >= g.n) continue;
    const uint16_t b = f2bf(val);
    if (g.kind == SHADOW_PLAIN) {
      g.dst[j] = b;
    } else {
      const int64_t row = j / g.cols, col = j - row * g.cols;
      const int64_t pr = packed_gate_row(row, g.H, g.slots);
      if (g.kind == SHADOW_GATES_IH) {
        if (col < g.E) g.dst[pr * (g.E + g.H) + col] = b;
        else if (g.dst2 != nullptr) g.dst2[pr * g.ld2 + (col - g.E)] = b;  // video columns
      } else {  // SHADOW_GATES_HH
        g.dst[pr * (g.E + g.H) + g.E + col] = b;
        g.dst2[pr * g.ld2 + col] = b;
      }
    }
  }
}

// The 4 consecutive parameters [e0, e0 + 4) of one float4 of the update: per
// segment one range test; a float4 inside one segment (the common case) takes
// one int32 row division and 4 contiguous bf16 stores (the per-element path
// cost a 64-bit division and a segment scan per parameter: VALU-bound
// update pass); float4s straddling a segment or row boundary fall back.
__device__ __forceinline__ void shadow_store4(const ShadowSegs& ss, int64_t e0, const float4& v) {
  const float vals[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < SHADOW_MAX_SEGS; ++k) {
    if (k >= ss.n) break;
    const ShadowSeg& g = ss.s[k];
    const int64_t j0 = e0 - g.off;
    if (j0 < -3 || j0 >= g.n) continue;  // no overlap
    if (j0 < 0 || j0 + 3 >= g.n) {       // partial overlap: per parameter
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (j0 + q >= 0 && j0 + q < g.n) shadow_store(ss, e0 + q, vals[q]);
      continue;
    }
    if (g.kind == SHADOW_PLAIN) {
      uint16_t* d = g.dst + j0;
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = f2bf(vals[q]);
      continue;
    }
    const int jj = (int)j0, row = jj / g.cols, col = jj - row * g.cols;
    if (col + 3 >= g.cols) {  // crosses a source row
#pragma unroll
      for (int q = 0; q < 4; ++q) shadow_store(ss, e0 + q, vals[q]);
      continue;
    }
    const int64_t pr = packed_gate_row(row, g.H, g.slots);
    if (g.kind == SHADOW_GATES_IH) {
      if (col + 3 < g.E) {
        uint16_t* d = g.dst + pr * (g.E + g.H) + col;
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = f2bf(vals[q]);
      } else if (g.dst2 != nullptr && col >= g.E) {  // packed video columns
        uint16_t* d = g.dst2 + pr * g.ld2 + (col - g.E);
#pragma unroll
        for (int q = 0; q < 4; ++q) d[q] = f2bf(vals[q]);
      } else {  // straddles the token / video boundary, or no video shadow
#pragma unroll
        for (int q = 0; q < 4; ++q) shadow_store(ss, e0 + q, vals[q]);
      }
    } else {  // SHADOW_GATES_HH
      uint16_t* d = g.dst + pr * (g.E + g.H) + g.E + col;
      uint16_t* d2 = g.dst2 + pr * g.ld2 + col;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint16_t bq = f2bf(vals[q]);
        d[q] = bq;
        d2[q] = bq;
      }
    }
  }
}

__global__ __launch_bounds__(256) void shadow_refresh_kernel(const float* __restrict__ p,
                                                             ShadowSegs ss, int seg) {
  const ShadowSeg& g = ss.s[seg];
  for (int64_t j = blockIdx.x * 256ll + threadIdx.x; j < g.n; j += (int64_t)gridDim.x * 256)
    shadow_store(ss, g.off + j, p[g.off + j]);
}

__device__ __forceinline__ void adam_one(float& p, float& m, float& v, float g, float coef,
                                         float lr_bc1, float b1, float b2, float eps,
                                         float inv_sqrt_bc2) {
  g *= coef;
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  const float denom = sqrtf(v) * inv_sqrt_bc2 + eps;
  p -= lr_bc1 * m / denom;
}

__global__ __launch_bounds__(ADAM_THREADS) void adam_update_kernel(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
    float* __restrict__ v, int64_t n, const float* __restrict__ partials, int nparts,
    const bool* __restrict__ skip, float* __restrict__ scal, float* __restrict__ hyper,
    float b1, float b2, float eps, float clip, float gscale, ShadowSegs ss) {
  __shared__ float sh[ADAM_THREADS / 64];
  __shared__ float s_coef;
  __shared__ int s_skip;
  const float t0 = hyper[1], t = t0 + 1.f;
  const float lr_bc1 = hyper[0] / (1.f - powf(b1, t));
  const float inv_sqrt_bc2 = 1.f / sqrtf(1.f - powf(b2, t));
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += ADAM_THREADS) acc += partials[i];
  const float tot = block_sum(acc, sh);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(tot) * gscale;
    const bool bad = *skip || !isfinite(norm);
    s_skip = bad;
    s_coef = fminf(1.f, clip / (norm + 1e-6f)) * gscale;
    if (blockIdx.x == 0) {
      scal[0] = norm;
      scal[1] = bad ? 0.f : s_coef / gscale;
      hyper[3] = bad ? t0 : t;
      if (bad) hyper[2] += 1.f;
    }
  }
  __syncthreads();
  if (s_skip) return;
  const float coef = s_coef;
  const int64_t n4 = n >> 2;
  float4* p4 = reinterpret_cast<float4*>(p);
  float4* m4 = reinterpret_cast<float4*>(m);
  float4* v4 = reinterpret_cast<float4*>(v);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = blockIdx.x * (int64_t)ADAM_THREADS + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * ADAM_THREADS) {
    float4 pp = p4[i], mm = m4[i], vv = v4[i];
    const float4 gg = g4[i];
    adam_one(pp.x, mm.x, vv.x, gg.x, coef, lr_bc1, b1, b2, eps, inv_sqrt_bc2);
    adam_one(pp.y, mm.y, vv.y, gg.y, coef, lr_bc1, b1, b2, eps, inv_sqrt_bc2);
    adam_one(pp.z, mm.z, vv.z, gg.z, coef, lr_bc1, b1, b2, eps, inv_sqrt_bc2);
    adam_one(pp.w, mm.w, vv.w, gg.w, coef, lr_bc1, b1, b2, eps, inv_sqrt_bc2);
    p4[i] = pp;
    m4[i] = mm;
    v4[i] = vv;
    if (ss.n > 0) shadow_store4(ss, 4 * i, pp);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += ADAM_THREADS) {
      adam_one(p[i], m[i], v[i], g[i], coef, lr_bc1, b1, b2, eps, inv_sqrt_bc2);
      if (ss.n > 0) shadow_store(ss, i, p[i]);
    }
  }
}

void launch_flat_adam(float* p, const float* g, float* m, float* v, int64_t n, float* partials,
                      const bool* skip, float* scal, float* hyper, float b1, float b2,
                      float eps, float clip, float gscale, int phase, const ShadowSegs& ss,
                      hipStream_t stream) {
  // (a sharded update: every rank's shard has the same n, so the same
  // number of partials, which the caller all-reduces between phases 1 and 2)
  int blocks = (int)std::min<int64_t>(ADAM_MAX_PARTIALS, std::max<int64_t>(1, (n / 4 + 255) / 256));
  if (phase != 2) {
    hipLaunchKernelGGL(adam_sumsq_kernel, dim3(blocks), dim3(ADAM_THREADS), 0, stream, g, n,
                       partials, hyper);
    post_launch("adam_sumsq_kernel", stream);
  }
  if (phase == 1) return;
  int ublocks = (int)std::min<int64_t>(2048, std::max<int64_t>(1, (n / 4 + 255) / 256));
  hipLaunchKernelGGL(adam_update_kernel, dim3(ublocks), dim3(ADAM_THREADS), 0, stream, p, g, m,
                     v, n, partials, blocks, skip, scal, hyper, b1, b2, eps, clip, gscale, ss);
  post_launch("adam_update_kernel", stream);
}

void launch_shadow_refresh(const float* p, const ShadowSegs& ss, hipStream_t stream) {
  for (int k = 0; k < ss.n; ++k) {
    const int blocks = (int)std::min<int64_t>(2048, std::max<int64_t>(1, (ss.s[k].n + 255) / 256));
    hipLaunchKernelGGL(shadow_refresh_kernel, dim3(blocks), dim3(256), 0, stream, p, ss, k);
    post_launch("shadow_refresh_kernel", stream);
  }
}

}  // namespace cst
