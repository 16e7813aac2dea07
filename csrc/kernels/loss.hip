// P19 + P21 on the device in two launches: the self-critical reward
// (sample CIDEr-D - greedy CIDEr-D, /root/reference/utils.py:215-224), the
// reference's reward mask (a row's first token always counts, later tokens
// while the previous one was not EOS; model.py RewardCriterion) and the
// REINFORCE loss  -sum(lp * reward * mask) / sum(mask), plus the logged means
// of the sample and greedy scores (train.py:223-246).  The PyTorch
// formulation is ~20 small launches between the CIDEr-D kernel and the
// backward on the critical path of every SCST step.
#include "../common.h"
#include "../launchers.h"

namespace cst {

constexpr int SL_THREADS = 1024;

__device__ __forceinline__ float block_sum_1024(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x < SL_THREADS / WAVE) t = sh[threadIdx.x];
  if (w == 0) t = wave_sum(t);
  return t;  // valid in thread 0
}

// one block: out = {loss, mean(sample), mean(greedy per row), sum(mask)},
// reward[r] = sample[r] - greedy[r / gdiv]
__global__ __launch_bounds__(SL_THREADS) void scst_loss_fwd_kernel(
    const int64_t* __restrict__ seq, const float* __restrict__ lp, int R, int T,
    const float* __restrict__ sample, const float* __restrict__ greedy, int gdiv,
    float* __restrict__ reward, float* __restrict__ out, float* __restrict__ loss) {
  __shared__ float sh[SL_THREADS / WAVE];
  float num = 0.f, den = 0.f, ssum = 0.f, gsum = 0.f;
  for (int r = threadIdx.x; r < R; r += SL_THREADS) {
    const float s = sample[r], g = greedy[r / gdiv];
    reward[r] = s - g;
    ssum += s;
    gsum += g;
  }
  for (int64_t i = threadIdx.x; i < (int64_t)R * T; i += SL_THREADS) {
    const int r = (int)(i / T), t = (int)(i % T);
    const float m = (t == 0 || seq[i - 1] > 0) ? 1.f : 0.f;
    const float rw = sample[r] - greedy[r / gdiv];
    num += lp[i] * rw * m;
    den += m;
  }
  num = block_sum_1024(num, sh);
  den = block_sum_1024(den, sh);
  ssum = block_sum_1024(ssum, sh);
  gsum = block_sum_1024(gsum, sh);
  if (threadIdx.x == 0) {
    out[0] = -num / den;
    loss[0] = out[0];
    out[1] = ssum / (float)R;
    out[2] = gsum / (float)R;
    out[3] = den;
  }
}

// dlp = -reward * mask / sum(mask) * dloss
__global__ __launch_bounds__(256) void scst_loss_bwd_kernel(const int64_t* __restrict__ seq,
                                                            const float* __restrict__ reward,
                                                            const float* __restrict__ out,
                                                            const float* __restrict__ dloss,
                                                            int R, int T, float* __restrict__ dlp) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)R * T) return;
  const int r = (int)(i / T), t = (int)(i % T);
  const float m = (t == 0 || seq[i - 1] > 0) ? 1.f : 0.f;
  dlp[i] = -reward[r] * m / out[3] * dloss[0];
}

void launch_scst_loss_fwd(const int64_t* seq, const float* lp, int R, int T, const float* sample,
                          const float* greedy, int gdiv, float* reward, float* out, float* loss,
                          hipStream_t stream) {
  hipLaunchKernelGGL(scst_loss_fwd_kernel, dim3(1), dim3(SL_THREADS), 0, stream, seq, lp, R, T,
                     sample, greedy, gdiv, reward, out, loss);
  post_launch("scst_loss_fwd_kernel", stream);
}

void launch_scst_loss_bwd(const int64_t* seq, const float* reward, const float* out,
                          const float* dloss, int R, int T, float* dlp, hipStream_t stream) {
  const int64_t n = (int64_t)R * T;
  hipLaunchKernelGGL(scst_loss_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     seq, reward, out, dloss, R, T, dlp);
  post_launch("scst_loss_bwd_kernel", stream);
}

}  // namespace cst
