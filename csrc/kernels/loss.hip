// P19 + P21 (and P22, CST) on the device in two launches: the self-critical reward
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

// Forward: 16 rows per 256-thread workgroup (4 rows per wave, the row's
// T tokens across the lanes: no per-element division), per-workgroup partials
// {num, den, sum sample, sum greedy} stored write-through, then one lane's
// agent-scope ticket; the workgroup that draws the last ticket sums the
// partials in workgroup order (deterministic) and writes out / loss.  One
// launch of ~R / 16 workgroups instead of a single 1,024-thread block that
// walked all R x T elements (178 us at 1,280 x 28, profiles/r3).
constexpr int SL_ROWS = 16;  // rows per workgroup
int scst_loss_ws_ints(int R) { return 4 * ((R + SL_ROWS - 1) / SL_ROWS) + 64; }

__device__ __forceinline__ float block_sum_256(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) sh[w] = v;
  __syncthreads();
  const float t = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return t;
}

// The workgroup's partials {v0..v3} (block sums, thread 0's values count)
// are stored write-through and the last workgroup to draw the ticket sums all
// of them in workgroup order: returns true there, with a[] the totals (in wave
// 0); every other workgroup returns false.
__device__ bool total_of_partials(float v0, float v1, float v2, float v3, int* __restrict__ ws,
                                  float a[4]) {
  __shared__ int s_last;
  const int lane = threadIdx.x & 63;
  float* part = reinterpret_cast<float*>(ws + 64);
  if (threadIdx.x == 0) {
    __hip_atomic_store(part + 4 * blockIdx.x, v0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(part + 4 * blockIdx.x + 1, v1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(part + 4 * blockIdx.x + 2, v2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(part + 4 * blockIdx.x + 3, v3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // Hand-off of the partials (gfx950): they are stored write-through (sc1,
    // agent-scope relaxed atomic stores) and drained by s_waitcnt vmcnt(0)
    // before the ticket, and the last arriver reads them with sc1 loads only
    // (agent-scope relaxed atomic loads, which bypass the non-coherent L1).
    // That is the valid no-fence form of an inter-workgroup hand-off on this
    // chip (CDNA HIP guide, Guideline 16 / split-K seam): an agent-scope
    // release here would add an L2 write-back (buffer_wbl2) on the critical
    // path, an agent-scope acquire an L1 invalidate, neither needed.
    const int ticket = __hip_atomic_fetch_add(ws, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = ticket == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler order: loads after the ticket)
  // last workgroup: the partials in workgroup order, 4 per thread pass
  a[0] = a[1] = a[2] = a[3] = 0.f;
  if (threadIdx.x < 64) {
    for (int b = 0; b < (int)gridDim.x; b += 64) {
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (b + lane < (int)gridDim.x)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          v[k] = __hip_atomic_load(part + 4 * (b + lane) + k, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] += wave_sum(v[k]);
    }
  }
  return true;
}

// out = {loss, mean(sample), mean(baseline score per row), sum(mask)},
// reward[r] = sample[r] - greedy[r / gdiv] (SCST, cb.S == 0), or
// sample[r] - mean of the cb.k lowest of the video's cb.S reference scores
// (CST; the logged b: mean(bref) with GT consensus scores, mean(baseline)
// with the samples' own, 0 for k = 0); ws: scst_loss_ws_ints(R) ints,
// the ticket word (ws[0]) zero at the first launch (re-armed by the kernel)
__global__ __launch_bounds__(256) void scst_loss_fwd_kernel(
    const int64_t* __restrict__ seq, const float* __restrict__ lp, int R, int T,
    const float* __restrict__ sample, const float* __restrict__ greedy, int gdiv,
    float* __restrict__ reward, float* __restrict__ out, float* __restrict__ loss,
    int* __restrict__ ws, CstBase cb) {
  __shared__ float sh[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float num = 0.f, den = 0.f, ssum = 0.f, gsum = 0.f;
#pragma unroll
  for (int j = 0; j < SL_ROWS / 4; ++j) {
    const int r = blockIdx.x * SL_ROWS + w * (SL_ROWS / 4) + j;
    if (r >= R) break;
    const float sv = sample[r];
    float gv, gl;  // baseline of the row, its logged value
    if (cb.S > 0) {
      // CST (utils.py:292-324): the mean of the video's scb_captions lowest
      // reference scores (the GT consensus scores, or the samples' own).
      // Lane j holds score j of the video; its rank (ties by index) says
      // whether it is among the k lowest -- the selection of a stable sort
      // without sorting.
      float base = 0.f;
      if (cb.k > 0) {
        const int v0 = (r / cb.S) * cb.S;
        const float* ref = cb.bref != nullptr ? cb.bref : sample;
        const float x = lane < cb.S ? ref[v0 + lane] : 0.f;
        int rank = 0;
        for (int i = 0; i < cb.S; ++i) {
          const float y = __shfl(x, i, 64);
          rank += (y < x || (y == x && i < lane)) ? 1 : 0;
        }
        base = wave_sum(lane < cb.S && rank < cb.k ? x : 0.f) / (float)cb.k;
      }
      gv = base;
      gl = cb.k == 0 ? 0.f : (cb.bref != nullptr ? cb.bref[r] : base);
    } else {
      gv = gl = greedy[r / gdiv];
    }
    const float rw = sv - gv;
    if (lane == 0) {
      reward[r] = rw;
      ssum += sv;
      gsum += gl;
    }
    const int64_t* srow = seq + (int64_t)r * T;
    const float* lrow = lp + (int64_t)r * T;
    for (int t = lane; t < T; t += 64) {
      const float m = (t == 0 || srow[t - 1] > 0) ? 1.f : 0.f;
      num += lrow[t] * rw * m;
      den += m;
    }
  }
  num = block_sum_256(num, sh);
  den = block_sum_256(den, sh);
  ssum = block_sum_256(ssum, sh);
  gsum = block_sum_256(gsum, sh);
  float a[4];
  if (!total_of_partials(num, den, ssum, gsum, ws, a)) return;
  if (threadIdx.x == 0) {
    out[0] = -a[0] / a[1];
    loss[0] = out[0];
    out[1] = a[2] / (float)R;
    out[2] = a[3] / (float)R;
    out[3] = a[1];
    ws[0] = 0;  // re-arm for the next launch (stream-ordered)
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
                          int* ws, CstBase cb, hipStream_t stream) {
  hipLaunchKernelGGL(scst_loss_fwd_kernel, dim3((R + SL_ROWS - 1) / SL_ROWS), dim3(256), 0, stream,
                     seq, lp, R, T, sample, greedy, gdiv, reward, out, loss, ws, cb);
  post_launch("scst_loss_fwd_kernel", stream);
}

void launch_scst_loss_bwd(const int64_t* seq, const float* reward, const float* out,
                          const float* dloss, int R, int T, float* dlp, hipStream_t stream) {
  const int64_t n = (int64_t)R * T;
  hipLaunchKernelGGL(scst_loss_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     seq, reward, out, dloss, R, T, dlp);
  post_launch("scst_loss_bwd_kernel", stream);
}

// XE (CrossEntropyCriterion on the gathered GT log-probs, models/criteria.py,
// with the loader's masks, dataloader.py:158-163 / data/dataset.py gather):
// the mask of label row r covers positions j < nnz(labels[r]) + 1; the
// criterion reads it from column off on, so log-prob t counts while
// t < nnz + 1 - off =: cnt[r].  loss = -sum(lp * mask) / sum(mask), out =
// {loss, sum(mask)}.  One launch instead of the mask gather (a long-integer
// row count, compare, convert) and the criterion's sums: ~12 launches, and
// the row count sat behind the vocab head's X GEMM (profiles/r6/steps_xe*).
__global__ __launch_bounds__(256) void xe_loss_fwd_kernel(
    const int64_t* __restrict__ labels, int L, int off, const float* __restrict__ lp, int R, int T,
    float* __restrict__ cnt, float* __restrict__ out, float* __restrict__ loss,
    int* __restrict__ ws) {
  __shared__ float sh[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float num = 0.f, den = 0.f;
#pragma unroll
  for (int j = 0; j < SL_ROWS / 4; ++j) {
    const int r = blockIdx.x * SL_ROWS + w * (SL_ROWS / 4) + j;
    if (r >= R) break;
    const int64_t* lrow = labels + (int64_t)r * L;
    float nz = 0.f;
    for (int c = lane; c < L; c += 64) nz += lrow[c] != 0 ? 1.f : 0.f;
    const float n = wave_sum(nz) + 1.f - (float)off;
    if (lane == 0) cnt[r] = n;
    const float* prow = lp + (int64_t)r * T;
    for (int t = lane; t < T; t += 64) {
      const float m = (float)t < n ? 1.f : 0.f;
      num += prow[t] * m;
      den += m;
    }
  }
  num = block_sum_256(num, sh);
  den = block_sum_256(den, sh);
  float a[4];
  if (!total_of_partials(num, den, 0.f, 0.f, ws, a)) return;
  if (threadIdx.x == 0) {
    out[0] = -a[0] / a[1];
    out[1] = a[1];
    loss[0] = out[0];
    ws[0] = 0;  // re-arm (stream-ordered)
  }
}

// dlp = -mask / sum(mask) * dloss
__global__ __launch_bounds__(256) void xe_loss_bwd_kernel(const float* __restrict__ cnt,
                                                          const float* __restrict__ out,
                                                          const float* __restrict__ dloss, int R,
                                                          int T, float* __restrict__ dlp) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)R * T) return;
  const int r = (int)(i / T), t = (int)(i % T);
  dlp[i] = (float)t < cnt[r] ? -dloss[0] / out[1] : 0.f;
}

void launch_xe_loss_fwd(const int64_t* labels, int L, int off, const float* lp, int R, int T,
                        float* cnt, float* out, float* loss, int* ws, hipStream_t stream) {
  hipLaunchKernelGGL(xe_loss_fwd_kernel, dim3((R + SL_ROWS - 1) / SL_ROWS), dim3(256), 0, stream,
                     labels, L, off, lp, R, T, cnt, out, loss, ws);
  post_launch("xe_loss_fwd_kernel", stream);
}

void launch_xe_loss_bwd(const float* cnt, const float* out, const float* dloss, int R, int T,
                        float* dlp, hipStream_t stream) {
  const int64_t n = (int64_t)R * T;
  hipLaunchKernelGGL(xe_loss_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     cnt, out, dloss, R, T, dlp);
  post_launch("xe_loss_bwd_kernel", stream);
}

}  // namespace cst
