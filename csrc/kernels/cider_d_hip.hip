#include "hip/hip_runtime.h"
// K5: CIDEr-D of sampled captions, on the GPU.
//
// Replaces the per-iteration host round trip of the reference
// (/root/reference/train.py:185,198-199 -> utils.py:229-324 -> external
// pyciderevalcap CiderD on the CPU) with one launch.  Reference n-gram vectors
// (tf-idf values, per-order norms, bigram "lengths") are precomputed once per
// dataset by csrc/host/cider_host.cpp; this kernel only processes hypotheses.
//
// One wavefront per hypothesis (4 per 256-thread block):
//   1. token compaction with ballots, reproducing array_to_str
//      (utils.py:135-152): drop BOS (=1) anywhere, stop at the first EOS (=0)
//      and keep that "0" when use_eos;
//   2. packed n-gram keys (n<=4) in LDS; term frequencies by an in-wave
//      O(W) scan, counted once at the first occurrence (later duplicates get
//      value 0, which contributes exactly 0 to the clipped dot product);
//   3. idf from the df hash table in HBM, per-order norms by wave reduction;
//   4. for every reference of the video: lanes stride over the reference's
//      unique n-grams, look each up among the hypothesis n-grams in LDS
//      (broadcast reads), accumulate min(vh, vr) * vr per order, normalise,
//      apply exp(-(lh - lr)^2 / (2 * 6^2));
//   5. score = 10 * sum_refs mean_n(val_n) / n_refs.
// Deterministic: fixed-order wave reductions, no atomics.
#include "../common.h"
#include "../cider_common.h"

namespace cst {

constexpr int CIDER_WAVES = 4;
constexpr int CIDER_MAXT = 64;

__global__ __launch_bounds__(256) void cider_d_kernel(
    const int64_t* __restrict__ hyps, int T, const int64_t* __restrict__ hyp_video, int N,
    const int64_t* __restrict__ ht_keys, const float* __restrict__ ht_vals, uint32_t ht_cap,
    const int32_t* __restrict__ vid_ref_off, const int32_t* __restrict__ ref_ng_off,
    const float* __restrict__ ref_norm, const int32_t* __restrict__ ref_len,
    const int64_t* __restrict__ ng_key, const float* __restrict__ ng_val, float log_ref_len,
    int use_eos, float* __restrict__ out) {
  __shared__ int s_tok[CIDER_WAVES][CIDER_MAXT];
  __shared__ uint64_t s_key[CIDER_WAVES][4][CIDER_MAXT];
  __shared__ float s_val[CIDER_WAVES][4][CIDER_MAXT];

  const int w = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int hyp_raw = blockIdx.x * CIDER_WAVES + w;
  const bool valid = hyp_raw < N;  // invalid waves still take part in the barriers
  const int hyp = valid ? hyp_raw : N - 1;

  // -- 1. compaction ------------------------------------------------------------
  int tok = lane < T ? (int)hyps[(int64_t)hyp * T + lane] : 0;
  uint64_t zmask = __ballot(lane >= T || tok == 0);
  int e = zmask ? __ffsll((long long)zmask) - 1 : 64;  // first EOS (or end)
  bool keep = lane < e && tok != 1;
  uint64_t kmask = __ballot(keep);
  int pos = __popcll(kmask & ((1ull << lane) - 1ull));
  int W = __popcll(kmask);
  if (keep) s_tok[w][pos] = tok;
  if (use_eos && e < T) {
    if (lane == 0) s_tok[w][W] = 0;
    W += 1;
  }
  __syncthreads();

  // -- 2./3. hypothesis n-grams, tf, idf, norms ---------------------------------
  float norm_h[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int cnt = W - n;  // number of n-grams of order n+1
    uint64_t key = 0;
    if (lane < cnt) {
#pragma unroll
      for (int i = 0; i <= n; ++i) key |= (uint64_t)(s_tok[w][lane + i] + 1) << (16 * i);
    }
    s_key[w][n][lane] = key;
  }
  __syncthreads();
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int cnt = W - n;
    float v = 0.f;
    if (lane < cnt) {
      const uint64_t key = s_key[w][n][lane];
      int tf = 0;
      bool first = true;
      for (int j = 0; j < cnt; ++j) {
        const bool eq = s_key[w][n][j] == key;
        tf += eq;
        first = first && !(eq && j < lane);
      }
      if (first) {
        const float df = df_lookup(ht_keys, ht_vals, ht_cap, key);
        v = (float)tf * (log_ref_len - __logf(fmaxf(1.f, df)));
      }
    }
    s_val[w][n][lane] = v;
    norm_h[n] = sqrtf(wave_sum(v * v));
  }
  __syncthreads();
  const float len_h = (float)max(W - 1, 0);

  // -- 4./5. references --------------------------------------------------------
  const int v = (int)hyp_video[hyp];
  const int r0 = vid_ref_off[v], r1 = vid_ref_off[v + 1];
  float total = 0.f;
  for (int r = r0; r < r1; ++r) {
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
    const int g0 = ref_ng_off[r], g1 = ref_ng_off[r + 1];
    for (int g = g0 + lane; g < g1; g += 64) {
      const uint64_t key = (uint64_t)ng_key[g];
      const float vr = ng_val[g];
      const int n = ngram_order(key) - 1;
      const int cnt = W - n;
      float c = 0.f;
      for (int j = 0; j < cnt; ++j) {
        if (s_key[w][n][j] == key) c += fminf(s_val[w][n][j], vr) * vr;
      }
      acc0 += n == 0 ? c : 0.f;
      acc1 += n == 1 ? c : 0.f;
      acc2 += n == 2 ? c : 0.f;
      acc3 += n == 3 ? c : 0.f;
    }
    float acc[4] = {wave_sum(acc0), wave_sum(acc1), wave_sum(acc2), wave_sum(acc3)};
    const float delta = len_h - (float)ref_len[r];
    const float pen = __expf(-(delta * delta) / 72.f);
    float s = 0.f;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const float nr = ref_norm[r * 4 + n];
      float val = acc[n];
      if (norm_h[n] != 0.f && nr != 0.f) val /= (norm_h[n] * nr);
      s += val * pen;
    }
    total += s;
  }
  if (lane == 0 && valid) {
    const int nref = r1 - r0;
    out[hyp] = nref > 0 ? 10.f * total / (4.f * (float)nref) : 0.f;
  }
}

void launch_cider_d(const int64_t* hyps, int T, const int64_t* hyp_video, int N,
                    const int64_t* ht_keys, const float* ht_vals, uint32_t ht_cap,
                    const int32_t* vid_ref_off, const int32_t* ref_ng_off,
                    const float* ref_norm, const int32_t* ref_len, const int64_t* ng_key,
                    const float* ng_val, float log_ref_len, int use_eos, float* out,
                    hipStream_t stream) {
  if (N <= 0) return;
  dim3 grid((N + CIDER_WAVES - 1) / CIDER_WAVES), block(64 * CIDER_WAVES);
  hipLaunchKernelGGL(cider_d_kernel, grid, block, 0, stream, hyps, T, hyp_video, N, ht_keys,
                     ht_vals, ht_cap, vid_ref_off, ref_ng_off, ref_norm, ref_len, ng_key,
                     ng_val, log_ref_len, use_eos, out);
}

}  // namespace cst
