// K5: CIDEr-D of sampled captions, on the GPU.
//
// Replaces the per-iteration host round trip of the reference
// (/root/reference/train.py:185,198-199 -> utils.py:229-324 -> external
// pyciderevalcap CiderD on the CPU) with one launch.  Reference n-gram vectors
// (tf-idf values, per-order norms, bigram "lengths") are precomputed once per
// dataset by csrc/host/cider_host.cpp; this kernel only processes hypotheses.
//
// One 256-thread block per hypothesis:
//   1. token compaction with ballots, reproducing array_to_str
//      (utils.py:135-152): drop BOS (=1) anywhere, stop at the first EOS (=0)
//      and keep that "0" when use_eos;
//   2. packed n-gram keys (n<=4) in LDS; term frequencies by an in-wave
//      O(W) scan, counted once at the first occurrence (later duplicates get
//      value 0, which contributes exactly 0 to the clipped dot product);
//   3. idf from the df hash table in HBM, per-order norms by wave reduction;
//   4. the 4 waves split the video's references; for each one, lanes stride over its
//      unique n-grams, look each up among the hypothesis n-grams in LDS
//      (broadcast reads), accumulate min(vh, vr) * vr per order, normalise,
//      apply exp(-(lh - lr)^2 / (2 * 6^2));
//   5. score = 10 * sum_refs mean_n(val_n) / n_refs.
// Deterministic: fixed-order wave/block reductions, no atomics.
#include "../common.h"
#include "../cider_common.h"

namespace cst {

constexpr int CIDER_MAXT = 64;

// One 256-thread block per hypothesis: wave 0 builds the hypothesis vector
// (steps 1-3) in LDS, then the 4 waves split the video's references.
__global__ __launch_bounds__(256) void cider_d_kernel(
    const int64_t* __restrict__ hyps, int T, const int64_t* __restrict__ hyp_video, int N,
    const int64_t* __restrict__ ht_keys, const float* __restrict__ ht_vals, uint32_t ht_cap,
    const int32_t* __restrict__ vid_ref_off, const int32_t* __restrict__ ref_ng_off,
    const float* __restrict__ ref_norm, const int32_t* __restrict__ ref_len,
    const int64_t* __restrict__ ng_key, const float* __restrict__ ng_val, float log_ref_len,
    int use_eos, float* __restrict__ out) {
  __shared__ int s_tok[CIDER_MAXT];
  __shared__ uint64_t s_key[4][CIDER_MAXT];
  __shared__ float s_val[4][CIDER_MAXT];
  __shared__ float s_norm[4];
  __shared__ float s_part[4];
  __shared__ int s_W;

  const int w = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int hyp = blockIdx.x;

  // -- 1. compaction (wave 0) ----------------------------------------------------
  if (w == 0) {
    const int tok = lane < T ? (int)hyps[(int64_t)hyp * T + lane] : 0;
    const uint64_t zmask = __ballot(lane >= T || tok == 0);
    const int e = zmask ? __ffsll((long long)zmask) - 1 : 64;  // first EOS (or end)
    const bool keep = lane < e && tok != 1;
    const uint64_t kmask = __ballot(keep);
    const int pos = __popcll(kmask & ((1ull << lane) - 1ull));
    int W = __popcll(kmask);
    if (keep) s_tok[pos] = tok;
    if (use_eos && e < T) {
      if (lane == 0) s_tok[W] = 0;
      W += 1;
    }
    if (lane == 0) s_W = W;
  }
  __syncthreads();
  const int W = s_W;
  // -- 2. packed n-gram keys: wave n builds the order-(n+1) keys ------------------
  {
    const int n = w, cnt = W - n;
    uint64_t key = 0;
    if (lane < cnt) {
      for (int i = 0; i <= n; ++i) key |= (uint64_t)(s_tok[lane + i] + 1) << (16 * i);
    }
    s_key[n][lane] = key;
  }
  __syncthreads();
  // -- 3. tf (first occurrence), idf, per-order norm: wave n handles order n+1 ----
  {
    const int n = w, cnt = W - n;
    float v = 0.f;
    if (lane < cnt) {
      const uint64_t key = s_key[n][lane];
      int tf = 0;
      bool first = true;
      for (int j = 0; j < cnt; ++j) {
        const bool eq = s_key[n][j] == key;
        tf += eq;
        first = first && !(eq && j < lane);
      }
      if (first) {
        const float df = df_lookup(ht_keys, ht_vals, ht_cap, key);
        v = (float)tf * (log_ref_len - __logf(fmaxf(1.f, df)));
      }
    }
    s_val[n][lane] = v;
    const float nrm = sqrtf(wave_sum(v * v));
    if (lane == 0) s_norm[n] = nrm;
  }
  __syncthreads();
  const float len_h = (float)max(W - 1, 0);
  float norm_h[4] = {s_norm[0], s_norm[1], s_norm[2], s_norm[3]};

  // -- 4. references, split over the 4 waves --------------------------------------
  const int v = (int)hyp_video[hyp];
  const int r0 = vid_ref_off[v], r1 = vid_ref_off[v + 1];
  float total = 0.f;
  for (int r = r0 + w; r < r1; r += 4) {
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
    const int g0 = ref_ng_off[r], g1 = ref_ng_off[r + 1];
    for (int g = g0 + lane; g < g1; g += 64) {
      const uint64_t key = (uint64_t)ng_key[g];
      const float vr = ng_val[g];
      const int n = ngram_order(key) - 1;
      const int cnt = W - n;
      float c = 0.f;
      for (int j = 0; j < cnt; ++j) {
        if (s_key[n][j] == key) c += fminf(s_val[n][j], vr) * vr;
      }
      acc0 += n == 0 ? c : 0.f;
      acc1 += n == 1 ? c : 0.f;
      acc2 += n == 2 ? c : 0.f;
      acc3 += n == 3 ? c : 0.f;
    }
    const float acc[4] = {wave_sum(acc0), wave_sum(acc1), wave_sum(acc2), wave_sum(acc3)};
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
  if (lane == 0) s_part[w] = total;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nref = r1 - r0;
    const float t4 = (s_part[0] + s_part[1]) + (s_part[2] + s_part[3]);
    out[hyp] = nref > 0 ? 10.f * t4 / (4.f * (float)nref) : 0.f;
  }
}

void launch_cider_d(const int64_t* hyps, int T, const int64_t* hyp_video, int N,
                    const int64_t* ht_keys, const float* ht_vals, uint32_t ht_cap,
                    const int32_t* vid_ref_off, const int32_t* ref_ng_off,
                    const float* ref_norm, const int32_t* ref_len, const int64_t* ng_key,
                    const float* ng_val, float log_ref_len, int use_eos, float* out,
                    hipStream_t stream) {
  if (N <= 0) return;
  dim3 grid(N), block(256);
  hipLaunchKernelGGL(cider_d_kernel, grid, block, 0, stream, hyps, T, hyp_video, N, ht_keys,
                     ht_vals, ht_cap, vid_ref_off, ref_ng_off, ref_norm, ref_len, ng_key,
                     ng_val, log_ref_len, use_eos, out);
  post_launch("cider_d_kernel", stream);
}

}  // namespace cst
