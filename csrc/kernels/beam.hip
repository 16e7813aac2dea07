// K10: batched beam search step on the GPU.
//
// Reference (/root/reference/model.py:369-512): one video at a time; each
// step moves the K x V log-probs to the host, sorts every beam's row
// (torch.sort on the CPU), builds Python candidate dicts, re-forks the beams by
// copying histories and LSTM state, and harvests finished beams into lists.
//
// Here all B videos advance together and nothing leaves the GPU:
//   * the vocab projection runs through the fused vocab kernel (fp32 logits +
//     per-row LSE), then beam_topk_kernel takes each beam row's K best
//     log-probs (one wavefront per row, register top-K per lane + K rounds of
//     wave arg-max);
//   * beam_step_kernel (one wavefront per video) applies the reference's
//     selection rules exactly: at t = 1 only beam 0 expands; candidates are
//     ordered word-rank-major (for c: for q) and stably sorted by cumulative
//     log-prob; the K best fork their parent's history; a beam that emitted
//     EOS (0) -- or any beam at the last step -- is harvested, and the
//     harvested beam with the lowest perplexity exp(-sum / (t - 1)) (10000 at
//     t = 1) wins, earliest on ties.  Beams keep expanding after EOS, as in
//     the reference;
//   * the LSTM state is not copied: the next step's LSTM kernel reads h/c of
//     row `parent[r]` (row_map).
#include "../common.h"
#include "../launchers.h"
#include "vocab_common.h"

namespace cst {

constexpr int BEAM_MAXK = 16;

// top-K (value, index) of logit - lse for each of R rows; ties -> smaller
// index.  One 256-thread block per row: each thread keeps a sorted register
// list of its strided entries (a value not above the list's K-th is rejected
// with one compare, so after the first few entries almost nothing is
// inserted), each wave takes K rounds of wave arg-max over its lanes' list
// heads, and wave 0 merges the 4 waves' K candidates the same way.
__device__ __forceinline__ void wave_argmax(float& best, int& besti) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(besti, o, 64);
    if (ov > best || (ov == best && oi < besti)) best = ov, besti = oi;
  }
}

__global__ __launch_bounds__(256) void beam_topk_kernel(const float* __restrict__ logits,
                                                        int64_t ldl, int V, int R, int K,
                                                        const float* __restrict__ lse,
                                                        float* __restrict__ top_v,
                                                        int* __restrict__ top_i) {
  __shared__ float s_v[4 * BEAM_MAXK];
  __shared__ int s_i[4 * BEAM_MAXK];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = blockIdx.x;
  const float* x = logits + (int64_t)r * ldl;
  // lane-local sorted top-K by an unrolled insertion pass (static register
  // indices only; strict > keeps the earlier, smaller index on ties)
  float bv[BEAM_MAXK];
  int bi[BEAM_MAXK];
#pragma unroll
  for (int k = 0; k < BEAM_MAXK; ++k) bv[k] = -INFINITY, bi[k] = 0x7fffffff;
  float thr = -INFINITY;  // the list's K-th value
  // TK_U independent loads in flight per chunk, then the (mostly rejecting)
  // insertions: one load at a time left the scan latency-bound (~50 us)
  constexpr int TK_U = 8;
  for (int v0 = threadIdx.x; v0 < V; v0 += 256 * TK_U) {
    float xs[TK_U];
#pragma unroll
    for (int u = 0; u < TK_U; ++u) {
      const int v = v0 + 256 * u;
      xs[u] = v < V ? x[v] : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < TK_U; ++u) {
      float cv = xs[u];
      if (!(cv > thr)) continue;
      int ci = v0 + 256 * u;
#pragma unroll
      for (int p = 0; p < BEAM_MAXK; ++p) {
        if (p < K && cv > bv[p]) {
          const float tv = bv[p];
          const int ti = bi[p];
          bv[p] = cv, bi[p] = ci;
          cv = tv, ci = ti;
        }
      }
#pragma unroll
      for (int p = 0; p < BEAM_MAXK; ++p) thr = p == K - 1 ? bv[p] : thr;
    }
  }
  // K rounds of wave arg-max over the lanes' list heads; the winner shifts
  for (int k = 0; k < K; ++k) {
    float best = bv[0];
    int besti = bi[0];
    wave_argmax(best, besti);
    if (bi[0] == besti) {
#pragma unroll
      for (int p = 0; p + 1 < BEAM_MAXK; ++p) bv[p] = bv[p + 1], bi[p] = bi[p + 1];
      bv[BEAM_MAXK - 1] = -INFINITY, bi[BEAM_MAXK - 1] = 0x7fffffff;
    }
    if (lane == 0) s_v[w * BEAM_MAXK + k] = best, s_i[w * BEAM_MAXK + k] = besti;
  }
  __syncthreads();
  if (w != 0) return;
  // the 4 waves' sorted candidate lists: lane l < 4K holds candidate l
  const int ww = lane / BEAM_MAXK, kk = lane % BEAM_MAXK;
  const bool have = lane < 4 * BEAM_MAXK && kk < K;
  float cv = have ? s_v[ww * BEAM_MAXK + kk] : -INFINITY;
  int ci = have ? s_i[ww * BEAM_MAXK + kk] : 0x7fffffff;
  const float L = lse[r];
  for (int k = 0; k < K; ++k) {
    float best = cv;
    int besti = ci;
    wave_argmax(best, besti);
    if (ci == besti && cv == best) cv = -INFINITY, ci = 0x7fffffff;
    if (lane == 0) {
      top_v[(int64_t)r * K + k] = best - L;
      top_i[(int64_t)r * K + k] = besti;
    }
  }
}

// The same top-K from the vocab launch's per-tile candidates (VF_TOPK:
// n_vt x K (logit, index) per row, each tile's list sorted): one wavefront per
// row merges n_vt * K candidates instead of scanning V fp32 logits.
__global__ __launch_bounds__(256) void beam_topk_cand_kernel(const float2* __restrict__ cand,
                                                             int n_vt, int R, int K,
                                                             const float* __restrict__ lse,
                                                             float* __restrict__ top_v,
                                                             int* __restrict__ top_i) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  constexpr int MK = 8;  // (VF_TOPK_MAXK)
  float bv[MK];
  int bi[MK];
#pragma unroll
  for (int k = 0; k < MK; ++k) bv[k] = -INFINITY, bi[k] = 0x7fffffff;
  const int n = n_vt * K;
  float thr = -INFINITY;
  for (int c0 = lane; c0 < n; c0 += 64 * 4) {
    float2 xs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + 64 * u;
      // candidate c = (tile c / K, rank c % K) of row r
      xs[u] = c < n ? cand[((int64_t)(c / K) * R + r) * K + c % K]
                    : make_float2(-INFINITY, __int_as_float(0x7fffffff));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float cv = xs[u].x;
      int ci = __float_as_int(xs[u].y);
      if (!(cv > thr || (cv == thr && ci < 0x7fffffff))) continue;
#pragma unroll
      for (int p = 0; p < MK; ++p) {
        if (p < K && (cv > bv[p] || (cv == bv[p] && ci < bi[p]))) {
          const float tv = bv[p];
          const int tix = bi[p];
          bv[p] = cv, bi[p] = ci;
          cv = tv, ci = tix;
        }
      }
#pragma unroll
      for (int p = 0; p < MK; ++p) thr = p == K - 1 ? bv[p] : thr;
    }
  }
  const float L = lse[r];
  for (int k = 0; k < K; ++k) {
    float best = bv[0];
    int besti = bi[0];
    wave_argmax(best, besti);
    if (bi[0] == besti) {
#pragma unroll
      for (int p = 0; p + 1 < MK; ++p) bv[p] = bv[p + 1], bi[p] = bi[p + 1];
      bv[MK - 1] = -INFINITY, bi[MK - 1] = 0x7fffffff;
    }
    if (lane == 0) {
      top_v[(int64_t)r * K + k] = best - L;
      top_i[(int64_t)r * K + k] = besti;
    }
  }
}

void launch_beam_topk_cand(const void* cand, int n_vt, int R, int K, const float* lse,
                           float* top_v, int* top_i, hipStream_t stream) {
  if (K < 1 || K > 8) throw std::runtime_error("beam_topk_cand: K must be in [1, 8]");
  hipLaunchKernelGGL(beam_topk_cand_kernel, dim3((R + 3) / 4), dim3(256), 0, stream,
                     (const float2*)cand, n_vt, R, K, lse, top_v, top_i);
  post_launch("beam_topk_cand_kernel", stream);
}

// One wavefront per video.  State (per video b, beam q):
//   beam_sum[b*K+q], seq/lp histories [2][B*K][T] (double-buffered by step
//   parity), best_ppl[b], best_seq[b][T], best_lp[b][T].
// Writes tok[b*K+v] (next input token) and parent[b*K+v] (row whose h/c the
// new beam continues).
__global__ __launch_bounds__(64) void beam_step_kernel(
    const float* __restrict__ top_v, const int* __restrict__ top_i, int B, int K, int T, int t,
    float* __restrict__ beam_sum, int64_t* __restrict__ seq_hist, float* __restrict__ lp_hist,
    float* __restrict__ best_ppl, int64_t* __restrict__ best_seq, float* __restrict__ best_lp,
    int64_t* __restrict__ tok_out, int* __restrict__ parent_out) {
  __shared__ float s_p[BEAM_MAXK * BEAM_MAXK];
  __shared__ int s_sel[BEAM_MAXK];
  __shared__ float s_sum_old[BEAM_MAXK];
  const int b = blockIdx.x, lane = threadIdx.x;
  const int rows = t == 1 ? 1 : K;
  const int ncand = rows * K;
  if (lane < K) s_sum_old[lane] = beam_sum[b * K + lane];
  __syncthreads();
  // candidate j = c * rows + q  (word rank c of beam q): the reference order
  for (int j = lane; j < ncand; j += 64) {
    const int c = j / rows, q = j % rows;
    s_p[j] = s_sum_old[q] + top_v[(int64_t)(b * K + q) * K + c];
  }
  __syncthreads();
  // stable selection of the K best: K rounds of (max p, then smallest j)
  for (int v = 0; v < K; ++v) {
    float best = -INFINITY;
    int bj = 0x7fffffff;
    for (int j = lane; j < ncand; j += 64) {
      bool taken = false;
      for (int u = 0; u < v; ++u) taken |= (s_sel[u] == j);
      const float p = s_p[j];
      if (!taken && (p > best || (p == best && j < bj))) best = p, bj = j;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oj = __shfl_xor(bj, o, 64);
      if (ov > best || (ov == best && oj < bj)) best = ov, bj = oj;
    }
    if (lane == 0) s_sel[v] = bj;
    __syncthreads();
  }
  // fork: new beam v continues parent q with word rank c
  const int64_t* sh_old = seq_hist + (int64_t)((t + 1) & 1) * B * K * T;
  const float* lh_old = lp_hist + (int64_t)((t + 1) & 1) * B * K * T;
  int64_t* sh_new = seq_hist + (int64_t)(t & 1) * B * K * T;
  float* lh_new = lp_hist + (int64_t)(t & 1) * B * K * T;
  for (int e = lane; e < K * T; e += 64) {
    const int v = e / T, pos = e % T;
    const int j = s_sel[v], c = j / rows, q = j % rows;
    const int64_t src = (int64_t)(b * K + q) * T + pos, dst = (int64_t)(b * K + v) * T + pos;
    if (pos < t - 1) {
      sh_new[dst] = sh_old[src];
      lh_new[dst] = lh_old[src];
    } else if (pos == t - 1) {
      sh_new[dst] = top_i[(int64_t)(b * K + q) * K + c];
      lh_new[dst] = top_v[(int64_t)(b * K + q) * K + c];
    } else {
      sh_new[dst] = 0;
      lh_new[dst] = 0.f;
    }
  }
  __syncthreads();
  if (lane < K) {
    const int v = lane, j = s_sel[v], c = j / rows, q = j % rows;
    beam_sum[b * K + v] = s_p[j];
    tok_out[b * K + v] = top_i[(int64_t)(b * K + q) * K + c];
    parent_out[b * K + v] = b * K + q;
  }
  // harvest, in beam order (earliest wins ties): lane 0 picks the winning
  // beam, then the lanes copy its history in parallel (this block wrote it
  // above; the barrier orders the copy after those stores)
  __shared__ int s_win;
  if (lane == 0) {
    int win = -1;
    float bp = best_ppl[b];
    for (int v = 0; v < K; ++v) {
      const int j = s_sel[v], c = j / rows, q = j % rows;
      const int w = top_i[(int64_t)(b * K + q) * K + c];
      if (w == 0 || t == T - 2) {
        const float ppl = t > 1 ? __expf(-s_p[j] / (float)(t - 1)) : 10000.f;
        if (ppl < bp) bp = ppl, win = v;
      }
    }
    if (win >= 0) best_ppl[b] = bp;
    s_win = win;
  }
  __syncthreads();
  const int win = s_win;
  if (win >= 0)
    for (int pos = lane; pos < T; pos += 64) {
      best_seq[(int64_t)b * T + pos] = sh_new[(int64_t)(b * K + win) * T + pos];
      best_lp[(int64_t)b * T + pos] = lh_new[(int64_t)(b * K + win) * T + pos];
    }
}

// Fused beam step (one 512-thread workgroup per video, beam size K <= 8),
// replacing combine + candidate top-K + beam step + LSTM step (4 launches):
//   0. prefetch of everything that does not depend on this step's selection:
//      the cell operands of the video's K current rows for this thread's
//      hidden units (pre = h_t W_hh^T + video gates, computed by the
//      recurrent tiles of the vocab launch; c_t) and the K history rows (LDS);
//   A. wavefront q < K, row q of the video: its candidate and partial loads
//      are issued together (one round trip), then the LSE from the vocab
//      launch's tile partials and the row's K best log-probs from its
//      n_vt x K tile candidates (VF_TOPK), into LDS;
//   B. the reference's selection / fork / harvest (beam_step_kernel's rules),
//      the new history rows written from LDS;
//   C. the next step's LSTM cell for the K new beams: gates = pre[parent] +
//      P[token] (the only gather left after the selection), c from the
//      parent's c -> h (bf16), c; the parent's operands are picked from the
//      prefetched registers by unrolled selects (no dynamic register index).
// Per decode step: this launch + the vocab launch (which also carries the
// next step's recurrent GEMM).  (The 256-thread form with per-phase loads --
// two rows per wavefront, two candidate batches, cell operands loaded after
// the selection -- was ~10 dependent memory round trips per step: 30.4 us,
// profiles/r5/steps_head_beam.txt.)
constexpr int BF_THREADS = 512, BF_MAXK = 8, BF_MAXC = 12, BF_MAXP = 2, BF_MAXT = 64;
template <int UPT, int KP>
__global__ __launch_bounds__(BF_THREADS) void beam_fused_step_kernel(BeamFusedArgs a, int t) {
  __shared__ float s_tv[BF_MAXK * BF_MAXK];
  __shared__ int s_ti[BF_MAXK * BF_MAXK];
  __shared__ float s_p[BF_MAXK * BF_MAXK];
  __shared__ int s_sel[BF_MAXK];
  __shared__ float s_sum_old[BF_MAXK];
  __shared__ int s_win;
  __shared__ int64_t s_sh[BF_MAXK * BF_MAXT];
  __shared__ float s_lh[BF_MAXK * BF_MAXT];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int K = a.K, R = a.R, T = a.T, n_vt = a.n_vt, H = a.H;
  const int rows = t == 1 ? 1 : K;
  // -- 0. prefetch ------------------------------------------------------------------
  const bool cell = a.pre != nullptr;
  float4 ppre[KP][UPT];
  float pc[KP][UPT];
  const bool att = a.vg16 != nullptr;
  if (cell) {
#pragma unroll
    for (int q = 0; q < KP; ++q)
#pragma unroll
      for (int j = 0; j < UPT; ++j) {
        const int u = min(tid + BF_THREADS * j, H - 1);
        const int64_t r = (int64_t)b * K + min(q, K - 1);
        ppre[q][j] = *reinterpret_cast<const float4*>(a.pre + r * 4 * H + 4 * u);
        pc[q][j] = a.c_in[r * H + u];
      }
    if (att) {  // (uniform) the rows' video gates (temporal attention), added to pre
      uint2 pv[KP][UPT];
#pragma unroll
      for (int q = 0; q < KP; ++q)
#pragma unroll
        for (int j = 0; j < UPT; ++j) {
          const int u = min(tid + BF_THREADS * j, H - 1);
          const int64_t r = (int64_t)b * K + min(q, K - 1);
          pv[q][j] = *reinterpret_cast<const uint2*>(a.vg16 + r * 4 * H + 4 * u);
        }
#pragma unroll
      for (int q = 0; q < KP; ++q)
#pragma unroll
        for (int j = 0; j < UPT; ++j) {
          ppre[q][j].x += bf2f(pv[q][j].x & 0xffff);
          ppre[q][j].y += bf2f(pv[q][j].x >> 16);
          ppre[q][j].z += bf2f(pv[q][j].y & 0xffff);
          ppre[q][j].w += bf2f(pv[q][j].y >> 16);
        }
    }
  }
  // the beams' running sums and the video's best perplexity (read after the
  // selection; loaded now)
  const float sum_old = a.beam_sum[b * K + min(tid, K - 1)];
  const float ppl_old = a.best_ppl[b];
  const int64_t* sh_old = a.seq_hist + (int64_t)((t + 1) & 1) * R * T;
  const float* lh_old = a.lp_hist + (int64_t)((t + 1) & 1) * R * T;
  for (int e = tid; e < K * T; e += BF_THREADS) {
    s_sh[e] = sh_old[(int64_t)b * K * T + e];
    s_lh[e] = lh_old[(int64_t)b * K * T + e];
  }
  // -- A. per-row LSE and top-K, one wavefront per row -------------------------------
  if (w < K) {
    const int r = b * K + w, n = n_vt * K;
    float2 xs[BF_MAXC];
#pragma unroll
    for (int i = 0; i < BF_MAXC; ++i) {  // (clamped, masked below)
      const int c = min(lane + 64 * i, n - 1);
      xs[i] = a.cand[((int64_t)(c / K) * R + r) * K + c % K];
    }
    float2 pp[BF_MAXP];
#pragma unroll
    for (int i = 0; i < BF_MAXP; ++i)
      pp[i] = *reinterpret_cast<const float2*>(a.part + (int64_t)min(lane + 64 * i, n_vt - 1) * R + r);
    float m = -INFINITY, sm = 0.f;
#pragma unroll
    for (int i = 0; i < BF_MAXP; ++i) {
      if (lane + 64 * i < n_vt) {
        const float pm = pp[i].x, ps = pp[i].y;
        const float M = fmaxf(m, pm);
        sm = (m == -INFINITY ? 0.f : sm * __expf(m - M)) + (pm == -INFINITY ? 0.f : ps * __expf(pm - M));
        m = M;
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(sm, o, 64);
      const float M = fmaxf(m, m2);
      sm = (m == -INFINITY ? 0.f : sm * __expf(m - M)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - M));
      m = M;
    }
    const float L = m + __logf(sm);
    float bv[BF_MAXK];
    int bi[BF_MAXK];
#pragma unroll
    for (int k = 0; k < BF_MAXK; ++k) bv[k] = -INFINITY, bi[k] = 0x7fffffff;
    float thr = -INFINITY;
#pragma unroll
    for (int i = 0; i < BF_MAXC; ++i) {
      const bool ok = lane + 64 * i < n;
      float cv = ok ? xs[i].x : -INFINITY;
      int ci = ok ? __float_as_int(xs[i].y) : 0x7fffffff;
      if (!(cv > thr || (cv == thr && ci < 0x7fffffff))) continue;
#pragma unroll
      for (int p = 0; p < BF_MAXK; ++p) {
        if (p < K && (cv > bv[p] || (cv == bv[p] && ci < bi[p]))) {
          const float tv = bv[p];
          const int tix = bi[p];
          bv[p] = cv, bi[p] = ci;
          cv = tv, ci = tix;
        }
      }
#pragma unroll
      for (int p = 0; p < BF_MAXK; ++p) thr = p == K - 1 ? bv[p] : thr;
    }
    for (int k = 0; k < K; ++k) {
      float best = bv[0];
      int besti = bi[0];
      wave_argmax(best, besti);
      if (bi[0] == besti) {
#pragma unroll
        for (int p = 0; p + 1 < BF_MAXK; ++p) bv[p] = bv[p + 1], bi[p] = bi[p + 1];
        bv[BF_MAXK - 1] = -INFINITY, bi[BF_MAXK - 1] = 0x7fffffff;
      }
      if (lane == 0) s_tv[w * K + k] = best - L, s_ti[w * K + k] = besti;
    }
  }
  if (tid < K) s_sum_old[tid] = sum_old;
  __syncthreads();
  // the token-table rows of every candidate (K rows x K tokens, known now)
  // for this thread's units, requested before the selection: after it only
  // register selects remain
  // (register budget: only for K <= 5 beams at H <= 512; else gathered after
  // the selection)
  // (measured slower: 25 candidate rows per thread -- 5x the gathered bytes
  // -- cost more than the round trip they save: 1.428 vs 1.172 ms per beam-5
  // decode of 64 videos)
  constexpr bool PFC = false;
  float4 xc[PFC ? KP * KP : 1][UPT];
  if (PFC && cell) {
#pragma unroll
    for (int e = 0; e < KP * KP; ++e) {
      const int q = min(e / KP, K - 1), c = min(e % KP, K - 1);
      const int64_t tk = s_ti[q * K + c];
#pragma unroll
      for (int jj = 0; jj < UPT; ++jj) {
        const int u = min(tid + BF_THREADS * jj, H - 1);
        xc[e][jj] = ld_h4(a.ptab + tk * 4 * H + 4 * u);
      }
    }
  }
  // -- B. selection (beam_step_kernel's rules), every thread at the barriers ------
  const int ncand = rows * K;
  if (tid < ncand) {
    const int c = tid / rows, q = tid % rows;
    s_p[tid] = s_sum_old[q] + s_tv[q * K + c];
  }
  __syncthreads();
  // the K best candidates in one pass: candidate j's rank is the number of
  // candidates ahead of it (higher sum, or equal sum and lower index -- the
  // order of the reference's repeated pick-the-best rounds), and the first K
  // ranks are the selection in order (ncand <= 64: one wavefront, one barrier
  // instead of K rounds of an argmax and a barrier)
  if (tid < ncand) {
    const float p = s_p[tid];
    int rank = 0;
    for (int i = 0; i < ncand; ++i) {
      const float pi = s_p[i];
      rank += (pi > p || (pi == p && i < tid)) ? 1 : 0;
    }
    if (rank < K) s_sel[rank] = tid;
  }
  __syncthreads();
  int64_t* sh_new = a.seq_hist + (int64_t)(t & 1) * R * T;
  float* lh_new = a.lp_hist + (int64_t)(t & 1) * R * T;
  for (int e = tid; e < K * T; e += BF_THREADS) {
    const int v = e / T, pos = e % T;
    const int j = s_sel[v], c = j / rows, q = j % rows;
    const int64_t dst = (int64_t)(b * K + v) * T + pos;
    sh_new[dst] = pos < t - 1 ? s_sh[q * T + pos] : (pos == t - 1 ? (int64_t)s_ti[q * K + c] : 0);
    lh_new[dst] = pos < t - 1 ? s_lh[q * T + pos] : (pos == t - 1 ? s_tv[q * K + c] : 0.f);
  }
  if (tid < K) {
    const int v = tid, j = s_sel[v], c = j / rows, q = j % rows;
    a.beam_sum[b * K + v] = s_p[j];
    a.tok_out[b * K + v] = s_ti[q * K + c];
  }
  if (tid == 0) {  // harvest, in beam order (earliest wins ties)
    int win = -1;
    float bp = ppl_old;
    for (int v = 0; v < K; ++v) {
      const int j = s_sel[v], c = j / rows, q = j % rows;
      if (s_ti[q * K + c] == 0 || t == T - 2) {
        const float ppl = t > 1 ? __expf(-s_p[j] / (float)(t - 1)) : 10000.f;
        if (ppl < bp) bp = ppl, win = v;
      }
    }
    if (win >= 0) a.best_ppl[b] = bp;
    s_win = win;
  }
  __syncthreads();
  const int win = s_win;
  if (win >= 0) {  // the winner's new row, formed from LDS like the history rows
    const int j = s_sel[win], c = j / rows, q = j % rows;
    for (int pos = tid; pos < T; pos += BF_THREADS) {
      a.best_seq[(int64_t)b * T + pos] =
          pos < t - 1 ? s_sh[q * T + pos] : (pos == t - 1 ? (int64_t)s_ti[q * K + c] : 0);
      a.best_lp[(int64_t)b * T + pos] =
          pos < t - 1 ? s_lh[q * T + pos] : (pos == t - 1 ? s_tv[q * K + c] : 0.f);
    }
  }
  if (!cell) return;
  // -- C. the next step's cell for the K new beams ---------------------------------
  float4 xv[KP][UPT];
  int par[KP];
#pragma unroll
  for (int v = 0; v < KP; ++v) {  // the selected candidates' token-table rows
    const int vv = min(v, K - 1), j = s_sel[vv], c = j / rows, q = j % rows;
    par[v] = q;
    if constexpr (PFC) {  // prefetched: register selects
      const int e = q * KP + c;
#pragma unroll
      for (int jj = 0; jj < UPT; ++jj) {
        float4 x = xc[0][jj];
#pragma unroll
        for (int f = 1; f < KP * KP; ++f)
          if (e == f) x = xc[f][jj];
        xv[v][jj] = x;
      }
    } else {  // all gathers out at once
      const int64_t tk = s_ti[q * K + c];
#pragma unroll
      for (int jj = 0; jj < UPT; ++jj) {
        const int u = min(tid + BF_THREADS * jj, H - 1);
        xv[v][jj] = ld_h4(a.ptab + tk * 4 * H + 4 * u);
      }
    }
  }
#pragma unroll
  for (int v = 0; v < KP; ++v) {
    if (v < K) {
#pragma unroll
      for (int jj = 0; jj < UPT; ++jj) {
        const int u = tid + BF_THREADS * jj;
        if (u < H) {
          float4 pv = ppre[0][jj];
          float cv = pc[0][jj];
#pragma unroll
          for (int q = 1; q < KP; ++q)
            if (par[v] == q) pv = ppre[q][jj], cv = pc[q][jj];
          const CellFwd cf = cell_fwd(a.cell, pv.x + xv[v][jj].x, pv.y + xv[v][jj].y,
                                      pv.z + xv[v][jj].z, pv.w + xv[v][jj].w, cv);
          const int64_t o = (int64_t)(b * K + v) * H + u;
          a.c_out[o] = cf.c;
          a.h_out[o] = f2bf(cf.h);
        }
      }
    }
  }
}

void launch_beam_fused_step(const BeamFusedArgs& a, int t, hipStream_t stream) {
  if (a.K < 1 || a.K > BF_MAXK || a.T > BF_MAXT || a.n_vt > 64 * BF_MAXP ||
      a.n_vt * a.K > 64 * BF_MAXC || (a.pre != nullptr && a.H > 2 * BF_THREADS))
    throw std::runtime_error("beam_fused_step: K <= 8, T <= 64, n_vt <= 128, n_vt K <= 768, H <= 1024");
  // register budget: K <= 4 / 8 beams, H <= 512 / 1024 units per workgroup
  const bool one = a.pre == nullptr || a.H <= BF_THREADS;
  if (a.K <= 4 && one)
    hipLaunchKernelGGL((beam_fused_step_kernel<1, 4>), dim3(a.B), dim3(BF_THREADS), 0, stream, a, t);
  else if (a.K <= 5 && one)
    hipLaunchKernelGGL((beam_fused_step_kernel<1, 5>), dim3(a.B), dim3(BF_THREADS), 0, stream, a, t);
  else if (one)
    hipLaunchKernelGGL((beam_fused_step_kernel<1, 8>), dim3(a.B), dim3(BF_THREADS), 0, stream, a, t);
  else
    hipLaunchKernelGGL((beam_fused_step_kernel<2, 8>), dim3(a.B), dim3(BF_THREADS), 0, stream, a, t);
  post_launch("beam_fused_step_kernel", stream);
}

void launch_beam_topk(const float* logits, int64_t ldl, int V, int R, int K, const float* lse,
                      float* top_v, int* top_i, hipStream_t stream) {
  hipLaunchKernelGGL(beam_topk_kernel, dim3(R), dim3(256), 0, stream, logits, ldl, V, R, K, lse,
                     top_v, top_i);
  post_launch("beam_topk_kernel", stream);
}

void launch_beam_step(const float* top_v, const int* top_i, int B, int K, int T, int t,
                      float* beam_sum, int64_t* seq_hist, float* lp_hist, float* best_ppl,
                      int64_t* best_seq, float* best_lp, int64_t* tok_out, int* parent_out,
                      hipStream_t stream) {
  hipLaunchKernelGGL(beam_step_kernel, dim3(B), dim3(64), 0, stream, top_v, top_i, B, K, T, t,
                     beam_sum, seq_hist, lp_hist, best_ppl, best_seq, best_lp, tok_out,
                     parent_out);
  post_launch("beam_step_kernel", stream);
}

}  // namespace cst
