// Input-token gradients (reference: nn.Embedding backward and the input half
// of the LSTM weight gradient, /root/reference/model.py:271-278): rows grouped
// by input token with a counting sort over the vocabulary (token ids < V <=
// 65536): histogram -> one-block exclusive scan -> scatter, three small
// launches (a full-width radix sort of the int64 ids cost ~320 us per training
// step), then per-token sums of the gate-gradient rows (token_group_sum).
// The scatter takes slots with atomics, so the order of rows inside a token's
// group varies between runs (summation order, as with PyTorch's own embedding
// backward on GPUs).
#include "../common.h"

namespace cst {

// ---- per-token sums of bf16 rows (input-token gradients) ----------------------
// S[v] = sum of the rows x[srow[i]] (first C columns, row stride ld) whose
// sorted token stok[i] is v, as bf16 (V x C).  The embedding gradient is then
// S W_ie and the input-weight gradient S^T emb: GEMMs over V rows instead of
// the n*R rollout rows (3.4x fewer rows at V = 10.5k, R = 1280, 28 steps).
//
// Ownership instead of scratch: block b walks the sorted entries from the
// start of the first group that begins in its chunk [GS_CHUNK b, GS_CHUNK (b +
// 1)) to the END of the last such group, even past the chunk, so every group
// of at most GS_LONG entries is summed by exactly one block, in a fixed order,
// and stored once as bf16 (no atomics, no fp32 scratch).  Only
// long groups (more than GS_LONG entries: the BOS token of step 0 has R of
// them) are split at chunk boundaries; each chunk adds its part into the fp32
// row S32[v] (zeroed by token_long_zero right after the sort, off the
// critical path) and the finalize pass converts those rows and zero-fills the
// tokens without entries.  (The former design zeroed a V x C fp32 scratch and
// a flag array every step -- 86 MB -- and sent every chunk-spanning group
// through atomics.)
// Thread t owns the 8-column chunks t + 256 j of every row (one 16-byte load
// per thread and row, GS_PF rows in flight); the block's entry indices are
// staged in LDS.
constexpr int GS_CHUNK = 64, GS_LONG = 192, GS_PF = 8;
constexpr int GS_SPAN = GS_CHUNK + GS_LONG;  // entries one block can own

template <int MAXJ>
__global__ __launch_bounds__(256) void token_group_sum_kernel(
    const uint16_t* __restrict__ x, int C, int64_t ld, const int* __restrict__ stok,
    const int* __restrict__ srow, const int* __restrict__ ws, int V, uint16_t* __restrict__ S,
    float* __restrict__ S32) {
  __shared__ int s_tok[GS_SPAN];
  __shared__ int s_row[GS_SPAN];
  const int* count = ws;
  const int* gend = ws + V;  // after the scatter: end of each token's group
  const int N = ws[2 * V];   // sorted entries
  const int c0 = blockIdx.x * GS_CHUNK;
  if (c0 >= N) return;
  const int c1 = min(c0 + GS_CHUNK, N);
  const int tid = threadIdx.x;
  // owned range [lo, hi)
  const int t0 = stok[c0], n0 = count[t0];
  const int lo = (gend[t0] - n0 == c0 || n0 > GS_LONG) ? c0 : gend[t0];
  const int tl = stok[c1 - 1], nl = count[tl];
  const int hi = nl > GS_LONG ? c1 : (gend[tl] - nl >= c0 ? gend[tl] : c1);
  const int n = hi - lo;
  if (n <= 0) return;  // the chunk lies inside a short group begun earlier
  CST_DCHECK(n <= GS_SPAN);
  // s_tok carries the long-group flag in bit 31 (so the flush branch reads no
  // global count: a vector load there would wait for every row load before it)
  for (int i = tid; i < n; i += 256) {
    const int t = stok[lo + i];
    s_tok[i] = t | (count[t] > GS_LONG ? (int)0x80000000u : 0);
    s_row[i] = srow[lo + i];
  }
  __syncthreads();
  const int nch = C >> 3;
  float acc[MAXJ][8];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[j][k] = 0.f;
  auto flush = [&](int tf) {
    const int v = tf & 0x7fffffff;
    if (tf >= 0) {  // whole group in this block: final value
#pragma unroll
      for (int j = 0; j < MAXJ; ++j) {
        const int c = tid + 256 * j;
        if (c < nch) {
          uint4 o;
          o.x = (uint32_t)f2bf(acc[j][0]) | ((uint32_t)f2bf(acc[j][1]) << 16);
          o.y = (uint32_t)f2bf(acc[j][2]) | ((uint32_t)f2bf(acc[j][3]) << 16);
          o.z = (uint32_t)f2bf(acc[j][4]) | ((uint32_t)f2bf(acc[j][5]) << 16);
          o.w = (uint32_t)f2bf(acc[j][6]) | ((uint32_t)f2bf(acc[j][7]) << 16);
          *reinterpret_cast<uint4*>(S + (int64_t)v * C + 8 * c) = o;
        }
      }
    } else {  // this chunk's part of a long group
      // (zero partials skip their atomics: the longest group of a teacher-
      // forced XE step is the padding token 0 after the captions end, ~25k
      // rows whose gate gradients are all zero -- 390 chunks x 2,048 atomics
      // on the same row serialised at the memory side)
#pragma unroll
      for (int j = 0; j < MAXJ; ++j) {
        const int c = tid + 256 * j;
        if (c < nch)
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (acc[j][k] != 0.f) atomicAdd(S32 + (int64_t)v * C + 8 * c + k, acc[j][k]);
      }
    }
#pragma unroll
    for (int j = 0; j < MAXJ; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[j][k] = 0.f;
  };
  // Double-buffered batches of GS_PF rows: the next batch's loads are issued
  // before the current batch is summed, every load unconditional (row index
  // clamped to the last owned entry, column chunk clamped to the last one,
  // surplus values masked at the add), and compiler barriers keep the loads
  // where they are.  (With conditional refills the compiler could not count
  // the loads issued after a buffer's and waited vmcnt(0) at every row, and it
  // sank the prefetches next to their uses: the loop was serialised on memory
  // latency, 365 us per step for a 147 MB pass.)
  auto load = [&](int i, uint4 (&r)[MAXJ]) {
    const uint16_t* row = x + (int64_t)s_row[min(i, n - 1)] * ld;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j)
      r[j] = *reinterpret_cast<const uint4*>(row + 8 * min(tid + 256 * j, nch - 1));
  };
  uint4 cb[GS_PF][MAXJ], nb[GS_PF][MAXJ];
#pragma unroll
  for (int p = 0; p < GS_PF; ++p) load(p, cb[p]);
  int cur = s_tok[0];
  for (int i0 = 0; i0 < n; i0 += GS_PF) {
    const bool more = i0 + GS_PF < n;
#pragma unroll
    for (int p = 0; p < GS_PF; ++p) load(i0 + GS_PF + p, nb[p]);  // clamped past n
    asm volatile("" ::: "memory");
#pragma unroll
    for (int p = 0; p < GS_PF; ++p) {
      const int i = i0 + p;
      if (i < n) {
        const int tk = s_tok[i];
        if (tk != cur) {
          flush(cur);
          cur = tk;
        }
#pragma unroll
        for (int j = 0; j < MAXJ; ++j) {
          const bool live = tid + 256 * j < nch;
          const uint32_t w[4] = {cb[p][j].x, cb[p][j].y, cb[p][j].z, cb[p][j].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            acc[j][2 * k] += live ? bf2f(w[k] & 0xffff) : 0.f;
            acc[j][2 * k + 1] += live ? bf2f(w[k] >> 16) : 0.f;
          }
        }
      }
    }
    asm volatile("" ::: "memory");
    if (!more) break;
#pragma unroll
    for (int p = 0; p < GS_PF; ++p)
#pragma unroll
      for (int j = 0; j < MAXJ; ++j) cb[p][j] = nb[p][j];
  }
  flush(cur);
}

// one wavefront per token: zero the fp32 rows of long groups (before the sums)
__global__ __launch_bounds__(256) void token_long_zero_kernel(int V, int C,
                                                              const int* __restrict__ count,
                                                              float* __restrict__ S32) {
  const int v = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (v >= V || count[v] <= GS_LONG) return;
  for (int c = lane; c < (C >> 2); c += 64)
    reinterpret_cast<float4*>(S32 + (int64_t)v * C)[c] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// one wavefront per token: zero rows of tokens without entries, convert the
// long groups' rows from the fp32 scratch
__global__ __launch_bounds__(256) void token_group_finalize_kernel(
    int V, int C, const int* __restrict__ count, const float* __restrict__ S32,
    uint16_t* __restrict__ S) {
  const int v = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (v >= V) return;
  const int cnt = count[v];
  if (cnt > 0 && cnt <= GS_LONG) return;
  const bool empty = cnt == 0;
  for (int c = lane; c < (C >> 3); c += 64) {
    uint4 o = make_uint4(0, 0, 0, 0);
    if (!empty) {
      const float4 a = reinterpret_cast<const float4*>(S32 + (int64_t)v * C + 8 * c)[0];
      const float4 b = reinterpret_cast<const float4*>(S32 + (int64_t)v * C + 8 * c)[1];
      o.x = (uint32_t)f2bf(a.x) | ((uint32_t)f2bf(a.y) << 16);
      o.y = (uint32_t)f2bf(a.z) | ((uint32_t)f2bf(a.w) << 16);
      o.z = (uint32_t)f2bf(b.x) | ((uint32_t)f2bf(b.y) << 16);
      o.w = (uint32_t)f2bf(b.z) | ((uint32_t)f2bf(b.w) << 16);
    }
    *reinterpret_cast<uint4*>(S + (int64_t)v * C + 8 * c) = o;
  }
}

void launch_token_long_zero(const int* ws, int V, int C, float* S32, hipStream_t stream) {
  if (C % 4 != 0) throw std::runtime_error("token_long_zero: C must be a multiple of 4");
  hipLaunchKernelGGL(token_long_zero_kernel, dim3((V + 3) / 4), dim3(256), 0, stream, V, C, ws,
                     S32);
  post_launch("token_long_zero_kernel", stream);
}

void launch_token_group_sum(const uint16_t* x, int C, int64_t ld, const int* stok,
                            const int* srow, int N, const int* ws, int V, uint16_t* S, float* S32,
                            hipStream_t stream) {
  if (C % 8 != 0 || C > 256 * 8 * 2 || ld % 8 != 0)
    throw std::runtime_error("token_group_sum: C and ld multiples of 8, C <= 4096");
  // grid over the N input entries (the sorted count ws[2V] <= N is read on
  // the device; chunks past it exit)
  const dim3 grid((N + GS_CHUNK - 1) / GS_CHUNK);
  if (C <= 256 * 8)
    hipLaunchKernelGGL(token_group_sum_kernel<1>, grid, dim3(256), 0, stream, x, C, ld, stok, srow,
                       ws, V, S, S32);
  else
    hipLaunchKernelGGL(token_group_sum_kernel<2>, grid, dim3(256), 0, stream, x, C, ld, stok, srow,
                       ws, V, S, S32);
  post_launch("token_group_sum_kernel", stream);
  hipLaunchKernelGGL(token_group_finalize_kernel, dim3((V + 3) / 4), dim3(256), 0, stream, V, C,
                     ws, S32, S);
  post_launch("token_group_finalize_kernel", stream);
}

// ---- counting sort of the input tokens ----------------------------------------
constexpr int TS_THREADS = 1024;

// Same-token lanes of a wave are aggregated before the atomics: the wave's
// most common repeats are the padding / end token 0 (teacher-forced XE rows
// after their caption ends: ~2/3 of the 37k entries) and the token of the
// wave's first lane (BOS at step 0: every row).  With one atomic per lane on
// one address those serialised at the memory side: 317 / 295 us for the
// histogram / scatter of an XE step, profiles/r6/steps_xe_before.txt.
struct TokAgg {
  int t;        // this lane's token (-1: none)
  uint64_t m;   // lanes sharing this lane's aggregated token (0: not aggregated)
  bool leader;  // the lowest lane of m
};
__device__ __forceinline__ TokAgg token_aggregate(int t) {
  const int lane = threadIdx.x & 63;
  const uint64_t m0 = __ballot(t == 0);
  const int tf = __shfl(t, __ffsll((unsigned long long)__ballot(t >= 0)) - 1, 64);
  const uint64_t mf = tf > 0 ? __ballot(t == tf) : 0ull;
  TokAgg a{t, 0ull, false};
  if (t == 0) a.m = m0;
  else if (t == tf && t > 0) a.m = mf;
  if (a.m != 0ull) a.leader = lane == __ffsll((unsigned long long)a.m) - 1;
  return a;
}

__global__ __launch_bounds__(256) void token_hist_kernel(const int64_t* __restrict__ toks, int N,
                                                         int V, int* __restrict__ count) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  int t = -1;
  if (i < N) {
    const int64_t x = toks[i];
    t = (x >= 0 && x < V) ? (int)x : -1;  // ids outside [0, V): no entry
  }
  const TokAgg a = token_aggregate(t);
  if (a.m != 0ull) {
    if (a.leader) atomicAdd(count + t, __popcll(a.m));
  } else if (t >= 0) {
    atomicAdd(count + t, 1);
  }
}

// one block: exclusive scan of count[0, V) into cursor[0, V) (V <= 65536).
// Chunks of 1024 consecutive counts (one coalesced load per thread), each
// scanned by wave shuffles + a 16-entry LDS scan of the wave totals, with the
// running total carried between chunks.  (A per-thread serial scan over
// contiguous runs made every load a separate cache line: 135-170 us per step
// next to the bandwidth-heavy backward, against a few us here.)
__global__ __launch_bounds__(TS_THREADS) void token_scan_kernel(const int* __restrict__ count,
                                                                int V, int* __restrict__ cursor) {
  constexpr int NW = TS_THREADS / WAVE;
  __shared__ int s_w[NW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int carry = 0;
  for (int base = 0; base < V; base += TS_THREADS) {
    const int v = base + (int)threadIdx.x;
    const int c = v < V ? count[v] : 0;
    int x = c;  // inclusive wave scan
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
      const int y = __shfl_up(x, o, WAVE);
      if (lane >= o) x += y;
    }
    if (lane == WAVE - 1) s_w[w] = x;
    __syncthreads();
    int before = 0, total = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int t = s_w[k];
      before += k < w ? t : 0;
      total += t;
    }
    if (v < V) cursor[v] = carry + before + x - c;
    carry += total;
    __syncthreads();  // s_w reused by the next chunk
  }
  if (threadIdx.x == 0) cursor[V] = carry;  // number of sorted entries
}

__global__ __launch_bounds__(256) void token_scatter_kernel(const int64_t* __restrict__ toks,
                                                            int N, int V, int* __restrict__ cursor,
                                                            int* __restrict__ stok,
                                                            int* __restrict__ srow) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  int t = -1;
  if (i < N) {
    const int64_t x = toks[i];
    t = (x >= 0 && x < V) ? (int)x : -1;
  }
  const TokAgg a = token_aggregate(t);
  const int lane = threadIdx.x & 63;
  int pos = -1;
  if (a.m != 0ull) {
    // one atomic per aggregated group; the lanes take consecutive slots
    int base = 0;
    if (a.leader) base = atomicAdd(cursor + t, __popcll(a.m));
    base = __shfl(base, __ffsll((unsigned long long)a.m) - 1, 64);
    pos = base + __popcll(a.m & ((1ull << lane) - 1ull));
  } else if (t >= 0) {
    pos = atomicAdd(cursor + t, 1);
  }
  if (pos >= 0) {
    stok[pos] = t;
    srow[pos] = i;
  }
}

// ws: 2 * V + 1 ints (histogram, then cursors, then the number of entries);
// ids outside [0, V) are left out (the sorted arrays hold ws[2V] entries)
void launch_token_sort(const int64_t* toks, int N, int V, int* ws, int* stok, int* srow,
                       hipStream_t stream) {
  if (V > 65536) throw std::runtime_error("token_sort: vocabulary larger than 65536");
  (void)hipMemsetAsync(ws, 0, sizeof(int) * (size_t)V, stream);
  const int nb = (N + 255) / 256;
  hipLaunchKernelGGL(token_hist_kernel, dim3(nb), dim3(256), 0, stream, toks, N, V, ws);
  post_launch("token_hist_kernel", stream);
  hipLaunchKernelGGL(token_scan_kernel, dim3(1), dim3(TS_THREADS), 0, stream, ws, V, ws + V);
  post_launch("token_scan_kernel", stream);
  hipLaunchKernelGGL(token_scatter_kernel, dim3(nb), dim3(256), 0, stream, toks, N, V, ws + V,
                     stok, srow);
  post_launch("token_scatter_kernel", stream);
}

// ---- video-gate gradient (mean-pooled features) -----------------------------
// d_vgate[b] = sum over steps t and the vdiv rows of video b of dG_t[row, 0:G4]
// (the per-video gate term W_iv . v enters every step's cell of every caption
// row of the video, lstm.hip).  One pass over the bf16 gate-gradient rows
// (n_steps x R x ld) straight into the (Bv, G4) fp32 result: the former
// dG.sum over time (fp32 R x G4 intermediate, 147 MB read) plus a second
// reduction over the rows of each video are one launch.  Block (video b,
// 256-column chunk): thread = 8 consecutive columns (one 16-byte load) of
// every 8th row of the video's n_steps * vdiv rows, RG_PF loads in flight;
// the 8 row partials are summed through LDS.
constexpr int RG_PF = 4;
__global__ __launch_bounds__(256) void video_gate_grad_kernel(const uint16_t* __restrict__ dG,
                                                              int64_t ld, int n_steps, int R,
                                                              int vdiv, int G4,
                                                              float* __restrict__ out) {
  __shared__ float s_part[8][256];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int cg = tid & 31, rs = tid >> 5;
  const int col = blockIdx.y * 256 + 8 * cg;
  const int colc = min(col, G4 - 8);  // (clamped: loads stay unconditional)
  const int nrows = n_steps * vdiv;
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  auto row_ptr = [&](int i) {
    const int t = i / vdiv, j = i - t * vdiv;
    return reinterpret_cast<const uint4*>(dG + ((int64_t)t * R + (int64_t)b * vdiv + j) * ld + colc);
  };
  for (int i0 = rs; i0 < nrows; i0 += 8 * RG_PF) {
    uint4 q[RG_PF];
#pragma unroll
    for (int k = 0; k < RG_PF; ++k) q[k] = *row_ptr(min(i0 + 8 * k, nrows - 1));
#pragma unroll
    for (int k = 0; k < RG_PF; ++k) {
      if (i0 + 8 * k < nrows) {
        const uint32_t w[4] = {q[k].x, q[k].y, q[k].z, q[k].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[2 * e] += bf2f(w[e] & 0xffff);
          acc[2 * e + 1] += bf2f(w[e] >> 16);
        }
      }
    }
  }
  // column chunk of 8 -> LDS row rs, then column tid sums the 8 row partials
#pragma unroll
  for (int k = 0; k < 8; ++k) s_part[rs][8 * cg + k] = acc[k];
  __syncthreads();
  const int c = blockIdx.y * 256 + tid;
  if (c < G4) {  // (chunks past G4 loaded clamped columns into LDS slots >= G4: unused)
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) v += s_part[r][tid];
    out[(int64_t)b * G4 + c] = v;
  }
}

void launch_video_gate_grad(const uint16_t* dG, int64_t ld, int n_steps, int R, int vdiv, int G4,
                            float* out, hipStream_t stream) {
  if (G4 % 8 != 0 || G4 < 8 || R % vdiv != 0 || ld % 8 != 0)
    throw std::runtime_error("video_gate_grad: unsupported shape");
  const dim3 grid(R / vdiv, (G4 + 255) / 256);
  hipLaunchKernelGGL(video_gate_grad_kernel, grid, dim3(256), 0, stream, dG, ld, n_steps, R, vdiv,
                     G4, out);
  post_launch("video_gate_grad_kernel", stream);
}

}  // namespace cst
