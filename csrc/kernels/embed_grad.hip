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
// One 256-thread block per GS_CHUNK consecutive sorted entries, thread t
// owning the 8-column chunks t + 256 j of every row (one 16-byte load per
// thread and row, GS_PF rows in flight); the chunk's token / row indices are
// staged in LDS.  A group that lies entirely in the chunk is stored directly
// as bf16; a group that spans chunks (its first or last entry outside) is
// added into the fp32 scratch S32 (zeroed by the caller) and flagged, and the
// finalize pass converts flagged rows and zero-fills tokens without rows.
// Atomics only at chunk boundaries, none per row.
constexpr int GS_CHUNK = 64, GS_MAXJ = 2, GS_PF = 4;  // C <= 8 * 256 * GS_MAXJ = 4096

__global__ __launch_bounds__(256) void token_group_sum_kernel(
    const uint16_t* __restrict__ x, int C, int64_t ld, const int* __restrict__ stok,
    const int* __restrict__ srow, int N, uint16_t* __restrict__ S, float* __restrict__ S32,
    int* __restrict__ flag) {
  __shared__ int s_tok[GS_CHUNK + 2];  // [0]: entry before the chunk, [n + 1]: after
  __shared__ int s_row[GS_CHUNK];
  const int c0 = blockIdx.x * GS_CHUNK;
  const int n = min(GS_CHUNK, N - c0);
  const int tid = threadIdx.x;
  if (tid < n) {
    s_tok[tid + 1] = stok[c0 + tid];
    s_row[tid] = srow[c0 + tid];
  }
  if (tid == 64) s_tok[0] = c0 > 0 ? stok[c0 - 1] : -1;
  if (tid == 65) s_tok[n + 1] = c0 + n < N ? stok[c0 + n] : -1;
  __syncthreads();
  const int nch = C >> 3;
  float acc[GS_MAXJ][8];
#pragma unroll
  for (int j = 0; j < GS_MAXJ; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[j][k] = 0.f;
  auto flush = [&](int v, bool inside) {
    if (inside) {  // whole group in this chunk: final value
#pragma unroll
      for (int j = 0; j < GS_MAXJ; ++j) {
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
    } else {  // spans chunks: partial sum into the fp32 scratch
#pragma unroll
      for (int j = 0; j < GS_MAXJ; ++j) {
        const int c = tid + 256 * j;
        if (c < nch)
#pragma unroll
          for (int k = 0; k < 8; ++k) atomicAdd(S32 + (int64_t)v * C + 8 * c + k, acc[j][k]);
      }
      if (tid == 0) flag[v] = 1;
    }
#pragma unroll
    for (int j = 0; j < GS_MAXJ; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[j][k] = 0.f;
  };
  auto load = [&](int i, uint4 (&r)[GS_MAXJ]) {
    const uint16_t* row = x + (int64_t)s_row[i] * ld;
#pragma unroll
    for (int j = 0; j < GS_MAXJ; ++j) {
      const int c = tid + 256 * j;
      r[j] = c < nch ? *reinterpret_cast<const uint4*>(row + 8 * c) : make_uint4(0, 0, 0, 0);
    }
  };
  uint4 buf[GS_PF][GS_MAXJ];
#pragma unroll
  for (int p = 0; p < GS_PF; ++p)
    if (p < n) load(p, buf[p]);
  int cur = s_tok[1];
  bool first = true;  // cur is the chunk's first group
  for (int i0 = 0; i0 < n; i0 += GS_PF) {
#pragma unroll
    for (int p = 0; p < GS_PF; ++p) {
      const int i = i0 + p;
      if (i < n) {
        const int tk = s_tok[i + 1];
        if (tk != cur) {
          flush(cur, !first || s_tok[0] != cur);
          cur = tk;
          first = false;
        }
#pragma unroll
        for (int j = 0; j < GS_MAXJ; ++j) {
          const uint32_t w[4] = {buf[p][j].x, buf[p][j].y, buf[p][j].z, buf[p][j].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            acc[j][2 * k] += bf2f(w[k] & 0xffff);
            acc[j][2 * k + 1] += bf2f(w[k] >> 16);
          }
        }
        if (i + GS_PF < n) load(i + GS_PF, buf[p]);
      }
    }
  }
  flush(cur, (!first || s_tok[0] != cur) && s_tok[n + 1] != cur);
}

// one wavefront per token: zero rows of tokens without entries, convert the
// flagged (chunk-spanning) rows from the fp32 scratch
__global__ __launch_bounds__(256) void token_group_finalize_kernel(
    int V, int C, const int* __restrict__ count, const int* __restrict__ flag,
    const float* __restrict__ S32, uint16_t* __restrict__ S) {
  const int v = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (v >= V) return;
  const bool empty = count[v] == 0;
  if (!empty && flag[v] == 0) return;
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

void launch_token_group_sum(const uint16_t* x, int C, int64_t ld, const int* stok,
                            const int* srow, int N, const int* ws, int V, uint16_t* S, float* S32,
                            int* flag, hipStream_t stream) {
  if (C % 8 != 0 || C > 256 * 8 * GS_MAXJ || ld % 8 != 0)
    throw std::runtime_error("token_group_sum: C and ld multiples of 8, C <= 4096");
  hipLaunchKernelGGL(token_group_sum_kernel, dim3((N + GS_CHUNK - 1) / GS_CHUNK), dim3(256), 0,
                     stream, x, C, ld, stok, srow, N, S, S32, flag);
  post_launch("token_group_sum_kernel", stream);
  hipLaunchKernelGGL(token_group_finalize_kernel, dim3((V + 3) / 4), dim3(256), 0, stream, V, C,
                     ws, flag, S32, S);
  post_launch("token_group_finalize_kernel", stream);
}

// ---- counting sort of the input tokens ----------------------------------------
constexpr int TS_THREADS = 1024;

__global__ __launch_bounds__(256) void token_hist_kernel(const int64_t* __restrict__ toks, int N,
                                                         int V, int* __restrict__ count) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < N) {
    const int64_t t = toks[i];
    if (t >= 0 && t < V) atomicAdd(count + t, 1);  // ids outside [0, V): no entry
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
  if (i < N) {
    const int64_t t = toks[i];
    if (t >= 0 && t < V) {
      const int pos = atomicAdd(cursor + t, 1);
      stok[pos] = (int)t;
      srow[pos] = i;
    }
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

}  // namespace cst
