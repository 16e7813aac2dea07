// Embedding gradient: d_emb[tok] = sum of the dX rows whose input token is
// tok (reference: nn.Embedding backward, /root/reference/model.py:271).
//
// Rows are grouped by token with a counting sort over the vocabulary (token
// ids < V <= 65536): histogram -> one-block exclusive scan -> scatter, three
// small launches (a full-width radix sort of the int64 ids cost ~320 us per
// training step).  The scatter takes slots with atomics, so the order of rows
// inside a token's group varies between runs; token_rows_sum_kernel already
// merges groups that span blocks with fp32 atomics, so the embedding
// gradient's summation order was never run-to-run deterministic (as with
// PyTorch's own embedding backward on GPUs).
//
// PyTorch's index_add_ issues one fp32 atomic per element (rows x E).  Here
// rows arrive sorted by token; a block sums EG_ROWS consecutive sorted rows in
// registers and issues one atomic row per token change, so the atomic count
// drops to (#blocks + #distinct tokens) x E and a frequent token (EOS, "a")
// is split across blocks instead of serialised.  Thread t owns columns
// t + 256 j: every wave-instruction (load or atomic) covers 256 contiguous
// bytes, the full-rate access shape for both.
#include "../common.h"

namespace cst {

constexpr int EG_ROWS = 64, EG_GROUP = 8, EG_MAXJ = 4;  // <= 1024 columns per launch

__global__ __launch_bounds__(256) void token_rows_sum_kernel(
    const float* __restrict__ x, int C, int ld, const int* __restrict__ stok,
    const int* __restrict__ srow, int N, float* __restrict__ out) {
  __shared__ int s_tok[EG_ROWS];
  __shared__ int s_row[EG_ROWS];
  const int i0 = blockIdx.x * EG_ROWS;
  const int n = min(EG_ROWS, N - i0);
  if ((int)threadIdx.x < n) {
    s_tok[threadIdx.x] = stok[i0 + threadIdx.x];
    s_row[threadIdx.x] = srow[i0 + threadIdx.x];
    CST_DCHECK(s_tok[threadIdx.x] >= 0 && s_row[threadIdx.x] >= 0 && s_row[threadIdx.x] < N);
  }
  __syncthreads();
  const int nj = (C + 255) >> 8;
  const int tcol = threadIdx.x;
  float acc[EG_MAXJ];
#pragma unroll
  for (int j = 0; j < EG_MAXJ; ++j) acc[j] = 0.f;
  int cur = s_tok[0];
  for (int g = 0; g < n; g += EG_GROUP) {
    float v[EG_GROUP][EG_MAXJ];
#pragma unroll
    for (int k = 0; k < EG_GROUP; ++k)  // the group's loads are in flight together
#pragma unroll
      for (int j = 0; j < EG_MAXJ; ++j)
        v[k][j] = (g + k < n && j < nj && tcol + 256 * j < C)
                      ? x[(int64_t)s_row[g + k] * ld + tcol + 256 * j]
                      : 0.f;
#pragma unroll
    for (int k = 0; k < EG_GROUP; ++k) {
      if (g + k < n) {
        const int tk = s_tok[g + k];
        if (tk != cur) {
#pragma unroll
          for (int j = 0; j < EG_MAXJ; ++j)
            if (j < nj && tcol + 256 * j < C) {
              atomicAdd(out + (int64_t)cur * ld + tcol + 256 * j, acc[j]);
              acc[j] = 0.f;
            }
          cur = tk;
        }
#pragma unroll
        for (int j = 0; j < EG_MAXJ; ++j) acc[j] += v[k][j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < EG_MAXJ; ++j)
    if (j < nj && tcol + 256 * j < C) atomicAdd(out + (int64_t)cur * ld + tcol + 256 * j, acc[j]);
}

void launch_token_rows_sum(const float* x, int C, const int* stok, const int* srow, int N,
                           float* out, hipStream_t stream) {
  // column chunks of <= 1024 (an embedding wider than that, e.g. the
  // 'standard' model's E = F * H, takes several launches)
  for (int c0 = 0; c0 < C; c0 += EG_MAXJ * 256) {
    hipLaunchKernelGGL(token_rows_sum_kernel, dim3((N + EG_ROWS - 1) / EG_ROWS), dim3(256), 0,
                       stream, x + c0, min(C - c0, EG_MAXJ * 256), C, stok, srow, N, out + c0);
    post_launch("token_rows_sum_kernel", stream);
  }
}

// ---- counting sort of the input tokens ----------------------------------------
constexpr int TS_THREADS = 1024;

__global__ __launch_bounds__(256) void token_hist_kernel(const int64_t* __restrict__ toks, int N,
                                                         int V, int* __restrict__ count) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < N) {
    const int t = (int)toks[i];
    CST_DCHECK(t >= 0 && t < V);
    atomicAdd(count + min(max(t, 0), V - 1), 1);
  }
}

// one block: exclusive scan of count[0, V) into cursor[0, V) (V <= 65536);
// every thread scans a contiguous run, then the run totals are scanned in LDS
__global__ __launch_bounds__(TS_THREADS) void token_scan_kernel(const int* __restrict__ count,
                                                                int V, int* __restrict__ cursor) {
  __shared__ int s_tot[TS_THREADS];
  const int per = (V + TS_THREADS - 1) / TS_THREADS;
  const int b = threadIdx.x * per, e = min(b + per, V);
  int tot = 0;
  for (int v = b; v < e; ++v) tot += count[v];
  s_tot[threadIdx.x] = tot;
  __syncthreads();
  for (int o = 1; o < TS_THREADS; o <<= 1) {  // Hillis-Steele inclusive scan
    const int add = threadIdx.x >= o ? s_tot[threadIdx.x - o] : 0;
    __syncthreads();
    s_tot[threadIdx.x] += add;
    __syncthreads();
  }
  int run = s_tot[threadIdx.x] - tot;  // exclusive prefix of this run
  for (int v = b; v < e; ++v) {
    cursor[v] = run;
    run += count[v];
  }
}

__global__ __launch_bounds__(256) void token_scatter_kernel(const int64_t* __restrict__ toks,
                                                            int N, int V, int* __restrict__ cursor,
                                                            int* __restrict__ stok,
                                                            int* __restrict__ srow) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < N) {
    const int t = min(max((int)toks[i], 0), V - 1);
    const int pos = atomicAdd(cursor + t, 1);
    stok[pos] = t;
    srow[pos] = i;
  }
}

// ws: 2 * V ints (histogram, then cursors); histogram zeroed here
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
