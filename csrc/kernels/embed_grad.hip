// Embedding gradient: d_emb[tok] = sum of the dX rows whose input token is
// tok (reference: nn.Embedding backward, /root/reference/model.py:271).
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

constexpr int EG_ROWS = 64, EG_GROUP = 8, EG_MAXJ = 4;  // C <= 1024

__global__ __launch_bounds__(256) void token_rows_sum_kernel(
    const float* __restrict__ x, int C, const int64_t* __restrict__ stok,
    const int64_t* __restrict__ srow, int N, float* __restrict__ out) {
  __shared__ int s_tok[EG_ROWS];
  __shared__ int s_row[EG_ROWS];
  const int i0 = blockIdx.x * EG_ROWS;
  const int n = min(EG_ROWS, N - i0);
  if ((int)threadIdx.x < n) {
    s_tok[threadIdx.x] = (int)stok[i0 + threadIdx.x];
    s_row[threadIdx.x] = (int)srow[i0 + threadIdx.x];
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
                      ? x[(int64_t)s_row[g + k] * C + tcol + 256 * j]
                      : 0.f;
#pragma unroll
    for (int k = 0; k < EG_GROUP; ++k) {
      if (g + k < n) {
        const int tk = s_tok[g + k];
        if (tk != cur) {
#pragma unroll
          for (int j = 0; j < EG_MAXJ; ++j)
            if (j < nj && tcol + 256 * j < C) {
              atomicAdd(out + (int64_t)cur * C + tcol + 256 * j, acc[j]);
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
    if (j < nj && tcol + 256 * j < C) atomicAdd(out + (int64_t)cur * C + tcol + 256 * j, acc[j]);
}

void launch_token_rows_sum(const float* x, int C, const int64_t* stok, const int64_t* srow, int N,
                           float* out, hipStream_t stream) {
  hipLaunchKernelGGL(token_rows_sum_kernel, dim3((N + EG_ROWS - 1) / EG_ROWS), dim3(256), 0,
                     stream, x, C, stok, srow, N, out);
  post_launch("token_rows_sum_kernel", stream);
}

}  // namespace cst
