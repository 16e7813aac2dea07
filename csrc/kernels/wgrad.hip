// K13: weight-gradient GEMM for K-major operands on gfx950.
//
//   C[m][n] = sum_k A[k][m] * B[k][n]      (A: K x M rows, B: K x N rows, bf16)
//
// Every weight gradient of the decoder backward has this form: the rows are
// caption rows / steps (K), the columns are the weight's two dimensions
// (dW_hh = dG^T h_prev, dW_ie = S^T emb).  PyTorch's bmm runs them as
// transposed-A vendor GEMMs on a handful of output tiles (2048 x 512 outputs)
// with a 35k-long K (profiles/r5/README_r5.md "weight gradients").  Here:
//
// * both operands are staged in their natural row-major layout (one 256-byte
//   row of 128 columns per K row) by LDS-DMA (buffer_load ... lds), the
//   16-byte chunks XOR-swizzled on the SOURCE side (chunk ^ f(row),
//   f(row) = ((row & 3) << 2) | ((row >> 2) & 3): the CDNA HIP guide's T10
//   image (b)), so the copy stays lane-linear;
// * the MFMA operand fragments (lane l: column l & 31, 8 consecutive K rows
//   8 (l >> 5) ...) are read with ds_read_b64_tr_b16 -- the hardware transpose
//   read: a 16-lane group gets 4 rows x 16 columns delivered column-major --,
//   two per fragment, conflict-free on that image;
// * v_mfma_f32_32x32x16_bf16, 128 x 128 output tile per 256-thread block (4
//   waves of 64 x 64), BK = 64 K rows per stage, double-buffered with counted
//   vmcnt and one raw barrier per K-tile (gemm_tile.h's pipeline);
// * split-K over S slabs so the chip holds >= 2 blocks per CU: the partial
//   tiles go to an fp32 workspace and one reduce launch sums them in a fixed
//   order (deterministic, bit-identical run to run) into the output rows --
//   two row ranges with their own destinations and strides (the dW_hh / dW_q
//   split of [dG | dq]^T h_prev);
// * K need not be a multiple of 64: the buffer resource of each split ends at
//   row K, so the DMA returns zeros for the rows past it;
// * blocks are numbered split-major through the XCD remap, so the blocks of one
//   split (which share its A and B rows) sit on one XCD's L2.
#include "gemm_tile.h"
#include "../launchers.h"

namespace cst {

namespace {

constexpr int WG_BM = 128, WG_BN = 128, WG_BK = 64;
constexpr int WG_A_BYTES = WG_BK * WG_BM * 2, WG_STAGE = WG_A_BYTES + WG_BK * WG_BN * 2;
// fused column sums (CS): per stage the K tile's 64 weights (one 1 KB DMA
// instruction, the first 256 bytes used) behind the operand stages
constexpr int WG_AL_BYTES = 1024;
// LDS-DMA wave-instructions per operand per stage per wave: 64 rows x 256 B =
// 16 KiB = 16 instructions of 1 KiB (4 rows each), over 4 waves
constexpr int WG_NI = WG_BK * 256 / 1024 / 4;

__device__ __forceinline__ int tr_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

__device__ __forceinline__ int xcd_remap_w(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// one MFMA operand fragment: two transposed reads (K rows +0..3, +4..7)
__device__ __forceinline__ bf16x8 tr_frag(const char* base, int off0, int off1) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + off1));
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// CS: the block also sums al[k] A[k][m] over its K range for the 32 columns
// [m0 + 32 tn, m0 + 32 tn + 32) of its A tile (N = 512: the 4 column tiles of
// an m tile split its 128 columns), from the A stage already in LDS: thread
// (column c = tid & 31, K group kg = tid >> 5) adds 8 rows per K tile.
template <int STAGES, bool CS>
__global__ __launch_bounds__(256, 2) void wgrad_tn_kernel(WgradArgs g) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tiles_n = g.N / WG_BN, tiles = ((g.M + WG_BM - 1) / WG_BM) * tiles_n;
  const int b = xcd_remap_w((int)blockIdx.x, tiles * g.S);
  const int s = b / tiles, t = b - s * tiles;
  const int tm = t / tiles_n, tn = t - tm * tiles_n;
  const int m0 = tm * WG_BM, n0 = tn * WG_BN;
  const int nkt = (g.K + WG_BK - 1) / WG_BK;
  const int kt0 = s * g.kts;
  const int nk = min(g.kts, nkt - kt0);
  const int64_t kb = (int64_t)kt0 * WG_BK;
  // this split's rows [kb, K): the resource ends at row K (zeros past it)
  const rsrc_t ra = make_rsrc(g.A + kb * g.lda, (int64_t)(g.K - kb) * g.lda * 2);
  const rsrc_t rb = make_rsrc(g.B + kb * g.ldb, (int64_t)(g.K - kb) * g.ldb * 2);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wr = w >> 1, wc = w & 1;

  // LDS-DMA sources: instruction I = w + 4 i fills rows 4 I .. 4 I + 3; lane l
  // writes physical chunk l & 15 of row 4 I + l / 16, i.e. logical chunk
  // (l & 15) ^ f(row)
  int va[WG_NI], vb[WG_NI];
#pragma unroll
  for (int i = 0; i < WG_NI; ++i) {
    const int row = 4 * (w + 4 * i) + (lane >> 4);
    const int ch = (lane & 15) ^ tr_swz(row);
    va[i] = row * (int)g.lda * 2 + m0 * 2 + ch * 16;
    vb[i] = row * (int)g.ldb * 2 + n0 * 2 + ch * 16;
  }
  const int sa = WG_BK * (int)g.lda * 2, sb = WG_BK * (int)g.ldb * 2;  // bytes per K-tile
  const rsrc_t ral = CS ? make_rsrc(g.al + kb, (int64_t)(g.K - kb) * 4) : ra;
  char* s_al = lds + STAGES * WG_STAGE;
  auto issue = [&](int buf, int kt) {
    char* A = lds + buf * WG_STAGE;
    char* B = A + WG_A_BYTES;
#pragma unroll
    for (int i = 0; i < WG_NI; ++i) glds16(ra, va[i], kt * sa, A + 1024 * (w + 4 * i));
#pragma unroll
    for (int i = 0; i < WG_NI; ++i) glds16(rb, vb[i], kt * sb, B + 1024 * (w + 4 * i));
    if (CS && w == 0)  // the tile's 64 weights (lanes >= 16 duplicate, unused)
      glds16(ral, 16 * (lane & 15), kt * WG_BK * 4, s_al + buf * WG_AL_BYTES);
  };
  const int cs_c = threadIdx.x & 31, cs_kg = threadIdx.x >> 5;
  const int cs_m = 32 * tn + cs_c;  // column within the A tile
  float cs_acc = 0.f;

  // transposed-read offsets (within a 16-row K sub-step): group gq = l / 16
  // reads rows 8 (gq >> 1) + 4 jj + q, columns c0 + 16 (gq & 1) + 4 p .. + 3
  // of the wave's 32-column sub-tile c0 (lane 4 q + p of the group)
  const int gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  int oa[2][2], ob[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int row = 8 * (gq >> 1) + 4 * jj + q;
      const int cx = 2 * (gq & 1) + (p >> 1);
      oa[i][jj] = 256 * row + 16 * ((wr * 8 + i * 4 + cx) ^ tr_swz(row)) + 8 * (p & 1);
      ob[i][jj] = 256 * row + 16 * ((wc * 8 + i * 4 + cx) ^ tr_swz(row)) + 8 * (p & 1);
    }

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll
  for (int pp = 0; pp < STAGES - 1; ++pp)
    if (pp < nk) issue(pp, pp);
  for (int kt = 0; kt < nk; ++kt) {
    if (STAGES > 2 && kt + 1 < nk) {
      wait_vmcnt<2 * WG_NI * (STAGES - 2)>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (kt + STAGES - 1 < nk) issue((kt + STAGES - 1) % STAGES, kt + STAGES - 1);
    const char* A = lds + (kt % STAGES) * WG_STAGE;
    const char* B = A + WG_A_BYTES;
    if (CS) {
      const float* al = reinterpret_cast<const float*>(s_al + (kt % STAGES) * WG_AL_BYTES);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = 8 * cs_kg + i;
        const uint16_t x = *reinterpret_cast<const uint16_t*>(
            A + 256 * row + 16 * ((cs_m >> 3) ^ tr_swz(row)) + 2 * (cs_m & 7));
        cs_acc = fmaf(al[row], bf2f(x), cs_acc);
      }
    }
#pragma unroll
    for (int ks = 0; ks < WG_BK / 16; ++ks) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = tr_frag(A + ks * 4096, oa[i][0], oa[i][1]);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = tr_frag(B + ks * 4096, ob[j][0], ob[j][1]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  if (CS) {  // the 8 K groups' sums of each column, through LDS
    __syncthreads();  // (every wave is past its last LDS read of the stages)
    float* s_red = reinterpret_cast<float*>(lds);
    s_red[cs_kg * 32 + cs_c] = cs_acc;
    __syncthreads();
    const int m = m0 + cs_m;
    if (threadIdx.x < 32 && m < g.M) {
      float v = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) v += s_red[k * 32 + cs_c];
      if (g.S > 1)
        g.ws_db[(int64_t)s * g.M + m] = v;
      else
        g.db[m] = v;
    }
  }
  // lane: column n0 + 64 wc + 32 j + (l & 31), rows m0 + 64 wr + 32 i + (r & 3) + 8 (r >> 2) + 4 (l >> 5)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 64 * wc + 32 * j + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 64 * wr + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= g.M) continue;  // (ragged last m tile)
        float* dst;
        if (g.S > 1)
          dst = g.ws + ((int64_t)s * g.M + m) * g.N + n;
        else
          dst = m < g.M0 ? g.C0 + (int64_t)m * g.ldc0 + n : g.C1 + (int64_t)(m - g.M0) * g.ldc1 + n;
        *dst = acc[i][j][r];
      }
    }
}

// C rows = the S slabs summed in split order (float4 per thread)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(WgradArgs g) {
  const int n4 = g.N / 4;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g.db != nullptr && idx < g.M) {  // fused column sums: the S partials in split order
    float v = g.ws_db[idx];
    for (int s = 1; s < g.S; ++s) v += g.ws_db[(int64_t)s * g.M + idx];
    g.db[idx] = v;
  }
  if (idx >= (int64_t)g.M * n4) return;
  const int m = (int)(idx / n4), c = (int)(idx - (int64_t)m * n4) * 4;
  const int64_t slab = (int64_t)g.M * g.N;
  const float* src = g.ws + (int64_t)m * g.N + c;
  float4 a = *reinterpret_cast<const float4*>(src);
  for (int s = 1; s < g.S; ++s) {
    const float4 x = *reinterpret_cast<const float4*>(src + s * slab);
    a.x += x.x, a.y += x.y, a.z += x.z, a.w += x.w;
  }
  float* dst = m < g.M0 ? g.C0 + (int64_t)m * g.ldc0 + c : g.C1 + (int64_t)(m - g.M0) * g.ldc1 + c;
  *reinterpret_cast<float4*>(dst) = a;
}

}  // namespace

// M need not be a multiple of 128: the last m tile reads up to 128 columns
// of every A row (past M they run into the row stride / the next row, or
// past the last row's end, where the buffer resource returns zeros) and
// stores only the columns < M
bool wgrad_tn_ok(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const void* A,
                 const void* B) {
  return M > 0 && N > 0 && K > 0 && N % WG_BN == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         lda >= M && ldb >= N && (reinterpret_cast<uintptr_t>(A) & 15) == 0 &&
         (reinterpret_cast<uintptr_t>(B) & 15) == 0 &&
         K * std::max(lda, ldb) * 2 + 256 < (1LL << 31);
}

int wgrad_tn_splits(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ((M + WG_BM - 1) / WG_BM) * (N / WG_BN);
  const int64_t nkt = (K + WG_BK - 1) / WG_BK;
  int64_t S = std::max<int64_t>(1, (512 + tiles - 1) / tiles);  // >= 2 blocks per CU
  S = std::min<int64_t>(S, std::max<int64_t>(1, nkt / 4));      // >= 4 K-tiles per split
  const int64_t kts = (nkt + S - 1) / S;
  return (int)((nkt + kts - 1) / kts);
}

void launch_wgrad_tn(WgradArgs g, hipStream_t stream) {
  const int64_t nkt = (g.K + WG_BK - 1) / WG_BK;
  if (g.S < 1) g.S = 1;
  g.kts = (int)((nkt + g.S - 1) / g.S);
  g.S = (int)((nkt + g.kts - 1) / g.kts);
  if (g.S > 1 && g.ws == nullptr) throw std::runtime_error("wgrad_tn: split-K needs a workspace");
  const bool cs = g.db != nullptr;
  if (cs && (g.N != 512 || g.al == nullptr || (g.S > 1 && g.ws_db == nullptr)))
    throw std::runtime_error("wgrad_tn: fused column sums need N = 512, weights and a workspace");
  const int blocks = ((g.M + WG_BM - 1) / WG_BM) * (g.N / WG_BN) * g.S;
  constexpr int STAGES = 2;
  if (cs) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)wgrad_tn_kernel<STAGES, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                STAGES * (WG_STAGE + WG_AL_BYTES));
      attr = true;
    }
    hipLaunchKernelGGL((wgrad_tn_kernel<STAGES, true>), dim3(blocks), dim3(256),
                       STAGES * (WG_STAGE + WG_AL_BYTES), stream, g);
  } else {
    hipLaunchKernelGGL((wgrad_tn_kernel<STAGES, false>), dim3(blocks), dim3(256), STAGES * WG_STAGE,
                       stream, g);
  }
  post_launch("wgrad_tn_kernel", stream);
  if (g.S > 1) {
    const int64_t n = std::max<int64_t>((int64_t)g.M * (g.N / 4), cs ? g.M : 0);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, g);
    post_launch("wgrad_reduce_kernel", stream);
  }
}

}  // namespace cst
