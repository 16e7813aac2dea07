// Persistent "NT" GEMM for the vocabulary head's backward on gfx950:
//
//   C (M x N, fp32, row-major) = A (M x K, bf16, K-contiguous)
//                               . B (N x K, bf16, K-contiguous)^T
//
// used for X = E W of a training step (A = the bf16 exp store, 35,840 x 10,560;
// B = W_logit^T zero-padded to 10,560 columns; N = 512): 386 GFLOP, the largest
// vendor GEMM on the headline step's critical path (verdict r3, missing 2).
//
// Why not one workgroup per tile: 256 x 256 tiles give (35,840 / 256) x 2 =
// 280 tiles for 256 CUs -- a second round that keeps 24 CUs busy (55 % of the
// chip over the launch); smaller tiles re-read the 753 MB exp store more often.
// So the grid is one workgroup per CU and the work is split in two phases:
//   1. floor(tiles / G) rounds of whole tiles, data parallel: every
//      workgroup sweeps K in step with the others (W^T tiles shared through
//      L2/MALL), the two N-tiles of one M block on one XCD (the exp-store rows
//      are read from HBM once and hit L2 for the second tile);
//   2. the remaining tiles' K-iterations divided evenly over all G
//      workgroups (stream-K): a workgroup that covers part of a tile writes
//      its fp32 partial to a slab in the accumulator's own lane order (256-B
//      stores), takes a ticket, and the tile's last arriver sums the slabs in
//      piece order (deterministic) and stores the tile.
// At the headline shape phase 2 adds 24 x 165 / 256 = 15.5 K-iterations per
// workgroup to phase 1's 165: 1.09 tile-times instead of 2.
//
// Main loop: 512 threads = 8 waves as 2 (M) x 4 (N), v_mfma_f32_32x32x16_bf16,
// K staged 64 wide through LDS by LDS-DMA (buffer_load ... lds, 16 B per lane)
// into STAGES buffers with 16-byte-chunk XOR swizzle (gemm_tile.h swz), a raw
// s_barrier per K-tile and a counted vmcnt (the next tiles' copies stay in
// flight across it).
//
// Hand-off (phase 2), the counter form of the split-K reduction: plain slab
// stores -> vmcnt(0) in every wave -> barrier -> one lane: agent-scope release
// fence, vmcnt(0), relaxed agent-scope fetch_add on the tile's counter; the
// last arriver: agent-scope acquire fence, vmcnt(0), barrier, plain slab loads.
// The counters are zeroed by the caller before every launch (a memset node
// inside a captured graph).
#include "../common.h"
#include "gemm_tile.h"

#include <algorithm>

namespace cst {

namespace {

// TRANS_: operand layout.  false ("NT"): A (M x K) and B (N x K) K-contiguous,
// LDS images [row][64 k] read by ds_read_b128.  true ("TN"): A stored (K x M)
// and B (K x N), M / N contiguous (dW = E'^T Hs: both operands have the
// reduction index as their row); LDS images [64 k][BM or BN] filled by the
// same lane-linear LDS-DMA, 16-byte chunks XOR-swizzled by (k & 3) << 2, and
// the MFMA fragments read with ds_read_b64_tr_b16 (two per fragment).
template <int BN_, int STAGES_, bool TRANS_ = false>
struct SkCfg {
  static constexpr bool TRANS = TRANS_;
  static constexpr int BM = 256, BN = BN_, BK = 64, THREADS = 512, STAGES = STAGES_;
  static constexpr int WAVES_M = 2, WAVES_N = 4;
  static constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;  // per-wave sub-tile
  static constexpr int TM = WM / 32, TN = WN / 32;
  static constexpr int A_INS = BM / 64, B_INS = BN / 64;  // DMA wave-instructions per wave per K-tile
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  static constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int LDS_BYTES = STAGES * STAGE_BYTES + 16;  // + the last-arriver flag
  static constexpr int NI = A_INS + B_INS;
  // TN images: 16-byte chunks per k-row, k-rows per DMA wave-instruction
  static constexpr int A_CPR = BM / 8, B_CPR = BN / 8;
  static constexpr int A_RPI = 64 / A_CPR, B_RPI = 64 / B_CPR;
  static_assert(!TRANS || (A_CPR >= 16 && B_CPR >= 16 && 64 % A_CPR == 0 && 64 % B_CPR == 0),
                "TN images: >= 16 chunks per k-row");
  static_assert(TM >= 1 && TN >= 1 && WN % 32 == 0, "tile");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

struct SkArgs {
  const uint16_t* A;  // NT: M x K, row stride lda (elements); TN: K x M
  const uint16_t* B;  // NT: N x K, row stride ldb; TN: K x N
  int64_t a_bytes, b_bytes;  // readable bytes from A / B (buffer-resource bounds)
  float* C;           // M x N, row stride ldc
  float* slab;        // phase-2 partials: [rem tile][piece][BM * BN]
  int* cnt;           // phase-2 tickets, one per remainder tile (zeroed by the caller)
  int64_t lda, ldb, ldc;
  int M, N, nk;       // nk = K / 64
  int tiles_n;        // N / BN (tiles_m = ceil(M / BM))
  int full_rounds;    // phase 1: whole tiles per workgroup
  int rem;            // phase 2: tiles split over all workgroups
  int pmax;           // slab pieces reserved per remainder tile
};

// first workgroup whose K-iteration range [floor(b I / G), floor((b+1) I / G))
// contains iteration x
__device__ __forceinline__ int sk_owner(int64_t x, int64_t I, int G) {
  return (int)(((x + 1) * G + I - 1) / I - 1);
}

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));

// TN image byte offset of (k-row, column): chunk XOR (row & 3) << 2
template <int ROWB>
__device__ __forceinline__ int tn_off(int row, int col) {
  return row * ROWB + ((((col >> 3) ^ ((row & 3) << 2))) << 4) + ((col & 7) << 1);
}

// one 32x32x16 operand fragment from a TN image: lane l holds column
// c0 + (l & 31), k = k0 + 8 (l >> 5) + j; ds_read_b64_tr_b16 per 16-lane
// group g delivers 4 k-rows x 16 columns, lane 4q + p addressing row q,
// columns 4p .. 4p + 3 (two reads: k-rows 0-3 and 4-7 of the lane's half)
template <int ROWB>
__device__ __forceinline__ bf16x8 tn_frag(const char* img, int c0, int k0, int lane) {
  const int g = lane >> 4, li = lane & 15;
  const int row = k0 + 8 * (g >> 1) + (li >> 2);
  const int col = c0 + 16 * (g & 1) + 4 * (li & 3);
  typedef __attribute__((address_space(3))) v4i16 lds_v4;
  const char* p0 = img + tn_off<ROWB>(row, col);
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(p0));
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(p0 + 4 * ROWB));
  const v8i16 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

template <class CF>
__device__ __forceinline__ void sk_mainloop(int kt0, int kt1, rsrc_t ra, const int (&va)[CF::A_INS],
                                            rsrc_t rb, const int (&vb)[CF::B_INS], int sa, int sb,
                                            char* lds, f32x16 (&acc)[CF::TM][CF::TN]) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wr = w / CF::WAVES_N, wc = w % CF::WAVES_N;
#pragma unroll
  for (int i = 0; i < CF::TM; ++i)
#pragma unroll
    for (int j = 0; j < CF::TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto issue = [&](int buf, int kt) {
    char* As = lds + buf * CF::STAGE_BYTES;
    char* Bs = As + CF::A_BYTES;
#pragma unroll
    for (int i = 0; i < CF::A_INS; ++i) glds16(ra, va[i], kt * sa, As + 1024 * (w + 8 * i));
#pragma unroll
    for (int i = 0; i < CF::B_INS; ++i) glds16(rb, vb[i], kt * sb, Bs + 1024 * (w + 8 * i));
  };
  const int n = kt1 - kt0;
#pragma unroll
  for (int p = 0; p < CF::STAGES - 1; ++p)
    if (p < n) issue(p, kt0 + p);
  for (int t = 0; t < n; ++t) {
    if (CF::STAGES > 2 && t + 1 < n)
      wait_vmcnt<CF::NI * (CF::STAGES - 2)>();
    else
      wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (t + CF::STAGES - 1 < n) issue((t + CF::STAGES - 1) % CF::STAGES, kt0 + t + CF::STAGES - 1);
    const char* As = lds + (t % CF::STAGES) * CF::STAGE_BYTES;
    const char* Bs = As + CF::A_BYTES;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int c = 2 * s + (lane >> 5);
      bf16x8 af[CF::TM], bfr[CF::TN];
      if constexpr (CF::TRANS) {
#pragma unroll
        for (int i = 0; i < CF::TM; ++i)
          af[i] = tn_frag<CF::BM * 2>(As, wr * CF::WM + i * 32, 16 * s, lane);
#pragma unroll
        for (int j = 0; j < CF::TN; ++j)
          bfr[j] = tn_frag<CF::BN * 2>(Bs, wc * CF::WN + j * 32, 16 * s, lane);
      } else {
#pragma unroll
        for (int i = 0; i < CF::TM; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(As + swz(wr * CF::WM + i * 32 + (lane & 31), c));
#pragma unroll
        for (int j = 0; j < CF::TN; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + swz(wc * CF::WN + j * 32 + (lane & 31), c));
      }
#pragma unroll
      for (int i = 0; i < CF::TM; ++i)
#pragma unroll
        for (int j = 0; j < CF::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // every wave done with the staging buffers before the next tile's DMA
}

// per-lane DMA source offsets (bytes from the tile's origin) and the buffer
// resources of one tile (bounded by the operand's last byte: reads past it
// return 0)
template <class CF>
__device__ __forceinline__ void sk_tile_src(const SkArgs& g, int m0, int n0, rsrc_t& ra,
                                            int (&va)[CF::A_INS], rsrc_t& rb,
                                            int (&vb)[CF::B_INS]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t la = g.lda * 2, lb = g.ldb * 2;
  if constexpr (CF::TRANS) {
    // origin = column m0 (n0) of k-row 0; DMA instruction i of wave w fills
    // k-rows RPI (w + 8 i) .. +RPI-1, lane l physical chunk l % CPR
    ra = make_rsrc(g.A + m0, g.a_bytes - 2 * (int64_t)m0);
    rb = make_rsrc(g.B + n0, g.b_bytes - 2 * (int64_t)n0);
#pragma unroll
    for (int i = 0; i < CF::A_INS; ++i) {
      const int row = CF::A_RPI * (w + 8 * i) + lane / CF::A_CPR;
      va[i] = (int)(row * la) + 16 * ((lane % CF::A_CPR) ^ ((row & 3) << 2));
    }
#pragma unroll
    for (int i = 0; i < CF::B_INS; ++i) {
      const int row = CF::B_RPI * (w + 8 * i) + lane / CF::B_CPR;
      vb[i] = (int)(row * lb) + 16 * ((lane % CF::B_CPR) ^ ((row & 3) << 2));
    }
  } else {
    ra = make_rsrc(g.A + (int64_t)m0 * g.lda, g.a_bytes - (int64_t)m0 * la);
    rb = make_rsrc(g.B + (int64_t)n0 * g.ldb, g.b_bytes - (int64_t)n0 * lb);
#pragma unroll
    for (int i = 0; i < CF::A_INS; ++i) {
      const int row = 8 * (w + 8 * i) + (lane >> 3);
      va[i] = (int)(row * la) + 16 * dma_chunk(row, lane);
    }
#pragma unroll
    for (int i = 0; i < CF::B_INS; ++i) {
      const int row = 8 * (w + 8 * i) + (lane >> 3);
      vb[i] = (int)(row * lb) + 16 * dma_chunk(row, lane);
    }
  }
}

// accumulators -> C rows < M (fp32, 2 x 128-byte row segments per store):
// buffer stores through a resource that ends at row M, so the rows of an
// edge tile past M are dropped by the hardware (no per-element branches)
template <class CF>
__device__ __forceinline__ void sk_store(const SkArgs& g, int m0, int n0,
                                         const f32x16 (&acc)[CF::TM][CF::TN]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wr = w / CF::WAVES_N, wc = w % CF::WAVES_N;
  const rsrc_t rc = make_rsrc(g.C + (int64_t)m0 * g.ldc, (int64_t)(g.M - m0) * g.ldc * 4);
  const int ldc4 = (int)g.ldc * 4;
#pragma unroll
  for (int i = 0; i < CF::TM; ++i) {
    const int rl = wr * CF::WM + i * 32 + 4 * (lane >> 5);
#pragma unroll
    for (int j = 0; j < CF::TN; ++j) {
      const int off = rl * ldc4 + 4 * (n0 + wc * CF::WN + j * 32 + (lane & 31));
#pragma unroll
      for (int r = 0; r < 16; ++r)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[i][j][r]), rc, off,
                                              ((r & 3) + 8 * (r >> 2)) * ldc4, 0);
    }
  }
}

template <int BN, int STAGES, bool TRANS>
__global__ __launch_bounds__(512, 1) void gemm_sk_kernel(SkArgs g) {
  using CF = SkCfg<BN, STAGES, TRANS>;
  // K-tile advance of the DMA source (scalar offset): 64 columns (NT) or 64
  // k-rows (TN)
  const int sa = CF::TRANS ? (int)(64 * g.lda * 2) : 128;
  const int sb = CF::TRANS ? (int)(64 * g.ldb * 2) : 128;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int* s_flag = reinterpret_cast<int*>(lds + CF::STAGES * CF::STAGE_BYTES);
  const int G = gridDim.x, b = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  f32x16 acc[CF::TM][CF::TN];
  rsrc_t ra, rb;
  int va[CF::A_INS], vb[CF::B_INS];

  // phase 1: whole tiles; workgroups b, b + 8, b + 16 ... share an XCD, so
  // consecutive tile numbers (the N-tiles of one M block) go to them
  const int per_xcd = G / 8;
  const int xslot = (b % 8) * per_xcd + b / 8;
  for (int f = 0; f < g.full_rounds; ++f) {
    const int u = f * G + xslot;
    const int m0 = (u / g.tiles_n) * CF::BM, n0 = (u % g.tiles_n) * CF::BN;
    sk_tile_src<CF>(g, m0, n0, ra, va, rb, vb);
    sk_mainloop<CF>(0, g.nk, ra, va, rb, vb, sa, sb, lds, acc);
    sk_store<CF>(g, m0, n0, acc);
  }
  if (g.rem == 0) return;

  // phase 2: remainder tiles, K-iterations split evenly over min(G, I)
  // workgroups (every one of them gets >= 1 iteration, so every piece a tile
  // counts arrives)
  const int64_t I = (int64_t)g.rem * g.nk;
  const int G2 = (int)min<int64_t>(G, I);
  if (b >= G2) return;
  const int64_t lo = (int64_t)b * I / G2, hi = (int64_t)(b + 1) * I / G2;
  int64_t it = lo;
  while (it < hi) {
    const int q = (int)(it / g.nk);
    const int k0 = (int)(it % g.nk);
    const int k1 = (int)min<int64_t>(g.nk, k0 + (hi - it));
    const int u = g.full_rounds * G + q;
    const int m0 = (u / g.tiles_n) * CF::BM, n0 = (u % g.tiles_n) * CF::BN;
    sk_tile_src<CF>(g, m0, n0, ra, va, rb, vb);
    sk_mainloop<CF>(k0, k1, ra, va, rb, vb, sa, sb, lds, acc);
    it += k1 - k0;
    const int fb = sk_owner((int64_t)q * g.nk, I, G2);
    const int lb = sk_owner((int64_t)(q + 1) * g.nk - 1, I, G2);
    const int P = lb - fb + 1, p = b - fb;
    if (P == 1) {
      sk_store<CF>(g, m0, n0, acc);
      continue;
    }
    // this piece -> its slab, in the accumulator's lane order
    const int64_t TILE = (int64_t)CF::BM * CF::BN;
    float* slab_q = g.slab + (int64_t)q * g.pmax * TILE;
    {
      float* s = slab_q + (int64_t)p * TILE + (int64_t)w * (CF::TM * CF::TN * 16 * 64) + lane;
#pragma unroll
      for (int i = 0; i < CF::TM; ++i)
#pragma unroll
        for (int j = 0; j < CF::TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) s[((i * CF::TN + j) * 16 + r) * 64] = acc[i][j][r];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int ticket =
          __hip_atomic_fetch_add(g.cnt + q, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_flag = ticket == P - 1;
      if (ticket == P - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    if (!*s_flag) continue;
    // last arriver: the pieces summed in piece order from the slabs (its own
    // included), so the result does not depend on the arrival order
#pragma unroll
    for (int i = 0; i < CF::TM; ++i)
#pragma unroll
      for (int j = 0; j < CF::TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    for (int pp = 0; pp < P; ++pp) {
      const float* s =
          slab_q + (int64_t)pp * TILE + (int64_t)w * (CF::TM * CF::TN * 16 * 64) + lane;
#pragma unroll
      for (int i = 0; i < CF::TM; ++i)
#pragma unroll
        for (int j = 0; j < CF::TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] += s[((i * CF::TN + j) * 16 + r) * 64];
    }
    sk_store<CF>(g, m0, n0, acc);
  }
}

template <int BN, int STAGES, bool TRANS>
void launch_sk(const SkArgs& g, int G, hipStream_t stream) {
  using CF = SkCfg<BN, STAGES, TRANS>;
  hipLaunchKernelGGL((gemm_sk_kernel<BN, STAGES, TRANS>), dim3(G), dim3(CF::THREADS),
                     CF::LDS_BYTES, stream, g);
}

}  // namespace

// Sizes the caller allocates before the launch: the tickets (ints, zeroed)
// and the phase-2 slabs (floats).  variant: 0 = 256 x 256 tiles / 2 stages,
// 1 = 256 x 128 tiles / 3 stages.
void gemm_sk_plan(int M, int N, int K, int G, int variant, int64_t* n_cnt, int64_t* n_slab) {
  const int BN = variant == 1 ? 128 : 256;
  const int tiles = ((M + 255) / 256) * (N / BN);
  const int full = tiles / G, rem = tiles - full * G;
  const int nk = K / 64;
  int pmax = 0;
  if (rem > 0) {
    const int64_t I = (int64_t)rem * nk;
    const int64_t G2 = std::min<int64_t>(G, I);
    for (int q = 0; q < rem; ++q) {
      const int64_t a = (int64_t)q * nk, z = (int64_t)(q + 1) * nk - 1;
      const int fb = (int)(((a + 1) * G2 + I - 1) / I - 1), lb = (int)(((z + 1) * G2 + I - 1) / I - 1);
      pmax = std::max(pmax, lb - fb + 1);
    }
  }
  *n_cnt = rem;
  *n_slab = (int64_t)rem * pmax * 256 * BN;
}

// trans = false: C = A B^T, A (M x K), B (N x K); trans = true: C = A^T B,
// A (K x M), B (K x N).  a_bytes / b_bytes: readable bytes from A / B.
void launch_gemm_sk(const uint16_t* A, int64_t lda, int64_t a_bytes, const uint16_t* B,
                    int64_t ldb, int64_t b_bytes, float* C, int64_t ldc, int M, int N, int K,
                    bool trans, int G, int variant, float* slab, int* cnt, hipStream_t stream) {
  const int BN = variant == 1 ? 128 : 256;
  SkArgs g;
  g.A = A, g.B = B, g.C = C, g.slab = slab, g.cnt = cnt;
  g.a_bytes = a_bytes, g.b_bytes = b_bytes;
  g.lda = lda, g.ldb = ldb, g.ldc = ldc;
  g.M = M, g.N = N, g.nk = K / 64;
  g.tiles_n = N / BN;
  const int tiles = ((M + 255) / 256) * g.tiles_n;
  g.full_rounds = tiles / G;
  g.rem = tiles - g.full_rounds * G;
  int64_t nc, ns;
  gemm_sk_plan(M, N, K, G, variant, &nc, &ns);
  g.pmax = g.rem > 0 ? (int)(ns / ((int64_t)g.rem * 256 * BN)) : 0;
  if (trans) {
    if (variant == 1)
      launch_sk<128, 3, true>(g, G, stream);
    else
      launch_sk<256, 2, true>(g, G, stream);
  } else {
    if (variant == 1)
      launch_sk<128, 3, false>(g, G, stream);
    else
      launch_sk<256, 2, false>(g, G, stream);
  }
}

// W (rows x cols, bf16 row-major) -> W^T (cols x ldo), columns rows .. ldo-1
// zero (64 x 64 tiles through LDS)
__global__ __launch_bounds__(256) void transpose_pad_bf16_kernel(const uint16_t* __restrict__ in,
                                                                 int rows, int cols,
                                                                 uint16_t* __restrict__ out,
                                                                 int64_t ldo) {
  __shared__ uint16_t t[64][66];
  const int r0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int rr = i / 64, cc = i % 64;
    const int r = r0 + rr, c = c0 + cc;
    t[rr][cc] = (r < rows && c < cols) ? in[(int64_t)r * cols + c] : (uint16_t)0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int cc = i / 64, rr = i % 64;
    const int r = r0 + rr, c = c0 + cc;
    if (c < cols && r < ldo) out[(int64_t)c * ldo + r] = t[rr][cc];
  }
}

void launch_transpose_pad_bf16(const uint16_t* in, int rows, int cols, uint16_t* out, int64_t ldo,
                               hipStream_t stream) {
  dim3 grid((unsigned)((ldo + 63) / 64), (unsigned)((cols + 63) / 64));
  hipLaunchKernelGGL(transpose_pad_bf16_kernel, grid, dim3(256), 0, stream, in, rows, cols, out,
                     ldo);
}

}  // namespace cst
