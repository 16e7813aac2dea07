// Fused vocab-head backward: dS = dG (onehot - softmax) formed on the fly from
// the saved fp16 logits, multiplied straight into dHd = dS W, with dS (bf16,
// in place over the logits) and the bias-gradient column sums as side outputs.
//
// Reference semantics: the backward of log_softmax(logit(dropout(h)))
// (/root/reference/model.py:281) under the RL / XE criteria
// (/root/reference/model.py:7-43).  The two-pass route (vocab_bwd_ds_kernel
// in vocab.hip, then a BLAS GEMM) moves the NR x V operand through HBM three
// times: fp16 read + bf16 write by the dS pass, bf16 read by the GEMM.  Here
// the GEMM's A-operand producer IS the dS pass: one fp16 read, one bf16
// write (kept for the dW_logit GEMM), and the matrix cores run under it.
//
//   dHd[r][h] = sum_v dS[r][v] W[v][h],  dS[r][v] = -(a+b) p[r][v] + a [v == y_s] + b [v == y_x]
//
// Geometry (MI355X, gfx950): block tile 128 rows x 512 (= H) columns, so every
// dS element is produced by exactly one thread (the in-place write is
// race-free and each softmax value is evaluated once); 512 threads = 8 waves
// in a 2 x 4 grid, 64 x 128 per wave (2 x 4 MFMA 32x32x16 bf16 tiles, 128 fp32
// accumulators).  K (= vocab) is staged 32 at a time through LDS, 3 stages:
//   A: buffer_load fp16 -> registers (one K-tile ahead) -> softmax residual in
//      fp32 -> bf16 -> LDS, and -> HBM in place;
//   B: W^T (H x Vp bf16, K-contiguous) by LDS-DMA (buffer_load ... lds) two
//      K-tiles ahead; one raw s_barrier per K-tile.
// Every VMEM instruction is issued unconditionally (out-of-range lanes use
// out-of-range buffer offsets, which the hardware drops), so the counted
// vmcnt waits for the DMA tiles are exact.
// 64-byte LDS rows are 16-byte-chunk XOR-swizzled (chunk ^ ((row >> 2) & 3)):
// the 16-lane groups of ds_read_b128 then hit 16 distinct bank slots.
// Column sums of the bf16 dS (bias gradient): each wave re-reads its own 16
// rows of the tile from LDS and stores one partial per (wave, column); the
// host sums the partials.  dS goes back to HBM two K-tiles (128 bytes of a
// row) at a time.  Split-K over the vocabulary (grid.y) writes one dHd partial per
// split; the reverse LSTM step adds the partials in its epilogue.
#include "../common.h"

namespace cst {

constexpr int VBD_BM = 128, VBD_BN = 512, VBD_BK = 32, VBD_STAGES = 4, VBD_THREADS = 512;
constexpr int VBD_A_BYTES = VBD_BM * VBD_BK * 2, VBD_B_BYTES = VBD_BN * VBD_BK * 2;
constexpr int VBD_STAGE_BYTES = VBD_A_BYTES + VBD_B_BYTES;
constexpr int VBD_LDS_BYTES = VBD_STAGES * VBD_STAGE_BYTES;                  // 160 KiB
constexpr int VBD_B_INS = VBD_B_BYTES / 1024 / (VBD_THREADS / 64);          // DMA ops / wave / tile
constexpr int VBD_OOB = 0x7ffffff0;      // dropped buffer offset
constexpr int VBD_OOB_ADD = 0x70000000;  // added to an in-range base: still dropped, no overflow
constexpr int VBD_AD = 4;  // A register prefetch depth (K-tiles)
// vector-memory ops per pipeline step: B DMA, column-sum store, A load, and
// the dS stores (two on odd steps, none on even ones): any two consecutive
// steps issue 2 * VBD_STEP_OPS
constexpr int VBD_STEP_OPS = VBD_B_INS + 3;
int vocab_bwd_dhd_mblocks(int64_t NR);

typedef __amdgpu_buffer_rsrc_t vbd_rsrc_t;
typedef __attribute__((address_space(3))) void* vbd_lds_ptr_t;
typedef unsigned int vbd_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int vbd_swz(int row, int chunk) {
  return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4);
}

template <int N>
__device__ __forceinline__ void vbd_wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// this wave's LDS operations done, then the workgroup barrier; the empty asm
// statements keep the compiler from moving memory operations across it
__device__ __forceinline__ void vbd_barrier() {
  __builtin_amdgcn_s_waitcnt(0xF | (0x3 << 14) | (0x7 << 4));  // lgkmcnt(0)
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct VbdRow {  // per-row scalars of the softmax residual
  float a, b;    // weights of the sampled / teacher token terms
  float lc, sg;  // -(a+b) p = sg * exp2(x log2e - lc)
  int ys, yx;
};

// 8 consecutive logits (fp16) of one row -> bf16 dS (d[] keeps the fp32
// values for the column sums).  tail: the K-tile crosses V (mask columns).
__device__ __forceinline__ vbd_u32x4 vbd_transform(vbd_u32x4 x, const VbdRow& s, int v0, int V,
                                                   bool tail, float (&d)[8]) {
  constexpr float LOG2E = 1.4426950408889634f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    d[2 * k] = s.sg * __builtin_amdgcn_exp2f(__builtin_fmaf(h2f(x[k] & 0xffff), LOG2E, -s.lc));
    d[2 * k + 1] = s.sg * __builtin_amdgcn_exp2f(__builtin_fmaf(h2f(x[k] >> 16), LOG2E, -s.lc));
  }
  const int dy = s.ys - v0, dx = s.yx - v0;
  if (__any((unsigned)dy < 8u || (unsigned)dx < 8u)) {  // ~5% of the wave-tiles
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] += (k == dy ? s.a : 0.f) + (k == dx ? s.b : 0.f);
  }
  if (tail) {
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = v0 + k < V ? d[k] : 0.f;
  }
  vbd_u32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    o[k] = (uint32_t)f2bf(d[2 * k]) | ((uint32_t)f2bf(d[2 * k + 1]) << 16);
  return o;
}

__global__ __launch_bounds__(VBD_THREADS, 1) void vocab_bwd_dhd_kernel(
    uint16_t* __restrict__ logits, int64_t ldl, int V, int NR, int R, int T_sel,
    const float* __restrict__ lse, const int64_t* __restrict__ y_sel, int64_t ysel_rs,
    const float* __restrict__ dg_sel, int64_t dgsel_rs, const int64_t* __restrict__ y_xe,
    int64_t yxe_rs, const float* __restrict__ dg_xe, int64_t dgxe_rs,
    const uint16_t* __restrict__ wT, int ldw, float* __restrict__ dhd, float* __restrict__ colsum,
    int dbg) {
  // dbg (microbenchmark ablations, 0 in production): 1 no A loads, 2 no dS
  // store, 4 no MFMA, 8 no B DMA, 16 no transform, 32 no column sums, 64 no
  // dHd store
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;  // 2 x 4 wave grid, 64 x 128 per wave
  const int mblk = blockIdx.x, split = blockIdx.y, S = gridDim.y;
  const int m0 = mblk * VBD_BM;
  const int NK = ldw / VBD_BK;
  const int kt0 = split * NK / S, nk = (split + 1) * NK / S - kt0;

  // this thread's transform slot: row m0 + tid/4, 8 columns at 8 (tid & 3)
  const int arow = tid >> 2, achunk = tid & 3;
  VbdRow rs;
  {
    // rows past NR: zero weights (dS = 0, so the column sums skip them);
    // their loads and stores fall outside the buffer range below
    const bool ok = m0 + arow < NR;
    const int rid = min(m0 + arow, NR - 1);
    const int t = rid / R, r = rid % R;
    const bool has_sel = dg_sel != nullptr && t < T_sel;
    rs.a = ok && has_sel ? dg_sel[(int64_t)r * dgsel_rs + t] : 0.f;
    rs.b = ok && dg_xe ? dg_xe[(int64_t)r * dgxe_rs + t] : 0.f;
    rs.ys = has_sel ? (int)y_sel[(int64_t)r * ysel_rs + t] : -1;
    rs.yx = dg_xe ? (int)y_xe[(int64_t)r * yxe_rs + t] : -1;
    const float nab = -(rs.a + rs.b);
    rs.sg = nab < 0.f ? -1.f : 1.f;
    rs.lc = lse[rid] * 1.4426950408889634f - __log2f(fabsf(nab));  // +inf when a + b == 0
  }
  // A: one buffer resource over this block's valid rows; K-tiles outside
  // [0, nk) get out-of-range offsets (their loads return 0, stores drop)
  const int nrows = min(VBD_BM, NR - m0);
  const vbd_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc(
      logits + (int64_t)m0 * ldl, (short)0, (int)((int64_t)nrows * ldl * 2), 0x00020000);
  const int abase = arow * (int)ldl * 2 + 16 * achunk;
  // wave-uniform byte offset of K-tile j (out of range outside [0, nk))
  auto tile_off = [&](int j) { return j >= 0 && j < nk ? (kt0 + j) * VBD_BK * 2 : VBD_OOB_ADD; };
  auto a_off = [&](int j) {
    const int off = abase + tile_off(j);
    if ((kt0 + j + 1) * VBD_BK <= ldl) return off;  // uniform: no chunk past the row
    return (kt0 + j) * VBD_BK + 8 * achunk < ldl ? off : VBD_OOB;
  };
  // The A loads are issued through inline asm so that the compiler's
  // wait-count pass does not track them: its merge at the loop back-edge
  // would otherwise wait for nearly every in-flight load before each
  // transform.  Tile j is loaded VBD_AD steps before its transform, so the
  // counted wait at the top of every iteration (all but the two youngest
  // steps' ops) already covers it; the prologue waits for vmcnt(0).
  typedef int vbd_i32x4 __attribute__((ext_vector_type(4)));
  vbd_i32x4 ars4;
  {
    const uint64_t base = reinterpret_cast<uint64_t>(logits + (int64_t)m0 * ldl);
    ars4[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)base);
    ars4[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(base >> 32) & 0xffff);  // stride 0
    ars4[2] = __builtin_amdgcn_readfirstlane((int)((int64_t)nrows * ldl * 2));
    ars4[3] = 0x00020000;
  }
  auto load_a = [&](int kt) -> vbd_u32x4 {
    vbd_u32x4 x = {0x3c003c00u, 0x3c003c00u, 0x3c003c00u, 0x3c003c00u};
    if (dbg & 1) return x;
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, %2, 0 offen"
                 : "=v"(x)
                 : "v"(a_off(kt)), "s"(ars4));
    return x;
  };
  // per-wave column-sum partials: row (mblk * 8 + w) of colsum
  const vbd_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
      colsum + ((int64_t)mblk * (VBD_THREADS / 64) + w) * V, (short)0, V * 4, 0x00020000);

  // B (W^T rows = output columns) by LDS-DMA: instruction i of wave w fills
  // tile rows 16 (w + 8 i) .. +15, lane l -> row + l/4, physical chunk l & 3
  const vbd_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(wT), (short)0, (int)((int64_t)VBD_BN * ldw * 2), 0x00020000);
  int bvoff[VBD_B_INS];
#pragma unroll
  for (int i = 0; i < VBD_B_INS; ++i) {
    const int row = 16 * (w + 8 * i) + (lane >> 2);
    bvoff[i] = row * ldw * 2 + (((lane & 3) ^ ((row >> 2) & 3)) << 4);
  }

  // One pipeline step for tile j (j may lie outside [0, nk): then every
  // access is out of range but still issued, so the vector-memory op count
  // per step is fixed, see VBD_STEP_OPS).
  float d_unused[8];
  vbd_u32x4 pend = {0u, 0u, 0u, 0u};
  auto produce = [&](int j, vbd_u32x4 x, vbd_u32x4& pend) {
    char* A = lds + ((j + VBD_STAGES) % VBD_STAGES) * VBD_STAGE_BYTES;
    const int bk = tile_off(j);
    if (!(dbg & 8))
#pragma unroll
    for (int i = 0; i < VBD_B_INS; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          brs, (vbd_lds_ptr_t)(A + VBD_A_BYTES + 1024 * (w + 8 * i)), 16, bvoff[i] + bk, 0, 0, 0);
    const int v0 = (kt0 + j) * VBD_BK + 8 * achunk;
    vbd_u32x4 o = x;
    if (!(dbg & 16)) o = vbd_transform(x, rs, v0, V, (kt0 + j + 1) * VBD_BK > V, d_unused);
    *reinterpret_cast<vbd_u32x4*>(A + vbd_swz(arow, achunk)) = o;
    // dS back to HBM in place, two K-tiles (128 bytes of a row) at a time
    if (j & 1) {
      if (!(dbg & 2)) {
        __builtin_amdgcn_raw_buffer_store_b128(pend, ars, a_off(j - 1), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(o, ars, a_off(j), 0, 0);
      }
    } else {
      pend = o;
    }
    if (dbg & 32) return;
    // bias-gradient column sums over this wave's 16 rows, read back from the
    // bf16 tile it just wrote (same wave: LDS order, no barrier): lane l sums
    // columns 2 (l & 15), +1 over rows 4 (l >> 4) .. +3, then across the
    // four row groups
    const int p2 = lane & 15, g = lane >> 4;
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * w + 4 * g + r;
      const uint32_t u = *reinterpret_cast<const uint32_t*>(
          A + vbd_swz(row, p2 >> 2) + ((p2 & 3) << 2));
      s0 += bf2f(u & 0xffff);
      s1 += bf2f(u >> 16);
    }
    s0 += __shfl_xor(s0, 16);
    s1 += __shfl_xor(s1, 16);
    s0 += __shfl_xor(s0, 32);
    s1 += __shfl_xor(s1, 32);
    const int v = (kt0 + j) * VBD_BK + 2 * p2;
    typedef unsigned int vbd_u32x2 __attribute__((ext_vector_type(2)));
    vbd_u32x2 cs;
    cs[0] = __builtin_bit_cast(unsigned int, s0);
    cs[1] = __builtin_bit_cast(unsigned int, s1);
    // V may be odd: a pair straddling V stores one float (the b64 store
    // would be dropped whole), through a second, rarely-taken offset
    const bool ok = lane < 16 && j >= 0 && j < nk;
    __builtin_amdgcn_raw_buffer_store_b64(cs, crs, ok && v + 1 < V ? v * 4 : VBD_OOB, 0, 0);
    if (ok && v + 1 == V) colsum[((int64_t)mblk * (VBD_THREADS / 64) + w) * V + v] = s0;
  };

  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // A register ring: tile j lives in areg[j % VBD_AD] from its load (issued
  // VBD_AD steps ahead) to its transform.  Prologue = steps -3..-1.
  vbd_u32x4 areg[VBD_AD];
#pragma unroll
  for (int j = 0; j < VBD_AD; ++j) areg[j] = load_a(j);
  vbd_wait_vmcnt<0>();
#pragma unroll
  for (int j = 0; j < VBD_STAGES - 1; ++j) {
    produce(j, areg[j % VBD_AD], pend);
    areg[j % VBD_AD] = load_a(j + VBD_AD);
  }

  for (int kb = 0; kb < nk; kb += VBD_AD) {
#pragma unroll
    for (int u = 0; u < VBD_AD; ++u) {
      const int kt = kb + u;
      if (kt < nk) {
        // B(kt) landed: the two later steps issued VBD_STEP_OPS ops each after
        // it (its own step's trailing ops are waited for too, whatever order
        // the compiler gave them)
        vbd_wait_vmcnt<VBD_STEP_OPS * (VBD_STAGES - 2)>();
        vbd_barrier();
        // MFMAs of tile kt first: the matrix core works through them while
        // this wave's VALU transforms tile kt + STAGES - 1 below
        const char* A = lds + (kt % VBD_STAGES) * VBD_STAGE_BYTES;
        const char* B = A + VBD_A_BYTES;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int c = 2 * s + (lane >> 5);
          bf16x8 af[2], bfr[4];
#pragma unroll
          for (int i = 0; i < 2; ++i)
            af[i] = *reinterpret_cast<const bf16x8*>(A + vbd_swz(wr * 64 + i * 32 + (lane & 31), c));
#pragma unroll
          for (int j = 0; j < 4; ++j)
            bfr[j] = *reinterpret_cast<const bf16x8*>(B + vbd_swz(wc * 128 + j * 32 + (lane & 31), c));
          if (!(dbg & 4))
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
          else
            acc[0][0][0] += (float)af[0][0] + (float)bfr[0][0];
        }
        // tile kt + STAGES - 1 into the stage MFMA(kt - 1) released at the barrier
        constexpr int P = (VBD_STAGES - 1) % VBD_AD;
        produce(kt + VBD_STAGES - 1, areg[(u + P) % VBD_AD], pend);
        areg[(u + P) % VBD_AD] = load_a(kt + VBD_STAGES - 1 + VBD_AD);
      }
    }
  }

  if (dbg & 64) {
    if (acc[0][0][0] == 12345.f) dhd[0] = acc[1][3][5];  // keep the accumulators live
    return;
  }
  float* out = dhd + (int64_t)split * NR * VBD_BN;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wc * 128 + j * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < NR) out[(int64_t)row * VBD_BN + col] = acc[i][j][r];
      }
    }
}

int vocab_bwd_dhd_colsum_rows(int64_t NR) { return vocab_bwd_dhd_mblocks(NR) * (VBD_THREADS / 64); }

int vocab_bwd_dhd_mblocks(int64_t NR) { return (int)((NR + VBD_BM - 1) / VBD_BM); }
int vocab_bwd_dhd_kpad() { return VBD_BK; }

void launch_vocab_bwd_dhd(uint16_t* logits, int64_t ldl, int V, int R, int T, int T_sel,
                          const float* lse, const int64_t* y_sel, int64_t ysel_rs,
                          const float* dg_sel, int64_t dgsel_rs, const int64_t* y_xe,
                          int64_t yxe_rs, const float* dg_xe, int64_t dgxe_rs, const uint16_t* wT,
                          int ldw, int H, int splits, float* dhd, float* colsum,
                          hipStream_t stream, int dbg) {
  const int64_t NR = (int64_t)T * R;
  if (H != VBD_BN || ldw % VBD_BK != 0 || ldw < V || ldl % 8 != 0 || ldl < V || splits < 1 ||
      NR <= 0 || (int64_t)VBD_BM * ldl * 2 >= VBD_OOB || (int64_t)VBD_BN * ldw * 2 >= VBD_OOB)
    throw std::runtime_error("vocab_bwd_dhd: unsupported shape");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)vocab_bwd_dhd_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, VBD_LDS_BYTES);
    attr = true;
  }
  hipLaunchKernelGGL(vocab_bwd_dhd_kernel, dim3(vocab_bwd_dhd_mblocks(NR), splits),
                     dim3(VBD_THREADS), VBD_LDS_BYTES, stream, logits, ldl, V, (int)NR, R, T_sel,
                     lse, y_sel, ysel_rs, dg_sel, dgsel_rs, y_xe, yxe_rs, dg_xe, dgxe_rs, wT, ldw,
                     dhd, colsum, dbg);
  post_launch("vocab_bwd_dhd_kernel", stream);
}

}  // namespace cst
