// K1 (reverse loop): the whole reverse LSTM recurrence of the decoder
// backward as ONE persistent launch.
//
// Reference: the autograd backward of the per-step cuDNN LSTM cell
// (/root/reference/model.py:234-282, train.py:216): for t = T-1 .. 0
//   dh_t  = dG_{t+1} W_hh + dropout_mask * dh_logit_t      (K = 4H)
//   dG_t, dc_{t-1} = cell backward(dh_t, dc_t, gates_t, c_t, c_{t-1}).
//
// The step-per-launch form (lstm.hip lstm_step_bwd_kernel) spends ~25-30 us
// per step on a GEMM whose operands are 0.5 MB per workgroup: every launch
// re-streams W_hh^T and dG_{t+1} from L2 / MALL and pays a kernel boundary.
// The recurrence is independent per caption row, so here:
//
// * the rows are split into 8 groups (one per XCD under round-robin dispatch:
//   block b runs on XCD b % 8, so group g = b % 8; a speed assumption only)
//   and each group's rows into row blocks of <= 48 rows; a TEAM = one row
//   block x all H / 64 unit blocks (8 workgroups at H = 512) -- the only
//   workgroups that exchange data: team members read each other's dG rows;
// * each workgroup (512 threads, one per CU, grid <= CU count, all resident)
//   keeps its W_hh^T slice (64 hidden units x 4H, 256 KB bf16 at H = 512) in
//   VGPRs for the whole loop as v_mfma_f32_16x16x32_bf16 A fragments, the 8
//   waves splitting K = 4H eight ways;
// * per step each wave loads its K range of the row block's dG_{t+1} rows
//   (B fragments, 16-byte sc1 loads -- written through by the team this
//   launch), the 8 K-partials are summed through LDS, and the cell backward
//   runs on the sum; the state-gradient carry dc stays in registers (the
//   thread owns the same (row, 4 units) every step);
// * the epilogue operands of step t (gates, c_t, c_{t-1}, dh_logit rows:
//   nothing written in this launch) are staged by LDS-DMA at the start of
//   the step, under the team wait and the GEMM;
// * hand-off (CDNA HIP guide, Guideline 16, valid form "one lane of each
//   storing workgroup: an agent-scope atomic add / an sc1 load poll"): dG_t
//   stored write-through (16-byte sc1 buffer stores), every storing wave
//   drains vmcnt(0), a workgroup barrier, ONE lane adds 1 to the team
//   counter; before step t - 1 one lane polls the counter (relaxed, sc1)
//   until all team members finished step t, the workgroup barrier releases
//   the other waves, and every load of dG rows is an sc1 load.  The poll is
//   bounded: a wait that gives up counts itself in the device error word.
#include "gemm_tile.h"
#include "../launchers.h"

namespace cst {

namespace {

constexpr int LP_THREADS = 512, LP_WAVES = 8;
constexpr int LP_UT = 4;       // 16-unit tiles per workgroup (64 units)
constexpr int LP_RT = 3;       // 16-row tiles per workgroup (<= 48 rows)
constexpr int LP_MAXR = 16 * LP_RT;
constexpr int LP_NF = LP_UT * LP_RT;  // accumulator fragments per wave
constexpr int LP_PF = 3;              // K-steps of B fragments in flight
// LDS: the K-partials [wave][fragment][lane] float4, then per fragment the
// staged epilogue operands of the wave that owns it (private to that wave:
// it stages them itself, so no barrier orders their reuse): gates (2 KB:
// 16 rows x 16 units x 4 gates bf16), two rotating c buffers (c_t and
// c_{t-1}: step t's c_{t-1} is step t - 1's c_t) and the h gradient rows
// dl (1 KB each: 16 rows x 16 units fp32).  Layout = the reader's lanes
// (lane = 16 ku + ru reads 16-byte chunk 16 ku + ru of each 1 KB piece).
constexpr int LP_PART_BYTES = LP_WAVES * LP_NF * 64 * 16;
constexpr int LP_FRAG_BYTES = 5 * 1024;  // gates 2 KB, c x 2, dl
constexpr int LP_LDS = LP_PART_BYTES + LP_NF * LP_FRAG_BYTES;
static_assert(LP_LDS <= 160 * 1024, "persistent reverse loop: LDS budget");
constexpr int LP_CNT_STRIDE = 32;  // ints between team counters (128 B)

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 ld_sc1_b128(rsrc_t r, int voff) {
  const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 16);  // 16: sc1
  return __builtin_bit_cast(bf16x8, v);
}
// (microbenchmark variants only, BwdLoopArgs::dbg: plain loads / no loads)
__device__ __forceinline__ bf16x8 ld_dbg_b128(rsrc_t r, int voff, int dbg) {
  if (dbg & 2) return __builtin_bit_cast(bf16x8, u32x4v{(uint32_t)voff, 0u, 0u, 0u});
  const u32x4v v = (dbg & 1) ? __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0)
                             : __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 16);
  return __builtin_bit_cast(bf16x8, v);
}

// one LDS-DMA instruction: lane l moves the 16 bytes at voff(l) to dst + 16 l
__device__ __forceinline__ void dma16(rsrc_t r, int voff, char* dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)dst, 16, voff, 0, 0, 0);
}

template <int KS, bool DBG = false>
__global__ __launch_bounds__(LP_THREADS, 1) void lstm_bwd_loop_kernel(BwdLoopArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int H = a.H, R = a.R, T = a.T, KD = 4 * H;
  const int g = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int ub = j % a.nub, rb = j / a.nub;
  const int team = g * a.nrb + rb;
  const int u0 = 64 * ub;
  const int rg0 = g * a.rows_per_group, rg1 = min(rg0 + a.rows_per_group, R);
  const int r_lo = rg0 + rb * a.rows_per_block;
  const int r_hi = min(r_lo + a.rows_per_block, rg1);
  const int nrows = r_hi - r_lo;  // >= 1 (launcher)
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ru = lane & 15, ku = lane >> 4;
  const int k0 = w * KS * 32;

  // W_hh^T slice: A fragments of the 4 unit tiles over this wave's K range
  bf16x8 wf[LP_UT][KS];
#pragma unroll
  for (int ut = 0; ut < LP_UT; ++ut)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[ut][ks] = *reinterpret_cast<const bf16x8*>(a.whhT + (int64_t)(u0 + 16 * ut + ru) * KD +
                                                    k0 + 32 * ks + 8 * ku);

  // epilogue ownership: waves 0-3 -> fragments (ut = w, rt 0) and (ut = w,
  // rt 2); waves 4-7 -> (ut = w - 4, rt 1).  Lane: units 4 ku .. 4 ku + 3 of
  // the unit tile, row ru of the row tile.
  const int e_ut = w & 3;
  const int nslot = w < 4 ? 2 : 1;
  int e_rt[2], e_row[2], e_src[2];
  bool e_ok[2];
  e_rt[0] = w < 4 ? 0 : 1;
  e_rt[1] = 2;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    e_row[s] = 16 * e_rt[s] + ru;  // local row
    e_ok[s] = s < nslot && e_row[s] < nrows;
    e_src[s] = r_lo + min(e_row[s], nrows - 1);  // (staging source row, clamped)
  }
  const int uq = u0 + 16 * e_ut + 4 * ku;  // first global unit of the lane's quad
  f32x4v dcr[2];
  dcr[0] = dcr[1] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const rsrc_t r_dg = make_rsrc(a.dG, (int64_t)T * R * KD * 2);
  const rsrc_t r_gates = make_rsrc(a.gates, (int64_t)T * R * KD * 2);
  const rsrc_t r_c = make_rsrc(a.c_all, (int64_t)T * R * H * 4);
  const rsrc_t r_dl = make_rsrc(a.dh, (int64_t)T * R * H * 4);
  const float inv_keep = a.drop_p > 0.f ? 1.f / (1.f - a.drop_p) : 1.f;
  const uint32_t seed = rng_seed(a.rng, RNG_SLOT_DROPOUT);
  int* cnt = a.cnt + team * LP_CNT_STRIDE;
  f32x4v* part = reinterpret_cast<f32x4v*>(lds);
  char* fr[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) fr[s] = lds + LP_PART_BYTES + (e_ut * LP_RT + e_rt[s]) * LP_FRAG_BYTES;
  // staging of the wave's own fragments (wave-uniform): gates / dl of step
  // ts, c of step tc into rotating buffer tc & 1
  auto stage = [&](int ts, int tc, bool with_gd) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s >= nslot) continue;
      const int64_t row = (int64_t)e_src[s];
      if (with_gd) {
        const int gb = (int)(((ts * (int64_t)R + row) * KD + 4 * uq) * 2);
        dma16(r_gates, gb, fr[s]);
        dma16(r_gates, gb + 16, fr[s] + 1024);
        dma16(r_dl, (int)(((ts * (int64_t)R + row) * H + uq) * 4), fr[s] + 4096);
      }
      if (tc >= 0) dma16(r_c, (int)(((tc * (int64_t)R + row) * H + uq) * 4), fr[s] + 2048 + 1024 * (tc & 1));
    }
  };
  // (microbenchmark: per-step phase stamps of every workgroup, lane 0 of wave 0)
  int64_t* ph = a.phases != nullptr ? a.phases + (int64_t)blockIdx.x * T * 4 : nullptr;
#define LP_STAMP(t, k) \
  if (ph != nullptr && tid == 0) ph[(int64_t)(T - 1 - (t)) * 4 + (k)] = (int64_t)wall_clock64();

  // prologue: step T-1's operands and c_{T-2}
  stage(T - 1, T - 1, true);
  if (T >= 2) stage(0, T - 2, false);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  for (int t = T - 1; t >= 0; --t) {
    LP_STAMP(t, 0)
    // 1. dh_rec = dG_{t+1} W_hh over this wave's K range, summed over waves
    f32x4v acc[LP_UT][LP_RT];
#pragma unroll
    for (int ut = 0; ut < LP_UT; ++ut)
#pragma unroll
      for (int rt = 0; rt < LP_RT; ++rt) acc[ut][rt] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const bool gemm = t + 1 < T;
    if (gemm) {
      if (tid == 0) {
        const int target = a.nub * (T - 1 - t);
        bool ok = false;
        for (int it = 0; it < a.poll_bound; ++it) {
          if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) {
            ok = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (!ok && a.err != nullptr)
          __hip_atomic_fetch_add(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler order only)
      LP_STAMP(t, 1)
      int boff[LP_RT];
#pragma unroll
      for (int rt = 0; rt < LP_RT; ++rt)
        boff[rt] = (int)((((int64_t)(t + 1) * R + r_lo + min(16 * rt + ru, nrows - 1)) * KD + k0 +
                          8 * ku) * 2);
      // LP_PF K-steps of B fragments in flight ahead of the MFMAs
      bf16x8 bq[LP_PF][LP_RT];
#pragma unroll
      for (int p = 0; p < LP_PF - 1; ++p)
        if (p < KS)
#pragma unroll
          for (int rt = 0; rt < LP_RT; ++rt)
            bq[p][rt] = DBG ? ld_dbg_b128(r_dg, boff[rt] + 64 * p, a.dbg) : ld_sc1_b128(r_dg, boff[rt] + 64 * p);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + LP_PF - 1 < KS) {
#pragma unroll
          for (int rt = 0; rt < LP_RT; ++rt)
            bq[(ks + LP_PF - 1) % LP_PF][rt] =
                DBG ? ld_dbg_b128(r_dg, boff[rt] + 64 * (ks + LP_PF - 1), a.dbg)
                    : ld_sc1_b128(r_dg, boff[rt] + 64 * (ks + LP_PF - 1));
        }
#pragma unroll
        for (int ut = 0; ut < LP_UT; ++ut)
#pragma unroll
          for (int rt = 0; rt < LP_RT; ++rt)
            acc[ut][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ut][ks], bq[ks % LP_PF][rt],
                                                                  acc[ut][rt], 0, 0, 0);
      }
#pragma unroll
      for (int ut = 0; ut < LP_UT; ++ut)
#pragma unroll
        for (int rt = 0; rt < LP_RT; ++rt) part[(w * LP_NF + ut * LP_RT + rt) * 64 + lane] = acc[ut][rt];
      __syncthreads();
    }
    LP_STAMP(t, 2)

    // 2. cell backward of the lane's (row, 4 units) slots; the operands were
    // staged (and drained) during step t + 1
    uint32_t ow[2][8];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s >= nslot) continue;
      f32x4v dh4 = f32x4v{0.f, 0.f, 0.f, 0.f};
      if (gemm) {
        const int f = e_ut * LP_RT + e_rt[s];
#pragma unroll
        for (int ww = 0; ww < LP_WAVES; ++ww) dh4 += part[(ww * LP_NF + f) * 64 + lane];
      }
      const uint4 gq0 = reinterpret_cast<const uint4*>(fr[s])[lane];
      const uint4 gq1 = reinterpret_cast<const uint4*>(fr[s] + 1024)[lane];
      const f32x4v ct = reinterpret_cast<const f32x4v*>(fr[s] + 2048 + 1024 * (t & 1))[lane];
      const f32x4v cp = t > 0 ? reinterpret_cast<const f32x4v*>(fr[s] + 2048 + 1024 * ((t - 1) & 1))[lane]
                              : f32x4v{0.f, 0.f, 0.f, 0.f};
      const f32x4v dl = reinterpret_cast<const f32x4v*>(fr[s] + 4096)[lane];
      const uint32_t gw[8] = {gq0.x, gq0.y, gq0.z, gq0.w, gq1.x, gq1.y, gq1.z, gq1.w};
      const int r = r_lo + e_row[s];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int u = uq + k;
        const bool keep = a.drop_p <= 0.f || dropout_keep(seed, t, r, u, a.drop_p);
        const float dh = dh4[k] + (keep ? dl[k] * inv_keep : 0.f);
        const uint32_t g01 = gw[2 * k], g23 = gw[2 * k + 1];
        const CellBwd cb = cell_bwd(a.cell, dh, dcr[s][k], bf2f(g01 & 0xffff), bf2f(g01 >> 16),
                                    bf2f(g23 & 0xffff), bf2f(g23 >> 16), ct[k], cp[k]);
        dcr[s][k] = cb.carry;
        ow[s][2 * k] = (uint32_t)f2bf(cb.d0) | ((uint32_t)f2bf(cb.d1) << 16);
        ow[s][2 * k + 1] = (uint32_t)f2bf(cb.d2) | ((uint32_t)f2bf(cb.d3) << 16);
      }
    }
    // 3. step t - 1's operands into this wave's own fragments (its reads of
    // them are done: their values are in registers), then the dG_t rows
    if (t > 0) stage(t - 1, t - 2, true);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (!e_ok[s]) continue;
      const int voff = (int)((((int64_t)t * R + r_lo + e_row[s]) * KD + 4 * uq) * 2);
      // write-through (sc1): team members read these rows in step t - 1
      if (DBG && (a.dbg & 4)) {  // (microbenchmark: plain stores)
        __builtin_amdgcn_raw_buffer_store_b128(u32x4v{ow[s][0], ow[s][1], ow[s][2], ow[s][3]},
                                               r_dg, voff, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4v{ow[s][4], ow[s][5], ow[s][6], ow[s][7]},
                                               r_dg, voff + 16, 0, 0);
        continue;
      }
      __builtin_amdgcn_raw_buffer_store_b128(u32x4v{ow[s][0], ow[s][1], ow[s][2], ow[s][3]}, r_dg,
                                             voff, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4v{ow[s][4], ow[s][5], ow[s][6], ow[s][7]}, r_dg,
                                             voff + 16, 0, 16);
    }
    // 4. publish step t: every storing wave drains (its staging too), then
    // ONE lane signals
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    LP_STAMP(t, 3)
    if (t > 0 && tid == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#undef LP_STAMP
  if (a.dc_out != nullptr) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if (e_ok[s])
        *reinterpret_cast<f32x4v*>(a.dc_out + (int64_t)(r_lo + e_row[s]) * H + uq) = dcr[s];
  }
}

// ---------------------------------------------------------------------------
// K-split form (CSTCAP_BWD_LOOP=2; measured slower than the row-read form
// above, 361.8 vs 331.6 us per loop: the partials' write-through round trip
// through MALL costs what the redundant row reads did): the team's nub
// workgroups split K = 4H instead
// of the hidden units.  Workgroup j of a team owns hidden units [64 j, 64 j +
// 64) for the cell backward, so it PRODUCES the dG columns [256 j, 256 j +
// 256) (4 packed gates x 64 units) -- exactly its K slice of the next step's
// GEMM.  Per step:
//   1. dh partials P_j[rows][all H units] over its own K slice, with the
//      B operand (its dG_{t+1} columns, bf16) already in LDS from its own
//      epilogue -- no global read of dG at all; wave w computes the 64 units
//      of unit block w (A operand: the W_hh^T slice [64 w .. +64) x [256 j ..
//      +256), 128 VGPRs, resident for the whole loop);
//   2. wave w hands P_j[rows][unit block w] (fp32, 12 KB) to workgroup w of
//      the team: write-through (sc1) stores into a parity-double-buffered
//      exchange slab, every wave drains, one lane adds to the team counter
//      (its own partial stays in LDS);
//   3. after the team counter shows every member's partials of this step,
//      the epilogue lanes sum the nub - 1 partials (sc1 loads) and their own,
//      run the cell backward, write dG_t to global memory (plain stores: only
//      later kernels read it) and their K slice of it into the LDS B operand.
// Per step a workgroup moves 7 x 12 KB out and in (headline) instead of
// reading the row block's whole dG rows (160 KB, the same rows by all 8 team
// members).  The exchange slab of parity p is rewritten two steps later, when
// every member has published the step in between -- i.e. finished reading it.
constexpr int LK_BSTRIDE = 528;   // bytes per LDS B row: 256 bf16 + 16 (conflict-free)
constexpr int LK_B_BYTES = LP_MAXR * LK_BSTRIDE;
constexpr int LK_OWN_BYTES = LP_NF * 64 * 16;  // own partial [frag][lane] float4
constexpr int LK_B_OFF = 0, LK_OWN_OFF = LK_B_BYTES, LK_FR_OFF = LK_OWN_OFF + LK_OWN_BYTES;
constexpr int LK_LDS = LK_FR_OFF + LP_NF * LP_FRAG_BYTES;
static_assert(LK_LDS <= 160 * 1024, "K-split reverse loop: LDS budget");
constexpr int LK_SLAB = LP_NF * 64 * 4;  // floats per (dst, src) partial: 12 frags x 64 lanes x 4

__global__ __launch_bounds__(LP_THREADS, 1) void lstm_bwd_ksplit_kernel(BwdLoopArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int H = a.H, R = a.R, T = a.T, KD = 4 * H, nub = a.nub;
  const int g = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int ub = j % nub, rb = j / nub;
  const int team = g * a.nrb + rb;
  const int u0 = 64 * ub;
  const int rg0 = g * a.rows_per_group, rg1 = min(rg0 + a.rows_per_group, R);
  const int r_lo = rg0 + rb * a.rows_per_block;
  const int r_hi = min(r_lo + a.rows_per_block, rg1);
  const int nrows = r_hi - r_lo;  // >= 1 (launcher)
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ru = lane & 15, ku = lane >> 4;
  const bool gemm_wave = w < nub;  // wave w: the partial of unit block w

  // W_hh^T[64 w + 16 ut + ru][256 ub + 32 ks + 8 ku ..]: A fragments, resident
  bf16x8 wf[LP_UT][8];
#pragma unroll
  for (int ut = 0; ut < LP_UT; ++ut)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      wf[ut][ks] = *reinterpret_cast<const bf16x8*>(
          a.whhT + (int64_t)(64 * min(w, nub - 1) + 16 * ut + ru) * KD + 256 * ub + 32 * ks + 8 * ku);

  // epilogue ownership as in lstm_bwd_loop_kernel
  const int e_ut = w & 3;
  const int nslot = w < 4 ? 2 : 1;
  int e_rt[2], e_row[2], e_src[2];
  bool e_ok[2];
  e_rt[0] = w < 4 ? 0 : 1;
  e_rt[1] = 2;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    e_row[s] = 16 * e_rt[s] + ru;
    e_ok[s] = s < nslot && e_row[s] < nrows;
    e_src[s] = r_lo + min(e_row[s], nrows - 1);
  }
  const int uq = u0 + 16 * e_ut + 4 * ku;
  f32x4v dcr[2];
  dcr[0] = dcr[1] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const rsrc_t r_gates = make_rsrc(a.gates, (int64_t)T * R * KD * 2);
  const rsrc_t r_c = make_rsrc(a.c_all, (int64_t)T * R * H * 4);
  const rsrc_t r_dl = make_rsrc(a.dh, (int64_t)T * R * H * 4);
  const float inv_keep = a.drop_p > 0.f ? 1.f / (1.f - a.drop_p) : 1.f;
  const uint32_t seed = rng_seed(a.rng, RNG_SLOT_DROPOUT);
  int* cnt = a.cnt + team * LP_CNT_STRIDE;
  char* b_lds = lds + LK_B_OFF;
  f32x4v* own = reinterpret_cast<f32x4v*>(lds + LK_OWN_OFF);
  char* fr[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) fr[s] = lds + LK_FR_OFF + (e_ut * LP_RT + e_rt[s]) * LP_FRAG_BYTES;
  // exchange slabs: xb[parity][team][dst][src][frag][lane] float4
  const int64_t team_floats = (int64_t)nub * nub * LK_SLAB;
  const int nteams = 8 * a.nrb;
  auto slab = [&](int par, int dst, int src) -> float* {
    return a.xb + ((int64_t)par * nteams + team) * team_floats + ((int64_t)dst * nub + src) * LK_SLAB;
  };
  const rsrc_t r_xb = make_rsrc(a.xb, (int64_t)2 * nteams * team_floats * 4);
  auto stage = [&](int ts, int tc, bool with_gd) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s >= nslot) continue;
      const int64_t row = (int64_t)e_src[s];
      if (with_gd) {
        const int gb = (int)(((ts * (int64_t)R + row) * KD + 4 * uq) * 2);
        dma16(r_gates, gb, fr[s]);
        dma16(r_gates, gb + 16, fr[s] + 1024);
        dma16(r_dl, (int)(((ts * (int64_t)R + row) * H + uq) * 4), fr[s] + 4096);
      }
      if (tc >= 0) dma16(r_c, (int)(((tc * (int64_t)R + row) * H + uq) * 4), fr[s] + 2048 + 1024 * (tc & 1));
    }
  };
  int64_t* ph = a.phases != nullptr ? a.phases + (int64_t)blockIdx.x * T * 4 : nullptr;
#define LK_STAMP(t, k) \
  if (ph != nullptr && tid == 0) ph[(int64_t)(T - 1 - (t)) * 4 + (k)] = (int64_t)wall_clock64();

  stage(T - 1, T - 1, true);
  if (T >= 2) stage(0, T - 2, false);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int t = T - 1; t >= 0; --t) {
    LK_STAMP(t, 0)
    const bool gemm = t + 1 < T;
    const int par = t & 1;
    if (gemm) {
      // 1. partial of unit block w over this workgroup's K slice
      if (gemm_wave) {
        f32x4v acc[LP_UT][LP_RT];
#pragma unroll
        for (int ut = 0; ut < LP_UT; ++ut)
#pragma unroll
          for (int rt = 0; rt < LP_RT; ++rt) acc[ut][rt] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          bf16x8 bq[LP_RT];
#pragma unroll
          for (int rt = 0; rt < LP_RT; ++rt)
            bq[rt] = *reinterpret_cast<const bf16x8*>(b_lds + (16 * rt + ru) * LK_BSTRIDE +
                                                      2 * (32 * ks + 8 * ku));
#pragma unroll
          for (int ut = 0; ut < LP_UT; ++ut)
#pragma unroll
            for (int rt = 0; rt < LP_RT; ++rt)
              acc[ut][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ut][ks], bq[rt], acc[ut][rt],
                                                                    0, 0, 0);
        }
        LK_STAMP(t, 1)
        // 2. hand-off: own unit block into LDS, the others write-through
        if (w == ub) {
#pragma unroll
          for (int ut = 0; ut < LP_UT; ++ut)
#pragma unroll
            for (int rt = 0; rt < LP_RT; ++rt) own[(ut * LP_RT + rt) * 64 + lane] = acc[ut][rt];
        } else {
          const int base = (int)((slab(par, w, ub) - a.xb) * 4);
#pragma unroll
          for (int ut = 0; ut < LP_UT; ++ut)
#pragma unroll
            for (int rt = 0; rt < LP_RT; ++rt)
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, acc[ut][rt]), r_xb,
                                                     base + ((ut * LP_RT + rt) * 64 + lane) * 16, 0,
                                                     16);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
      __syncthreads();
      if (tid == 0) {
        __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int target = nub * (T - 1 - t);
        bool ok = false;
        for (int it = 0; it < a.poll_bound; ++it) {
          if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) {
            ok = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (!ok && a.err != nullptr)
          __hip_atomic_fetch_add(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler order only)
    }
    LK_STAMP(t, 2)

    // 3. the sum of the team's partials + cell backward of the lane's slots
    uint32_t ow[2][8];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s >= nslot) continue;
      const int f = e_ut * LP_RT + e_rt[s];
      f32x4v dh4 = f32x4v{0.f, 0.f, 0.f, 0.f};
      if (gemm) {
        f32x4v pv[7];
#pragma unroll
        for (int q = 0; q < 7; ++q) {  // (sources past nub - 1: loaded clamped, not added)
          const int src = min(q < ub ? q : q + 1, nub - 1);
          const int off = (int)((slab(par, ub, src) - a.xb) * 4) + (f * 64 + lane) * 16;
          pv[q] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r_xb, off, 0, 16));
        }
        dh4 = own[f * 64 + lane];
#pragma unroll
        for (int q = 0; q < 7; ++q)
          if (q < nub - 1) dh4 += pv[q];
      }
      const uint4 gq0 = reinterpret_cast<const uint4*>(fr[s])[lane];
      const uint4 gq1 = reinterpret_cast<const uint4*>(fr[s] + 1024)[lane];
      const f32x4v ct = reinterpret_cast<const f32x4v*>(fr[s] + 2048 + 1024 * (t & 1))[lane];
      const f32x4v cp = t > 0 ? reinterpret_cast<const f32x4v*>(fr[s] + 2048 + 1024 * ((t - 1) & 1))[lane]
                              : f32x4v{0.f, 0.f, 0.f, 0.f};
      const f32x4v dl = reinterpret_cast<const f32x4v*>(fr[s] + 4096)[lane];
      const uint32_t gw[8] = {gq0.x, gq0.y, gq0.z, gq0.w, gq1.x, gq1.y, gq1.z, gq1.w};
      const int r = r_lo + e_row[s];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int u = uq + k;
        const bool keep = a.drop_p <= 0.f || dropout_keep(seed, t, r, u, a.drop_p);
        const float dh = dh4[k] + (keep ? dl[k] * inv_keep : 0.f);
        const uint32_t g01 = gw[2 * k], g23 = gw[2 * k + 1];
        const CellBwd cb = cell_bwd(a.cell, dh, dcr[s][k], bf2f(g01 & 0xffff), bf2f(g01 >> 16),
                                    bf2f(g23 & 0xffff), bf2f(g23 >> 16), ct[k], cp[k]);
        dcr[s][k] = cb.carry;
        ow[s][2 * k] = (uint32_t)f2bf(cb.d0) | ((uint32_t)f2bf(cb.d1) << 16);
        ow[s][2 * k + 1] = (uint32_t)f2bf(cb.d2) | ((uint32_t)f2bf(cb.d3) << 16);
      }
    }
    // 4. step t - 1's staged operands (this wave's own fragments), dG_t out:
    // global (later kernels) and this workgroup's K slice into the B operand
    if (t > 0) stage(t - 1, t - 2, true);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s >= nslot) continue;
      // B row 16 rt + ru, K bytes [2 x 4 x (uq - u0), + 32): padding rows get
      // their values too (harmless: their partials are never read)
      char* bp = b_lds + e_row[s] * LK_BSTRIDE + 8 * (uq - u0);
      *reinterpret_cast<u32x4v*>(bp) = u32x4v{ow[s][0], ow[s][1], ow[s][2], ow[s][3]};
      *reinterpret_cast<u32x4v*>(bp + 16) = u32x4v{ow[s][4], ow[s][5], ow[s][6], ow[s][7]};
      if (e_ok[s]) {
        uint16_t* dst = a.dG + (((int64_t)t * R + r_lo + e_row[s]) * KD + 4 * uq);
        *reinterpret_cast<u32x4v*>(dst) = u32x4v{ow[s][0], ow[s][1], ow[s][2], ow[s][3]};
        *reinterpret_cast<u32x4v*>(dst + 8) = u32x4v{ow[s][4], ow[s][5], ow[s][6], ow[s][7]};
      }
    }
    // the B operand complete (LDS writes); the staging DMA and the dG stores
    // are drained by the next step's hand-off wait, before its epilogue
    __syncthreads();
    LK_STAMP(t, 3)
  }
#undef LK_STAMP
  if (a.dc_out != nullptr) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if (e_ok[s])
        *reinterpret_cast<f32x4v*>(a.dc_out + (int64_t)(r_lo + e_row[s]) * H + uq) = dcr[s];
  }
}

// dl = scale * dh + a W[ys] + b W[yx] in place, one wavefront per row (the
// loop reads the folded rows; lstm_bwd_loop_fold)
__global__ __launch_bounds__(256) void lstm_bwd_fold_kernel(BwdLoopArgs a, int64_t NR) {
  if (blockIdx.x == 0)  // the loop's team counters (the loop launch follows on this stream)
    for (int i = threadIdx.x; i < 8 * a.nrb * LP_CNT_STRIDE; i += 256) a.cnt[i] = 0;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= NR) return;
  const int lane = threadIdx.x & 63, H = a.H;
  const float sc = a.scale != nullptr ? a.scale[row] : 1.f;
  const float wa = a.oh_a != nullptr ? a.oh_a[row] : 0.f;
  const float wb = a.oh_b != nullptr ? a.oh_b[row] : 0.f;
  const int ys = a.oh_a != nullptr ? max(a.oh_ys[row], 0) : 0;
  const int yx = a.oh_b != nullptr ? max(a.oh_yx[row], 0) : 0;
  float* d = const_cast<float*>(a.dh) + row * H;
  for (int u = 4 * lane; u < H; u += 256) {
    f32x4v x = *reinterpret_cast<const f32x4v*>(d + u) * sc;
    if (a.oh_a != nullptr) {
      const uint2 q = *reinterpret_cast<const uint2*>(a.oh_W + (int64_t)ys * H + u);
      x[0] = fmaf(wa, bf2f(q.x & 0xffff), x[0]);
      x[1] = fmaf(wa, bf2f(q.x >> 16), x[1]);
      x[2] = fmaf(wa, bf2f(q.y & 0xffff), x[2]);
      x[3] = fmaf(wa, bf2f(q.y >> 16), x[3]);
    }
    if (a.oh_b != nullptr) {
      const uint2 q = *reinterpret_cast<const uint2*>(a.oh_W + (int64_t)yx * H + u);
      x[0] = fmaf(wb, bf2f(q.x & 0xffff), x[0]);
      x[1] = fmaf(wb, bf2f(q.x >> 16), x[1]);
      x[2] = fmaf(wb, bf2f(q.y & 0xffff), x[2]);
      x[3] = fmaf(wb, bf2f(q.y >> 16), x[3]);
    }
    *reinterpret_cast<f32x4v*>(d + u) = x;
  }
}

struct LoopGeom {
  int nub, nrb, rows_per_group, rows_per_block, grid;
};

LoopGeom loop_geom(int R, int H) {
  LoopGeom g{};
  g.nub = H / 64;
  g.rows_per_group = (R + 7) / 8;
  g.nrb = (g.rows_per_group + LP_MAXR - 1) / LP_MAXR;
  g.rows_per_block = (g.rows_per_group + g.nrb - 1) / g.nrb;
  g.grid = 8 * g.nub * g.nrb;
  return g;
}

int cu_count() {
  static int n = -1;
  if (n < 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 0;
  }
  return n;
}

}  // namespace

bool lstm_bwd_loop_ok(int R, int H, int T) {
  if (T < 1 || R < 8 || (H != 128 && H != 256 && H != 512)) return false;
  const LoopGeom g = loop_geom(R, H);
  // every group and row block non-empty; one workgroup per CU, all resident
  if (g.rows_per_group * 7 >= R || (g.nrb - 1) * g.rows_per_block >= g.rows_per_group) return false;
  if ((int64_t)T * R * 4 * H * 2 >= (1LL << 31) || (int64_t)T * R * H * 4 >= (1LL << 31)) return false;
  return g.grid <= cu_count();
}

int lstm_bwd_loop_counter_ints(int R, int H) {
  const LoopGeom g = loop_geom(R, H);
  return 8 * g.nrb * LP_CNT_STRIDE;
}

int64_t lstm_bwd_loop_xb_floats(int R, int H) {
  const LoopGeom g = loop_geom(R, H);
  return (int64_t)2 * 8 * g.nrb * g.nub * g.nub * LK_SLAB;
}

void launch_lstm_bwd_loop(BwdLoopArgs a, hipStream_t stream) {
  if (!lstm_bwd_loop_ok(a.R, a.H, a.T)) throw std::runtime_error("lstm_bwd_loop: unsupported shape");
  const LoopGeom g = loop_geom(a.R, a.H);
  a.nub = g.nub;
  a.nrb = g.nrb;
  a.rows_per_group = g.rows_per_group;
  a.rows_per_block = g.rows_per_block;
  if (a.scale != nullptr || a.oh_a != nullptr) {
    // the row scales and one-hot rows folded into dh (in place) first; the
    // fold also zeroes the team counters (one memset node less between X and
    // the loop)
    const int64_t NR = (int64_t)a.T * a.R;
    hipLaunchKernelGGL(lstm_bwd_fold_kernel, dim3((unsigned)((NR + 3) / 4)), dim3(256), 0, stream,
                       a, NR);
    post_launch("lstm_bwd_fold_kernel", stream);
  } else {
    // team counters: zeroed by a memset node ahead of every launch
    (void)hipMemsetAsync(a.cnt, 0, sizeof(int) * 8 * g.nrb * LP_CNT_STRIDE, stream);
  }
#define LP_LAUNCH(KSV, DB)                                                                      \
  {                                                                                             \
    static bool attr = false;                                                                   \
    if (!attr) {                                                                                \
      (void)hipFuncSetAttribute((const void*)lstm_bwd_loop_kernel<KSV, DB>,                     \
                                hipFuncAttributeMaxDynamicSharedMemorySize, LP_LDS);            \
      attr = true;                                                                              \
    }                                                                                           \
    hipLaunchKernelGGL((lstm_bwd_loop_kernel<KSV, DB>), dim3(g.grid), dim3(LP_THREADS), LP_LDS,    \
                       stream, a);                                                              \
  }
  if (a.form == 0) {  // K-split (CSTCAP_BWD_LOOP=2)
    if (a.xb == nullptr) throw std::runtime_error("lstm_bwd_loop: K-split form needs the exchange slabs");
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)lstm_bwd_ksplit_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, LK_LDS);
      attr = true;
    }
    hipLaunchKernelGGL(lstm_bwd_ksplit_kernel, dim3(g.grid), dim3(LP_THREADS), LK_LDS, stream, a);
  } else if (a.dbg != 0) {
    if (a.H != 512) throw std::runtime_error("lstm_bwd_loop: debug variants at H = 512 only");
    LP_LAUNCH(8, true)
  } else {
    switch (a.H) {
      case 128: LP_LAUNCH(2, false) break;
      case 256: LP_LAUNCH(4, false) break;
      default: LP_LAUNCH(8, false) break;
    }
  }
#undef LP_LAUNCH
  post_launch("lstm_bwd_loop_kernel", stream);
}

}  // namespace cst
