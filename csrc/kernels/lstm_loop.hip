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
// LDS: K-partials [wave][fragment][lane] float4, then the staged epilogue
// operands, rows padded by one 16-byte chunk (conflict-free ds_read_b128 of
// 16 consecutive rows at the same column)
constexpr int LP_PART_BYTES = LP_WAVES * LP_NF * 64 * 16;
constexpr int LP_GSTRIDE = 33, LP_CSTRIDE = 17;  // 16-byte chunks per staged row
// (each staged operand reserves whole 1 KB DMA instructions)
constexpr int LP_G_BYTES = (LP_MAXR * LP_GSTRIDE + 63) / 64 * 1024;
constexpr int LP_C_BYTES = (LP_MAXR * LP_CSTRIDE + 63) / 64 * 1024;
constexpr int LP_G_OFF = LP_PART_BYTES;
constexpr int LP_CT_OFF = LP_G_OFF + LP_G_BYTES;
constexpr int LP_CP_OFF = LP_CT_OFF + LP_C_BYTES;
constexpr int LP_DL_OFF = LP_CP_OFF + LP_C_BYTES;
constexpr int LP_LDS = LP_DL_OFF + LP_C_BYTES;
static_assert(LP_LDS <= 160 * 1024, "persistent reverse loop: LDS budget");
constexpr int LP_CNT_STRIDE = 32;  // ints between team counters (128 B)

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 ld_sc1_b128(rsrc_t r, int voff) {
  const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 16);  // 16: sc1
  return __builtin_bit_cast(bf16x8, v);
}

// one staged operand: rows [0, nrows) x `chunks` 16-byte chunks of the
// global rows (row stride `gstride` bytes, column offset `goff`), to LDS rows
// of `stride` chunks; instruction k of the operand fills LDS chunks
// [64 k, 64 k + 64)
__device__ __forceinline__ void stage_rows(rsrc_t r, int64_t row0_bytes, int gstride, int goff,
                                           int nrows, int chunks, int stride, char* lds, int k,
                                           int lane) {
  const int p = 64 * k + lane;
  int row = p / stride, c = p - row * stride;
  // padding chunks and rows past the block reload a valid chunk (harmless)
  c = c < chunks ? c : chunks - 1;
  row = row < nrows ? row : nrows - 1;
  const int voff = (int)(row0_bytes + (int64_t)row * gstride) + goff + 16 * c;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(lds + 1024 * k), 16, voff, 0, 0, 0);
}

template <int KS>
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
  int e_rt[2], e_row[2];
  bool e_ok[2];
  e_rt[0] = w < 4 ? 0 : 1;
  e_rt[1] = 2;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    e_row[s] = 16 * e_rt[s] + ru;  // local row
    e_ok[s] = s < nslot && e_row[s] < nrows;
  }
  const int q = 4 * e_ut + ku;  // unit quad within the 64 units
  const int uq = u0 + 4 * q;    // first global unit of the quad
  f32x4v dcr[2];
  dcr[0] = dcr[1] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const rsrc_t r_dg = make_rsrc(a.dG, (int64_t)T * R * KD * 2);
  const rsrc_t r_gates = make_rsrc(a.gates, (int64_t)T * R * KD * 2);
  const rsrc_t r_c = make_rsrc(a.c_all, (int64_t)T * R * H * 4);
  const rsrc_t r_dl = make_rsrc(a.dh, (int64_t)T * R * H * 4);
  const int n_g = (nrows * LP_GSTRIDE + 63) / 64, n_c = (nrows * LP_CSTRIDE + 63) / 64;
  const float inv_keep = a.drop_p > 0.f ? 1.f / (1.f - a.drop_p) : 1.f;
  const uint32_t seed = rng_seed(a.rng, RNG_SLOT_DROPOUT);
  int* cnt = a.cnt + team * LP_CNT_STRIDE;
  f32x4v* part = reinterpret_cast<f32x4v*>(lds);
  // (microbenchmark: per-step phase stamps of every workgroup, lane 0 of wave 0)
  int64_t* ph = a.phases != nullptr ? a.phases + (int64_t)blockIdx.x * T * 4 : nullptr;
#define LP_STAMP(t, k) \
  if (ph != nullptr && tid == 0) ph[(int64_t)(T - 1 - (t)) * 4 + (k)] = (int64_t)wall_clock64();

  for (int t = T - 1; t >= 0; --t) {
    LP_STAMP(t, 0)
    // 1. stage step t's epilogue operands (waves 1..7; wave 0 polls)
    if (w > 0) {
      const int n_ins = n_g + n_c * (t > 0 ? 3 : 2);
      for (int k = w - 1; k < n_ins; k += LP_WAVES - 1) {
        if (k < n_g) {
          stage_rows(r_gates, ((int64_t)t * R + r_lo) * KD * 2, KD * 2, u0 * 8, nrows, 32,
                     LP_GSTRIDE, lds + LP_G_OFF, k, lane);
        } else {
          const int kk = k - n_g, which = kk / n_c, kc = kk - which * n_c;
          // which: 0 = dh_logit, 1 = c_t, 2 = c_{t-1}
          const int ts = which == 2 ? t - 1 : t;
          stage_rows(which == 0 ? r_dl : r_c, ((int64_t)ts * R + r_lo) * H * 4, H * 4, u0 * 4,
                     nrows, 16, LP_CSTRIDE,
                     lds + (which == 0 ? LP_DL_OFF : which == 1 ? LP_CT_OFF : LP_CP_OFF), kc,
                     lane);
        }
      }
    }
    // the per-row scalars of the thread's rows (plain loads: not written here)
    float e_sc[2], e_a[2], e_b[2];
    uint2 e_w[2], e_wx[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int r = r_lo + min(e_row[s], nrows - 1);
      const int64_t tr = (int64_t)t * R + r;
      e_sc[s] = a.scale != nullptr ? a.scale[tr] : 1.f;
      e_a[s] = 0.f;
      e_b[s] = 0.f;
      e_w[s] = e_wx[s] = make_uint2(0u, 0u);
      if (a.oh_a != nullptr) {
        e_a[s] = a.oh_a[tr];
        e_w[s] = *reinterpret_cast<const uint2*>(a.oh_W + (int64_t)max(a.oh_ys[tr], 0) * H + uq);
      }
      if (a.oh_b != nullptr) {
        e_b[s] = a.oh_b[tr];
        e_wx[s] = *reinterpret_cast<const uint2*>(a.oh_W + (int64_t)max(a.oh_yx[tr], 0) * H + uq);
      }
    }

    // 2. dh_rec = dG_{t+1} W_hh over this wave's K range, summed over waves
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
      // two K-steps of B fragments in flight ahead of the MFMAs
      bf16x8 bq[2][LP_RT];
#pragma unroll
      for (int rt = 0; rt < LP_RT; ++rt) bq[0][rt] = ld_sc1_b128(r_dg, boff[rt]);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + 1 < KS) {
#pragma unroll
          for (int rt = 0; rt < LP_RT; ++rt)
            bq[(ks + 1) & 1][rt] = ld_sc1_b128(r_dg, boff[rt] + 64 * (ks + 1));
        }
#pragma unroll
        for (int ut = 0; ut < LP_UT; ++ut)
#pragma unroll
          for (int rt = 0; rt < LP_RT; ++rt)
            acc[ut][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ut][ks], bq[ks & 1][rt],
                                                                  acc[ut][rt], 0, 0, 0);
      }
#pragma unroll
      for (int ut = 0; ut < LP_UT; ++ut)
#pragma unroll
        for (int rt = 0; rt < LP_RT; ++rt) part[(w * LP_NF + ut * LP_RT + rt) * 64 + lane] = acc[ut][rt];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // staged operands landed (every wave)
    __syncthreads();
    LP_STAMP(t, 2)

    // 3. cell backward of the thread's (row, 4 units) slots
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (!e_ok[s]) continue;
      const int i = e_row[s], r = r_lo + i;
      f32x4v dh4 = f32x4v{0.f, 0.f, 0.f, 0.f};
      if (gemm) {
        const int f = e_ut * LP_RT + e_rt[s];
#pragma unroll
        for (int ww = 0; ww < LP_WAVES; ++ww) dh4 += part[(ww * LP_NF + f) * 64 + lane];
      }
      const uint4 gq0 = reinterpret_cast<const uint4*>(lds + LP_G_OFF)[i * LP_GSTRIDE + 2 * q];
      const uint4 gq1 = reinterpret_cast<const uint4*>(lds + LP_G_OFF)[i * LP_GSTRIDE + 2 * q + 1];
      const f32x4v ct = reinterpret_cast<const f32x4v*>(lds + LP_CT_OFF)[i * LP_CSTRIDE + q];
      const f32x4v cp = t > 0 ? reinterpret_cast<const f32x4v*>(lds + LP_CP_OFF)[i * LP_CSTRIDE + q]
                              : f32x4v{0.f, 0.f, 0.f, 0.f};
      f32x4v dl = reinterpret_cast<const f32x4v*>(lds + LP_DL_OFF)[i * LP_CSTRIDE + q] * e_sc[s];
      dl[0] = fmaf(e_a[s], bf2f(e_w[s].x & 0xffff), fmaf(e_b[s], bf2f(e_wx[s].x & 0xffff), dl[0]));
      dl[1] = fmaf(e_a[s], bf2f(e_w[s].x >> 16), fmaf(e_b[s], bf2f(e_wx[s].x >> 16), dl[1]));
      dl[2] = fmaf(e_a[s], bf2f(e_w[s].y & 0xffff), fmaf(e_b[s], bf2f(e_wx[s].y & 0xffff), dl[2]));
      dl[3] = fmaf(e_a[s], bf2f(e_w[s].y >> 16), fmaf(e_b[s], bf2f(e_wx[s].y >> 16), dl[3]));
      const uint32_t gw[8] = {gq0.x, gq0.y, gq0.z, gq0.w, gq1.x, gq1.y, gq1.z, gq1.w};
      uint32_t ow[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int u = uq + k;
        const bool keep = a.drop_p <= 0.f || dropout_keep(seed, t, r, u, a.drop_p);
        const float dh = dh4[k] + (keep ? dl[k] * inv_keep : 0.f);
        const uint32_t g01 = gw[2 * k], g23 = gw[2 * k + 1];
        const CellBwd cb = cell_bwd(a.cell, dh, dcr[s][k], bf2f(g01 & 0xffff), bf2f(g01 >> 16),
                                    bf2f(g23 & 0xffff), bf2f(g23 >> 16), ct[k], cp[k]);
        dcr[s][k] = cb.carry;
        ow[2 * k] = (uint32_t)f2bf(cb.d0) | ((uint32_t)f2bf(cb.d1) << 16);
        ow[2 * k + 1] = (uint32_t)f2bf(cb.d2) | ((uint32_t)f2bf(cb.d3) << 16);
      }
      const int voff = (int)((((int64_t)t * R + r) * KD + 4 * uq) * 2);
      // write-through (sc1): team members read these rows in step t - 1
      __builtin_amdgcn_raw_buffer_store_b128(u32x4v{ow[0], ow[1], ow[2], ow[3]}, r_dg, voff, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4v{ow[4], ow[5], ow[6], ow[7]}, r_dg, voff + 16, 0,
                                             16);
    }
    // 4. publish step t: every storing wave drains, then ONE lane signals
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

void launch_lstm_bwd_loop(BwdLoopArgs a, hipStream_t stream) {
  if (!lstm_bwd_loop_ok(a.R, a.H, a.T)) throw std::runtime_error("lstm_bwd_loop: unsupported shape");
  const LoopGeom g = loop_geom(a.R, a.H);
  a.nub = g.nub;
  a.nrb = g.nrb;
  a.rows_per_group = g.rows_per_group;
  a.rows_per_block = g.rows_per_block;
  // team counters: zeroed by a memset node ahead of every launch
  (void)hipMemsetAsync(a.cnt, 0, sizeof(int) * 8 * g.nrb * LP_CNT_STRIDE, stream);
#define LP_LAUNCH(KSV)                                                                          \
  {                                                                                             \
    static bool attr = false;                                                                   \
    if (!attr) {                                                                                \
      (void)hipFuncSetAttribute((const void*)lstm_bwd_loop_kernel<KSV>,                         \
                                hipFuncAttributeMaxDynamicSharedMemorySize, LP_LDS);            \
      attr = true;                                                                              \
    }                                                                                           \
    hipLaunchKernelGGL(lstm_bwd_loop_kernel<KSV>, dim3(g.grid), dim3(LP_THREADS), LP_LDS, stream, \
                       a);                                                                      \
  }
  switch (a.H) {
    case 128: LP_LAUNCH(2) break;
    case 256: LP_LAUNCH(4) break;
    default: LP_LAUNCH(8) break;
  }
#undef LP_LAUNCH
  post_launch("lstm_bwd_loop_kernel", stream);
}

}  // namespace cst
