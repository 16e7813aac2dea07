// Temporal attention, forward of one decode step, on MFMA (K11-ext; the
// model and its reference anchors are described in attention.hip).  Used as
// extra workgroups of the merged decode launch (vocab.hip
// vocab_lstm_fwd_kernel): the attention of step t+1 depends only on h_t, like
// the recurrent GEMM of that launch, so it runs concurrently with the
// vocabulary tiles of step t instead of as a launch of its own between the
// decode launch and the combine.
//
// A video's attention is split over NS = A / 64 workgroups of 256 threads
// (4 waves): workgroup (b, s) owns the 64 query units [64 s, 64 s + 64) and
// all rows of video b (rows_per_video <= 32: two 16-row MFMA column tiles).
//   1. q^T = W_q[units] h_t^T     (64 x 32, K = H)  v_mfma_f32_16x16x32_bf16.
//      The video's h_t rows (32 x H bf16) are staged ONCE per workgroup in LDS
//      by LDS-DMA (16-byte chunks XOR-swizzled by row on the source address,
//      so the B-fragment ds_read_b128 of 16 rows is bank-conflict free); wave
//      w streams its 16 W_q rows straight into registers, every k-step's
//      fragment requested up front (one memory round trip for the GEMM).
//      In the output layout a lane holds 4 consecutive units of one row per
//      column tile, so the tanh scorer's sum over units is register-local;
//   2. partial scores sum_{a in slice} w_a tanh(P[b, c, a] + q_r[a]) (P / w_a
//      of the slice in LDS, 16-byte broadcast reads), combined over the 4 lane
//      groups and the 4 waves, stored to the workgroup's slot with
//      write-through (sc1) stores; one agent-scope ticket add per workgroup;
//   3. the video's LAST workgroup (ticket NS - 1; the hand-off is write-through
//      (sc1) slot stores, drained by every storing wave's s_waitcnt vmcnt(0)
//      and a workgroup barrier before ONE lane's agent-scope ticket add, and
//      sc1 loads of the slots by the workgroup that drew the last ticket: no
//      L1 line of another CU and no unflushed L2 line of another XCD is ever
//      read) sums the NS slots, adds b_a, takes the softmax over
//      frames and forms vgate^T = Gv[b]^T alpha^T (4H x 32, K = 16 frames) on
//      MFMA (v_mfma_f32_32x32x16_bf16): A operand = the per-frame gate table
//      in frame-minor bf16 layout gv16[b][n][CP], requested before the slot
//      loads; B operand = alpha (bf16, LDS).  A lane's output registers
//      4g..4g+3 are the 4 packed gates of one hidden unit of its row: one
//      8-byte store each into the bf16 per-row video-gate buffer that the
//      combine's cell epilogue adds.  It re-arms the ticket.
// No load is conditional (the compiler branches around, and waits for, each
// conditional load): indices are clamped and values masked instead.
// Training also stores alpha (R x C) and q (R x A, fp32) for the backward.
#pragma once
#include "gemm_tile.h"
#include "../launchers.h"

namespace cst {

constexpr int ATT_SLICE = 64;  // query units per workgroup

// LDS bytes of one attention workgroup: h rows (32 x H bf16), P slice
// (C x 64 fp32), w_a slice, wave partial scores (4 x 32 x CP), alpha bf16
// (32 x 16), ticket flag
__host__ __device__ constexpr int att_mfma_lds_bytes(int C, int CP, int H) {
  return 32 * H * 2 + (C * ATT_SLICE + ATT_SLICE + 4 * 32 * CP) * 4 + 32 * 16 * 2 + 16;
}

__device__ __forceinline__ bf16x8 ld_bf16x8(const uint16_t* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

typedef float f32x4v __attribute__((ext_vector_type(4)));

// phase stamp of a workgroup (microbenchmark only: AttMfmaArgs::dbg)
__device__ __forceinline__ void att_phase(const AttMfmaArgs& g, int blk, int k) {
  if (g.dbg != nullptr && threadIdx.x == 0) g.dbg[blk * 8 + k] = (int64_t)wall_clock64();
}

// CP: frames padded to 8 / 16.  blk = b * NS + s.
template <int CP>
__device__ __forceinline__ void att_mfma_fwd_block(int blk, const AttMfmaArgs& g, char* lds) {
  const int A = g.A, H = g.H, C = g.C, G4 = g.G4, vdiv = g.vdiv, NS = A / ATT_SLICE;
  const int b = blk / NS, s = blk - b * NS;
  uint16_t* s_h = reinterpret_cast<uint16_t*>(lds);  // [32][H], chunks swizzled
  float* s_P = reinterpret_cast<float*>(lds + 32 * H * 2);  // [C][64]
  float* s_wa = s_P + C * ATT_SLICE;
  float* s_e = s_wa + ATT_SLICE;
  uint16_t* s_alb = reinterpret_cast<uint16_t*>(s_e + 4 * 32 * CP);
  int* s_flag = reinterpret_cast<int*>(s_alb + 32 * 16);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row0 = b * vdiv, a0 = s * ATT_SLICE;
  att_phase(g, blk, 0);
  // h rows of the video -> LDS by LDS-DMA (rows >= vdiv repeat the last row)
  const int cpr = H / 8;  // 16-byte chunks per row
  const int swm = (cpr < 16 ? cpr : 16) - 1;
  {
    const rsrc_t rh = make_rsrc(g.h + (int64_t)row0 * H, (int64_t)vdiv * H * 2);
    const int nins = 32 * H * 2 / 1024;  // 1 KiB wave-instructions
    for (int i = w; i < nins; i += 4) {
      const int e = i * 64 + lane;  // chunk of the LDS image
      const int row = e / cpr, ch = e % cpr;
      const int src = min(row, vdiv - 1) * cpr + (ch ^ (row & swm));
      glds16(rh, src * 16, 0, reinterpret_cast<char*>(s_h) + 1024 * i);
    }
  }
  // W_q fragments of this wave (16 units), all k-steps requested at once
  const int ku = lane >> 4, ru = lane & 15;  // k group / row within a 16-row tile
  constexpr int MAXK = 16;                   // H <= 512: K / 32 k-steps
  const int nks = H / 32;
  const uint16_t* wrow = g.wq + (int64_t)(a0 + 16 * w + ru) * H + 8 * ku;
  bf16x8 af[MAXK];
#pragma unroll
  for (int k = 0; k < MAXK; ++k) af[k] = ld_bf16x8(wrow + 32 * min(k, nks - 1));
  // P slice and w_a
  for (int i = tid; i < C * (ATT_SLICE / 4); i += 256) {
    const int c = i / (ATT_SLICE / 4), k = i % (ATT_SLICE / 4);
    reinterpret_cast<float4*>(s_P)[i] =
        reinterpret_cast<const float4*>(g.P + ((int64_t)b * C + c) * A + a0)[k];
  }
  if (tid < ATT_SLICE / 4)
    reinterpret_cast<float4*>(s_wa)[tid] = reinterpret_cast<const float4*>(g.wa + a0)[tid];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // h rows, P, w_a in LDS
  att_phase(g, blk, 1);
  // 1. q^T tiles (16 units x 16 rows) x 2 row tiles
  f32x4v acc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) acc[j] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    if (k < nks) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = 16 * j + ru, ch = 4 * k + ku;
        const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(
            reinterpret_cast<const char*>(s_h) + row * H * 2 + ((ch ^ (row & swm)) << 4));
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k], bfr, acc[j], 0, 0, 0);
      }
    }
  }
  // lane: units u0 .. u0 + 3 (registers 0..3) of rows 16 j + ru
  const int u0 = 16 * w + 4 * ku;
  att_phase(g, blk, 2);
  if (g.q_out != nullptr) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = 16 * j + ru;
      if (row < vdiv)
        *reinterpret_cast<float4*>(g.q_out + (int64_t)(row0 + row) * A + a0 + u0) =
            make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
    }
  }
  // 2. partial scores of the slice, one frame per iteration
  const float4 wv = *reinterpret_cast<const float4*>(s_wa + u0);
  for (int c = 0; c < C; ++c) {
    const float4 p = *reinterpret_cast<const float4*>(s_P + c * ATT_SLICE + u0);
    float ec[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float t0 = tanh_fast(p.x + acc[j][0]), t1 = tanh_fast(p.y + acc[j][1]);
      const float t2 = tanh_fast(p.z + acc[j][2]), t3 = tanh_fast(p.w + acc[j][3]);
      ec[j] = wv.x * t0;
      ec[j] = fmaf(wv.y, t1, ec[j]);
      ec[j] = fmaf(wv.z, t2, ec[j]);
      ec[j] = fmaf(wv.w, t3, ec[j]);
      const int row = 16 * j + ru;
      if (g.u_out != nullptr && row < vdiv)  // the backward's scorer values (fp16, u_enc)
        *reinterpret_cast<uint2*>(g.u_out + ((int64_t)(row0 + row) * C + c) * A + a0 + u0) =
            make_uint2((uint32_t)u_enc(t0) | ((uint32_t)u_enc(t1) << 16),
                       (uint32_t)u_enc(t2) | ((uint32_t)u_enc(t3) << 16));
      ec[j] += __shfl_xor(ec[j], 16, 64);
      ec[j] += __shfl_xor(ec[j], 32, 64);
    }
    if (ku == 0) {
      s_e[(w * 32 + ru) * CP + c] = ec[0];
      s_e[(w * 32 + 16 + ru) * CP + c] = ec[1];
    }
  }
  __syncthreads();
  att_phase(g, blk, 3);
  // the slice's partial (rows x frames) -> its slot, write-through (sc1)
  float* slot = g.e_part + ((int64_t)b * NS + s) * 32 * CP;
  for (int i = tid; i < 32 * CP; i += 256) {
    const int rr = i / CP, c = i % CP;
    const float v = s_e[rr * CP + c] + s_e[(32 + rr) * CP + c] + s_e[(64 + rr) * CP + c] +
                    s_e[(96 + rr) * CP + c];
    __hip_atomic_store(slot + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    // sc1 slot stores drained by vmcnt(0) above, sc1 slot loads below: the
    // no-fence hand-off form (see loss.hip scst_loss_fwd_kernel)
    const int ticket = __hip_atomic_fetch_add(g.cnt + b, 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    *s_flag = ticket == NS - 1;
  }
  __syncthreads();
  att_phase(g, blk, 4);
  if (!*s_flag) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler order only)
  // 3. last workgroup of the video: scores, softmax, vgate.  The gate-table
  // tiles do not depend on alpha: all of this wave's are requested first, so
  // their latency overlaps the slot loads and the softmax.
  const int hh = lane >> 5, r = lane & 31;
  const int ntw = G4 / 128;  // vgate tiles per wave
  constexpr int MAXT = 16;   // 4H <= 2048
  const uint16_t* gvb = g.gv16 + (int64_t)b * G4 * CP;
  const bool ghalf = CP == 16 || hh == 0;  // CP = 8: frames 8..15 are zero
  bf16x8 ga[MAXT];
#pragma unroll
  for (int i = 0; i < MAXT; ++i) {
    const int n0 = (w * ntw + min(i, ntw - 1)) * 32;
    ga[i] = ld_bf16x8(gvb + (int64_t)(n0 + r) * CP + (CP == 16 ? 8 * hh : 0));
  }
  if (tid == 0) g.cnt[b] = 0;  // re-arm for the next step (stream-ordered)
  const float ba = g.ba[0];      // (requested with the slot loads)
  // the NS slots summed per (row, frame): one pair per thread, all slot loads
  // of a thread out together (sc1, the hand-off's loads)
  {
    constexpr int MAXS = 16;  // A <= 1024
    for (int i = tid; i < 32 * CP; i += 256) {
      const float* sl = g.e_part + (int64_t)b * NS * 32 * CP + i;
      float v[MAXS];
#pragma unroll
      for (int k = 0; k < MAXS; ++k)
        v[k] = __hip_atomic_load(sl + (int64_t)min(k, NS - 1) * 32 * CP, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < MAXS; ++k) t += k < NS ? v[k] : 0.f;
      s_e[i] = t;  // (the wave partials are consumed: reused)
    }
  }
  __syncthreads();
  att_phase(g, blk, 5);
  if (tid < 32) {
    float x[CP], mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < CP; ++c) x[c] = s_e[tid * CP + c] + ba;
#pragma unroll
    for (int c = 0; c < CP; ++c)
      if (c < C) mx = fmaxf(mx, x[c]);
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < CP; ++c) {
      x[c] = c < C ? __expf(x[c] - mx) : 0.f;
      sum += x[c];
    }
    const float inv = 1.f / sum;
    const bool ok = tid < vdiv;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const float al = (c < CP && c < C && ok) ? x[c < CP ? c : 0] * inv : 0.f;
      s_alb[tid * 16 + c] = f2bf(al);
      if (c < C && ok && g.alpha_out != nullptr) g.alpha_out[(int64_t)(row0 + tid) * C + c] = al;
    }
  }
  __syncthreads();
  att_phase(g, blk, 7);
  // vgate tiles (32 rows x 32 gate columns): 4H / 32 tiles over the 4 waves.
  // A = alpha (rows), B = the gate table (columns): a lane then holds one
  // gate column of 16 rows, so each store instruction writes two rows' 64-byte
  // runs (32 lanes = 32 consecutive columns).  (With the gate table as A a
  // lane held 16 columns of ONE row: every store instruction scattered 64
  // 8-byte pieces over 32 rows, ~7 us of the last workgroup's tail at the
  // headline shape, scripts/microbench_att.py phase stamps.)
  const bf16x8 bal = ld_bf16x8(s_alb + r * 16 + 8 * hh);
  const bf16x8 zero8 = {};
  // the 16 output rows of this lane: one pointer each, formed once (the
  // tile's column offset is then an immediate of the store)
  uint16_t* prow[16];
  bool vrow[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int row = (k & 3) + 8 * (k >> 2) + 4 * hh;
    vrow[k] = row < vdiv;
    prow[k] = g.vg_out + (int64_t)(row0 + min(row, vdiv - 1)) * G4 + w * ntw * 32 + r;
  }
#pragma unroll
  for (int i = 0; i < MAXT; ++i) {
    f32x16 o;
#pragma unroll
    for (int k = 0; k < 16; ++k) o[k] = 0.f;
    o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bal, ghalf ? ga[i] : zero8, o, 0, 0, 0);
    if (i < ntw) {
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (vrow[k]) prow[k][32 * i] = f2bf(o[k]);
    }
  }
  att_phase(g, blk, 6);
}

// Whole-video form (AttMfmaArgs::whole): ONE workgroup per video loops over
// the A / 64 query slices -- the video's h rows staged once, each slice's W_q
// fragments requested while the previous slice's scores are formed -- and
// accumulates the scores in LDS: no partial-score slots, no ticket, no
// last-arriver hand-off, and Bv instead of Bv * A / 64 workgroups ahead of the
// vocabulary tiles of the decode launch (at the att8 shape 64 instead of 512
// workgroups holding CU slots while the vocabulary tiles wait).  Then the
// softmax and vgate^T = Gv^T alpha^T exactly as the last arriver above.
// Opt-in (CSTCAP_ATT_WHOLE=1): the slices in sequence outlast the vocabulary
// tiles (att8 decode launch 63.8 vs 48.9 us, profiles/r6/s2/att_whole/).
__host__ __device__ constexpr int att_mfma_video_lds_bytes(int C, int CP, int H) {
  return att_mfma_lds_bytes(C, CP, H) + 32 * CP * 4;
}

template <int CP>
__device__ __forceinline__ void att_mfma_fwd_video(int b, const AttMfmaArgs& g, char* lds) {
  const int A = g.A, H = g.H, C = g.C, G4 = g.G4, vdiv = g.vdiv, NS = A / ATT_SLICE;
  uint16_t* s_h = reinterpret_cast<uint16_t*>(lds);  // [32][H], chunks swizzled
  float* s_P = reinterpret_cast<float*>(lds + 32 * H * 2);  // [C][64]
  float* s_wa = s_P + C * ATT_SLICE;
  float* s_e = s_wa + ATT_SLICE;
  uint16_t* s_alb = reinterpret_cast<uint16_t*>(s_e + 4 * 32 * CP);
  float* s_acc = reinterpret_cast<float*>(lds + att_mfma_lds_bytes(C, CP, H));  // [32][CP]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row0 = b * vdiv;
  const int cpr = H / 8;
  const int swm = (cpr < 16 ? cpr : 16) - 1;
  {
    const rsrc_t rh = make_rsrc(g.h + (int64_t)row0 * H, (int64_t)vdiv * H * 2);
    const int nins = 32 * H * 2 / 1024;
    for (int i = w; i < nins; i += 4) {
      const int e = i * 64 + lane;
      const int row = e / cpr, ch = e % cpr;
      const int src = min(row, vdiv - 1) * cpr + (ch ^ (row & swm));
      glds16(rh, src * 16, 0, reinterpret_cast<char*>(s_h) + 1024 * i);
    }
  }
  for (int i = tid; i < 32 * CP; i += 256) s_acc[i] = 0.f;
  const int ku = lane >> 4, ru = lane & 15;
  constexpr int MAXK = 16;
  const int nks = H / 32;
  const int u0 = 16 * w + 4 * ku;
  bf16x8 af[MAXK];
  auto load_wq = [&](int s) {
    const uint16_t* wrow = g.wq + (int64_t)(s * ATT_SLICE + 16 * w + ru) * H + 8 * ku;
#pragma unroll
    for (int k = 0; k < MAXK; ++k) af[k] = ld_bf16x8(wrow + 32 * min(k, nks - 1));
  };
  load_wq(0);
  for (int s = 0; s < NS; ++s) {
    const int a0 = s * ATT_SLICE;
    for (int i = tid; i < C * (ATT_SLICE / 4); i += 256) {
      const int c = i / (ATT_SLICE / 4), k = i % (ATT_SLICE / 4);
      reinterpret_cast<float4*>(s_P)[i] =
          reinterpret_cast<const float4*>(g.P + ((int64_t)b * C + c) * A + a0)[k];
    }
    if (tid < ATT_SLICE / 4)
      reinterpret_cast<float4*>(s_wa)[tid] = reinterpret_cast<const float4*>(g.wa + a0)[tid];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // h rows (first slice), P, w_a in LDS; s_acc zeroed
    f32x4v acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < MAXK; ++k) {
      if (k < nks) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int row = 16 * j + ru, ch = 4 * k + ku;
          const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(
              reinterpret_cast<const char*>(s_h) + row * H * 2 + ((ch ^ (row & swm)) << 4));
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k], bfr, acc[j], 0, 0, 0);
        }
      }
    }
    // the next slice's W_q fragments, in flight under this slice's scores
    if (s + 1 < NS) load_wq(s + 1);
    if (g.q_out != nullptr) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = 16 * j + ru;
        if (row < vdiv)
          *reinterpret_cast<float4*>(g.q_out + (int64_t)(row0 + row) * A + a0 + u0) =
              make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
      }
    }
    const float4 wv = *reinterpret_cast<const float4*>(s_wa + u0);
    for (int c = 0; c < C; ++c) {
      const float4 p = *reinterpret_cast<const float4*>(s_P + c * ATT_SLICE + u0);
      float ec[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float t0 = tanh_fast(p.x + acc[j][0]), t1 = tanh_fast(p.y + acc[j][1]);
        const float t2 = tanh_fast(p.z + acc[j][2]), t3 = tanh_fast(p.w + acc[j][3]);
        ec[j] = wv.x * t0;
        ec[j] = fmaf(wv.y, t1, ec[j]);
        ec[j] = fmaf(wv.z, t2, ec[j]);
        ec[j] = fmaf(wv.w, t3, ec[j]);
        const int row = 16 * j + ru;
        if (g.u_out != nullptr && row < vdiv)
          *reinterpret_cast<uint2*>(g.u_out + ((int64_t)(row0 + row) * C + c) * A + a0 + u0) =
              make_uint2((uint32_t)u_enc(t0) | ((uint32_t)u_enc(t1) << 16),
                         (uint32_t)u_enc(t2) | ((uint32_t)u_enc(t3) << 16));
        ec[j] += __shfl_xor(ec[j], 16, 64);
        ec[j] += __shfl_xor(ec[j], 32, 64);
      }
      if (ku == 0) {
        s_e[(w * 32 + ru) * CP + c] = ec[0];
        s_e[(w * 32 + 16 + ru) * CP + c] = ec[1];
      }
    }
    __syncthreads();  // s_e complete; s_P / s_wa reads done
    for (int i = tid; i < 32 * CP; i += 256) {
      const int rr = i / CP, c = i % CP;
      s_acc[i] += s_e[rr * CP + c] + s_e[(32 + rr) * CP + c] + s_e[(64 + rr) * CP + c] +
                  s_e[(96 + rr) * CP + c];
    }
  }
  // softmax over frames and vgate (as the last arriver of att_mfma_fwd_block)
  const int hh = lane >> 5, r = lane & 31;
  const int ntw = G4 / 128;
  constexpr int MAXT = 16;
  const uint16_t* gvb = g.gv16 + (int64_t)b * G4 * CP;
  const bool ghalf = CP == 16 || hh == 0;
  bf16x8 ga[MAXT];
#pragma unroll
  for (int i = 0; i < MAXT; ++i) {
    const int n0 = (w * ntw + min(i, ntw - 1)) * 32;
    ga[i] = ld_bf16x8(gvb + (int64_t)(n0 + r) * CP + (CP == 16 ? 8 * hh : 0));
  }
  const float ba = g.ba[0];
  __syncthreads();  // s_acc complete
  if (tid < 32) {
    float x[CP], mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < CP; ++c) x[c] = s_acc[tid * CP + c] + ba;
#pragma unroll
    for (int c = 0; c < CP; ++c)
      if (c < C) mx = fmaxf(mx, x[c]);
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < CP; ++c) {
      x[c] = c < C ? __expf(x[c] - mx) : 0.f;
      sum += x[c];
    }
    const float inv = 1.f / sum;
    const bool ok = tid < vdiv;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const float al = (c < CP && c < C && ok) ? x[c < CP ? c : 0] * inv : 0.f;
      s_alb[tid * 16 + c] = f2bf(al);
      if (c < C && ok && g.alpha_out != nullptr) g.alpha_out[(int64_t)(row0 + tid) * C + c] = al;
    }
  }
  __syncthreads();
  const bf16x8 bal = ld_bf16x8(s_alb + r * 16 + 8 * hh);
  const bf16x8 zero8 = {};
  uint16_t* prow[16];
  bool vrow[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int row = (k & 3) + 8 * (k >> 2) + 4 * hh;
    vrow[k] = row < vdiv;
    prow[k] = g.vg_out + (int64_t)(row0 + min(row, vdiv - 1)) * G4 + w * ntw * 32 + r;
  }
#pragma unroll
  for (int i = 0; i < MAXT; ++i) {
    f32x16 o;
#pragma unroll
    for (int k = 0; k < 16; ++k) o[k] = 0.f;
    o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bal, ghalf ? ga[i] : zero8, o, 0, 0, 0);
    if (i < ntw) {
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (vrow[k]) prow[k][32 * i] = f2bf(o[k]);
    }
  }
}

// attention variant of a kernel template: 0 = none, else the padded frame
// count CP (8 or 16)
constexpr int att_variant(int C) { return C <= 8 ? 8 : 16; }
// workgroups of one step's attention
__host__ __device__ constexpr int att_mfma_blocks(int Bv, int A) { return Bv * (A / ATT_SLICE); }
__host__ __device__ inline int att_mfma_nblocks(const AttMfmaArgs& a) {
  return a.whole ? a.Bv : att_mfma_blocks(a.Bv, a.A);
}
// one attention workgroup of either form
template <int CP>
__device__ __forceinline__ void att_mfma_fwd_any(int blk, const AttMfmaArgs& g, char* lds) {
  if (g.whole)
    att_mfma_fwd_video<CP>(blk, g, lds);
  else
    att_mfma_fwd_block<CP>(blk, g, lds);
}

}  // namespace cst
