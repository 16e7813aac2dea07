// Temporal-attention forward block (K11-ext), shared by the stand-alone
// kernel (attention.hip) and the merged decode launch (vocab.hip), where
// these blocks ride behind the vocabulary tiles; see attention.hip for the
// design.
#pragma once
#include "../common.h"
#include "../launchers.h"

namespace cst {


constexpr int ATT_THREADS = 256, ATT_RPW = 4, ATT_WAVES = ATT_THREADS / WAVE;

// Butterfly all-reduce of N (32 or 64) per-lane partial sums across the 64
// lanes of a wave in log2(64) exchange steps: each step a lane keeps half of
// its values and adds the partner's copy of them, so the wave spends N-1
// shuffles instead of 6 N for N separate reductions.  Afterwards lane l holds
// the total of value index (l >> (6 - log2 N)) in v[0].
template <int N, int M>
struct Bfly {
  static __device__ __forceinline__ void run(float* v, int lane) {
    constexpr int H = N / 2;
    const bool up = (lane & M) != 0;
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const float send = up ? v[i] : v[i + H];
      const float keep = up ? v[i + H] : v[i];
      v[i] = keep + __shfl_xor(send, M, WAVE);
    }
    Bfly<H, M / 2>::run(v, lane);
  }
};
template <int M>
struct Bfly<1, M> {
  static __device__ __forceinline__ void run(float* v, int lane) {
    v[0] += __shfl_xor(v[0], M, WAVE);
    Bfly<1, M / 2>::run(v, lane);
  }
};
template <>
struct Bfly<1, 0> {
  static __device__ __forceinline__ void run(float*, int) {}
};

// Sum of RPW x MAXC per-thread partials over the whole block -> s_out
// (index s * MAXC + c); s_red holds ATT_WAVES x RPW x MAXC floats.
template <int MAXC, int RPW = ATT_RPW>
__device__ __forceinline__ void block_sum_partials(float (&part)[RPW][MAXC], float* s_red,
                                                   float* s_out) {
  constexpr int N = RPW * MAXC;
  constexpr int CH = N < 64 ? N : 64;  // butterfly chunk (a power of two, >= 2)
  static_assert((CH & (CH - 1)) == 0 && CH >= 2, "butterfly chunk");
  // after the butterfly lane l holds value (l >> SH): one writer per value
  constexpr int SH = CH == 64 ? 0 : CH == 32 ? 1 : CH == 16 ? 2 : CH == 8 ? 3 : CH == 4 ? 4 : 5;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* flat = &part[0][0];
#pragma unroll
  for (int c0 = 0; c0 < N; c0 += CH) {
    Bfly<CH, 32>::run(flat + c0, lane);
    if ((lane & ((1 << SH) - 1)) == 0) s_red[w * N + c0 + (lane >> SH)] = flat[c0];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < N; i += ATT_THREADS) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < ATT_WAVES; ++k) t += s_red[k * N + i];
    s_out[i] = t;
  }
  __syncthreads();
}

// Column groups (float4) of the 4H gate vector a thread prefetches into
// registers: 2 x 256 threads x 4 = 2048 = 4H at H = 512 (larger H loops).
constexpr int ATT_GPF = 2;

// grid: Bv * ngroups blocks; block (b, g) owns rows b*vdiv + g*RPW ... (< (b+1)*vdiv)
// Scores: thread t owns attention units a = t + 256 j and accumulates the
// partial dot products of all RPW x C (row, frame) pairs over them (its own
// columns of P[b] and q: coalesced loads, no LDS staging), then one butterfly
// + cross-wave sum finishes every score at once.
template <int MAXC, int RPW>
__device__ __forceinline__ void att_fwd_block(int bid, const AttFwdArgs& args) {
  const float* __restrict__ gv = args.gv;
  const float* __restrict__ pre = args.pre;
  const float* __restrict__ q = args.q;
  const int* __restrict__ q_rowmap = args.q_rowmap;
  const float* __restrict__ wa = args.wa;
  const float* __restrict__ ba = args.ba;
  const int wa_ld = args.wa_ld, ba_ld = args.ba_ld, vdiv = args.vdiv, ngroups = args.ngroups;
  const int C = args.C, A = args.A, G4 = args.G4, accumulate = args.accumulate;
  float* __restrict__ vg_out = args.vg_out;
  float* __restrict__ alpha_out = args.alpha_out;
  __shared__ float s_red[ATT_WAVES * RPW * MAXC];
  __shared__ float s_e[RPW * MAXC];
  const int b = bid / ngroups, g = bid % ngroups;
  const int r0 = b * vdiv + g * RPW, nr = min(RPW, vdiv - g * RPW);
  const int tid = threadIdx.x;
  const float4* G = reinterpret_cast<const float4*>(gv + (int64_t)b * C * G4);
  const int G44 = G4 >> 2;
  // the video's frame gate rows (L2-resident, shared by its row groups) are
  // requested first: their latency hides under the scores
  // (register prefetch only for C <= 8: 2 x 8 float4 = 64 VGPRs)
  const bool gpf = MAXC <= 8 && G44 <= ATT_GPF * ATT_THREADS;
  float4 gr[ATT_GPF][MAXC];
  if (gpf) {
#pragma unroll
    for (int j = 0; j < ATT_GPF; ++j)
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
        gr[j][c] = (c < C && tid + j * ATT_THREADS < G44)
                       ? G[(int64_t)c * G44 + tid + j * ATT_THREADS]
                       : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // accumulate: the rows' current pre-activations (written by the previous
  // launch) are requested up front too, so the final add does not wait on a
  // second memory round trip
  float4 acc0[ATT_GPF][RPW];
  if (gpf && accumulate) {
#pragma unroll
    for (int j = 0; j < ATT_GPF; ++j)
#pragma unroll
      for (int s = 0; s < RPW; ++s)
        acc0[j][s] = (s < nr && tid + j * ATT_THREADS < G44)
                         ? reinterpret_cast<const float4*>(vg_out + (int64_t)(r0 + s) * G4)[tid + j * ATT_THREADS]
                         : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // the softmax thread's frame biases, requested now (not after the reduction)
  float bap[MAXC <= 8 ? MAXC : 1];
  if (MAXC <= 8 && tid < nr) {
#pragma unroll
    for (int c = 0; c < (MAXC <= 8 ? MAXC : 1); ++c) bap[c] = c < C ? ba[c * ba_ld] : 0.f;
  }
  int qrow[RPW];
#pragma unroll
  for (int s = 0; s < RPW; ++s) {
    const int r = r0 + min(s, nr - 1);
    qrow[s] = q_rowmap ? q_rowmap[r] : r;
    CST_DCHECK(qrow[s] >= 0);
  }
  CST_DCHECK(nr >= 1 && g * RPW + nr <= vdiv);
  float part[RPW][MAXC];
#pragma unroll
  for (int s = 0; s < RPW; ++s)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) part[s][c] = 0.f;
  const float* P = pre + (int64_t)b * C * A;
  // A <= 512 (C <= 8): every unit's query / frame / scorer operand is
  // requested in ONE batch (a single memory round trip instead of one per
  // unit group); the latency-bound kernel has registers to spare
  constexpr int AJ = 2;
  if (MAXC <= 8 && A <= AJ * ATT_THREADS) {
    float qv[AJ][RPW], pcv[AJ][MAXC], wav[AJ][MAXC];
#pragma unroll
    for (int j = 0; j < AJ; ++j) {
      const int a = tid + j * ATT_THREADS;
      const bool ok = a < A;
#pragma unroll
      for (int s = 0; s < RPW; ++s)
        qv[j][s] = (ok && q != nullptr) ? q[(int64_t)qrow[s] * A + a] : 0.f;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        wav[j][c] = (ok && c < C) ? wa[c * wa_ld + a] : 0.f;  // 0: no contribution
        pcv[j][c] = (ok && c < C) ? P[(int64_t)c * A + a] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < AJ; ++j)
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int s = 0; s < RPW; ++s) part[s][c] += wav[j][c] * tanhf_(pcv[j][c] + qv[j][s]);
  } else {
    for (int a = tid; a < A; a += ATT_THREADS) {
      float qv[RPW];
#pragma unroll
      for (int s = 0; s < RPW; ++s) qv[s] = q != nullptr ? q[(int64_t)qrow[s] * A + a] : 0.f;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        if (c < C) {
          const float wa_a = wa[c * wa_ld + a];
          const float pc = P[(int64_t)c * A + a];
#pragma unroll
          for (int s = 0; s < RPW; ++s) part[s][c] += wa_a * tanhf_(pc + qv[s]);
        }
      }
    }
  }
  block_sum_partials<MAXC, RPW>(part, s_red, s_e);
  if (tid < nr) {  // softmax over frames, one thread per row
    float* e = s_e + tid * MAXC;
    float m = -INFINITY;
    if (MAXC <= 8) {
#pragma unroll
      for (int c = 0; c < (MAXC <= 8 ? MAXC : 1); ++c)
        if (c < C) {
          e[c] += bap[c];
          m = fmaxf(m, e[c]);
        }
    } else {
      for (int c = 0; c < C; ++c) {
        e[c] += ba[c * ba_ld];
        m = fmaxf(m, e[c]);
      }
    }
    float sum = 0.f;
    for (int c = 0; c < C; ++c) {
      const float x = __expf(e[c] - m);
      e[c] = x;
      sum += x;
    }
    const float inv = 1.f / sum;
    for (int c = 0; c < C; ++c) {
      e[c] *= inv;
      if (alpha_out) alpha_out[(int64_t)(r0 + tid) * C + c] = e[c];
    }
  }
  __syncthreads();
  // vgate_r = sum_c alpha_rc Gv[b, c]: each thread owns float4 column groups
  auto emit = [&](int cg, const float4* gcol, int pj) {  // pj: prefetched group, or -1
    float4 acc[RPW];
#pragma unroll
    for (int s = 0; s < RPW; ++s) acc[s] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c < C) {
        const float4 v = gcol[c];
#pragma unroll
        for (int s = 0; s < RPW; ++s) {
          const float al = s_e[min(s, nr - 1) * MAXC + c];
          acc[s].x += al * v.x;
          acc[s].y += al * v.y;
          acc[s].z += al * v.z;
          acc[s].w += al * v.w;
        }
      }
    }
#pragma unroll
    for (int s = 0; s < RPW; ++s) {
      if (s < nr) {
        float4* dst = reinterpret_cast<float4*>(vg_out + (int64_t)(r0 + s) * G4) + cg;
        if (accumulate) {
          float4 o;
          if (pj >= 0) {
#pragma unroll
            for (int j = 0; j < ATT_GPF; ++j)
              if (j == pj) o = acc0[j][s];
          } else {
            o = *dst;
          }
          acc[s].x += o.x, acc[s].y += o.y, acc[s].z += o.z, acc[s].w += o.w;
        }
        *dst = acc[s];
      }
    }
  };
  if (gpf) {
#pragma unroll
    for (int j = 0; j < ATT_GPF; ++j)
      if (tid + j * ATT_THREADS < G44) emit(tid + j * ATT_THREADS, gr[j], j);
  } else {
    for (int cg = tid; cg < G44; cg += ATT_THREADS) {
      float4 gcol[MAXC];
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
        gcol[c] = c < C ? G[(int64_t)c * G44 + cg] : make_float4(0.f, 0.f, 0.f, 0.f);
      emit(cg, gcol, -1);
    }
  }
}


}  // namespace cst
