// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels.
//
// Conventions used by every kernel in csrc/kernels:
//   * wavefront = 64 lanes; block sizes are multiples of 64;
//   * bf16 values travel as raw 16-bit patterns (uint16_t / short vectors) and
//     are bit-cast to __bf16 vectors only at the MFMA call;
//   * all launchers take an explicit hipStream_t (the caller passes PyTorch's
//     current HIP stream) and never synchronise or allocate, so the whole
//     decoder step can be captured in a HIP graph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <stdexcept>
#include <string>

namespace cst {

// ---- debugging aids -------------------------------------------
// Device-side bounds checks, compiled in by the debug build
// (CSTCAP_KERNEL_DEBUG=1 python setup.py build_ext --inplace, which adds
// -DCST_KERNEL_DEBUG): a failed check prints the condition and the block /
// thread and execution continues on the kernel's own clamped index (no trap:
// a trapping wave can take the whole node down on the shared pool).
#ifdef CST_KERNEL_DEBUG
#define CST_DCHECK(cond)                                                               \
  do {                                                                                 \
    if (!(cond))                                                                       \
      printf("CST_DCHECK failed %s:%d: %s (block %d, thread %d)\n", __FILE__, __LINE__, \
             #cond, (int)blockIdx.x, (int)threadIdx.x);                                \
  } while (0)
#else
#define CST_DCHECK(cond) \
  do {                   \
  } while (0)
#endif

// Host-side launch checking, after every kernel launch of the runtime:
// CSTCAP_LAUNCH_CHECK=1 -> hipGetLastError (bad grid / LDS / arguments);
// CSTCAP_LAUNCH_CHECK=2 -> also synchronise the stream, so an asynchronous
// fault is reported against the kernel that caused it (HIP_LAUNCH_BLOCKING
// for this runtime only).  Raises std::runtime_error (RuntimeError in Python).
inline int launch_check_mode() {
  static const int mode = [] {
    const char* e = getenv("CSTCAP_LAUNCH_CHECK");
    return e ? atoi(e) : 0;
  }();
  return mode;
}
inline void post_launch(const char* kernel, hipStream_t stream) {
  const int mode = launch_check_mode();
  if (mode == 0) return;
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && mode > 1) {
    // (a stream being captured into a graph cannot be synchronised: the
    // launch is checked, the fault check happens when the graph runs)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(stream, &cs);
    if (cs == hipStreamCaptureStatusNone) e = hipStreamSynchronize(stream);
  }
  if (e != hipSuccess)
    throw std::runtime_error(std::string("HIP error after ") + kernel + ": " +
                             hipGetErrorString(e));
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int WAVE = 64;

__device__ __forceinline__ float bf2f(uint16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}

// round-to-nearest-even f32 -> bf16 (hardware v_cvt_pk_bf16_f32; NaN stays NaN)
__device__ __forceinline__ uint16_t f2bf(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}

__device__ __forceinline__ float h2f(uint16_t h) {
  return (float)__builtin_bit_cast(_Float16, h);
}
__device__ __forceinline__ uint16_t f2h(float f) {
  return __builtin_bit_cast(uint16_t, (_Float16)f);
}
// 4 consecutive fp16 values (8 bytes) as a float4 (the fp16 gate tables:
// the projected-embedding table P and the recurrent pre-activations)
__device__ __forceinline__ float4 ld_h4(const uint16_t* p) {
  const uint2 q = *reinterpret_cast<const uint2*>(p);
  return make_float4(h2f(q.x & 0xffff), h2f(q.x >> 16), h2f(q.y & 0xffff), h2f(q.y >> 16));
}
__device__ __forceinline__ uint2 pack_h4(float a, float b, float c, float d) {
  return make_uint2((uint32_t)f2h(a) | ((uint32_t)f2h(b) << 16),
                    (uint32_t)f2h(c) | ((uint32_t)f2h(d) << 16));
}

// fast gate nonlinearities: one exp + one reciprocal each (rel. err ~1e-6)
__device__ __forceinline__ float sigmoidf_(float x) {
  return __builtin_amdgcn_rcpf(1.f + __expf(-x));
}
__device__ __forceinline__ float tanhf_(float x) {
  const float e = __expf(-2.f * fabsf(x));
  const float t = (1.f - e) * __builtin_amdgcn_rcpf(1.f + e);
  return copysignf(t, x);
}
// attention scorer tanh: tanh(x) = 1 - 2 / (exp(2x) + 1): one exp, one
// reciprocal, three plain ops (saturates to +-1 through exp -> inf / 0); the
// forward (att_mfma.h) and backward scorers use the same form
__device__ __forceinline__ float tanh_fast(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);
  return fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
}

// Scorer value u = tanh(.) of the temporal attention as ONE fp16 word for the
// backward: v = 1 - |u| with u's sign.  The backward needs u and 1 - u^2 =
// v (2 - v); stored as u itself, 1 - u^2 cancels near saturation (|u| -> 1:
// fp16 spacing 2^-11 below 1, up to 100 % relative error of the tanh
// derivative), while v keeps fp16's relative precision exactly there; for
// small |u| the absolute error of u stays below 2^-12.
__device__ __forceinline__ uint16_t u_enc(float u) { return f2h(copysignf(1.f - fabsf(u), u)); }
struct UDec {
  float u, d;  // u and 1 - u^2
};
__device__ __forceinline__ UDec u_dec(uint16_t h) {
  const float x = h2f(h), v = fabsf(x);
  return UDec{copysignf(1.f - v, x), v * (2.f - v)};
}

// murmur3 32-bit finaliser: avalanche hash used as a counter-based RNG for
// the per-element sampling draws (hash(row-key ^ v * odd constant)).
__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// ---- wave64 reductions --------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- Philox4x32-10 counter-based RNG ------------------------------------------
// Deterministic per (seed, counter): the same draw is regenerated in backward
// (dropout masks) and is independent of launch geometry.
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32(u32x4 ctr, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    u32x4 n;
    n.x = hi1 ^ ctr.y ^ k0;
    n.y = lo1;
    n.z = hi0 ^ ctr.w ^ k1;
    n.w = lo0;
    ctr = n;
    k0 += W0;
    k1 += W1;
  }
  return ctr;
}

// uniform in (0, 1]: never 0, so log() is finite
__device__ __forceinline__ float u01(uint32_t r) {
  return ((float)(r >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// RNG streams (the `z` word of the counter)
enum RngStream : uint32_t {
  RNG_GUMBEL = 1,     // multinomial rollout sampling (Gumbel-max)
  RNG_DROPOUT_H = 2,  // dropout on h before the vocab projection
  RNG_SS = 3,         // scheduled-sampling coin per row
};

// Per-pass RNG seeds live in DEVICE memory (int32[2], drawn by the caller with
// torch.randint on the GPU), not in kernel arguments: a captured HIP graph
// replays its kernel arguments verbatim, so seeds passed by value would repeat
// the same dropout masks and samples on every replay.  The backward reads the
// same two words as its forward, so it regenerates the forward's masks.
enum RngSlot : int { RNG_SLOT_DROPOUT = 0, RNG_SLOT_SAMPLE = 1 };
__device__ __forceinline__ uint32_t rng_seed(const uint32_t* rng, int slot) {
  return rng != nullptr ? rng[slot] : 0u;
}

// ---- recurrent cells ------------------------------------------------------------
// Every cell is computed from 4 packed pre-activation slots per hidden unit
// (packed row 4u + g of the gate GEMMs; the caller packs the weights):
//   LSTM (PyTorch i, f, g, o):  c = f c' + i g,  h = o tanh(c)
//   GRU  (PyTorch r, z, n):     slots (r, z, n_x, n_h) -- the input part of n
//        (x / video terms) and its recurrent part (W_hn h) stay separate:
//        n = tanh(n_x + r n_h),  h = (1 - z) n + z h'
//   RNN  (tanh):                slot 0 only, h = tanh(a0)
// The "c" state buffers carry h in fp32 for GRU / RNN.  Saved gate slots
// (bf16) for the backward: LSTM (i, f, g, o); GRU (r, z, n, n_h); RNN (h, -).
enum CellType : int { CELL_LSTM = 0, CELL_GRU = 1, CELL_RNN_TANH = 2 };

struct CellFwd {
  float h, c, s0, s1, s2, s3;
};
__device__ __forceinline__ CellFwd cell_fwd(int cell, float a0, float a1, float a2, float a3,
                                            float cp) {
  CellFwd o;
  if (cell == CELL_LSTM) {
    const float gi = sigmoidf_(a0), gf = sigmoidf_(a1), gg = tanhf_(a2), go = sigmoidf_(a3);
    o.c = gf * cp + gi * gg;
    o.h = go * tanhf_(o.c);
    o.s0 = gi, o.s1 = gf, o.s2 = gg, o.s3 = go;
  } else if (cell == CELL_GRU) {
    const float r = sigmoidf_(a0), z = sigmoidf_(a1);
    const float n = tanhf_(a2 + r * a3);
    o.h = (1.f - z) * n + z * cp;
    o.c = o.h;
    o.s0 = r, o.s1 = z, o.s2 = n, o.s3 = a3;
  } else {
    o.h = tanhf_(a0);
    o.c = o.h;
    o.s0 = o.h, o.s1 = o.s2 = o.s3 = 0.f;
  }
  return o;
}

// Cell backward: dh = gradient reaching h_t (recurrent GEMM + logit path),
// carry = the state gradient carried from step t+1 (LSTM: into c_t; GRU /
// RNN: into h_t); c_t / cp = this / previous step's state.  Returns the
// 4 packed slot gradients and the carry for step t-1.
struct CellBwd {
  float d0, d1, d2, d3, carry;
};
__device__ __forceinline__ CellBwd cell_bwd(int cell, float dh, float carry, float s0, float s1,
                                            float s2, float s3, float c_t, float cp) {
  CellBwd o;
  if (cell == CELL_LSTM) {
    const float tc = tanhf_(c_t);
    const float dc = carry + dh * s3 * (1.f - tc * tc);
    o.d0 = dc * s2 * s0 * (1.f - s0);
    o.d1 = dc * cp * s1 * (1.f - s1);
    o.d2 = dc * s0 * (1.f - s2 * s2);
    o.d3 = dh * tc * s3 * (1.f - s3);
    o.carry = dc * s1;
  } else if (cell == CELL_GRU) {
    const float r = s0, z = s1, n = s2, nh = s3;
    const float d = dh + carry;
    const float dz = d * (cp - n);
    const float da2 = d * (1.f - z) * (1.f - n * n);
    const float dr = da2 * nh;
    o.d0 = dr * r * (1.f - r);
    o.d1 = dz * z * (1.f - z);
    o.d2 = da2;
    o.d3 = da2 * r;
    o.carry = d * z;
  } else {
    const float d = dh + carry;
    o.d0 = d * (1.f - s0 * s0);
    o.d1 = o.d2 = o.d3 = 0.f;
    o.carry = 0.f;
  }
  return o;
}

// Keep-mask of dropout on element (row, col) of step t: a counter hash, so the
// backward regenerates exactly the forward's mask.
__device__ __forceinline__ bool dropout_keep(uint32_t seed, int step, int row, int col,
                                             float p) {
  const uint32_t h = mix32(mix32(seed ^ ((uint32_t)step * 0x9E3779B1u) ^ (uint32_t)row * 0x7FEB352Du) ^
                           (uint32_t)col * 0x846CA68Bu);
  return u01(h) > p;
}

}  // namespace cst
