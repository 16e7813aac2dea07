// Device timeline stamps (SURVEY.md 5.1 tracing): a one-thread kernel that
// writes the GPU's constant-rate wall clock (100 MHz on MI355X) into a slot
// of a device buffer, enqueued at phase boundaries on the stream that runs
// the phase.  Inside a replayed HIP graph the stamps are graph nodes on the
// branches they were captured on, so unlike a profiler (rocprofv3 serialises
// a replayed graph onto one queue) they show the step's real concurrency:
// when the greedy branch starts, how long the reverse loop waits, which side
// stream ends last before Adam.  Disabled (no buffer registered) the
// launcher enqueues nothing, so a captured graph has no stamp nodes.
#include "../common.h"
#include "../launchers.h"

namespace cst {

static int64_t* g_stamp_buf = nullptr;
static int g_stamp_slots = 0;

__global__ void stamp_kernel(int64_t* __restrict__ buf, int slot) {
  buf[slot] = (int64_t)wall_clock64();
}

void set_stamp_buffer(int64_t* buf, int slots) {
  g_stamp_buf = buf;
  g_stamp_slots = buf != nullptr ? slots : 0;
}

bool stamps_enabled() { return g_stamp_buf != nullptr; }

void launch_stamp(int slot, hipStream_t stream) {
  if (g_stamp_buf == nullptr || slot < 0 || slot >= g_stamp_slots) return;
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(1), 0, stream, g_stamp_buf, slot);
}

// Stand-in for a collective's kernel (tests / scripts of the DP overlap): a
// grid of `blocks` 256-thread workgroups that stream copies through their own
// slice of `buf` (one 16-byte load + store per thread and pass, HBM traffic
// like a ring all-reduce's channels) until `ticks` of the wall clock have
// passed since each workgroup started.  Every wave reaches the exit: the loop
// condition is the wave's own clock read.
__global__ __launch_bounds__(256) void busy_copy_kernel(float4* __restrict__ buf, int64_t n4_per_block,
                                                         int64_t ticks) {
  float4* seg = buf + (int64_t)blockIdx.x * n4_per_block;
  const int64_t half = n4_per_block / 2;
  const int64_t t0 = (int64_t)wall_clock64();
  int64_t i = threadIdx.x;
  while ((int64_t)wall_clock64() - t0 < ticks) {
    for (int k = 0; k < 16; ++k) {
      seg[half + i] = seg[i];
      i += 256;
      if (i >= half) i = threadIdx.x;
    }
  }
}

void launch_busy_copy(float* buf, int64_t n_floats, int blocks, double us, hipStream_t stream) {
  if (blocks < 1 || n_floats < (int64_t)blocks * 2048)
    throw std::runtime_error("busy_copy: buffer smaller than 8 KB per workgroup");
  int khz = 0;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  if (khz <= 0) khz = 100000;
  const int64_t ticks = (int64_t)(us * 1e-3 * khz);
  const int64_t n4 = (n_floats / 4) / blocks / 512 * 512;
  hipLaunchKernelGGL(busy_copy_kernel, dim3(blocks), dim3(256), 0, stream,
                     reinterpret_cast<float4*>(buf), n4, ticks);
  post_launch("busy_copy_kernel", stream);
}

}  // namespace cst
