// Device timeline stamps (SURVEY.md 5.1 tracing): a one-thread kernel that
// writes the GPU's constant-rate wall clock (100 MHz on MI355X) into a slot
// of a device buffer, enqueued at phase boundaries on the stream that runs
// the phase.  Inside a replayed HIP graph the stamps are graph nodes on the
// branches they were captured on, so unlike a profiler (rocprofv3 serialises
// a replayed graph onto one queue) they show the step's real concurrency:
// when the greedy branch starts, how long the reverse loop waits, which side
// stream ends last before Adam.  Disabled (no buffer registered) the
// launcher enqueues nothing, so a captured graph has no stamp nodes.
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

}  // namespace cst
