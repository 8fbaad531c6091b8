// Hardware-queue probe: do two HIP streams share a hardware queue?
//
// HIP maps every stream onto one of a bounded set of hardware queues when the stream is
// created (GPU_MAX_HW_QUEUES per priority level); streams that land on the same queue
// serialise, whatever their event dependencies say.  For the pipeline runtime that is a
// correctness question, not only a performance one: an RCCL kernel blocks its queue until
// the peer rank arrives, so a compute or channel stream stuck behind it on a shared queue
// can close a cross-rank wait cycle (parallel/queues.py).
//
// The probe is a bounded spin/flag pair:
//   waiter stream:  spin_kernel polls a device word until it holds `expect`, or until
//                   `timeout_us` of wall clock (the 100 MHz constant counter) have passed;
//   setter stream:  set_kernel stores `expect` into the word (launched after the spinner).
// If the setter could run while the spinner was resident (separate queues), the spinner
// sees the flag within microseconds; if the two streams share a queue, the setter is
// queued behind the spinner and the spinner times out.  Every wave exits on its own
// deadline, so the probe can never hang the device.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__global__ void spin_kernel(unsigned* flag, unsigned expect, uint64_t timeout_ticks, unsigned* result) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  unsigned seen = 0;
  uint64_t t = t0;
  // the iteration cap is a second exit in case the clock does not advance
  for (uint64_t it = 0; it < (1ull << 34); ++it) {
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == expect) {
      seen = 1;
      break;
    }
    t = wall_clock64();
    if (t - t0 > timeout_ticks) break;
    __builtin_amdgcn_s_sleep(4);
  }
  result[0] = seen;
  result[1] = (unsigned)(t - t0);  // ticks of the constant clock until the flag or the deadline
}

__global__ void set_kernel(unsigned* flag, unsigned value) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

extern "C" {

// Enqueue the spinner on `waiter` (flag/result are device buffers of >= 1 / 2 words; the
// caller zeroes the flag first).  Returns a HIP error code.
int mp_probe_spin(unsigned* flag, unsigned expect, int64_t timeout_us, unsigned* result, hipStream_t waiter) {
  int rate_khz = 0;
  int dev = 0;
  hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || rate_khz <= 0)
    rate_khz = 100000;  // MI300/MI355 constant clock: 100 MHz
  const uint64_t ticks = (uint64_t)timeout_us * (uint64_t)rate_khz / 1000ull;
  spin_kernel<<<1, 64, 0, waiter>>>(flag, expect, ticks, result);
  return (int)hipGetLastError();
}

int mp_probe_set(unsigned* flag, unsigned value, hipStream_t setter) {
  set_kernel<<<1, 64, 0, setter>>>(flag, value);
  return (int)hipGetLastError();
}

int mp_probe_clock_khz() {
  int rate_khz = 0, dev = 0;
  hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return 0;
  return rate_khz;
}
}
