// Host-only stand-in (csrc/tests/host_asan_test.cpp): the current stream is one fake stream.
#pragma once
#include <hip/hip_runtime.h>
#include <map>
namespace c10 {
namespace hip {
struct HIPStream {
  hipStream_t s = nullptr;
  hipStream_t stream() const { return s; }
};
// one current stream per device (two ranks of one test process sit on devices 0 and 1)
inline hipStream_t fake_current(int device) {
  static std::map<int, hipStream_t> s;
  auto it = s.find(device);
  if (it == s.end()) it = s.emplace(device, fake_hip::make_stream()).first;
  return it->second;
}
inline HIPStream getCurrentHIPStream(int device = 0) { return HIPStream{fake_current(device)}; }
inline HIPStream getStreamFromExternal(hipStream_t s, int) { return HIPStream{s}; }
}  // namespace hip
}  // namespace c10
