// Host-only stand-in for the HIP runtime API the native runtime uses (csrc/tests/host_asan_test.cpp).
//
// Streams are FIFOs of work items; events are HEAP objects (new / delete) so a use after
// hipEventDestroy, a double destroy or a leaked event is an AddressSanitizer / LeakSanitizer
// report.  Work runs when the test drains the streams (fake_drain): an event fires when its
// stream reaches it, a stream blocked by hipStreamWaitEvent resumes when that event fired.
#pragma once
#include <atomic>
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <set>

enum hipError_t { hipSuccess = 0, hipErrorNotReady = 600, hipErrorInvalidValue = 1 };
enum hipMemcpyKind { hipMemcpyDeviceToDevice = 3 };
constexpr unsigned hipEventDisableTiming = 2;
constexpr unsigned hipStreamNonBlocking = 1;

struct FakeEvent;
struct FakeStream {
  std::deque<std::function<bool()>> work;   // an item returns false while it must wait
};
struct FakeEvent {
  uint64_t magic = 0xe7e7e7e7e7e7e7e7ull;
  std::atomic<int64_t> generation{0};   // bumped by every record
  std::atomic<int64_t> fired{0};        // generation that fired (never recorded: complete, as in HIP)
  double t = 0.0;
};
typedef FakeStream* hipStream_t;
typedef FakeEvent* hipEvent_t;
typedef struct FakeGraphExec* hipGraphExec_t;

namespace fake_hip {
inline std::mutex mu;
inline std::set<FakeStream*>& streams() {
  static std::set<FakeStream*> s;
  return s;
}
inline int64_t graph_launches = 0, memcpys = 0, waits = 0, records = 0;
inline double clock = 0.0;
inline FakeStream* make_stream() {
  auto* s = new FakeStream();
  streams().insert(s);
  return s;
}
inline void free_stream(FakeStream* s) {
  streams().erase(s);
  delete s;
}
// run every stream's ready work until nothing moves; returns false if work is stuck
inline bool drain() {
  bool moved = true;
  while (moved) {
    moved = false;
    for (FakeStream* s : streams())
      while (!s->work.empty() && s->work.front()()) {
        s->work.pop_front();
        moved = true;
      }
  }
  for (FakeStream* s : streams())
    if (!s->work.empty()) return false;
  return true;
}
}  // namespace fake_hip

inline const char* hipGetErrorString(hipError_t e) { return e == hipSuccess ? "hipSuccess" : "hipError"; }
inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
  *e = new FakeEvent();
  return hipSuccess;
}
inline hipError_t hipEventCreate(hipEvent_t* e) {
  *e = new FakeEvent();
  return hipSuccess;
}
inline hipError_t hipEventDestroy(hipEvent_t e) {
  if (e->magic != 0xe7e7e7e7e7e7e7e7ull) return hipErrorInvalidValue;
  e->magic = 0;
  delete e;
  return hipSuccess;
}
inline hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
  ++fake_hip::records;
  const int64_t g = ++e->generation;
  s->work.push_back([e, g] {
    if (e->fired.load() < g) e->fired.store(g);
    e->t = (fake_hip::clock += 1.0);
    return true;
  });
  return hipSuccess;
}
inline hipError_t hipEventQuery(hipEvent_t e) {
  return e->fired >= e->generation ? hipSuccess : hipErrorNotReady;
}
inline hipError_t hipEventSynchronize(hipEvent_t e) {
  fake_hip::drain();
  return hipEventQuery(e);
}
inline hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b) {
  *ms = (float)(b->t - a->t);
  return hipSuccess;
}
inline hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned) {
  ++fake_hip::waits;
  const int64_t g = e->generation;   // the state captured at the call (as HIP does)
  s->work.push_back([e, g] { return e->fired >= g; });
  return hipSuccess;
}
inline hipError_t hipStreamSynchronize(hipStream_t) {
  fake_hip::drain();
  return hipSuccess;
}
namespace fake_hip {
// the body of a replayed graph: returns false while it is still "running" (a test holds a
// long kernel on a stream this way); default: completes at once
inline std::function<bool(hipGraphExec_t)> graph_body = [](hipGraphExec_t) { return true; };
}  // namespace fake_hip
inline hipError_t hipGraphLaunch(hipGraphExec_t g, hipStream_t s) {
  ++fake_hip::graph_launches;
  s->work.push_back([g] { return fake_hip::graph_body(g); });
  return hipSuccess;
}
inline hipError_t hipMemcpyAsync(void* d, const void* src, size_t n, hipMemcpyKind, hipStream_t s) {
  ++fake_hip::memcpys;
  s->work.push_back([d, src, n] {
    std::memmove(d, src, n);   // host buffers: ASan checks both ranges
    return true;
  });
  return hipSuccess;
}
inline hipError_t hipGetDevice(int* d) {
  *d = 0;
  return hipSuccess;
}
inline hipError_t hipSetDevice(int) { return hipSuccess; }
inline hipError_t hipDeviceGetStreamPriorityRange(int* lo, int* hi) {
  *lo = 0;
  *hi = -1;
  return hipSuccess;
}
inline hipError_t hipStreamCreateWithPriority(hipStream_t* s, unsigned, int) {
  *s = fake_hip::make_stream();
  return hipSuccess;
}
