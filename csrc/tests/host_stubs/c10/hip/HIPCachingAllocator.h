#pragma once
#include <c10/hip/HIPStream.h>
namespace c10 {
namespace hip {
namespace HIPCachingAllocator {
inline void recordStream(void*, const HIPStream&) {}
}  // namespace HIPCachingAllocator
}  // namespace hip
}  // namespace c10
