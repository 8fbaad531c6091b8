// Host-only stand-in for the RCCL types (csrc/tests/host_asan_test.cpp): the engine calls
// RCCL through its function table (mipipe_comm::g_rccl), which the test fills with fakes.
#pragma once
#include <cstddef>
#include <hip/hip_runtime.h>

enum ncclResult_t { ncclSuccess = 0, ncclInvalidArgument = 4, ncclInProgress = 7 };
enum ncclDataType_t { ncclInt8 = 0, ncclUint8 = 1, ncclInt32 = 2, ncclUint32 = 3, ncclInt64 = 4, ncclUint64 = 5,
                      ncclFloat16 = 6, ncclFloat32 = 7, ncclFloat64 = 8, ncclBfloat16 = 9 };
enum ncclRedOp_t { ncclSum = 0, ncclProd = 1, ncclMax = 2 };
typedef struct FakeComm* ncclComm_t;
struct ncclUniqueId {
  char internal[128];
};
ncclResult_t ncclGetUniqueId(ncclUniqueId*);
ncclResult_t ncclCommInitRank(ncclComm_t*, int, ncclUniqueId, int);
ncclResult_t ncclCommDestroy(ncclComm_t);
ncclResult_t ncclCommAbort(ncclComm_t);
ncclResult_t ncclCommGetAsyncError(ncclComm_t, ncclResult_t*);
ncclResult_t ncclSend(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
ncclResult_t ncclRecv(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
ncclResult_t ncclAllReduce(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
ncclResult_t ncclReduceScatter(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
ncclResult_t ncclAllGather(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
ncclResult_t ncclGroupStart();
ncclResult_t ncclGroupEnd();
const char* ncclGetErrorString(ncclResult_t);
