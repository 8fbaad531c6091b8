// Native RCCL point-to-point engine for the pipeline runtime (SURVEY §2.4 "P2P engine").
//
// One RCCL communicator per pipeline group, created from a unique id that the Python side
// broadcasts once over torch.distributed.  Every CommGroup of the lowered program becomes
// one ncclGroupStart/End on a dedicated high-priority HIP comm stream:
//
//   post(sends, recvs):  event(current compute stream) -> comm stream waits on it (send
//                        data produced, recv buffers free) -> grouped ncclSend/ncclRecv ->
//                        "done" event recorded on the comm stream; returns a handle
//   wait(handle):        the CURRENT stream waits on that event (no host block), exactly
//                        where the runtime consumes a received buffer
//
// so transfers overlap compute and never stall the host.  Tensors touched by the comm
// stream are registered with the caching allocator (recordStream), so their memory is not
// reused before the transfer completes.  The order of groups is the globally consistent
// order produced by parallel/lower.py, which is what RCCL's in-order semantics require.
#pragma once
#include <torch/extension.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <cstring>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace py = pybind11;

namespace mipipe_comm {

// RCCL entry points are resolved at run time from the librccl that PyTorch itself loaded
// (torch/lib/librccl.so, shared with ProcessGroupNCCL): the extension does not link a second
// RCCL into the process.  rccl.h only provides the types.
struct Rccl {
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
};

inline Rccl* g_rccl = nullptr;

inline void load_rccl(const std::string& path) {
  if (g_rccl != nullptr) return;
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);  // the copy torch already mapped
  if (h == nullptr) h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  TORCH_CHECK(h != nullptr, "RcclP2P: cannot open ", path, ": ", dlerror());
  auto* r = new Rccl();
#define MP_SYM(f)                                                                      \
  r->f = reinterpret_cast<decltype(r->f)>(dlsym(h, "nccl" #f));                        \
  TORCH_CHECK(r->f != nullptr, "RcclP2P: missing symbol nccl" #f " in ", path);
  MP_SYM(GetUniqueId) MP_SYM(CommInitRank) MP_SYM(CommDestroy) MP_SYM(Send) MP_SYM(Recv) MP_SYM(GroupStart)
  MP_SYM(GroupEnd) MP_SYM(GetErrorString)
#undef MP_SYM
  g_rccl = r;
}

#define MP_NCCL(x)                                                                                 \
  do {                                                                                             \
    ncclResult_t r_ = (x);                                                                         \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL call failed: ", g_rccl->GetErrorString(r_), " at ", #x);  \
  } while (0)
#define MP_HIP(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    TORCH_CHECK(e_ == hipSuccess, "HIP call failed: ", hipGetErrorString(e_), " at ", #x);          \
  } while (0)

inline ncclDataType_t nccl_type(const torch::Tensor& t) {
  switch (t.scalar_type()) {
    case torch::kBFloat16: return ncclBfloat16;
    case torch::kFloat32: return ncclFloat32;
    case torch::kFloat16: return ncclFloat16;
    case torch::kInt64: return ncclInt64;
    case torch::kInt32: return ncclInt32;
    case torch::kUInt8: return ncclUint8;
    case torch::kFloat64: return ncclFloat64;
    default: TORCH_CHECK(false, "RcclP2P: unsupported dtype ", t.scalar_type());
  }
  return ncclFloat32;
}

class RcclP2P {
 public:
  static void load(const std::string& path) { load_rccl(path); }

  static py::bytes unique_id() {
    TORCH_CHECK(g_rccl != nullptr, "RcclP2P.load(<torch/lib/librccl.so>) first");
    ncclUniqueId id;
    MP_NCCL(g_rccl->GetUniqueId(&id));
    return py::bytes(id.internal, sizeof(id.internal));
  }

  RcclP2P(const py::bytes& id, int nranks, int rank, int device) : nranks_(nranks), rank_(rank), device_(device) {
    TORCH_CHECK(g_rccl != nullptr, "RcclP2P.load(<torch/lib/librccl.so>) first");
    std::string s = id;
    TORCH_CHECK(s.size() == sizeof(ncclUniqueId::internal), "RcclP2P: bad unique id size ", s.size());
    ncclUniqueId uid;
    std::memcpy(uid.internal, s.data(), s.size());
    MP_HIP(hipSetDevice(device));
    MP_NCCL(g_rccl->CommInitRank(&comm_, nranks, uid, rank));
    // high-priority stream from torch's pool: comm kernels are scheduled ahead of compute, and
    // the stream outlives every tensor recordStream()-ed on it (the caching allocator records
    // events on it when those tensors are freed, possibly after close())
    comm_stream_ = c10::hip::getStreamFromPool(/*isHighPriority=*/true, device);
    stream_ = comm_stream_.stream();
  }

  ~RcclP2P() { close(); }

  void close() {
    if (stream_ != nullptr) {
      hipStreamSynchronize(stream_);
      for (auto& kv : pending_) hipEventDestroy(kv.second);
      pending_.clear();
      for (hipEvent_t e : pool_) hipEventDestroy(e);
      pool_.clear();
      stream_ = nullptr;
    }
    if (comm_ != nullptr) {
      g_rccl->CommDestroy(comm_);
      comm_ = nullptr;
    }
  }

  int64_t post(const std::vector<std::pair<torch::Tensor, int64_t>>& sends,
               const std::vector<std::pair<torch::Tensor, int64_t>>& recvs) {
    TORCH_CHECK(comm_ != nullptr, "RcclP2P is closed");
    hipStream_t cur = c10::hip::getCurrentHIPStream(device_).stream();
    hipEvent_t ready = event();
    MP_HIP(hipEventRecord(ready, cur));
    MP_HIP(hipStreamWaitEvent(stream_, ready, 0));
    pool_.push_back(ready);  // the wait above captured its state; reusable now
    const c10::hip::HIPStream& cs = comm_stream_;
    MP_NCCL(g_rccl->GroupStart());
    for (const auto& [t, peer] : sends) {
      TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RcclP2P: send tensors must be contiguous GPU tensors");
      MP_NCCL(g_rccl->Send(t.data_ptr(), t.numel(), nccl_type(t), (int)peer, comm_, stream_));
    }
    for (const auto& [t, peer] : recvs) {
      TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RcclP2P: recv tensors must be contiguous GPU tensors");
      MP_NCCL(g_rccl->Recv(t.data_ptr(), t.numel(), nccl_type(t), (int)peer, comm_, stream_));
    }
    MP_NCCL(g_rccl->GroupEnd());
    for (const auto& p : sends) c10::hip::HIPCachingAllocator::recordStream(p.first.storage().data_ptr(), cs);
    for (const auto& p : recvs) c10::hip::HIPCachingAllocator::recordStream(p.first.storage().data_ptr(), cs);
    hipEvent_t done = event();
    MP_HIP(hipEventRecord(done, stream_));
    const int64_t h = next_++;
    pending_[h] = done;
    return h;
  }

  // Raw form for the native stage runner (csrc/runtime/stage_runner.cpp): buffers by
  // device pointer, ordered after / consumed on an explicit compute stream.  The caller
  // keeps the buffers alive (they are persistent graph / runtime buffers).
  struct RawOp {
    void* ptr;
    size_t count;
    ncclDataType_t type;
    int peer;
  };
  int64_t post_raw(const std::vector<RawOp>& sends, const std::vector<RawOp>& recvs, hipStream_t compute) {
    TORCH_CHECK(comm_ != nullptr, "RcclP2P is closed");
    hipEvent_t ready = event();
    MP_HIP(hipEventRecord(ready, compute));
    MP_HIP(hipStreamWaitEvent(stream_, ready, 0));
    pool_.push_back(ready);
    MP_NCCL(g_rccl->GroupStart());
    for (const auto& o : sends) MP_NCCL(g_rccl->Send(o.ptr, o.count, o.type, o.peer, comm_, stream_));
    for (const auto& o : recvs) MP_NCCL(g_rccl->Recv(o.ptr, o.count, o.type, o.peer, comm_, stream_));
    MP_NCCL(g_rccl->GroupEnd());
    hipEvent_t done = event();
    MP_HIP(hipEventRecord(done, stream_));
    const int64_t h = next_++;
    pending_[h] = done;
    return h;
  }
  void wait_raw(int64_t h, hipStream_t compute) {
    auto it = pending_.find(h);
    if (it == pending_.end()) return;
    MP_HIP(hipStreamWaitEvent(compute, it->second, 0));
    pool_.push_back(it->second);
    pending_.erase(it);
  }

  // make the current stream wait for a posted group (idempotent)
  void wait(int64_t h) {
    auto it = pending_.find(h);
    if (it == pending_.end()) return;
    hipStream_t cur = c10::hip::getCurrentHIPStream(device_).stream();
    MP_HIP(hipStreamWaitEvent(cur, it->second, 0));
    pool_.push_back(it->second);
    pending_.erase(it);
  }

  bool query(int64_t h) {
    auto it = pending_.find(h);
    return it == pending_.end() || hipEventQuery(it->second) == hipSuccess;
  }

  void synchronize() {
    if (stream_ != nullptr) MP_HIP(hipStreamSynchronize(stream_));
  }

  int rank() const { return rank_; }
  int nranks() const { return nranks_; }

 private:
  hipEvent_t event() {
    if (!pool_.empty()) {
      hipEvent_t e = pool_.back();
      pool_.pop_back();
      return e;
    }
    hipEvent_t e;
    MP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
  }

  ncclComm_t comm_ = nullptr;
  c10::hip::HIPStream comm_stream_{c10::hip::getDefaultHIPStream()};
  hipStream_t stream_ = nullptr;
  int nranks_, rank_, device_;
  int64_t next_ = 1;
  std::unordered_map<int64_t, hipEvent_t> pending_;
  std::vector<hipEvent_t> pool_;
};

}  // namespace mipipe_comm
