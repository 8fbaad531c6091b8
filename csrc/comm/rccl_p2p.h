// Native RCCL point-to-point engine for the pipeline runtime (SURVEY §2.4 "P2P engine",
// §7.4-1 "separate communicators or streams per direction avoid head-of-line blocking").
//
// Two RCCL communicators per pipeline group, one per traffic DIRECTION, each driven from
// its own high-priority HIP stream:
//
//   channel 0 ("fwd"):  activations flowing down the pipeline (F messages, and the last
//                       stage's hidden rows to the distributed-head ranks, H messages)
//   channel 1 ("bwd"):  gradients flowing back up (B messages, head input grads D)
//
// RCCL runs the operations of one communicator in host-issue order and a large send
// completes only when the peer's matching receive runs.  With ONE stream for both
// directions an early-posted gradient receive (waiting on the downstream backward) holds
// back every activation send queued after it, so the downstream rank starves.  With one
// stream per direction the two flows never queue behind each other; parallel/simulate.py
// (check_lowered(..., channels=2)) proves the per-channel order of a lowered program
// cannot deadlock before the runtime uses it.  Each communicator is only ever used from
// its own stream, in host order, so RCCL's per-communicator ordering rule holds.
//
//   post(ch, sends, recvs): event(current compute stream) -> channel stream waits on it
//                           (send data produced, recv buffers free) -> grouped
//                           ncclSend/ncclRecv -> "done" event; returns a handle
//   wait(handle):           the CURRENT stream waits on that event (no host block)
//
// Tensors touched by a channel stream are registered with the caching allocator
// (recordStream), so their memory is not reused before the transfer completes.
// `abort()` (ncclCommAbort) tears both communicators down even with transfers in
// flight -- the pre-flight ping uses it to back out of a link that does not answer.
#pragma once
#include <torch/extension.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <array>
#include <cstring>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace py = pybind11;

namespace mipipe_comm {

constexpr int kChannels = 2;

// RCCL entry points are resolved at run time from the librccl that PyTorch itself loaded
// (torch/lib/librccl.so, shared with ProcessGroupNCCL): the extension does not link a second
// RCCL into the process.  rccl.h only provides the types.
struct Rccl {
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclCommAbort) CommAbort = nullptr;
  decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
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
  MP_SYM(GetUniqueId) MP_SYM(CommInitRank) MP_SYM(CommDestroy) MP_SYM(CommAbort) MP_SYM(CommGetAsyncError)
  MP_SYM(Send) MP_SYM(Recv) MP_SYM(GroupStart) MP_SYM(GroupEnd) MP_SYM(GetErrorString)
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
  static int64_t id_bytes() { return (int64_t)sizeof(ncclUniqueId::internal); }

  // ids: kChannels unique ids concatenated (one communicator per direction)
  RcclP2P(const py::bytes& ids, int nranks, int rank, int device) : nranks_(nranks), rank_(rank), device_(device) {
    TORCH_CHECK(g_rccl != nullptr, "RcclP2P.load(<torch/lib/librccl.so>) first");
    std::string s = ids;
    const size_t n = sizeof(ncclUniqueId::internal);
    TORCH_CHECK(s.size() == n * kChannels, "RcclP2P: expected ", kChannels, " unique ids (", n * kChannels,
                " bytes), got ", s.size());
    MP_HIP(hipSetDevice(device));
    int lo = 0, hi = 0;
    MP_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    for (int c = 0; c < kChannels; ++c) {
      ncclUniqueId uid;
      std::memcpy(uid.internal, s.data() + c * n, n);
      MP_NCCL(g_rccl->CommInitRank(&comm_[c], nranks, uid, rank));
      // A private high-priority stream per channel (not torch's round-robin pool, which
      // could hand both channels -- or a compute user -- the same stream).  Never destroyed:
      // the caching allocator may record events on it when recordStream()-ed tensors are
      // freed after close().
      MP_HIP(hipStreamCreateWithPriority(&stream_[c], hipStreamNonBlocking, hi));
      hstream_[c] = c10::hip::getStreamFromExternal(stream_[c], device);
    }
  }

  ~RcclP2P() { close(); }

  void close() {
    if (open_) {
      for (int c = 0; c < kChannels; ++c) hipStreamSynchronize(stream_[c]);
      release_events();
      for (int c = 0; c < kChannels; ++c)
        if (comm_[c] != nullptr) g_rccl->CommDestroy(comm_[c]);
      comm_ = {nullptr, nullptr};
      open_ = false;
    }
  }

  // Tear down with transfers possibly in flight (a peer that never answered).  Does not
  // synchronise the channel streams: ncclCommAbort makes their kernels return.
  void abort() {
    if (!open_) return;
    for (int c = 0; c < kChannels; ++c)
      if (comm_[c] != nullptr) g_rccl->CommAbort(comm_[c]);
    comm_ = {nullptr, nullptr};
    pending_.clear();  // events leaked on purpose: their streams may still be unwinding
    open_ = false;
  }

  // First asynchronous RCCL error of either communicator ("" if none).
  std::string async_error() {
    if (!open_) return "closed";
    for (int c = 0; c < kChannels; ++c) {
      ncclResult_t r = ncclSuccess;
      if (g_rccl->CommGetAsyncError(comm_[c], &r) != ncclSuccess) return "ncclCommGetAsyncError failed";
      if (r != ncclSuccess && r != ncclInProgress) return g_rccl->GetErrorString(r);
    }
    return "";
  }

  int64_t post(int channel, const std::vector<std::pair<torch::Tensor, int64_t>>& sends,
               const std::vector<std::pair<torch::Tensor, int64_t>>& recvs) {
    std::vector<RawOp> s, r;
    for (const auto& [t, peer] : sends) s.push_back(raw(t, peer));
    for (const auto& [t, peer] : recvs) r.push_back(raw(t, peer));
    const int64_t h = post_raw(channel, s, r, c10::hip::getCurrentHIPStream(device_).stream());
    const c10::hip::HIPStream& cs = hstream_[channel];
    for (const auto& p : sends) c10::hip::HIPCachingAllocator::recordStream(p.first.storage().data_ptr(), cs);
    for (const auto& p : recvs) c10::hip::HIPCachingAllocator::recordStream(p.first.storage().data_ptr(), cs);
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
  int64_t post_raw(int channel, const std::vector<RawOp>& sends, const std::vector<RawOp>& recvs,
                   hipStream_t compute) {
    TORCH_CHECK(open_, "RcclP2P is closed");
    TORCH_CHECK(channel >= 0 && channel < kChannels, "RcclP2P: bad channel ", channel);
    hipStream_t cs = stream_[channel];
    ncclComm_t comm = comm_[channel];
    hipEvent_t ready = event();
    MP_HIP(hipEventRecord(ready, compute));
    MP_HIP(hipStreamWaitEvent(cs, ready, 0));
    pool_.push_back(ready);  // the wait above captured its state; reusable now
    MP_NCCL(g_rccl->GroupStart());
    for (const auto& o : sends) {
      TORCH_CHECK(o.peer >= 0 && o.peer < nranks_, "RcclP2P: bad send peer ", o.peer);
      MP_NCCL(g_rccl->Send(o.ptr, o.count, o.type, o.peer, comm, cs));
    }
    for (const auto& o : recvs) {
      TORCH_CHECK(o.peer >= 0 && o.peer < nranks_, "RcclP2P: bad recv peer ", o.peer);
      MP_NCCL(g_rccl->Recv(o.ptr, o.count, o.type, o.peer, comm, cs));
    }
    MP_NCCL(g_rccl->GroupEnd());
    hipEvent_t done = event();
    MP_HIP(hipEventRecord(done, cs));
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
  void wait(int64_t h) { wait_raw(h, c10::hip::getCurrentHIPStream(device_).stream()); }

  // host-side completion test (pre-flight ping polls it against a deadline)
  bool query(int64_t h) {
    auto it = pending_.find(h);
    return it == pending_.end() || hipEventQuery(it->second) == hipSuccess;
  }

  void synchronize() {
    if (open_)
      for (int c = 0; c < kChannels; ++c) MP_HIP(hipStreamSynchronize(stream_[c]));
  }

  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  int channels() const { return kChannels; }
  int64_t stream_handle(int c) const { return reinterpret_cast<int64_t>(stream_[c]); }

 private:
  RawOp raw(const torch::Tensor& t, int64_t peer) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RcclP2P: tensors must be contiguous GPU tensors");
    return RawOp{t.data_ptr(), (size_t)t.numel(), nccl_type(t), (int)peer};
  }

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

  void release_events() {
    for (auto& kv : pending_) hipEventDestroy(kv.second);
    pending_.clear();
    for (hipEvent_t e : pool_) hipEventDestroy(e);
    pool_.clear();
  }

  std::array<ncclComm_t, kChannels> comm_{nullptr, nullptr};
  std::array<hipStream_t, kChannels> stream_{nullptr, nullptr};
  std::array<c10::hip::HIPStream, kChannels> hstream_{c10::hip::getDefaultHIPStream(),
                                                      c10::hip::getDefaultHIPStream()};
  bool open_ = true;
  int nranks_, rank_, device_;
  int64_t next_ = 1;
  std::unordered_map<int64_t, hipEvent_t> pending_;
  std::vector<hipEvent_t> pool_;
};

}  // namespace mipipe_comm
