// Native RCCL engine of the pipeline runtime: point-to-point transfers AND the collectives
// of a training step, each on a communicator + HIP stream the runtime controls (SURVEY §2.4
// "P2P engine", §7.1 comm/rccl_allreduce, §5.8).
//
// An engine owns one RCCL communicator per CHANNEL over one process group (the pipeline
// group, or the DP group of a stage).  Every channel issues on one of a small, process-wide
// set of COMM STREAM SLOTS -- private high-priority HIP streams created once per device and
// never destroyed, so every engine a process builds maps onto the same hardware queues:
//
//   slot 0 ("fwd"):  activations flowing down the pipeline (F, and the last stage's hidden
//                    rows to the distributed-head ranks, H)
//   slot 1 ("bwd"):  gradients flowing back up (B, head input grads D)
//   slot 2 ("coll"): every collective of the step, in one FIFO: the pipeline engine's
//                    head-gradient reduce-scatter / clip-norm sum / weight all-gather and
//                    the DP engine's per-stage gradient all-reduce (different
//                    communicators, one stream: their relative order is host issue order,
//                    the same on every rank -- parallel/simulate.py check_collectives)
//
// Why the split.  RCCL runs the operations of one communicator in host-issue order and a
// send / a collective completes only when the peers' matching calls run; an RCCL kernel
// holds its hardware queue until then.  Activations and gradients on separate streams never
// queue behind each other (check_lowered(channels=2) proves the per-channel order); the
// collectives never wait for p2p and nothing waits for them before the end of the step, so
// a blocked collective delays only the collective stream.  That argument needs the comm
// streams on hardware queues of their own, which parallel/queues.py verifies at start-up
// with the spin/flag probe (csrc/kernels/probe.hip) and the runtime degrades if not.
//
//   post(ch, sends, recvs):  event(current compute stream) -> channel stream waits on it
//                            (send data produced, recv buffers free) -> grouped
//                            ncclSend/ncclRecv -> "done" event; returns a handle
//   coll(ch, op, send, recv): same ordering, one ncclAllReduce / ReduceScatter / AllGather
//   wait(handle):            the CURRENT stream waits on that event (no host block)
//
// `abort()` (ncclCommAbort) tears the communicators down even with transfers in flight --
// the pre-flight ping uses it to back out of a link that does not answer.
#pragma once
#include <torch/extension.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace py = pybind11;

namespace mipipe_comm {

constexpr int kStreamSlots = 3;  // fwd, bwd, coll

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
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclReduceScatter) ReduceScatter = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
};

inline Rccl* g_rccl = nullptr;

inline void load_rccl(const std::string& path) {
  if (g_rccl != nullptr) return;
  void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);  // the copy torch already mapped
  if (h == nullptr) h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
  TORCH_CHECK(h != nullptr, "RcclEngine: cannot open ", path, ": ", dlerror());
  auto* r = new Rccl();
#define MP_SYM(f)                                                                      \
  r->f = reinterpret_cast<decltype(r->f)>(dlsym(h, "nccl" #f));                        \
  TORCH_CHECK(r->f != nullptr, "RcclEngine: missing symbol nccl" #f " in ", path);
  MP_SYM(GetUniqueId) MP_SYM(CommInitRank) MP_SYM(CommDestroy) MP_SYM(CommAbort) MP_SYM(CommGetAsyncError)
  MP_SYM(Send) MP_SYM(Recv) MP_SYM(AllReduce) MP_SYM(ReduceScatter) MP_SYM(AllGather) MP_SYM(GroupStart)
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
    default: TORCH_CHECK(false, "RcclEngine: unsupported dtype ", t.scalar_type());
  }
  return ncclFloat32;
}

inline size_t nccl_size(ncclDataType_t t) {
  switch (t) {
    case ncclBfloat16: case ncclFloat16: return 2;
    case ncclFloat32: case ncclInt32: return 4;
    case ncclInt64: case ncclFloat64: return 8;
    default: return 1;
  }
}

// Process-wide comm streams: slot k of device d is created on first use (high priority,
// non-blocking) and lives as long as the process.  Engines built later in the process (a
// test suite, a sweep, a bench retry in the same child) reuse them, so the stream ->
// hardware-queue mapping never drifts and no stream leaks per engine.
inline hipStream_t comm_stream(int device, int slot) {
  static std::mutex mu;
  static std::unordered_map<int, std::array<hipStream_t, kStreamSlots>> streams;
  TORCH_CHECK(slot >= 0 && slot < kStreamSlots, "comm_stream: bad slot ", slot);
  std::lock_guard<std::mutex> lk(mu);
  auto it = streams.find(device);
  if (it == streams.end()) it = streams.emplace(device, std::array<hipStream_t, kStreamSlots>{}).first;
  hipStream_t& s = it->second[slot];
  if (s == nullptr) {
    int cur = 0;
    MP_HIP(hipGetDevice(&cur));
    MP_HIP(hipSetDevice(device));
    int lo = 0, hi = 0;
    MP_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    MP_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
    MP_HIP(hipSetDevice(cur));
  }
  return s;
}

// collective kinds (python: parallel/collectives.py)
enum CollOp { ALLREDUCE_SUM = 0, REDUCE_SCATTER_SUM = 1, ALL_GATHER = 2, ALLREDUCE_MAX = 3 };

class RcclEngine {
 public:
  static void load(const std::string& path) { load_rccl(path); }

  static py::bytes unique_id() {
    TORCH_CHECK(g_rccl != nullptr, "RcclEngine.load(<torch/lib/librccl.so>) first");
    ncclUniqueId id;
    MP_NCCL(g_rccl->GetUniqueId(&id));
    return py::bytes(id.internal, sizeof(id.internal));
  }
  static int64_t id_bytes() { return (int64_t)sizeof(ncclUniqueId::internal); }

  // ids: one unique id per channel, concatenated; slots[c]: the comm stream slot of channel c
  RcclEngine(const py::bytes& ids, int nranks, int rank, int device, std::vector<int64_t> slots)
      : nranks_(nranks), rank_(rank), device_(device) {
    TORCH_CHECK(g_rccl != nullptr, "RcclEngine.load(<torch/lib/librccl.so>) first");
    TORCH_CHECK(!slots.empty(), "RcclEngine: at least one channel");
    std::string s = ids;
    const size_t n = sizeof(ncclUniqueId::internal);
    const size_t nch = slots.size();
    TORCH_CHECK(s.size() == n * nch, "RcclEngine: expected ", nch, " unique ids (", n * nch, " bytes), got ",
                s.size());
    MP_HIP(hipSetDevice(device));
    comm_.assign(nch, nullptr);
    for (size_t c = 0; c < nch; ++c) {
      ncclUniqueId uid;
      std::memcpy(uid.internal, s.data() + c * n, n);
      MP_NCCL(g_rccl->CommInitRank(&comm_[c], nranks, uid, rank));
      stream_.push_back(comm_stream(device, (int)slots[c]));
      slot_.push_back((int)slots[c]);
      hstream_.push_back(c10::hip::getStreamFromExternal(stream_.back(), device));
    }
  }

  ~RcclEngine() { close(); }

  void close() {
    if (open_) {
      for (auto st : stream_) hipStreamSynchronize(st);
      release_events();
      for (auto& c : comm_)
        if (c != nullptr) g_rccl->CommDestroy(c);
      std::fill(comm_.begin(), comm_.end(), nullptr);
      open_ = false;
    }
  }

  // Tear down with transfers possibly in flight (a peer that never answered).  Does not
  // synchronise the channel streams: ncclCommAbort makes their kernels return.
  void abort() {
    if (!open_) return;
    for (auto& c : comm_)
      if (c != nullptr) g_rccl->CommAbort(c);
    std::fill(comm_.begin(), comm_.end(), nullptr);
    // events kept (not destroyed) on purpose: their streams may still be unwinding; parked
    // where they stay reachable so the engine itself owns nothing afterwards
    std::vector<hipEvent_t>& park = abandoned_events();
    for (auto& kv : pending_) park.push_back(kv.second);
    pending_.clear();
    for (hipEvent_t e : pool_) park.push_back(e);
    pool_.clear();
    {
      std::lock_guard<std::mutex> lk(trace_mu_);
      for (auto& e : trace_)
        if (e.ev != nullptr) park.push_back(e.ev);
      trace_.clear();
      trace_head_ = 0;
    }
    open_ = false;
  }

  // First asynchronous RCCL error of any communicator ("" if none).
  std::string async_error() {
    if (!open_) return "closed";
    for (auto& c : comm_) {
      ncclResult_t r = ncclSuccess;
      if (g_rccl->CommGetAsyncError(c, &r) != ncclSuccess) return "ncclCommGetAsyncError failed";
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
    for (const auto& p : sends) record(p.first, channel);
    for (const auto& p : recvs) record(p.first, channel);
    return h;
  }

  // One collective on channel `channel` (torch form, current stream).  ALLREDUCE: send and
  // recv have the same numel (may alias: in place).  REDUCE_SCATTER: send holds nranks x
  // recv.numel() elements (in place: recv == send[rank * n : (rank+1) * n]).  ALL_GATHER:
  // recv holds nranks x send.numel() (in place: send == recv[rank * n : ...]).
  int64_t coll(int channel, int op, const torch::Tensor& send, const torch::Tensor& recv) {
    TORCH_CHECK(send.is_cuda() && recv.is_cuda() && send.is_contiguous() && recv.is_contiguous(),
                "RcclEngine.coll: contiguous GPU tensors");
    TORCH_CHECK(send.scalar_type() == recv.scalar_type(), "RcclEngine.coll: dtype mismatch");
    size_t count = 0;
    switch (op) {
      case ALLREDUCE_SUM: case ALLREDUCE_MAX:
        TORCH_CHECK(send.numel() == recv.numel(), "all_reduce: numel mismatch");
        count = (size_t)recv.numel();
        break;
      case REDUCE_SCATTER_SUM:
        TORCH_CHECK(send.numel() == recv.numel() * nranks_, "reduce_scatter: send must be nranks x recv");
        count = (size_t)recv.numel();
        break;
      case ALL_GATHER:
        TORCH_CHECK(recv.numel() == send.numel() * nranks_, "all_gather: recv must be nranks x send");
        count = (size_t)send.numel();
        break;
      default: TORCH_CHECK(false, "RcclEngine.coll: bad op ", op);
    }
    const int64_t h = coll_raw(channel, op, send.data_ptr(), recv.data_ptr(), count, nccl_type(send),
                               c10::hip::getCurrentHIPStream(device_).stream());
    record(send, channel);
    record(recv, channel);
    return h;
  }

  // Raw forms for the native stage runner (csrc/runtime/stage_runner.cpp): buffers by
  // device pointer, ordered after / consumed on an explicit compute stream.  The caller
  // keeps the buffers alive (they are persistent graph / runtime buffers).
  struct RawOp {
    void* ptr;
    size_t count;
    ncclDataType_t type;
    int peer;
  };
  // ``after`` (optional): for a RECEIVE-ONLY group, order the channel stream after that event
  // instead of after everything issued so far on the compute stream (a
  // pre-posted receive then starts at post time, so the peer's matching send is not held
  // behind this rank's unrelated compute).  The caller guarantees the receive buffers are
  // free once ``after`` has fired: the native stage runner passes an event recorded at the
  // start of the step, and every in-step message has a receive slot of its own
  // (PipelineRuntime._plan_recv_arena).  A group with sends always follows the compute.
  int64_t post_raw(int channel, const std::vector<RawOp>& sends, const std::vector<RawOp>& recvs,
                   hipStream_t compute, hipEvent_t after = nullptr) {
    check_channel(channel);
    // peers checked before anything is issued: a throw inside the group would leave this
    // thread's RCCL group open and fold the next post into it (csrc/tests/host_asan_test.cpp)
    for (const auto& o : sends) TORCH_CHECK(o.peer >= 0 && o.peer < nranks_, "RcclEngine: bad send peer ", o.peer);
    for (const auto& o : recvs) TORCH_CHECK(o.peer >= 0 && o.peer < nranks_, "RcclEngine: bad recv peer ", o.peer);
    hipStream_t cs = stream_[channel];
    ncclComm_t comm = comm_[channel];
    if (after != nullptr && sends.empty()) {
      MP_HIP(hipStreamWaitEvent(cs, after, 0));
    } else {
      order_after(compute, cs);
    }
    MP_NCCL(g_rccl->GroupStart());
    for (const auto& o : sends) MP_NCCL(g_rccl->Send(o.ptr, o.count, o.type, o.peer, comm, cs));
    for (const auto& o : recvs) MP_NCCL(g_rccl->Recv(o.ptr, o.count, o.type, o.peer, comm, cs));
    MP_NCCL(g_rccl->GroupEnd());
    const int64_t h = finish(cs);
    trace(channel, -1, cs, sends, recvs);
    return h;
  }

  int64_t coll_raw(int channel, int op, void* send, void* recv, size_t count, ncclDataType_t type,
                   hipStream_t compute) {
    check_channel(channel);
    hipStream_t cs = stream_[channel];
    ncclComm_t comm = comm_[channel];
    order_after(compute, cs);
    switch (op) {
      case ALLREDUCE_SUM: MP_NCCL(g_rccl->AllReduce(send, recv, count, type, ncclSum, comm, cs)); break;
      case ALLREDUCE_MAX: MP_NCCL(g_rccl->AllReduce(send, recv, count, type, ncclMax, comm, cs)); break;
      case REDUCE_SCATTER_SUM: MP_NCCL(g_rccl->ReduceScatter(send, recv, count, type, ncclSum, comm, cs)); break;
      case ALL_GATHER: MP_NCCL(g_rccl->AllGather(send, recv, count, type, comm, cs)); break;
      default: TORCH_CHECK(false, "RcclEngine: bad collective ", op);
    }
    const int64_t h = finish(cs);
    trace(channel, op, cs, {RawOp{send, count, type, -1}}, {});
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

  // non-consuming wait: every stream that reads a group's receives waits on its completion
  // event (microbatch lanes: one grouped post may feed computes on two streams); the
  // handle stays valid until `release`
  void wait_keep_raw(int64_t h, hipStream_t compute) {
    auto it = pending_.find(h);
    if (it == pending_.end()) return;
    MP_HIP(hipStreamWaitEvent(compute, it->second, 0));
  }
  void wait_keep(int64_t h) { wait_keep_raw(h, c10::hip::getCurrentHIPStream(device_).stream()); }
  // return a handle's event to the pool (after its last wait_keep)
  void release(int64_t h) {
    auto it = pending_.find(h);
    if (it == pending_.end()) return;
    pool_.push_back(it->second);
    pending_.erase(it);
  }

  // host-side completion test (pre-flight ping polls it against a deadline)
  bool query(int64_t h) {
    auto it = pending_.find(h);
    return it == pending_.end() || hipEventQuery(it->second) == hipSuccess;
  }

  // Hang diagnostics: the groups of the last kTrace posts / collectives (per engine) that
  // have not completed on their channel stream, oldest first -- channel, kind (-1 p2p,
  // else CollOp), peers, bytes, seconds since the host issued it.  A watchdog report then
  // names the transfer every rank is stuck in instead of only the Python stack.
  py::list progress() {
    py::list out;
    // the watchdog thread calls this while the native tape runner (GIL released) records
    // new groups: entries and head under trace_mu_, nothing once closed
    std::lock_guard<std::mutex> lk(trace_mu_);
    if (!trace_on_ || !open_) return out;
    const auto now = std::chrono::steady_clock::now();
    const size_t n = std::min<size_t>(trace_head_, kTrace);
    for (size_t i = trace_head_ - n; i < trace_head_; ++i) {
      const TraceEntry& e = trace_[i % kTrace];
      if (e.ev == nullptr || hipEventQuery(e.ev) != hipErrorNotReady) continue;
      py::dict d;
      d["seq"] = e.seq;
      d["channel"] = e.channel;
      d["kind"] = e.kind < 0 ? std::string("p2p") : std::string(coll_name(e.kind));
      d["sends"] = py::cast(std::vector<int>(e.send_peers, e.send_peers + e.nsend));
      d["recvs"] = py::cast(std::vector<int>(e.recv_peers, e.recv_peers + e.nrecv));
      d["bytes"] = (int64_t)e.bytes;
      d["age_s"] = std::chrono::duration<double>(now - e.t).count();
      out.append(d);
    }
    return out;
  }
  int64_t issued() {
    std::lock_guard<std::mutex> lk(trace_mu_);
    return (int64_t)trace_head_;
  }

  void synchronize() {
    if (open_)
      for (auto st : stream_) MP_HIP(hipStreamSynchronize(st));
  }

  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  int channels() const { return (int)comm_.size(); }
  int64_t stream_handle(int c) const { return reinterpret_cast<int64_t>(stream_.at(c)); }
  int slot(int c) const { return slot_.at(c); }

 private:
  void check_channel(int channel) const {
    TORCH_CHECK(open_, "RcclEngine is closed");
    TORCH_CHECK(channel >= 0 && channel < (int)comm_.size(), "RcclEngine: bad channel ", channel);
  }

  // the channel stream waits for everything issued so far on the compute stream
  void order_after(hipStream_t compute, hipStream_t cs) {
    hipEvent_t ready = event();
    MP_HIP(hipEventRecord(ready, compute));
    MP_HIP(hipStreamWaitEvent(cs, ready, 0));
    pool_.push_back(ready);  // the wait above captured its state; reusable now
  }

  int64_t finish(hipStream_t cs) {
    hipEvent_t done = event();
    MP_HIP(hipEventRecord(done, cs));
    const int64_t h = next_++;
    pending_[h] = done;
    return h;
  }

  // tensors touched by a channel stream are registered with the caching allocator, so
  // their memory is not reused before the transfer completes
  void record(const torch::Tensor& t, int channel) {
    c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), hstream_[channel]);
  }

  RawOp raw(const torch::Tensor& t, int64_t peer) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RcclEngine: tensors must be contiguous GPU tensors");
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
    {
      std::lock_guard<std::mutex> lk(trace_mu_);
      for (auto& e : trace_)
        if (e.ev != nullptr) hipEventDestroy(e.ev);
      trace_.clear();
      trace_head_ = 0;
    }
    for (auto& kv : pending_) hipEventDestroy(kv.second);
    pending_.clear();
    for (hipEvent_t e : pool_) hipEventDestroy(e);
    pool_.clear();
  }

  static std::vector<hipEvent_t>& abandoned_events() {
    static std::vector<hipEvent_t> v;
    return v;
  }

  static constexpr size_t kTrace = 256;
  static constexpr int kPeers = 8;
  struct TraceEntry {
    hipEvent_t ev = nullptr;
    int64_t seq = 0;
    int channel = 0, kind = -1, nsend = 0, nrecv = 0;
    int send_peers[kPeers], recv_peers[kPeers];
    size_t bytes = 0;
    std::chrono::steady_clock::time_point t;
  };
  static const char* coll_name(int op) {
    switch (op) {
      case ALLREDUCE_SUM: return "all_reduce";
      case ALLREDUCE_MAX: return "all_reduce_max";
      case REDUCE_SCATTER_SUM: return "reduce_scatter";
      case ALL_GATHER: return "all_gather";
      default: return "?";
    }
  }
  static size_t type_bytes(ncclDataType_t t) {
    switch (t) {
      case ncclInt8: case ncclUint8: return 1;
      case ncclFloat16: case ncclBfloat16: return 2;
      case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
      default: return 8;
    }
  }
  // one extra event record per group (MIPIPE_COMM_TRACE=0: none)
  void trace(int channel, int kind, hipStream_t cs, const std::vector<RawOp>& sends, const std::vector<RawOp>& recvs) {
    if (!trace_on_) return;
    std::lock_guard<std::mutex> lk(trace_mu_);
    if (trace_.empty()) trace_.resize(kTrace);
    TraceEntry& e = trace_[trace_head_ % kTrace];
    if (e.ev == nullptr) MP_HIP(hipEventCreateWithFlags(&e.ev, hipEventDisableTiming));
    MP_HIP(hipEventRecord(e.ev, cs));
    e.seq = (int64_t)trace_head_;
    e.channel = channel;
    e.kind = kind;
    e.nsend = e.nrecv = 0;
    e.bytes = 0;
    for (const auto& o : sends) {
      if (o.peer >= 0 && e.nsend < kPeers) e.send_peers[e.nsend++] = o.peer;
      e.bytes += o.count * type_bytes(o.type);
    }
    for (const auto& o : recvs) {
      if (e.nrecv < kPeers) e.recv_peers[e.nrecv++] = o.peer;
      e.bytes += o.count * type_bytes(o.type);
    }
    e.t = std::chrono::steady_clock::now();
    ++trace_head_;
  }
  bool trace_on_ = [] {
    const char* v = std::getenv("MIPIPE_COMM_TRACE");
    return v == nullptr || std::string(v) != "0";
  }();
  std::vector<TraceEntry> trace_;
  size_t trace_head_ = 0;
  std::mutex trace_mu_;     // trace_ / trace_head_: recorder thread vs watchdog (progress)

  std::vector<ncclComm_t> comm_;
  std::vector<hipStream_t> stream_;
  std::vector<int> slot_;
  std::vector<c10::hip::HIPStream> hstream_;
  std::atomic<bool> open_{true};   // read by the watchdog thread (progress / async_error)
  int nranks_, rank_, device_;
  int64_t next_ = 1;
  std::unordered_map<int64_t, hipEvent_t> pending_;
  std::vector<hipEvent_t> pool_;
};

}  // namespace mipipe_comm
