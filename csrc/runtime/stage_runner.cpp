// Native stage runner: replays one rank's pipeline step from C++ (SURVEY §7.1
// runtime/stage_runner; the executor role of torch's _PipelineScheduleRuntime,
// schedules.py:2037-2284, which the reference drives from Python).
//
// Once every compute action of the rank's lowered program has been captured as a HIP
// graph (parallel/graphs.py) and every buffer the program touches is persistent (static
// receive buffers, graph-pool outputs), a step is a fixed instruction tape:
//
//   GRAPH  g         hipGraphLaunch(g) on the compute stream
//   COPY   d, s, n   hipMemcpyAsync device -> device (a static graph input refreshed)
//   POST   e, c, ops one grouped ncclSend/ncclRecv on channel c (0: activations down the
//                    pipeline, 1: gradients up) of the RCCL engine -- that direction's own
//                    communicator and stream, ordered after the compute stream
//                    (RcclEngine::post_raw); fills a slot
//   COLL   e, c, op  one collective (all-reduce / reduce-scatter / all-gather) on channel c
//                    of an engine (the pipeline's or the DP group's): the gradient
//                    reductions of REDUCE_GRAD and of the distributed head, ordered after
//                    the compute stream on the collective stream slot; fills a slot
//   WAIT   slot, s   stream s (the compute stream or a lane) waits for that group's
//                    completion event
//   CALL   fn        a Python callable (anything not expressible above: gloo transfers and
//                    collectives on CPU) -- the GIL is taken only here; a GPU tape with the
//                    native engines holds none
//   SYNC   w, s      stream w waits for everything issued so far on stream s (an event)
//
// GRAPH, COPY and WAIT carry the stream they were issued on (0 = the compute stream): with
// microbatch lanes (parallel/runtime.py) the odd microbatches' graphs replay on a second
// stream, forked from and joined back into the compute stream by SYNCs; at PP > 1 a
// receive feeding a lane's compute is waited for on that lane, and a POST carrying a
// lane's output follows a SYNC of the compute stream on that lane.
//
// parallel/native_runner.py records the tape from one instrumented Python step and
// `run()` replays it with the GIL released: no per-action Python, no allocator calls, no
// host synchronisation -- the host issues the whole step in tens of microseconds and the
// GPU streams run ahead of it.
//
// Profiling (`set_profile(true)`): timing events are recorded on the compute stream at the
// start of the step, around every GRAPH and at the end, so the measured pipeline bubble
// (1 - busy / step) describes exactly the replayed execution that the benchmark times.
// A graph launch completes only when all its nodes have (including the dW GEMMs it forks
// onto the side stream), so its interval covers that work too.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "../comm/rccl_engine.h"

namespace py = pybind11;

namespace mipipe_runtime {

using mipipe_comm::RcclEngine;

#define MP_HIPCHK(x)                                                                         \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    TORCH_CHECK(e_ == hipSuccess, "stage runner: ", hipGetErrorString(e_), " at ", #x);      \
  } while (0)

class StageRunner {
 public:
  enum Kind { GRAPH = 0, COPY = 1, POST = 2, WAIT = 3, CALL = 4, SYNC = 5, COLL = 6 };

  explicit StageRunner(int device) : device_(device) {}
  StageRunner(const StageRunner&) = delete;
  StageRunner& operator=(const StageRunner&) = delete;
  // the SYNC / step / timing events (a still-pending event is released by HIP once it fired)
  ~StageRunner() {
    for (hipEvent_t e : sync_ev_) hipEventDestroy(e);
    for (hipEvent_t e : ev_) hipEventDestroy(e);
    if (step_ev_ != nullptr) hipEventDestroy(step_ev_);
  }

  void add_graph(int64_t graph_exec, const std::string& label, int64_t stream) {
    TORCH_CHECK(graph_exec != 0, "stage runner: null graph exec");
    Instr i;
    i.kind = GRAPH;
    i.a = graph_exec;
    i.label = label;
    i.stream = stream;
    tape_.push_back(std::move(i));
  }

  void add_copy(int64_t dst, int64_t src, int64_t nbytes, int64_t stream) {
    Instr i;
    i.kind = COPY;
    i.a = dst;
    i.b = src;
    i.c = nbytes;
    i.stream = stream;
    tape_.push_back(std::move(i));
  }

  // waiter / signal: HIP stream handles, 0 = the compute stream
  void add_sync(int64_t waiter, int64_t signal) {
    TORCH_CHECK(waiter != signal, "stage runner: SYNC of a stream with itself");
    Instr i;
    i.kind = SYNC;
    i.a = waiter;
    i.b = signal;
    i.slot = nsync_++;
    tape_.push_back(std::move(i));
  }

  // sends / recvs: (device pointer, element count, dtype code, peer); dtype codes follow
  // torch (bf16 15, f32 6, f16 5, i64 4, i32 3, u8 0, f64 7).  Returns the slot a WAIT names.
  int64_t add_post(py::object engine, int channel, const std::vector<std::tuple<int64_t, int64_t, int64_t, int64_t>>& sends,
                   const std::vector<std::tuple<int64_t, int64_t, int64_t, int64_t>>& recvs) {
    Instr i;
    i.kind = POST;
    i.engine = engine.cast<RcclEngine*>();
    i.keep = engine;
    i.channel = channel;
    for (const auto& [p, n, t, peer] : sends) i.sends.push_back({reinterpret_cast<void*>(p), (size_t)n, nccl(t), (int)peer});
    for (const auto& [p, n, t, peer] : recvs) i.recvs.push_back({reinterpret_cast<void*>(p), (size_t)n, nccl(t), (int)peer});
    i.slot = nslots_++;
    tape_.push_back(std::move(i));
    return tape_.back().slot;
  }

  // one collective: op (CollOp), send / recv device pointers, count (elements per the
  // RCCL call's convention), dtype code as in add_post.  Returns the slot a WAIT names.
  int64_t add_coll(py::object engine, int channel, int op, int64_t send, int64_t recv, int64_t count, int64_t dtype) {
    Instr i;
    i.kind = COLL;
    i.engine = engine.cast<RcclEngine*>();
    i.keep = engine;
    i.channel = channel;
    i.a = send;
    i.b = recv;
    i.c = count;
    i.op = op;
    i.dtype = nccl(dtype);
    i.slot = nslots_++;
    tape_.push_back(std::move(i));
    return tape_.back().slot;
  }

  // stream: the waiting stream (0 = the compute stream; a microbatch lane's stream when the
  // receive feeds a compute issued on that lane)
  void add_wait(int64_t slot, int64_t stream) {
    TORCH_CHECK(slot >= 0 && slot < nslots_, "stage runner: bad slot ", slot);
    Instr i;
    i.kind = WAIT;
    i.slot = slot;
    i.stream = stream;
    tape_.push_back(std::move(i));
  }

  void add_call(py::function fn) {
    Instr i;
    i.kind = CALL;
    i.fn = std::move(fn);
    tape_.push_back(std::move(i));
  }

  void set_profile(bool on) { profile_ = on; }
  // receive-only POSTs ordered after the step's start instead of the compute stream
  // (RcclEngine::post_raw ``after``; PipelineRuntime turns it on with MIPIPE_RECV_EARLY)
  void set_recv_early(bool on) { recv_early_ = on; }
  bool recv_early() const { return recv_early_; }

  // one step on the current HIP stream of `device`
  void run() {
    hipStream_t st = c10::hip::getCurrentHIPStream(device_).stream();
    std::vector<int64_t> handles(nslots_, -1);
    std::vector<RcclEngine*> engines(nslots_, nullptr);
    std::vector<char> waited(nslots_, 0);
    const bool prof = profile_;
    if (prof) prepare_events();
    while ((int64_t)sync_ev_.size() < nsync_) {
      hipEvent_t e;
      MP_HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      sync_ev_.push_back(e);
    }
    auto on = [st](int64_t s) { return s ? reinterpret_cast<hipStream_t>(s) : st; };
    if (recv_early_ && step_ev_ == nullptr) MP_HIPCHK(hipEventCreateWithFlags(&step_ev_, hipEventDisableTiming));
    py::gil_scoped_release nogil;
    int ng = 0;
    // everything before this step (the previous step's readers of every receive slot, its
    // lanes joined back, the optimizer) is ordered before this event
    if (recv_early_) MP_HIPCHK(hipEventRecord(step_ev_, st));
    if (prof) MP_HIPCHK(hipEventRecord(ev_[0], st));
    for (const Instr& i : tape_) {
      switch (i.kind) {
        case GRAPH: {
          hipStream_t gs = on(i.stream);
          if (prof) MP_HIPCHK(hipEventRecord(ev_[2 + 2 * ng], gs));
          MP_HIPCHK(hipGraphLaunch(reinterpret_cast<hipGraphExec_t>(i.a), gs));
          if (prof) MP_HIPCHK(hipEventRecord(ev_[3 + 2 * ng], gs));
          ++ng;
          break;
        }
        case COPY:
          MP_HIPCHK(hipMemcpyAsync(reinterpret_cast<void*>(i.a), reinterpret_cast<const void*>(i.b), (size_t)i.c,
                                   hipMemcpyDeviceToDevice, on(i.stream)));
          break;
        case SYNC:
          MP_HIPCHK(hipEventRecord(sync_ev_[i.slot], on(i.b)));
          MP_HIPCHK(hipStreamWaitEvent(on(i.a), sync_ev_[i.slot], 0));
          break;
        case POST:
          handles[i.slot] = i.engine->post_raw(i.channel, i.sends, i.recvs, st,
                                               (recv_early_ && i.sends.empty()) ? step_ev_ : nullptr);
          engines[i.slot] = i.engine;
          break;
        case COLL:
          handles[i.slot] = i.engine->coll_raw(i.channel, i.op, reinterpret_cast<void*>(i.a),
                                               reinterpret_cast<void*>(i.b), (size_t)i.c, i.dtype, st);
          engines[i.slot] = i.engine;
          break;
        case WAIT:
          // non-consuming: a group feeding computes on two lanes is waited on by both
          TORCH_CHECK(handles[i.slot] >= 0, "stage runner: WAIT before its POST (slot ", i.slot, ")");
          engines[i.slot]->wait_keep_raw(handles[i.slot], on(i.stream));
          waited[i.slot] = 1;
          break;
        case CALL: {
          py::gil_scoped_acquire gil;
          i.fn();
          break;
        }
      }
    }
    // groups whose completion nobody waited for (sends): order them before the next step;
    // then every handle's event goes back to its engine's pool
    for (int64_t s = 0; s < nslots_; ++s) {
      if (handles[s] < 0) continue;
      if (!waited[s]) engines[s]->wait_keep_raw(handles[s], st);
      engines[s]->release(handles[s]);
    }
    if (prof) {
      MP_HIPCHK(hipEventRecord(ev_[1], st));
      profiled_ = true;
    }
    ++runs_;
  }

  // Last profiled step: (label, start_ms, end_ms) per GRAPH relative to the step start,
  // and the step's total time on the compute stream.  Blocks until the step finished.
  std::pair<std::vector<std::tuple<std::string, double, double>>, double> timeline() {
    std::vector<std::tuple<std::string, double, double>> out;
    TORCH_CHECK(profiled_, "stage runner: no profiled step (set_profile(True) and run())");
    MP_HIPCHK(hipEventSynchronize(ev_[1]));
    float total = 0.f;
    MP_HIPCHK(hipEventElapsedTime(&total, ev_[0], ev_[1]));
    int ng = 0;
    for (const Instr& i : tape_) {
      if (i.kind != GRAPH) continue;
      float s = 0.f, e = 0.f;
      MP_HIPCHK(hipEventElapsedTime(&s, ev_[0], ev_[2 + 2 * ng]));
      MP_HIPCHK(hipEventElapsedTime(&e, ev_[0], ev_[3 + 2 * ng]));
      out.emplace_back(i.label, (double)s, (double)e);
      ++ng;
    }
    return {out, (double)total};
  }

  int64_t size() const { return (int64_t)tape_.size(); }
  int64_t runs() const { return runs_; }
  std::vector<int64_t> kinds() const {
    std::vector<int64_t> k;
    for (const auto& i : tape_) k.push_back(i.kind);
    return k;
  }
  std::vector<int64_t> channels() const {
    std::vector<int64_t> k;
    for (const auto& i : tape_)
      if (i.kind == POST) k.push_back(i.channel);
    return k;
  }
  // (channel, op) of every COLL, in tape order
  std::vector<std::pair<int64_t, int64_t>> collectives() const {
    std::vector<std::pair<int64_t, int64_t>> k;
    for (const auto& i : tape_)
      if (i.kind == COLL) k.emplace_back(i.channel, i.op);
    return k;
  }

 private:
  void prepare_events() {
    int64_t ng = 0;
    for (const auto& i : tape_) ng += i.kind == GRAPH;
    const size_t need = (size_t)(2 + 2 * ng);
    while (ev_.size() < need) {
      hipEvent_t e;
      MP_HIPCHK(hipEventCreate(&e));  // timing enabled
      ev_.push_back(e);
    }
  }

  struct Instr {
    int kind = GRAPH;
    int64_t a = 0, b = 0, c = 0;
    int64_t slot = -1;
    int64_t stream = 0;  // GRAPH / COPY / WAIT: issuing (waiting) stream (0 = compute stream)
    int channel = 0;
    int op = 0;
    ncclDataType_t dtype = ncclFloat32;
    std::string label;
    RcclEngine* engine = nullptr;
    py::object keep;  // keeps the engine alive
    std::vector<RcclEngine::RawOp> sends, recvs;
    py::function fn;
  };

  static ncclDataType_t nccl(int64_t code) {
    switch (code) {
      case 15: return ncclBfloat16;
      case 6: return ncclFloat32;
      case 5: return ncclFloat16;
      case 4: return ncclInt64;
      case 3: return ncclInt32;
      case 0: return ncclUint8;
      case 7: return ncclFloat64;
      default: TORCH_CHECK(false, "stage runner: unsupported dtype code ", code);
    }
    return ncclFloat32;
  }

  int device_;
  std::vector<Instr> tape_;
  int64_t nslots_ = 0;
  int64_t nsync_ = 0;
  std::vector<hipEvent_t> sync_ev_;
  int64_t runs_ = 0;
  bool profile_ = false;
  bool recv_early_ = false;
  hipEvent_t step_ev_ = nullptr;
  bool profiled_ = false;
  std::vector<hipEvent_t> ev_;
};

void register_runner(py::module& m) {
  py::class_<StageRunner>(m, "StageRunner")
      .def(py::init<int>(), py::arg("device"))
      .def("add_graph", &StageRunner::add_graph, py::arg("graph_exec"), py::arg("label") = "",
           py::arg("stream") = 0)
      .def("add_copy", &StageRunner::add_copy, py::arg("dst"), py::arg("src"), py::arg("nbytes"),
           py::arg("stream") = 0)
      .def("add_sync", &StageRunner::add_sync, py::arg("waiter"), py::arg("signal"))
      .def("add_post", &StageRunner::add_post)
      .def("add_coll", &StageRunner::add_coll)
      .def("add_wait", &StageRunner::add_wait, py::arg("slot"), py::arg("stream") = 0)
      .def("add_call", &StageRunner::add_call)
      .def("run", &StageRunner::run)
      .def("set_profile", &StageRunner::set_profile)
      .def("set_recv_early", &StageRunner::set_recv_early)
      .def("recv_early", &StageRunner::recv_early)
      .def("timeline", &StageRunner::timeline)
      .def("kinds", &StageRunner::kinds)
      .def("channels", &StageRunner::channels)
      .def("collectives", &StageRunner::collectives)
      .def_property_readonly("size", &StageRunner::size)
      .def_property_readonly("runs", &StageRunner::runs);
}

}  // namespace mipipe_runtime
