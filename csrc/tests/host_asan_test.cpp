// Host build of the native runtime under AddressSanitizer + UndefinedBehaviorSanitizer.
//
// stage_runner.cpp (and through it comm/rccl_engine.h) is compiled with plain g++ against the
// stand-in headers in host_stubs/: HIP streams become FIFOs of host work, events heap
// objects, RCCL a two-rank in-process fabric reached through the engine's own function
// table (mipipe_comm::g_rccl).  Two ranks then replay pipeline tapes -- COPY, GRAPH, SYNC,
// POST (send and receive-early), WAIT, COLL, CALL, profiled timelines -- for many steps,
// with a second thread polling the engines' progress() the way the watchdog does, then go
// through the error, close and abort paths.  Any heap misuse, leak (event pools, trace ring,
// runner events), data race on the trace ring that corrupts memory, or undefined behaviour
// is a sanitizer report and a non-zero exit.
//
//   python tools/build_ext.py --asan-host        (builds build/host_asan_test and runs it)
#include "../runtime/stage_runner.cpp"

#include <atomic>
#include <cmath>
#include <cstdio>
#include <thread>

#include <sanitizer/lsan_interface.h>

using mipipe_comm::RcclEngine;
using mipipe_runtime::StageRunner;

// ---------------------------------------------------------------- in-process RCCL fabric
struct FakeComm {
  std::string key;
  int nranks = 0, rank = 0;
  int64_t coll_seq = 0;
};

namespace fabric {
struct Message {
  std::vector<char> data;
};
// (key, src, dst) -> FIFO of messages
std::map<std::tuple<std::string, int, int>, std::deque<Message>> mail;
struct Coll {
  std::vector<std::vector<char>> part;
  int deposited = 0, done = 0;
};
std::map<std::pair<std::string, int64_t>, Coll> colls;
int64_t next_id = 0, sends = 0, recvs = 0, collectives = 0, group_depth = 0;
}  // namespace fabric

static ncclResult_t f_GetUniqueId(ncclUniqueId* id) {
  std::memset(id->internal, 0, sizeof(id->internal));
  std::snprintf(id->internal, sizeof(id->internal), "fake-comm-%lld", (long long)fabric::next_id++);
  return ncclSuccess;
}
static ncclResult_t f_CommInitRank(ncclComm_t* c, int nranks, ncclUniqueId id, int rank) {
  auto* fc = new FakeComm();
  fc->key = std::string(id.internal);
  fc->nranks = nranks;
  fc->rank = rank;
  *c = fc;
  return ncclSuccess;
}
static ncclResult_t f_CommDestroy(ncclComm_t c) {
  delete c;
  return ncclSuccess;
}
static ncclResult_t f_CommGetAsyncError(ncclComm_t, ncclResult_t* r) {
  *r = ncclSuccess;
  return ncclSuccess;
}
static ncclResult_t f_Send(const void* p, size_t n, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
  ++fabric::sends;
  const size_t bytes = n * mipipe_comm::nccl_size(t);
  const auto key = std::make_tuple(c->key, c->rank, peer);
  s->work.push_back([p, bytes, key] {
    fabric::Message m;
    m.data.resize(bytes);
    std::memcpy(m.data.data(), p, bytes);
    fabric::mail[key].push_back(std::move(m));
    return true;
  });
  return ncclSuccess;
}
static ncclResult_t f_Recv(void* p, size_t n, ncclDataType_t t, int peer, ncclComm_t c, hipStream_t s) {
  ++fabric::recvs;
  const size_t bytes = n * mipipe_comm::nccl_size(t);
  const auto key = std::make_tuple(c->key, peer, c->rank);
  s->work.push_back([p, bytes, key] {
    auto& q = fabric::mail[key];
    if (q.empty()) return false;
    if (q.front().data.size() != bytes) {
      std::fprintf(stderr, "fabric: message size %zu != receive %zu\n", q.front().data.size(), bytes);
      std::abort();
    }
    std::memcpy(p, q.front().data.data(), bytes);
    q.pop_front();
    return true;
  });
  return ncclSuccess;
}
// float32 sum / max, or byte gather; every rank deposits its send buffer, the last reader
// retires the entry
static ncclResult_t coll(int kind, const void* send, void* recv, size_t n, ncclDataType_t t, ncclComm_t c,
                         hipStream_t s) {
  ++fabric::collectives;
  if (kind != 2 && t != ncclFloat32) return ncclInvalidArgument;
  const size_t es = mipipe_comm::nccl_size(t);
  const int R = c->nranks, me = c->rank;
  const auto key = std::make_pair(c->key, c->coll_seq++);
  const size_t in_bytes = (kind == 1 ? n * R : n) * es;   // reduce-scatter sends R x n
  auto deposited = std::make_shared<bool>(false);
  s->work.push_back([=] {
    auto& e = fabric::colls[key];
    if (!*deposited) {
      if (e.part.empty()) e.part.resize(R);
      e.part[me].assign((const char*)send, (const char*)send + in_bytes);
      ++e.deposited;
      *deposited = true;
    }
    if (e.deposited < R) return false;
    if (kind == 2) {   // all-gather
      for (int r = 0; r < R; ++r) std::memcpy((char*)recv + r * n * es, e.part[r].data(), n * es);
    } else {
      float* out = (float*)recv;
      const size_t off = kind == 1 ? me * n : 0;
      for (size_t i = 0; i < n; ++i) {
        float acc = kind == 3 ? -INFINITY : 0.f;
        for (int r = 0; r < R; ++r) {
          const float v = ((const float*)e.part[r].data())[off + i];
          acc = kind == 3 ? std::max(acc, v) : acc + v;
        }
        out[i] = acc;
      }
    }
    if (++e.done == R) fabric::colls.erase(key);
    return true;
  });
  return ncclSuccess;
}
static ncclResult_t f_AllReduce(const void* a, void* b, size_t n, ncclDataType_t t, ncclRedOp_t op, ncclComm_t c,
                                hipStream_t s) {
  return coll(op == ncclMax ? 3 : 0, a, b, n, t, c, s);
}
static ncclResult_t f_ReduceScatter(const void* a, void* b, size_t n, ncclDataType_t t, ncclRedOp_t, ncclComm_t c,
                                    hipStream_t s) {
  return coll(1, a, b, n, t, c, s);
}
static ncclResult_t f_AllGather(const void* a, void* b, size_t n, ncclDataType_t t, ncclComm_t c, hipStream_t s) {
  return coll(2, a, b, n, t, c, s);
}
static ncclResult_t f_GroupStart() {
  ++fabric::group_depth;
  return ncclSuccess;
}
static ncclResult_t f_GroupEnd() {
  --fabric::group_depth;
  return ncclSuccess;
}
static const char* f_GetErrorString(ncclResult_t r) { return r == ncclSuccess ? "ok" : "fake rccl error"; }

static void install_fake_rccl() {
  static mipipe_comm::Rccl r;
  r.GetUniqueId = f_GetUniqueId;
  r.CommInitRank = f_CommInitRank;
  r.CommDestroy = f_CommDestroy;
  r.CommAbort = f_CommDestroy;
  r.CommGetAsyncError = f_CommGetAsyncError;
  r.Send = f_Send;
  r.Recv = f_Recv;
  r.AllReduce = f_AllReduce;
  r.ReduceScatter = f_ReduceScatter;
  r.AllGather = f_AllGather;
  r.GroupStart = f_GroupStart;
  r.GroupEnd = f_GroupEnd;
  r.GetErrorString = f_GetErrorString;
  mipipe_comm::g_rccl = &r;
}

// ---------------------------------------------------------------- helpers
static int failures = 0;
#define EXPECT(c)                                                                  \
  do {                                                                             \
    if (!(c)) {                                                                    \
      std::fprintf(stderr, "EXPECT failed %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      ++failures;                                                                  \
    }                                                                              \
  } while (0)

template <typename F>
static bool throws(F f) {
  try {
    f();
  } catch (const std::runtime_error&) {
    return true;
  }
  return false;
}

static pybind11::bytes ids(int n) {
  std::string s;
  for (int c = 0; c < n; ++c) s += RcclEngine::unique_id();
  return pybind11::bytes(s);
}
static int64_t h(const void* p) { return reinterpret_cast<int64_t>(p); }

// ---------------------------------------------------------------- the two-rank pipeline
// rank 0: x -> (COPY) act -> POST send ch0 -> POST recv grad ch1 (WAIT on a lane, SYNC back)
//         -> GRAPH -> COLL all-reduce(ch2) of w -> CALL
// rank 1: POST recv act ch0 (receive-early) -> WAIT -> COPY act -> grad -> GRAPH on a lane
//         -> SYNC -> POST send grad ch1 -> COLL all-reduce(ch2) of w
static void pipeline(bool recv_early, bool profile, int steps) {
  const int N = 1024;
  const pybind11::bytes uid = ids(3);
  auto e0 = std::make_shared<RcclEngine>(uid, 2, 0, 0, std::vector<int64_t>{0, 1, 2});
  auto e1 = std::make_shared<RcclEngine>(uid, 2, 1, 1, std::vector<int64_t>{0, 1, 2});
  pybind11::object o0 = pybind11::object::of(e0), o1 = pybind11::object::of(e1);
  std::vector<float> x(N), act0(N), grad0(N), w0(N), act1(N), grad1(N), w1(N);
  hipStream_t lane0 = fake_hip::make_stream(), lane1 = fake_hip::make_stream();
  int calls = 0;
  {
    StageRunner r0(0), r1(1);
    r0.add_copy(h(act0.data()), h(x.data()), N * 4, 0);
    const int64_t s_send = r0.add_post(o0, 0, {{h(act0.data()), N, 6, 1}}, {});
    const int64_t s_recv = r0.add_post(o0, 1, {}, {{h(grad0.data()), N, 6, 1}});
    r0.add_sync(h(lane0), 0);
    r0.add_wait(s_recv, h(lane0));
    r0.add_graph(0x1234, "B0", h(lane0));
    r0.add_sync(0, h(lane0));
    const int64_t s_ar = r0.add_coll(o0, 2, mipipe_comm::ALLREDUCE_SUM, h(w0.data()), h(w0.data()), N, 6);
    r0.add_wait(s_ar, 0);
    r0.add_call(pybind11::function([&calls] { ++calls; }));
    (void)s_send;

    const int64_t t_recv = r1.add_post(o1, 0, {}, {{h(act1.data()), N, 6, 0}});
    r1.add_wait(t_recv, h(lane1));
    r1.add_sync(h(lane1), 0);
    r1.add_copy(h(grad1.data()), h(act1.data()), N * 4, h(lane1));
    r1.add_graph(0x5678, "F0", h(lane1));
    r1.add_sync(0, h(lane1));
    r1.add_post(o1, 1, {{h(grad1.data()), N, 6, 0}}, {});
    const int64_t t_ar = r1.add_coll(o1, 2, mipipe_comm::ALLREDUCE_SUM, h(w1.data()), h(w1.data()), N, 6);
    r1.add_wait(t_ar, 0);
    r1.set_recv_early(recv_early);
    r0.set_profile(profile);
    EXPECT(r0.size() == 10 && r1.size() == 9);
    EXPECT(r1.recv_early() == recv_early);

    std::atomic<bool> stop{false};
    std::thread watchdog([&] {   // progress() / issued() race the recorder as in the real watchdog
      while (!stop.load()) {
        pybind11::list l0 = e0->progress(), l1 = e1->progress();
        (void)l0.size();
        (void)l1.size();
        (void)e0->issued();
        std::this_thread::yield();
      }
    });
    for (int step = 0; step < steps; ++step) {
      for (int i = 0; i < N; ++i) {
        x[i] = (float)(step * N + i);
        w0[i] = 1.f + i;
        w1[i] = 2.f * i;
      }
      r0.run();
      r1.run();
      EXPECT(fake_hip::drain());   // the tapes of both ranks complete: no cross-rank deadlock
      bool ok = true;
      for (int i = 0; i < N; ++i) {
        ok &= act1[i] == x[i];              // activation reached rank 1
        ok &= grad0[i] == x[i];             // and came back as the gradient
        ok &= w0[i] == 1.f + 3.f * i;       // all-reduced on both ranks
        ok &= w1[i] == 1.f + 3.f * i;
      }
      EXPECT(ok);
      if (profile && step % 7 == 0) {
        auto tl = r0.timeline();
        EXPECT(tl.first.size() == 1 && std::get<0>(tl.first[0]) == "B0");
        EXPECT(tl.second > 0.0);
      }
    }
    stop.store(true);
    watchdog.join();
    EXPECT(calls == steps);
    EXPECT(r0.runs() == steps && r1.runs() == steps);
    EXPECT(e0->issued() == 3 * steps);   // > 256: the trace ring wrapped
    EXPECT(e0->progress().size() == 0);   // nothing left in flight
    EXPECT(e0->async_error().empty());
  }   // runners destroyed: their SYNC / step / timing events freed
  e0->close();
  e1->close();
  EXPECT(e0->async_error() == "closed");
  EXPECT(throws([&] { e0->post_raw(0, {}, {}, c10::hip::getCurrentHIPStream(0).stream()); }));
  fake_hip::free_stream(lane0);
  fake_hip::free_stream(lane1);
}

// reduce-scatter / all-gather / max on the raw entry points, and the torch-form wrappers
static void collectives() {
  const int N = 256;
  const pybind11::bytes uid = ids(1);
  RcclEngine a(uid, 2, 0, 0, {2}), b(uid, 2, 1, 1, {2});
  std::vector<float> sa(2 * N), sb(2 * N), ra(N), rb(N), ga(2 * N), gb(2 * N);
  for (int i = 0; i < 2 * N; ++i) {
    sa[i] = (float)i;
    sb[i] = 10.f * i;
  }
  hipStream_t ca = c10::hip::getCurrentHIPStream(0).stream(), cb = c10::hip::getCurrentHIPStream(1).stream();
  int64_t ha = a.coll_raw(0, mipipe_comm::REDUCE_SCATTER_SUM, sa.data(), ra.data(), N, ncclFloat32, ca);
  int64_t hb = b.coll_raw(0, mipipe_comm::REDUCE_SCATTER_SUM, sb.data(), rb.data(), N, ncclFloat32, cb);
  a.wait_raw(ha, ca);
  b.wait_raw(hb, cb);
  EXPECT(fake_hip::drain());
  for (int i = 0; i < N; ++i) {
    EXPECT(ra[i] == 11.f * i);
    EXPECT(rb[i] == 11.f * (N + i));
  }
  // torch-form: tensors over the same host buffers
  torch::Tensor tra{ra.data(), N, torch::kFloat32}, tga{ga.data(), 2 * N, torch::kFloat32};
  torch::Tensor trb{rb.data(), N, torch::kFloat32}, tgb{gb.data(), 2 * N, torch::kFloat32};
  ha = a.coll(0, mipipe_comm::ALL_GATHER, tra, tga);
  hb = b.coll(0, mipipe_comm::ALL_GATHER, trb, tgb);
  a.wait(ha);
  b.wait_keep(hb);
  b.release(hb);
  EXPECT(fake_hip::drain());
  EXPECT(a.query(ha) && b.query(hb));
  for (int i = 0; i < N; ++i) EXPECT(ga[i] == 11.f * i && gb[N + i] == 11.f * (N + i));
  ha = a.coll(0, mipipe_comm::ALLREDUCE_MAX, tra, tra);
  hb = b.coll(0, mipipe_comm::ALLREDUCE_MAX, trb, trb);
  a.synchronize();
  EXPECT(a.query(ha) && b.query(hb));
  EXPECT(ra[5] == 11.f * (N + 5));
  // argument checks throw (and leak nothing)
  torch::Tensor bad{ra.data(), N + 1, torch::kFloat32};
  EXPECT(throws([&] { a.coll(0, mipipe_comm::ALLREDUCE_SUM, tra, bad); }));
  EXPECT(throws([&] { a.coll(0, mipipe_comm::ALL_GATHER, tra, tra); }));
  EXPECT(throws([&] { a.coll(0, 99, tra, tra); }));
  torch::Tensor host{ra.data(), N, torch::kFloat32, false};
  EXPECT(throws([&] { a.coll(0, mipipe_comm::ALLREDUCE_SUM, host, host); }));
  EXPECT(throws([&] { a.post_raw(0, {{ra.data(), 4, ncclFloat32, 2}}, {}, ca); }));   // bad peer
  EXPECT(throws([&] { a.post_raw(1, {}, {}, ca); }));                                  // bad channel
  // torch-form post: a group with one send and one receive each way
  std::vector<float> pa(N, 3.f), pb(N, 4.f), qa(N), qb(N);
  torch::Tensor tpa{pa.data(), N, torch::kFloat32}, tpb{pb.data(), N, torch::kFloat32};
  torch::Tensor tqa{qa.data(), N, torch::kFloat32}, tqb{qb.data(), N, torch::kFloat32};
  ha = a.post(0, {{tpa, 1}}, {{tqa, 1}});
  hb = b.post(0, {{tpb, 0}}, {{tqb, 0}});
  a.wait(ha);
  b.wait(hb);
  EXPECT(fake_hip::drain());
  EXPECT(qa[7] == 4.f && qb[7] == 3.f);
  EXPECT(fabric::group_depth == 0);
  fake_hip::drain();
}

// a runner whose tape is malformed or whose engine is gone
static void runner_errors() {
  const pybind11::bytes uid = ids(1);
  auto e = std::make_shared<RcclEngine>(uid, 1, 0, 0, std::vector<int64_t>{0});
  pybind11::object o = pybind11::object::of(e);
  StageRunner r(0);
  EXPECT(throws([&] { r.add_graph(0, "", 0); }));
  EXPECT(throws([&] { r.add_sync(5, 5); }));
  EXPECT(throws([&] { r.add_wait(0, 0); }));   // no slot yet
  EXPECT(throws([&] { r.add_post(o, 0, {{16, 1, 99, 0}}, {}); }));   // dtype code
  std::vector<float> buf(8);
  const int64_t s = r.add_post(o, 0, {{h(buf.data()), 8, 6, 0}}, {{h(buf.data()), 8, 6, 0}});
  r.add_wait(s, 0);
  r.set_recv_early(true);
  r.set_profile(true);
  EXPECT(throws([&] { r.timeline(); }));   // not profiled yet
  r.run();
  EXPECT(fake_hip::drain());
  auto tl = r.timeline();
  EXPECT(tl.first.empty());
  EXPECT(r.kinds().size() == 2 && r.channels() == std::vector<int64_t>{0});
  EXPECT(r.collectives().empty());
  e->close();
  EXPECT(throws([&] { r.run(); }));   // engine closed: the POST throws out of run()
  fake_hip::drain();
}

// abort with transfers in flight: receives that never get their message
static void abort_in_flight() {
  const pybind11::bytes uid = ids(2);
  RcclEngine e(uid, 2, 0, 0, {0, 1});
  std::vector<float> buf(64);
  hipStream_t c = c10::hip::getCurrentHIPStream(0).stream();
  for (int i = 0; i < 40; ++i) e.post_raw(i % 2, {}, {{buf.data(), 64, ncclFloat32, 1}}, c);
  EXPECT(!fake_hip::drain());   // stuck: rank 1 never sends
  EXPECT(e.progress().size() > 0);
  e.abort();
  EXPECT(e.async_error() == "closed");
  // the stuck receives are dropped with their stream's work (the comm stream is shared by
  // slot, so clear it for later tests)
  for (FakeStream* s : fake_hip::streams()) s->work.clear();
  fabric::mail.clear();
}

// with receive-early a receive-only POST does not wait for the compute the
// tape issued before it.  Rank 1's tape is [GRAPH (held running)] [POST recv] [WAIT]; rank 0
// sends.  The receive lands while the graph is still running only with receive-early on.
static void recv_early_semantics(bool early) {
  const int N = 512;
  const pybind11::bytes uid = ids(1);
  auto e0 = std::make_shared<RcclEngine>(uid, 2, 0, 0, std::vector<int64_t>{0});
  auto e1 = std::make_shared<RcclEngine>(uid, 2, 1, 1, std::vector<int64_t>{0});
  std::vector<float> act0(N, 7.f), act1(N, 0.f);
  bool running = true;
  hipGraphExec_t long_graph = reinterpret_cast<hipGraphExec_t>(0xbeef);
  fake_hip::graph_body = [&](hipGraphExec_t g) { return g != long_graph || !running; };
  {
    StageRunner r0(0), r1(1);
    r0.add_post(pybind11::object::of(e0), 0, {{h(act0.data()), N, 6, 1}}, {});
    r1.add_graph(h(long_graph), "F0", 0);
    const int64_t s = r1.add_post(pybind11::object::of(e1), 0, {}, {{h(act1.data()), N, 6, 0}});
    r1.add_wait(s, 0);
    r1.set_recv_early(early);
    r0.run();
    r1.run();
    EXPECT(!fake_hip::drain());          // rank 1's compute stream is held by the graph
    EXPECT((act1[3] == 7.f) == early);   // ... yet the receive landed iff receive-early
    running = false;
    EXPECT(fake_hip::drain());
    EXPECT(act1[3] == 7.f);
  }
  fake_hip::graph_body = [](hipGraphExec_t) { return true; };
  e0->close();
  e1->close();
}

int main() {
  install_fake_rccl();
  pipeline(false, false, 40);
  pipeline(true, true, 120);
  collectives();
  runner_errors();
  abort_in_flight();
  recv_early_semantics(false);
  recv_early_semantics(true);
  for (int i = 0; i < 3; ++i) pipeline(i % 2 == 0, i == 1, 10);
  EXPECT(fabric::colls.empty());
  // leak check now, while the process-wide statics (comm streams, parked events) still hold
  // what they own: exit-time destructors would free the containers and orphan their entries
  __lsan_do_leak_check();
  std::printf("host_asan_test: %lld sends, %lld recvs, %lld collectives, %lld graph launches, %lld events recorded; "
              "%d failures\n",
              (long long)fabric::sends, (long long)fabric::recvs, (long long)fabric::collectives,
              (long long)fake_hip::graph_launches, (long long)fake_hip::records, failures);
  return failures == 0 ? 0 : 1;
}
