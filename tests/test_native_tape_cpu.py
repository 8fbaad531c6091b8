"""The native stage runner's tape at PP=4, on CPU/gloo with stand-ins for the GPU parts.

On a GPU a step after graph capture is recorded into ``StageRunner``
(csrc/runtime/stage_runner.cpp) as GRAPH / COPY / POST / WAIT / CALL instructions and
replayed from C++.  Multi-rank RCCL cannot run on a one-GPU box, so this test swaps in:

* ``FakeGraphCache`` -- "captures" an action by running it and replays it by re-running it
  into the same persistent output tensors (what a HIP graph replay does);
* ``FakeEngine`` -- the native RCCL engine's interface (two channels, post/wait), moving
  data over one gloo group per channel;
* ``FakeRunner`` -- ``StageRunner``'s interface; ``run()`` replays the tape in Python.

* ``FakeEngine.coll`` -- the engines' collectives (the pipeline engine's collective
  channel, the DP engine), run on gloo.

It checks that a recorded PP=4 step (x DP=2, distributed ZeRO-1 head) holds only
GRAPH/COPY/POST/WAIT/COLL -- no Python CALL: the DP all-reduce of REDUCE_GRAD and the
head's reduce-scatter + shard all-reduce of REDUCE_HEAD are native COLL instructions --
that both p2p channels carry POSTs, and that replaying the tape trains exactly like the
Python executor.
"""
import queue
import threading
import types

import pytest
import torch
import torch.distributed as dist

import mipipe  # noqa: F401
from mipipe.engine import PipelineTrainer
from mipipe.models.config import NativeConfig
from mipipe.parallel import native_runner
from mipipe.parallel.graphs import GraphCache
from mipipe.parallel.runtime import PipelineRuntime

from dist_utils import run_world

GRAPH, COPY, POST, WAIT, CALL, SYNC, COLL = range(7)


def _nested_copy(dst, src):
    if isinstance(dst, torch.Tensor):
        dst.copy_(src)
    elif isinstance(dst, (tuple, list)):
        for d, s_ in zip(dst, src):
            _nested_copy(d, s_)


class FakeGraph:
    reg = {}

    def __init__(self, fn, static_in, out):
        self.fn, self.static_in, self.out = fn, static_in, out
        FakeGraph.reg[id(self)] = self

    def raw_cuda_graph_exec(self):
        return id(self)

    def replay(self):
        _nested_copy(self.out, self.fn(self.static_in))


class FakeGraphCache(GraphCache):
    def run(self, key, inputs, fn, keep=None, pool=None):
        rec = native_runner.active()
        entry = self.graphs.get(key)
        if entry is None:
            if rec is not None:
                rec.invalidate("capture during recording")
            static_in = list(inputs)
            out = fn(static_in)
            g = FakeGraph(fn, static_in, out)
            self.graphs[key] = entry = (g, static_in, out, [])
            self.captures += 1
            if rec is not None:
                rec.graph(g, self.label(key))
            return out
        g, static_in, out, _ = entry
        for s_, t in zip(static_in, inputs):
            if s_.data_ptr() != t.data_ptr():
                s_.copy_(t)
                if rec is not None:
                    rec.copy(s_, t)
        self.replays += 1
        g.replay()
        if rec is not None:
            rec.graph(g, self.label(key))
        return out


class _Job:
    def __init__(self, fn):
        self.fn, self.ev, self.err = fn, threading.Event(), None

    def wait(self):
        if not self.ev.wait(180):
            raise TimeoutError("collective FIFO job did not finish")
        if self.err is not None:
            raise self.err


class _CollFIFO:
    """One worker thread executing collectives in issue order (the comm stream)."""

    def __init__(self):
        self.q = queue.Queue()
        threading.Thread(target=self._run, daemon=True).start()

    def _run(self):
        while True:
            job = self.q.get()
            try:
                job.fn()
            except BaseException as e:  # noqa: BLE001 - re-raised at wait
                job.err = e
            job.ev.set()

    def submit(self, fn):
        job = _Job(fn)
        self.q.put(job)
        return job


_FIFO = []


def _fifo():
    if not _FIFO:
        _FIFO.append(_CollFIFO())
    return _FIFO[0]


class FakeEngine:
    """Native engine stand-in: channel c -> its own gloo group (independent matching)."""

    def __init__(self, groups, ranks):
        self.groups, self.ranks, self.channels = groups, ranks, len(groups)
        self.reg, self.pending, self.next = {}, {}, 1
        self.posts = [0] * len(groups)
        self.colls = 0

    def post(self, ch, sends, recvs):
        ops = []
        for t, p in sends:
            self.reg[t.data_ptr()] = t
            ops.append(dist.P2POp(dist.isend, t, self.ranks[p], self.groups[ch]))
        for t, p in recvs:
            self.reg[t.data_ptr()] = t
            ops.append(dist.P2POp(dist.irecv, t, self.ranks[p], self.groups[ch]))
        h = self.next
        self.next += 1
        self.pending[h] = dist.batch_isend_irecv(ops) if ops else []
        self.posts[ch] += 1
        return h

    def coll(self, ch, op, send, recv):
        """Collectives run in ONE FIFO per process, off the host thread -- the real engines
        issue every collective on one comm stream (a later collective always sees an
        earlier one's result) that runs independently of the p2p streams and the host
        (the overlapped placement's independent-queue model)."""
        # (by object, not pointer: an in-place reduce-scatter's block 0 shares the pointer)
        self.last_coll = (send, recv)
        g = self.groups[ch]

        def fn():
            if op in (0, 3):
                dist.all_reduce(recv, op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MAX, group=g)
            elif op == 1:     # reduce-scatter in place: recv is this rank's block of send
                dist.all_reduce(send, group=g)
            else:             # all-gather in place: send is this rank's block of recv
                parts = [torch.empty_like(send) for _ in range(dist.get_world_size(g))]
                dist.all_gather(parts, send.clone(), group=g)
                recv.copy_(torch.cat(parts).view_as(recv))
        self.colls += 1
        h = self.next
        self.next += 1
        self.pending[h] = [_fifo().submit(fn)]
        return h

    def wait(self, h):
        for w in self.pending.pop(h, []):
            w.wait()

    def wait_keep(self, h):     # host-side stand-in: completes the group (idempotent)
        self.wait(h)

    def release(self, h):
        self.pending.pop(h, None)

    def query(self, h):
        return True

    def abort(self):
        pass


class FakeRunner:
    def __init__(self, device):
        self.tape, self.nslots, self.runs = [], 0, 0
        self.labels = []

    def add_graph(self, g, label=""):
        self.tape.append((GRAPH, FakeGraph.reg[g]))
        self.labels.append((len(self.tape) - 1, label))

    def add_copy_t(self, dst, src):
        self.tape.append((COPY, (dst, src)))

    def add_post(self, engine, ch, sends, recvs):
        res = lambda lst: [(engine.reg[ptr], peer) for ptr, n, code, peer in lst]
        self.tape.append((POST, (engine, ch, res(sends), res(recvs), self.nslots)))
        self.nslots += 1
        return self.nslots - 1

    def add_coll(self, engine, ch, op, send, recv, count, code):
        snd, rcv = engine.last_coll    # recorded right after the live engine.coll call
        assert (snd.data_ptr(), rcv.data_ptr()) == (send, recv)
        self.tape.append((COLL, (engine, ch, op, snd, rcv, self.nslots)))
        self.nslots += 1
        return self.nslots - 1

    def collectives(self):
        return [(x[1], x[2]) for k, x in self.tape if k == COLL]

    def add_wait(self, slot, stream=0):
        self.tape.append((WAIT, slot))

    def add_call(self, fn):
        self.tape.append((CALL, fn))

    @property
    def size(self):
        return len(self.tape)

    def kinds(self):
        return [k for k, _ in self.tape]

    def channels(self):
        return [x[1] for k, x in self.tape if k == POST]

    def set_profile(self, on):
        pass

    def run(self):
        handles = {}
        for k, x in self.tape:
            if k == GRAPH:
                x.replay()
            elif k == COPY:
                x[0].copy_(x[1])
            elif k == POST:
                eng, ch, s_, r_, slot = x
                handles[slot] = (eng, eng.post(ch, s_, r_))
            elif k == COLL:
                eng, ch, op, snd, rcv, slot = x
                handles[slot] = (eng, eng.coll(ch, op, snd, rcv))
            elif k == WAIT:
                eng, h = handles[x]
                eng.wait_keep(h)
            else:
                x()
        for eng, h in handles.values():
            eng.wait(h)
        self.runs += 1


def _patch(monkeypatch_like):
    """Route the recorder to the fakes (runs inside each spawned rank)."""
    import mipipe.ops.kernels as K
    K.load_ext = lambda: types.SimpleNamespace(StageRunner=FakeRunner)
    native_runner.TapeRecorder.copy = lambda self, dst, src: self.runner.add_copy_t(dst, src)

    def possible(self, return_outputs):
        if not self.native_enabled or return_outputs or self.deps is not None:
            return False
        if any(getattr(st, "graphs", None) is None for st in self.stages.values()):
            return False
        if self.head is not None and self.head.graphs is None:
            return False
        return self._steps >= 2 and all(getattr(st, "step_id", 0) >= 2 for st in self.stages.values())
    PipelineRuntime._native_possible = possible


CFG = lambda: NativeConfig.gpt2("tiny", vocab_size=96, d_model=64, n_layers=8, n_heads=4, d_ff=128, max_seq_len=16,
                                dropout=0.0)
M, MBS, S = 8, 2, 16


def _worker(rank, world, pp, dp, schedule, v, native, steps, overlap="probe"):
    import os
    os.environ["MIPIPE_COLL_OVERLAP"] = overlap
    torch.manual_seed(0)
    if native:
        _patch(None)
    cfg = CFG()
    tr = PipelineTrainer(cfg, pp=pp, dp=dp, schedule=schedule, n_microbatches=M, mbs=MBS, seq_len=S, v=v,
                         device=torch.device("cpu"), dtype=torch.float32, lr=1e-3, head_align=8)
    eng = None
    if native:
        ranks = tr.mesh.pipe_ranks
        groups = []
        for d in range(dp):      # every rank creates every group, in the same order
            rr = [d * pp + i for i in range(pp)]
            gs = [dist.new_group(rr, backend="gloo") for _ in range(3)]   # fwd, bwd, coll
            if d == tr.mesh.dp_rank:
                groups = gs
        dgroup = None
        for i in range(pp):
            g_ = dist.new_group([d * pp + i for d in range(dp)], backend="gloo") if dp > 1 else None
            if i == tr.mesh.pp_rank:
                dgroup = g_
        eng = FakeEngine(groups, ranks)
        tr.runtime.p2p.engine = eng
        tr.runtime.p2p.channels = 2
        tr.coll.pipe_engine, tr.coll.pp_kind = eng, "native"
        if dp > 1:
            tr.coll.dp_engine, tr.coll.dp_kind = FakeEngine([dgroup], None), "native"
        for st in tr.stages:
            st.graphs = FakeGraphCache(str(st.stage_index))
        if tr.runtime.head is not None:
            tr.runtime.head.graphs = FakeGraphCache(str(tr.mesh.pp_rank))
    g = torch.Generator().manual_seed(11 + tr.mesh.dp_rank)
    x = torch.randint(0, cfg.vocab_size, (M * MBS, S), generator=g)
    y = torch.randint(0, cfg.vocab_size, (M * MBS, S), generator=g)
    losses = [float(tr.train_step(x, y)) for _ in range(steps)]
    out = dict(losses=losses, sd={k: v.numpy().copy() for k, v in tr.state_dict().items()})
    r = tr.runtime.native_runner
    if native:
        out.update(recorded=r is not None, kinds=r.kinds() if r else [], channels=r.channels() if r else [],
                   colls=r.collectives() if r else [], runs=r.runs if r else 0, reason=tr.runtime.native_reason,
                   n_reduce_grad=sum(1 for st in tr.stages if st.has_grad_reduction(True)),
                   head=tr.runtime.head_reduce is not None, placement=tr.runtime.coll_placement,
                   dp_zero=tr.dp_zero, labels=r.labels if r else [],
                   stages=[st.stage_index for st in tr.stages])
    return out


def _graphs_between_last_b_and_grad_coll(o):
    """Per local stage: compute graphs on the tape between the stage's last backward graph
    and its REDUCE_GRAD collective (None if the stage issues no gradient collective)."""
    kinds, out = o["kinds"], {}
    colls = [i for i, k in enumerate(kinds) if k == COLL]
    for s in o["stages"]:
        bs = [i for i, lab in o["labels"] if lab.startswith(f"{s}B") or lab.startswith(f"{s}I")
              or lab.startswith(f"{s}W")]
        if not bs or o["n_reduce_grad"] == 0:
            continue
        after = [c for c in colls if c > max(bs)]
        if not after:
            continue
        c = after[0]
        out[s] = sum(1 for i, k in enumerate(kinds) if k == GRAPH and max(bs) < i < c)
    return out


@pytest.mark.parametrize("overlap", ["0", "probe"])
@pytest.mark.parametrize("schedule,v,dp", [("1F1B", 1, 1), ("Interleaved1F1B", 2, 1), ("1F1B", 1, 2)])
def test_pp4_tape_is_native_and_replays_exactly(schedule, v, dp, overlap):
    """``overlap='0'``: every collective deferred to the step end; ``'probe'`` (the default):
    each collective stays where lowering put it -- a stage's DP reduction right after its
    last backward, overlapping the rest of the flush."""
    world = 4 * dp
    ref = run_world(_worker, world, 4, dp, schedule, v, False, 5, overlap)
    res = run_world(_worker, world, 4, dp, schedule, v, True, 5, overlap)
    for r in range(world):
        o = res[r]
        assert o["recorded"], o["reason"]
        assert o["runs"] == 2                   # steps 4 and 5 replayed from the tape
        kinds = o["kinds"]
        assert set(kinds) <= {GRAPH, COPY, POST, WAIT, COLL, SYNC}, kinds    # no CALL
        assert kinds.count(POST) > 0 and kinds.count(GRAPH) > 0
        # collectives: REDUCE_HEAD = reduce-scatter over the pipeline (+ the shard's DP
        # all-reduce), one DP reduction per stage at REDUCE_GRAD (a reduce-scatter with
        # ZeRO-1 over DP, else an all-reduce)
        head_colls = [(2, 1)] + ([(0, 0)] if dp > 1 else [])
        assert o["dp_zero"] == (dp > 1)
        grad_coll = (0, 1) if o["dp_zero"] else (0, 0)
        assert sorted(o["colls"]) == sorted(head_colls + [grad_coll] * o["n_reduce_grad"]), o["colls"]
        last_post = max(i for i, k in enumerate(kinds) if k == POST)
        if overlap == "0":
            assert all(i > last_post for i, k in enumerate(kinds) if k == COLL), "collectives after every p2p group"
            assert o["placement"].startswith("step end")
        else:
            assert o["placement"].startswith("overlapped"), o["placement"]
            g = _graphs_between_last_b_and_grad_coll(o)
            assert all(n == 0 for n in g.values()), (r, g)   # COLL right after the stage's last B
        # both directions use their own channel
        assert set(o["channels"]) == {0, 1}
        assert o["losses"] == pytest.approx(ref[r]["losses"], rel=1e-6, abs=1e-6)
        for k, w in o["sd"].items():
            torch.testing.assert_close(torch.from_numpy(w), torch.from_numpy(ref[r]["sd"][k]), atol=1e-6,
                                       rtol=1e-6)
    if overlap != "0":
        # the head's reduction (after the rank's last head chunk) runs while the flush still
        # moves gradients: on some rank a COLL precedes p2p POSTs and compute graphs
        early = [r for r in range(world)
                 if min(i for i, k in enumerate(res[r]["kinds"]) if k == COLL)
                 < max(i for i, k in enumerate(res[r]["kinds"]) if k == POST)]
        assert early, "no collective overlaps the flush"
