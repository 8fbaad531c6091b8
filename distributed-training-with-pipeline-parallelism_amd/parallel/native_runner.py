"""Native step replay: record one pipeline step as an instruction tape, run later steps in C++.

After HIP-graph capture (:mod:`.graphs`) every compute action of a rank's lowered program is
one graph launch on persistent buffers, so a training step's device work is a fixed
sequence: graph launches, device copies (static graph inputs, loss slots), grouped
point-to-point transfers and waits.  :class:`TapeRecorder` observes one real Python step
(the runtime, :class:`~.graphs.GraphCache` and :class:`~.comm.P2P` report to it) and builds
a ``StageRunner`` (csrc/runtime/stage_runner.cpp) that replays the step with the GIL
released: no per-action Python, no allocator traffic, no host synchronisation.

Transfers on the native RCCL engine (the default p2p transport on GPUs) become native
POST/WAIT instructions (one per direction channel), and the step's collectives on the native
engines (parallel/collectives.py: DP gradient all-reduce, head-gradient reduce-scatter) native
COLL/WAIT instructions.  Only transfers / collectives through ``torch.distributed`` (gloo on
CPU, or the torch p2p fallback) become CALL instructions that re-issue the same Python call on
the same persistent tensors, so the runner is exact for every backend.  Anything that would break
replay (a graph captured during the recording step, a dependency tracker or profiler
attached) invalidates the tape and the runtime stays on the Python path.

Dependency analogue: the executor loop of torch's ``_PipelineScheduleRuntime``
(schedules.py:2037-2284), which the reference runs from Python every step.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional

import torch

_ACTIVE: Optional["TapeRecorder"] = None

# torch dtype -> code understood by StageRunner.add_post (torch's ScalarType numbering)
_DTYPE_CODE = {torch.uint8: 0, torch.int32: 3, torch.int64: 4, torch.float16: 5, torch.float32: 6,
               torch.float64: 7, torch.bfloat16: 15}


def active() -> Optional["TapeRecorder"]:
    return _ACTIVE


class paused:
    """Run a block outside the active recording: its device work and collectives are NOT
    put on the tape.  For per-step work the runtime issues itself on every step, replayed
    or not (``StageBase.post_step``): recording it too would run it twice per replay."""

    def __enter__(self):
        global _ACTIVE
        self._saved, _ACTIVE = _ACTIVE, None
        return self

    def __exit__(self, *exc):
        global _ACTIVE
        _ACTIVE = self._saved
        return False


class TapeRecorder:
    def __init__(self, device: torch.device):
        from ..ops.kernels import load_ext
        ext = load_ext()
        if ext is None or not hasattr(ext, "StageRunner"):
            raise RuntimeError("the native stage runner needs the built extension (_C.so)")
        idx = device.index if device.index is not None else (torch.cuda.current_device() if device.type == "cuda" else 0)
        self.runner = ext.StageRunner(idx)
        # instructions issued on another stream than this one (microbatch lanes) carry it
        self.cuda = device.type == "cuda"
        self.main_stream = torch.cuda.current_stream(idx).cuda_stream if self.cuda else 0
        self.valid = True
        self.reason = ""
        self._holders: Dict[int, list] = {}
        self._next_holder = 0

    # ------------------------------------------------------------------ context
    def __enter__(self):
        global _ACTIVE
        _ACTIVE = self
        return self

    def __exit__(self, *exc):
        global _ACTIVE
        _ACTIVE = None
        if exc[0] is not None:
            self.invalidate(f"exception {exc[0].__name__}")
        return False

    def invalidate(self, why: str) -> None:
        if self.valid:
            self.valid, self.reason = False, why

    # ------------------------------------------------------------------ instructions
    def _stream(self) -> int:
        if not self.cuda:
            return 0
        s = torch.cuda.current_stream().cuda_stream
        return 0 if s == self.main_stream else int(s)

    def graph(self, g: torch.cuda.CUDAGraph, label: str = "") -> None:
        st = self._stream()
        if st:
            self.runner.add_graph(int(g.raw_cuda_graph_exec()), str(label), st)
        else:
            self.runner.add_graph(int(g.raw_cuda_graph_exec()), str(label))

    def sync(self, waiter: "torch.cuda.Stream", signal: "torch.cuda.Stream") -> None:
        """``waiter.wait_stream(signal)`` on the tape."""
        w, s = int(waiter.cuda_stream), int(signal.cuda_stream)
        self.runner.add_sync(0 if w == self.main_stream else w, 0 if s == self.main_stream else s)

    def copy(self, dst: torch.Tensor, src: torch.Tensor) -> None:
        if not (dst.is_contiguous() and src.is_contiguous() and dst.dtype == src.dtype
                and dst.numel() == src.numel()):
            self.invalidate("non-contiguous or mismatched copy")
            return
        self.runner.add_copy(dst.data_ptr(), src.data_ptr(), dst.numel() * dst.element_size(), self._stream())

    def native_post(self, engine, channel: int, sends, recvs) -> int:
        def ops(lst):
            out = []
            for t, peer in lst:
                code = _DTYPE_CODE.get(t.dtype)
                if code is None or not t.is_contiguous():
                    self.invalidate(f"unsupported p2p tensor {t.dtype}")
                    code = 6
                out.append((t.data_ptr(), t.numel(), code, int(peer)))
            return out
        return self.runner.add_post(engine, int(channel), ops(sends), ops(recvs))

    def native_coll(self, engine, channel: int, op: int, send: torch.Tensor, recv: torch.Tensor,
                    nranks: int) -> int:
        """A collective on a native engine (op codes of csrc/comm/rccl_engine.h CollOp)."""
        code = _DTYPE_CODE.get(send.dtype)
        if code is None or not (send.is_contiguous() and recv.is_contiguous()):
            self.invalidate(f"unsupported collective tensor {send.dtype}")
            code = 6
        count = send.numel() if op == 2 else recv.numel()   # ALL_GATHER counts the send block
        return self.runner.add_coll(engine, int(channel), int(op), send.data_ptr(), recv.data_ptr(), int(count),
                                    code)

    def native_wait(self, slot: int) -> None:
        """The current stream (compute, or a microbatch lane) waits for the slot's group."""
        self.runner.add_wait(slot, self._stream())

    def call(self, fn: Callable[[], None]) -> None:
        self.runner.add_call(fn)

    def holder(self) -> list:
        """A mutable cell shared by a recorded issuing CALL and its recorded waits."""
        h: list = []
        self._holders[self._next_holder] = h
        self._next_holder += 1
        return h


class RecordedWork:
    """Work handle of a recorded Python-issued transfer/collective: ``wait`` waits on the
    live handle now and records a CALL that waits on the handle of each replayed step."""

    def __init__(self, live, cell: list, idx: int, rec: TapeRecorder):
        self.live, self.cell, self.idx, self.rec = live, cell, idx, rec

    def wait(self):
        r = self.live.wait() if hasattr(self.live, "wait") else True
        cell, idx = self.cell, self.idx

        def _w():
            w = cell[0][idx]
            if hasattr(w, "wait"):
                w.wait()
        self.rec.call(_w)
        return r


def record_issue(rec: TapeRecorder, issue: Callable[[], List]) -> List:
    """Run ``issue()`` (returns a list of work handles) now, record a CALL that re-runs it
    on replay, and return recorded wrappers of the live handles."""
    cell = rec.holder()
    works = issue()
    cell.append(works)

    def _again():
        cell[0] = issue()
    rec.call(_again)
    return [RecordedWork(w, cell, i, rec) for i, w in enumerate(works)]


def copy_into(dst: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    """``dst.copy_(src)`` that a recording step also puts on the tape."""
    dst.copy_(src)
    r = _ACTIVE
    if r is not None:
        r.copy(dst, src)
    return dst
