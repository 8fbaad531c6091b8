"""HIP-graph capture of per-microbatch stage compute.

A stage's forward (or backward) for microbatch slot ``mb`` is the same sequence of
kernel launches on the same buffers every step: static shapes and, with the flat
parameter arena and persistent receive buffers, static pointers.  :class:`GraphCache`
captures each such action once (``torch.cuda.CUDAGraph`` = hipGraph on ROCm), then
replays it with one launch.  That removes the Python/launch overhead (~0.4 ms per
GPT-2 layer fwd+bwd, measured) that otherwise bounds small microbatches and deep
pipelines.  Design rules:

* every captured action has its own private memory pool, and all tensors the action
  saves for a later action (forward activations read by the backward) are kept
  referenced by the cache, so no later allocation can alias them;
* inputs are captured by pointer; if a later call passes a tensor at another address
  (e.g. the user's token chunk) it is copied into the captured buffer first;
* communication stays outside the graphs (RCCL work is posted by the runtime between
  replays, and ordered by stream waits), as do optimizer steps whose scalars change;
* capture never synchronises the device: actions are captured lazily in the middle of a
  pipeline step, when receives posted on the comm streams may still be waiting for a peer
  that itself waits for this rank (``torch.cuda.graph`` would ``torch.cuda.synchronize()``
  on entry -- a cross-rank deadlock on the first multi-GPU capture step).  The capture
  runs on a private stream ordered after the compute stream, in thread-local mode.

Graphs are off on CPU.  Dropout is graph-safe: the per-site seeds are static kernel
arguments, and every dropout kernel mixes in a device-side training-step counter
(``ops.set_dropout_step``, written before each step outside the graphs), so each replay
draws a new mask and the backward regenerates the forward's.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Hashable, List, Sequence

import torch


def _tensors(obj, out: List[torch.Tensor]) -> List[torch.Tensor]:
    if isinstance(obj, torch.Tensor):
        out.append(obj)
    elif isinstance(obj, dict):
        for v in obj.values():
            _tensors(v, out)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _tensors(v, out)
    elif hasattr(obj, "__dict__") and not callable(obj):
        _tensors(vars(obj), out)
    return out


_CAPTURE_STREAMS: Dict[int, torch.cuda.Stream] = {}
# streams that code running inside a capture may fork off the capture stream (the
# weight-gradient side stream, models/native.py WGradOverlap): on a failed capture they are
# joined back before the capture is ended, so ending it succeeds and leaves every stream
# out of capture mode
_SIDE_STREAMS: List[torch.cuda.Stream] = []


def register_side_stream(s: "torch.cuda.Stream") -> None:
    if all(x.cuda_stream != s.cuda_stream for x in _SIDE_STREAMS):
        _SIDE_STREAMS.append(s)


def _capturing(s: "torch.cuda.Stream") -> bool:
    with torch.cuda.stream(s):
        return torch.cuda.is_current_stream_capturing()


def _abort_capture(g: "torch.cuda.CUDAGraph", cs: "torch.cuda.Stream") -> None:
    """End a capture whose function raised: join every registered side stream still in
    capture mode (a fork the failure left open) into the capture stream, end the capture
    (a partial, discarded graph) and drop it.  Secondary errors are swallowed: the caller
    re-raises the original one."""
    try:
        for s in _SIDE_STREAMS:
            if s.cuda_stream != cs.cuda_stream and _capturing(s):
                cs.wait_stream(s)
        g.capture_end()
    except Exception:       # noqa: BLE001 - secondary to the error being raised
        pass


def capture(g: "torch.cuda.CUDAGraph", fn: Callable[[], Any], pool=None) -> Any:
    """Capture ``fn()`` into ``g`` without a device-wide synchronisation (module docstring):
    on a per-device capture stream that first waits for the current stream, thread-local
    capture mode, a private memory pool (``pool``: the pool of earlier captures to share --
    parallel/stash.py slot rings).  If ``fn`` raises (an allocation failing inside the
    capture, say), the capture is ended and discarded and THAT exception propagates -- not
    the ``hipErrorStreamCaptureUnjoined`` that ending a half-built capture reports when the
    failure left a forked side stream unjoined."""
    cur = torch.cuda.current_stream()
    idx = cur.device.index if cur.device.index is not None else torch.cuda.current_device()
    cs = _CAPTURE_STREAMS.get(idx)
    if cs is None:
        cs = _CAPTURE_STREAMS[idx] = torch.cuda.Stream(device=idx)
    cs.wait_stream(cur)
    with torch.cuda.stream(cs):
        if pool is not None:
            g.capture_begin(pool=pool, capture_error_mode="thread_local")
        else:
            g.capture_begin(capture_error_mode="thread_local")
        try:
            out = fn()
        except BaseException:
            _abort_capture(g, cs)
            raise
        g.capture_end()
    cur.wait_stream(cs)
    return out


class GraphCache:
    def __init__(self, name: str = ""):
        self.name = name
        self.graphs: Dict[Hashable, tuple] = {}
        self.captures = 0
        self.replays = 0

    def label(self, key) -> str:
        """Action label of a graph key on the tape, e.g. ('F', 3) -> 'F3' (prefixed by
        ``self.name``, the stage index or 'H')."""
        if isinstance(key, tuple) and len(key) == 2:
            return f"{self.name}{key[0]}{key[1]}"
        return f"{self.name}{key}"

    def __contains__(self, key) -> bool:
        return key in self.graphs

    def run(self, key: Hashable, inputs: Sequence[torch.Tensor], fn: Callable[[Sequence[torch.Tensor]], Any],
            keep: Callable[[], Any] = None, pool=None) -> Any:
        """Replay the graph captured for ``key`` (capturing it on first use).  ``keep``
        returns objects whose tensors must outlive the capture (saved activations) -- until
        :meth:`release`.  ``pool``: capture into this shared memory pool (a stash slot's,
        parallel/stash.py) instead of a private one."""
        from . import native_runner
        rec = native_runner.active()
        entry = self.graphs.get(key)
        if entry is None:
            if rec is not None:
                rec.invalidate(f"graph {key!r} captured during the recording step")
            g = torch.cuda.CUDAGraph()
            out = capture(g, lambda: fn(inputs), pool=pool)
            kept = _tensors(keep(), []) if keep is not None else []
            entry = (g, list(inputs), out, kept)
            self.graphs[key] = entry
            self.captures += 1
        else:
            g, static_in, out, _ = entry
            for s, t in zip(static_in, inputs):
                if s.data_ptr() != t.data_ptr():
                    s.copy_(t)
                    if rec is not None:
                        rec.copy(s, t)
            self.replays += 1
        entry[0].replay()
        if rec is not None:
            rec.graph(entry[0], self.label(key))
        return entry[2]

    def release(self, key: Hashable) -> None:
        """Drop the tensors ``keep`` pinned for ``key`` (its graph and outputs stay): once the
        last graph reading them is captured, their blocks return to the capture's pool, where
        the next capture into that pool (the slot's next occupant) reuses them."""
        entry = self.graphs.get(key)
        if entry is not None and entry[3]:
            self.graphs[key] = (entry[0], entry[1], entry[2], [])

    def clear(self) -> None:
        self.graphs.clear()
