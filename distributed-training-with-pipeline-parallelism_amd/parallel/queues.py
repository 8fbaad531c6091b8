"""Which HIP streams of a rank share a hardware queue?  (the spin/flag probe)

HIP maps each stream onto one of GPU_MAX_HW_QUEUES (4 on the MI355X boxes) hardware
queues per priority level when the stream is created; two streams on one queue
serialise in host issue order whatever their event dependencies say.  An RCCL kernel
holds its queue until every peer has arrived, so whether the comm streams of
csrc/comm/rccl_engine.h (fwd / bwd p2p, collectives) have queues of their own decides
which deadlock model the pipeline program must satisfy (:func:`.simulate.check_lowered`):

* every comm stream on its own queue, apart from compute -> the *independent* model:
  collectives may run mid-step on the collective stream, overlapping the flush;
* anything shared -> the *serial* model (one FIFO per rank, the worst case of any
  mapping): collectives are deferred to the end of the step
  (:func:`.lower.defer_collectives`).

:func:`shares_queue` launches a bounded spinner on one stream (csrc/kernels/probe.hip)
and a flag store on the other: separate queues -> the store lands while the spinner is
resident and it exits within microseconds; a shared queue -> the store waits behind the
spinner, which exits on its own deadline (never a hang).  ``tools/queue_probe.py`` runs
the probe over the exact stream set of a PP>1 rank and records the result.
"""
from __future__ import annotations

import logging
import os
from typing import Dict, List, Optional, Tuple

import torch

log = logging.getLogger("mipipe.queues")

COMM_SLOT_NAMES = ("comm:fwd", "comm:bwd", "comm:coll")


def _ext():
    from ..ops.kernels import load_ext
    ext = load_ext()
    if ext is None or not hasattr(ext, "probe_spin"):
        raise RuntimeError("the hardware-queue probe needs the built extension (_C.so)")
    return ext


def shares_queue(waiter: int, setter: int, device: torch.device, timeout_us: int = 20000,
                 graph: Optional[str] = None) -> Tuple[bool, float]:
    """(shared, microseconds the spinner waited).  ``waiter`` / ``setter``: raw HIP stream
    handles (0 = the current stream).  ``graph='waiter'|'setter'``: that side is issued as a
    captured HIP graph launched on the current stream whose kernel runs on a branch forked
    onto the given stream -- how the runtime's per-microbatch graphs replay their dW work."""
    ext = _ext()
    flag = torch.zeros(1, dtype=torch.int32, device=device)
    res = torch.zeros(2, dtype=torch.int32, device=device)
    torch.cuda.synchronize(device)
    g = None
    if graph is not None:
        side = torch.cuda.ExternalStream(waiter if graph == "waiter" else setter, device=device)
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(device=device)
        with torch.cuda.graph(g, stream=cap, capture_error_mode="thread_local"):
            side.wait_stream(cap)
            with torch.cuda.stream(side):
                if graph == "waiter":
                    ext.probe_spin(flag, 1, timeout_us, res, 0)
                else:
                    ext.probe_set(flag, 1, 0)
            cap.wait_stream(side)
        torch.cuda.synchronize(device)
        flag.zero_()
        res.zero_()
        torch.cuda.synchronize(device)
    if graph == "waiter":
        g.replay()
        ext.probe_set(flag, 1, setter)
    elif graph == "setter":
        ext.probe_spin(flag, 1, timeout_us, res, waiter)
        g.replay()
    else:
        ext.probe_spin(flag, 1, timeout_us, res, waiter)
        ext.probe_set(flag, 1, setter)
    torch.cuda.synchronize(device)
    seen, ticks = (int(x) for x in res.cpu().tolist())
    khz = max(1, int(ext.probe_clock_khz()) or 100000)
    return (seen == 0), ticks * 1000.0 / khz


def comm_streams(device: torch.device) -> Dict[str, int]:
    """The process-wide comm stream slots of csrc/comm/rccl_engine.h (created on first use)."""
    ext = _ext()
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return {name: int(ext.comm_stream(idx, k)) for k, name in enumerate(COMM_SLOT_NAMES)}


def rank_streams(device: torch.device, lanes: Optional[List[torch.cuda.Stream]] = None) -> Dict[str, int]:
    """The compute-side streams a rank drives: the compute stream, the dW side stream of
    the native model (models/native.py WGradOverlap, created here if not yet), lanes."""
    from ..models.native import WGradOverlap
    idx = device.index if device.index is not None else torch.cuda.current_device()
    out = {"compute": int(torch.cuda.current_stream(idx).cuda_stream)}
    try:
        out["dw_side"] = int(WGradOverlap(torch.device("cuda", idx)).side.cuda_stream)
    except Exception:   # noqa: BLE001 - no side stream configured (MIPIPE_WGRAD_STREAM=0)
        pass
    for i, s in enumerate(lanes or []):
        out[f"lane{i + 1}"] = int(s.cuda_stream)
    return out


def check_comm_queues(device: torch.device, lanes=None, timeout_us: int = 20000,
                      graphs: bool = True) -> dict:
    """Probe every comm stream slot against every other comm slot and every compute-side
    stream (plus, with ``graphs``, against a graph whose kernel replays on the dW side
    branch).  Returns ``{"independent": bool, "shared": [pairs], "pairs": {pair: us}}``;
    ``independent`` holds iff no comm stream shares a queue with anything."""
    comm = comm_streams(device)
    other = rank_streams(device, lanes)
    pairs: Dict[str, float] = {}
    shared: List[str] = []
    names = list(comm)
    for i, a in enumerate(names):
        targets = [(b, comm[b], None) for b in names[i + 1:]] + [(b, h, None) for b, h in other.items()]
        if graphs and "dw_side" in other:
            targets.append(("graph:dw_side", other["dw_side"], "setter"))
        for b, hb, g in targets:
            sh, us = shares_queue(comm[a], hb, device, timeout_us, graph=g)
            key = f"{a}|{b}"
            pairs[key] = round(us, 1)
            if sh:
                shared.append(key)
    return {"independent": not shared, "shared": shared, "pairs": pairs}


_CACHE: Dict[int, dict] = {}


def comm_queues_independent(device: torch.device, lanes=None) -> Tuple[bool, dict]:
    """Cached per device and process (stream -> queue mappings are fixed at stream
    creation; the comm slots and the dW side stream are process-wide).
    ``MIPIPE_QUEUE_MODEL=serial|independent`` overrides the probe (A/B, tests)."""
    forced = os.environ.get("MIPIPE_QUEUE_MODEL", "").lower()
    if forced in ("serial", "independent"):
        return forced == "independent", {"forced": forced}
    idx = device.index if device.index is not None else torch.cuda.current_device()
    rep = _CACHE.get(idx)
    if rep is None:
        rep = check_comm_queues(device, lanes)
        _CACHE[idx] = rep
        if rep["shared"]:
            log.warning("comm streams share hardware queues (%s): collectives deferred to the step end",
                        ", ".join(rep["shared"]))
    return bool(rep["independent"]), rep
