"""Point-to-point transport between pipeline stages.

On MI355X the transport is the native RCCL engine (csrc/comm/rccl_engine.h) over the
point-to-point xGMI links: one communicator and one high-priority HIP stream per
traffic direction (activations down, gradients up), grouped ``ncclSend``/``ncclRecv``,
plus a third communicator for the step's collectives (parallel/collectives.py),
pre-flight pinged at construction with an in-process fallback to torch p2p if any
pipeline rank fails.  On CPU it is gloo (reference plumbing config, helper:175).  The
executor hands this module :class:`~.ir.CommGroup` s whose per-peer order is already
globally consistent (:mod:`.lower`) and proven hang-free for the channel split in use
(:func:`.simulate.check_lowered`), so nothing here needs to sort or retry.

Static shapes: unlike the dependency's runtime shape inference with pickled
meta-tensors (stage.py:1410-1519, C4 in SURVEY §2.6), stages declare their tensor
specs; when a user module's specs are unknown, :func:`exchange_specs` ships them
as small int64 tensors once at init (no pickling).
"""
from __future__ import annotations

import logging
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

log = logging.getLogger("mipipe.comm")

_DTYPES = [torch.float32, torch.bfloat16, torch.float16, torch.int64, torch.int32, torch.float64, torch.uint8,
           torch.bool, torch.int8]
_MAX_DIMS = 8

Spec = Tuple[Tuple[int, ...], torch.dtype]


class _StagedRecv:
    """Receive into a host buffer, copied to the device tensor on ``wait``."""

    def __init__(self, work, host: torch.Tensor, dev: torch.Tensor):
        self.work, self.host, self.dev = work, host, dev

    def wait(self):
        self.work.wait()
        self.dev.copy_(self.host)
        return True


class _StagedSend:
    """Send of a host copy; keeps the copy alive until the transfer completed."""

    def __init__(self, work, host: torch.Tensor):
        self.work, self.host = work, host

    def wait(self):
        return self.work.wait()


class _NativeWork:
    """Handle of one grouped transfer on the native RCCL engine; ``wait`` makes the
    current stream wait (no host block), like torch's NCCL Work -- once per stream: a
    group whose receives feed computes on two microbatch lanes is waited on by both
    streams (a non-consuming engine wait; ``release`` returns the event at the step end).
    Under a recording step (:mod:`.native_runner`) each such wait is also put on the tape
    with its stream."""

    def __init__(self, engine, handle: int, rec=None, slot: int = -1):
        self.engine, self.handle, self.rec, self.slot = engine, handle, rec, slot
        self.streams = set()
        self.released = False

    def wait(self):
        sid = int(torch.cuda.current_stream().cuda_stream) if torch.cuda.is_available() else 0
        if sid in self.streams:
            return True
        self.streams.add(sid)
        self.engine.wait_keep(self.handle)
        if self.rec is not None:
            self.rec.native_wait(self.slot)
        return True

    def release(self):
        if not self.released:
            self.released = True
            self.engine.release(self.handle)


def load_native_rccl(ext) -> None:
    """Bind the engine to the librccl PyTorch loaded (one RCCL per process)."""
    ext.RcclEngine.load(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))


# message kind -> engine channel: 0 = activations down the pipeline (F, and the last
# stage's hidden rows to the head ranks, H), 1 = gradients back up (B, head grads D);
# channel 2 carries the pipeline group's collectives (parallel/collectives.py)
CHANNEL_OF_KIND = {"F": 0, "H": 0, "B": 1, "D": 1}
PIPE_CHANNEL_SLOTS = (0, 1, 2)   # channel c issues on comm stream slot c (rccl_engine.h)


def comm_progress_report(engines: Dict[str, object], limit: int = 6) -> str:
    """One block per native engine: groups issued, the incomplete ones (oldest first: channel,
    kind, peer ranks within the engine's group, bytes, seconds since issue) and any RCCL
    async error.  Read by the watchdog when a step stalls: the oldest incomplete group on
    every rank names the transfer the pipeline waits on (csrc/comm/rccl_engine.h progress)."""
    lines = []
    for name, eng in engines.items():
        if eng is None or not hasattr(eng, "progress"):
            continue
        try:
            pend, issued, err = eng.progress(), int(eng.issued()), eng.async_error()
        except Exception as e:  # pragma: no cover - diagnostics only
            lines.append(f"[comm] {name}: progress unavailable ({e})")
            continue
        lines.append(f"[comm] {name} engine (rank {eng.rank}/{eng.nranks}): {issued} groups issued, "
                     f"{len(pend)} incomplete" + (f", RCCL async error: {err}" if err else ""))
        for d in pend[:limit]:
            peers = (f" send->{d['sends']}" if d["sends"] else "") + (f" recv<-{d['recvs']}" if d["recvs"] else "")
            lines.append(f"[comm]   #{d['seq']} channel {d['channel']} {d['kind']}{peers} "
                         f"{d['bytes'] / 1e6:.2f} MB, issued {d['age_s']:.1f}s ago")
        if len(pend) > limit:
            lines.append(f"[comm]   ... {len(pend) - limit} more")
    return "\n".join(lines) if lines else "[comm] no native RCCL engine on this rank"


def make_native_engine(group, ranks: Sequence[int], my_pipe_rank: int, device: torch.device):
    """Collective over the pipeline group: pipeline rank 0 draws one RCCL unique id per
    channel, the group broadcasts them, every rank joins the three communicators
    (csrc/comm/rccl_engine.h).  RCCL's communicator init blocks until every peer joined:
    callers run it under a watchdog (bench.py) or a process-group timeout."""
    from ..ops.kernels import load_ext
    ext = load_ext()
    if ext is None or not hasattr(ext, "RcclEngine"):
        raise RuntimeError("the native RCCL engine needs the built extension (_C.so)")
    load_native_rccl(ext)
    nch = len(PIPE_CHANNEL_SLOTS)
    nb = int(ext.RcclEngine.id_bytes()) * nch
    buf = torch.zeros(nb, dtype=torch.uint8, device=device)
    if my_pipe_rank == 0:
        uid = b"".join(ext.RcclEngine.unique_id() for _ in range(nch))
        buf.copy_(torch.frombuffer(bytearray(uid), dtype=torch.uint8))
    if len(ranks) > 1:
        dist.broadcast(buf, src=ranks[0], group=group)
    uid = bytes(buf.cpu().tolist())
    return ext.RcclEngine(uid, len(ranks), my_pipe_rank, device.index if device.index is not None else 0,
                          list(PIPE_CHANNEL_SLOTS))


def preflight(engine, peers: Sequence[int], me: int, device: torch.device, timeout_s: float) -> Tuple[bool, str]:
    """Ping every peer on every channel of a native engine (one grouped send+recv per
    channel) and poll for completion against a host deadline.  Also establishes the RCCL
    connections up front (the role of torch's p2p warm-up, stage.py:925-979).
    Returns (ok, reason)."""
    peers = sorted(set(p for p in peers if p != me))
    if not peers:
        return True, ""
    handles, recvs = [], []
    for ch in range(engine.channels):
        s = [(torch.full((1,), float(me * 16 + ch), device=device), p) for p in peers]
        r = [(torch.full((1,), -1.0, device=device), p) for p in peers]
        handles.append(engine.post(ch, s, r))
        recvs.append(r)
    deadline = time.monotonic() + timeout_s
    while not all(engine.query(h) for h in handles):
        err = engine.async_error()
        if err:
            return False, f"RCCL async error: {err}"
        if time.monotonic() > deadline:
            return False, f"no answer from peers {peers} within {timeout_s:.0f}s"
        time.sleep(0.002)
    for h in handles:
        engine.wait(h)
    torch.cuda.current_stream(device).synchronize()
    for ch, r in enumerate(recvs):
        for t, p in r:
            if float(t.item()) != float(p * 16 + ch):
                return False, f"channel {ch}: wrong ping payload from peer {p}: {float(t.item())}"
    return True, ""


def agree(ok: bool, group, device: torch.device) -> bool:
    """True iff every rank of ``group`` reports ok (control plane: a gloo group when
    available, so a wedged RCCL channel cannot block the vote).  ``group=None`` is the
    world group (as everywhere in torch.distributed): every rank still votes."""
    if not dist.is_initialized() or dist.get_world_size(group) <= 1:
        return ok
    backend = dist.get_backend(group)
    dev = torch.device("cpu") if backend == "gloo" else device
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()) == 1)


class P2P:
    """Point-to-point transport of one pipeline group.

    ``ranks[i]`` is the global rank of pipeline rank ``i``.  Modes (``mode`` argument or
    ``MIPIPE_P2P``):

    * ``auto`` (default) / ``native`` -- on GPUs with the RCCL backend, the C++ engine
      (csrc/comm/rccl_engine.h): one communicator + stream per direction, grouped
      ncclSend/ncclRecv, posts replayed natively by the stage runner.  It is created and
      pinged (:func:`preflight`) at construction; if any rank of the pipeline fails, every
      rank agrees (:func:`agree`) to fall back to torch p2p in-process -- ``auto`` logs
      ``fallback_reason``, ``native`` raises.
    * ``torch`` -- ``torch.distributed.batch_isend_irecv`` (ProcessGroupNCCL = RCCL, or gloo).

    With the gloo backend and GPU tensors (``MIPIPE_DIST_BACKEND=gloo``: several ranks
    sharing one GPU, used to test the whole multi-process GPU stack on a single-GPU box)
    transfers are staged through host memory.
    """

    def __init__(self, group: Optional[dist.ProcessGroup], ranks: Sequence[int], device: torch.device,
                 mode: Optional[str] = None, ctrl_group=None, preflight_timeout: Optional[float] = None):
        self.group = group
        self.ranks = list(ranks)
        self.device = device
        self.host_staged = (device.type == "cuda" and dist.is_initialized()
                            and dist.get_backend(group) == "gloo")
        mode = (mode or os.environ.get("MIPIPE_P2P", "auto")).lower()
        if mode not in ("auto", "native", "torch"):
            raise ValueError(f"MIPIPE_P2P={mode}: expected auto, native or torch")
        self.engine = None
        self.channels = 1
        self.fallback_reason = ""
        self._live: List = []       # native works of the current step (release_works)
        self.audit = None           # parallel/audit.CommAudit while a step is audited
        capable = (device.type == "cuda" and dist.is_initialized() and not self.host_staged and len(self.ranks) > 1)
        if mode != "torch" and capable:
            timeout = preflight_timeout if preflight_timeout is not None else \
                float(os.environ.get("MIPIPE_P2P_PREFLIGHT_S", "60"))
            me = self.ranks.index(dist.get_rank())
            eng, ok, why = None, False, ""
            try:
                eng = make_native_engine(group, self.ranks, me, device)
                ok, why = preflight(eng, range(len(self.ranks)), me, device, timeout)
            except Exception as e:  # noqa: BLE001 - reported, then the whole pipeline falls back
                ok, why = False, f"{type(e).__name__}: {e}"
            all_ok = agree(ok, ctrl_group if ctrl_group is not None else group, device)
            if all_ok:
                self.engine = eng
                # p2p directions; the engine's last channel is the collective channel
                self.channels = min(2, int(eng.channels))
            else:
                if eng is not None:
                    eng.abort()
                self.fallback_reason = why or "a peer's native engine failed its pre-flight"
                if mode == "native":
                    raise RuntimeError(f"MIPIPE_P2P=native: {self.fallback_reason}")
                log.warning("native RCCL p2p engine not used (%s); torch p2p instead", self.fallback_reason)

    @property
    def kind(self) -> str:
        """Transport actually in use: native | torch | gloo-staged | none."""
        if self.engine is not None:
            return "native"
        if len(self.ranks) <= 1 or not dist.is_initialized():
            return "none"
        return "gloo-staged" if self.host_staged else "torch"

    def release_works(self) -> None:
        """End of a step: the native groups' completion events go back to the engine pool
        (their waits are stream-ordered, so releasing after the last one is issued is safe)."""
        for w in self._live:
            w.release()
        self._live.clear()

    def reset_channels(self) -> None:
        """Back to the engine's two direction channels (a transport reused by a new runtime
        whose program may be proven on both; see use_single_channel)."""
        if self.engine is not None:
            self.channels = min(2, int(self.engine.channels))

    def use_single_channel(self) -> None:
        """Post both directions on channel 0 (the lowered program's two-channel order was
        not proven deadlock-free, see simulate.check_lowered)."""
        self.channels = 1

    def global_rank(self, pipe_rank: int) -> int:
        return self.ranks[pipe_rank]

    def post(self, sends: Sequence[Tuple[torch.Tensor, int]], recvs: Sequence[Tuple[torch.Tensor, int]],
             send_ch: Optional[Sequence[int]] = None, recv_ch: Optional[Sequence[int]] = None):
        """Post one group; returns (send_works, recv_works) aligned with the inputs.
        ``send_ch``/``recv_ch`` give each op's channel (native engine: the group is split
        into one grouped call per channel; torch: ignored, one batch)."""
        from . import native_runner
        rec = native_runner.active()
        if self.engine is not None:
            if not sends and not recvs:
                return [], []
            sc = [0] * len(sends) if send_ch is None or self.channels == 1 else list(send_ch)
            rc = [0] * len(recvs) if recv_ch is None or self.channels == 1 else list(recv_ch)
            works_s: List = [None] * len(sends)
            works_r: List = [None] * len(recvs)
            for ch in sorted(set(sc) | set(rc)):
                s_ = [sends[i] for i in range(len(sends)) if sc[i] == ch]
                r_ = [recvs[i] for i in range(len(recvs)) if rc[i] == ch]
                if self.audit is not None:
                    self.audit.p2p(ch, [(t, self.global_rank(p)) for t, p in s_],
                                   [(t, self.global_rank(p)) for t, p in r_])
                h = self.engine.post(ch, s_, r_)
                slot = rec.native_post(self.engine, ch, s_, r_) if rec is not None else -1
                w = _NativeWork(self.engine, h, rec, slot)
                self._live.append(w)
                for i in range(len(sends)):
                    if sc[i] == ch:
                        works_s[i] = w
                for i in range(len(recvs)):
                    if rc[i] == ch:
                        works_r[i] = w
            return works_s, works_r
        if self.audit is not None and (sends or recvs):
            self.audit.p2p(0, [(t, self.global_rank(p)) for t, p in sends], [(t, self.global_rank(p)) for t, p in recvs])
        if rec is not None:
            # transfers through torch.distributed replay as CALLs on the same tensors
            ns = len(sends)
            works = native_runner.record_issue(rec, lambda: self._post_torch(sends, recvs))
            return works[:ns], works[ns:]
        return self._post_torch_split(sends, recvs)

    def _post_torch_split(self, sends, recvs):
        works = self._post_torch(sends, recvs)
        return works[: len(sends)], works[len(sends):]

    def _post_torch(self, sends, recvs) -> list:
        ops = []
        staged = []
        for t, peer in sends:
            if self.host_staged:
                t = t.detach().to("cpu")
                staged.append(t)
            ops.append(dist.P2POp(dist.isend, t, self.global_rank(peer), self.group))
        host_recv = []
        for t, peer in recvs:
            if self.host_staged:
                h = torch.empty(t.shape, dtype=t.dtype)
                host_recv.append((h, t))
                t = h
            ops.append(dist.P2POp(dist.irecv, t, self.global_rank(peer), self.group))
        if not ops:
            return []
        works = dist.batch_isend_irecv(ops)
        sw, rw = works[: len(sends)], works[len(sends):]
        if self.host_staged:
            sw = [_StagedSend(w, h) for w, h in zip(sw, staged)]
            rw = [_StagedRecv(w, h, d) for w, (h, d) in zip(rw, host_recv)]
        return list(sw) + list(rw)

    # -------------------------------------------------------------- spec exchange
    def _pack(self, specs: Sequence[Spec]) -> torch.Tensor:
        buf = torch.zeros(1 + 8 * (2 + _MAX_DIMS), dtype=torch.int64)
        buf[0] = len(specs)
        for i, (shape, dtype) in enumerate(specs):
            base = 1 + i * (2 + _MAX_DIMS)
            buf[base] = _DTYPES.index(dtype)
            buf[base + 1] = len(shape)
            for j, d in enumerate(shape):
                buf[base + 2 + j] = d
        return buf if self.host_staged else buf.to(self.device)

    @staticmethod
    def _unpack(buf: torch.Tensor) -> List[Spec]:
        buf = buf.cpu().tolist()
        out = []
        for i in range(int(buf[0])):
            base = 1 + i * (2 + _MAX_DIMS)
            dt = _DTYPES[int(buf[base])]
            nd = int(buf[base + 1])
            out.append((tuple(int(x) for x in buf[base + 2: base + 2 + nd]), dt))
        return out

    def send_specs(self, specs: Sequence[Spec], peer: int) -> None:
        if len(specs) > 8:
            raise ValueError("at most 8 tensors per stage boundary")
        dist.send(self._pack(specs), self.global_rank(peer), group=self.group)

    def recv_specs(self, peer: int) -> List[Spec]:
        buf = torch.zeros(1 + 8 * (2 + _MAX_DIMS), dtype=torch.int64,
                          device="cpu" if self.host_staged else self.device)
        dist.recv(buf, self.global_rank(peer), group=self.group)
        return self._unpack(buf)

    def warmup(self, peers: Sequence[int], my_rank: int) -> None:
        """Establish the communicators to every neighbor once (torch stage.py:925-979).

        Pairs are exchanged in ascending (low, high) order on both sides so the
        first RCCL p2p on each link cannot cross-wait.
        """
        if self.engine is not None:
            return      # every link of both channels was pinged by preflight()
        for peer in sorted(set(peers)):
            if peer == my_rank:
                continue
            dev = "cpu" if self.host_staged else self.device
            t_send = torch.ones(1, device=dev)
            t_recv = torch.zeros(1, device=dev)
            s, r = self.post([(t_send, peer)], [(t_recv, peer)])
            for w in s + r:
                w.wait()
