"""Point-to-point transport between pipeline stages.

On MI355X the backend is RCCL (``torch.distributed`` backend ``"nccl"``) over the
point-to-point xGMI links; on CPU it is gloo (reference plumbing config,
helper:175).  The executor hands this module :class:`~.ir.CommGroup` s whose
per-peer order is already globally consistent (:mod:`.lower`), so each group is
posted as one ``batch_isend_irecv`` (= one RCCL group: both directions of a link
progress together) and nothing here needs to sort or retry.

Static shapes: unlike the dependency's runtime shape inference with pickled
meta-tensors (stage.py:1410-1519, C4 in SURVEY §2.6), stages declare their tensor
specs; when a user module's specs are unknown, :func:`exchange_specs` ships them
as small int64 tensors once at init (no pickling).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

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
    current stream wait (no host block), like torch's NCCL Work.  Under a recording step
    (:mod:`.native_runner`) the wait is also put on the tape."""

    def __init__(self, engine, handle: int, rec=None, slot: int = -1):
        self.engine, self.handle, self.rec, self.slot = engine, handle, rec, slot

    def wait(self):
        self.engine.wait(self.handle)
        if self.rec is not None:
            self.rec.native_wait(self.slot)
            self.rec = None     # one WAIT per handle, however often it is waited on
        return True


def load_native_rccl(ext) -> None:
    """Bind the engine to the librccl PyTorch loaded (one RCCL per process)."""
    ext.RcclP2P.load(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"))


def make_native_engine(group, ranks: Sequence[int], my_pipe_rank: int, device: torch.device):
    """Collective over the pipeline group: pipeline rank 0 draws an RCCL unique id, the
    group broadcasts it, every rank joins the communicator (csrc/comm/rccl_p2p.cpp)."""
    from ..ops.kernels import load_ext
    ext = load_ext()
    if ext is None or not hasattr(ext, "RcclP2P"):
        raise RuntimeError("MIPIPE_P2P=native needs the built extension (_C.so)")
    load_native_rccl(ext)
    n = 128
    buf = torch.zeros(n, dtype=torch.uint8, device=device)
    if my_pipe_rank == 0:
        uid = ext.RcclP2P.unique_id()
        buf.copy_(torch.frombuffer(bytearray(uid), dtype=torch.uint8))
    if len(ranks) > 1:
        dist.broadcast(buf, src=ranks[0], group=group)
    uid = bytes(buf.cpu().tolist())
    return ext.RcclP2P(uid, len(ranks), my_pipe_rank, device.index if device.index is not None else 0)


class P2P:
    """Thin wrapper around ``torch.distributed`` p2p for one pipeline group.

    ``ranks[i]`` is the global rank of pipeline rank ``i``.  With the gloo backend and
    GPU tensors (``MIPIPE_DIST_BACKEND=gloo``: several ranks sharing one GPU, used to
    test the whole multi-process GPU stack on a single-GPU box) transfers are staged
    through host memory; with RCCL they go device to device over xGMI.
    """

    def __init__(self, group: Optional[dist.ProcessGroup], ranks: Sequence[int], device: torch.device):
        self.group = group
        self.ranks = list(ranks)
        self.device = device
        self.host_staged = (device.type == "cuda" and dist.is_initialized()
                            and dist.get_backend(group) == "gloo")
        # MIPIPE_P2P=native: grouped ncclSend/ncclRecv from the C++ engine on its own comm
        # stream instead of torch.distributed.batch_isend_irecv
        self.engine = None
        if (os.environ.get("MIPIPE_P2P", "torch") == "native" and device.type == "cuda" and dist.is_initialized()
                and not self.host_staged and len(self.ranks) > 1):
            me = self.ranks.index(dist.get_rank())
            self.engine = make_native_engine(group, self.ranks, me, device)

    def global_rank(self, pipe_rank: int) -> int:
        return self.ranks[pipe_rank]

    def post(self, sends: Sequence[Tuple[torch.Tensor, int]], recvs: Sequence[Tuple[torch.Tensor, int]]):
        """Post one group; returns (send_works, recv_works) aligned with the inputs."""
        from . import native_runner
        rec = native_runner.active()
        if self.engine is not None:
            if not sends and not recvs:
                return [], []
            h = self.engine.post([(t, p) for t, p in sends], [(t, p) for t, p in recvs])
            slot = rec.native_post(self.engine, sends, recvs) if rec is not None else -1
            w = _NativeWork(self.engine, h, rec, slot)
            return [w] * len(sends), [w] * len(recvs)
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
        for peer in sorted(set(peers)):
            if peer == my_rank:
                continue
            dev = "cpu" if self.host_staged else self.device
            t_send = torch.ones(1, device=dev)
            t_recv = torch.zeros(1, device=dev)
            s, r = self.post([(t_send, peer)], [(t_recv, peer)])
            for w in s + r:
                w.wait()
