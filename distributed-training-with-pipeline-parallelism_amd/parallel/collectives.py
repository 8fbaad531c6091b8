"""Collectives of a training step on the native RCCL engines (SURVEY §7.1 comm/rccl_allreduce, §5.8).

Every reduction a step performs goes through one :class:`Collectives` object per rank:

=====================  ========  ============================================================
what                   scope     where
=====================  ========  ============================================================
stage grad all-reduce  ``dp``    ``REDUCE_GRAD`` (models/stage.py ``reduce_grad``)
head grad reduce       ``pp``    ``REDUCE_HEAD``: reduce-scatter of the replicated head's
                                 gradient, then ``dp`` all-reduce of this rank's shard
                                 (ZeRO-1 head, engine.py)
clip-norm sum          ``pp``    FlatAdamW.step (4 bytes)
loss sum               ``pp``    PipelineTrainer.train_step (one float per microbatch)
head weight gather     ``pp``    all-gather of the updated bf16 head shards
tied embedding sum     ``embed`` first + last stage (no distributed head): NativeStage.post_step
=====================  ========  ============================================================

On GPUs with the RCCL backend the pipeline group's collectives run on the pipeline
engine's collective channel (csrc/comm/rccl_engine.h, stream slot "coll") and the DP
group's on a one-channel DP engine issuing on the SAME stream slot, so all collectives
of a rank form one FIFO in host issue order -- identical on DP replicas, and checked by
:func:`.simulate.check_lowered`.  Inside a recorded step (parallel/native_runner.py) they
become native COLL / WAIT instructions: the tape of a GPU step holds no Python CALL.
Elsewhere (CPU / gloo, torch p2p fallback) they are ``torch.distributed`` calls.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

# csrc/comm/rccl_engine.h CollOp
ALLREDUCE_SUM, REDUCE_SCATTER_SUM, ALL_GATHER, ALLREDUCE_MAX = 0, 1, 2, 3
COLL_SLOT = 2           # the collective stream slot
PIPE_COLL_CHANNEL = 2   # channel of the pipeline engine that issues on it


class _Done:
    def wait(self):
        return True


class _EngineWork:
    """A collective posted on a native engine; ``wait`` makes the current stream wait (no
    host block) and, inside a recording step, puts the WAIT on the tape."""

    def __init__(self, engine, handle: int, rec=None, slot: int = -1):
        self.engine, self.handle, self.rec, self.slot = engine, handle, rec, slot

    def wait(self):
        self.engine.wait(self.handle)
        if self.rec is not None:
            self.rec.native_wait(self.slot)
            self.rec = None
        return True


class _Then:
    """Work whose completion runs ``finish`` (a copy out of a staging buffer)."""

    def __init__(self, work, finish):
        self.work, self.finish = work, finish

    def wait(self):
        from . import native_runner
        if self.work is not None:
            self.work.wait()
        if self.finish is not None:
            self.finish()
            rec = native_runner.active()
            if rec is not None:
                rec.call(self.finish)     # replayed after the recorded wait
            self.finish = None
        return True


def make_dp_engine(dp_group, dp_ranks: List[int], my_dp_rank: int, device: torch.device):
    """One-channel RCCL engine over a DP group, issuing on the collective stream slot."""
    from ..ops.kernels import load_ext
    from .comm import load_native_rccl
    ext = load_ext()
    load_native_rccl(ext)
    nb = int(ext.RcclEngine.id_bytes())
    buf = torch.zeros(nb, dtype=torch.uint8, device=device)
    if my_dp_rank == 0:
        buf.copy_(torch.frombuffer(bytearray(ext.RcclEngine.unique_id()), dtype=torch.uint8))
    dist.broadcast(buf, src=dp_ranks[0], group=dp_group)
    uid = bytes(buf.cpu().tolist())
    return ext.RcclEngine(uid, len(dp_ranks), my_dp_rank, device.index if device.index is not None else 0,
                          [COLL_SLOT])


class Collectives:
    """Collectives over this rank's pipeline group (``"pp"``) and DP group (``"dp"``).

    ``pipe_engine``: the pipeline's native engine (parallel/comm.py P2P.engine) when it has
    a collective channel; the DP engine is built here when the pipeline's is native (same
    backend, GPUs) and ``dp > 1``.  Each call returns a work handle (``wait()``), or one
    that is already complete when the group has a single rank."""

    def __init__(self, mesh, device: torch.device, pipe_engine=None, embed: bool = False):
        self.mesh = mesh
        self.device = torch.device(device)
        self.pp_group, self.dp_group = mesh.pp_group, mesh.dp_group
        self.pp, self.dp = mesh.pp, mesh.dp
        self.pipe_engine = pipe_engine if (pipe_engine is not None and
                                           int(pipe_engine.channels) > PIPE_COLL_CHANNEL) else None
        self.dp_engine = None
        # element type of the ZeRO-1 DP gradient reduce-scatter: f32 (default) or bf16
        # (MIPIPE_DP_REDUCE_DTYPE=bf16: half the bytes on the per-link-bound xGMI ring)
        rd = os.environ.get("MIPIPE_DP_REDUCE_DTYPE", "f32").lower()
        if rd not in ("f32", "fp32", "bf16"):
            raise ValueError(f"MIPIPE_DP_REDUCE_DTYPE={rd}: f32 or bf16")
        self.dp_reduce_dtype = torch.bfloat16 if rd == "bf16" else torch.float32
        if self.dp > 1 and self.dp_transport_native(mesh):
            dp_ranks = [d * self.pp + mesh.pp_rank for d in range(self.dp)]
            self.dp_engine = make_dp_engine(self.dp_group, dp_ranks, mesh.dp_rank, self.device)
        # the tied embedding's two copies (first + last stage, no distributed head): a
        # 2-rank engine over mesh.embed_group on the same collective slot
        self.embed_group = getattr(mesh, "embed_group", None) if embed else None
        self.embed_engine = None
        if (self.embed_group is not None and self.pipe_engine is not None and self.device.type == "cuda"
                and os.environ.get("MIPIPE_COLL", "native") != "torch"):
            d = mesh.dp_rank
            ranks = sorted({d * self.pp, d * self.pp + self.pp - 1})
            self.embed_engine = make_dp_engine(self.embed_group, ranks, ranks.index(mesh.rank), self.device)
        if self.pp > 1 and self.pipe_engine is None:
            self.pp_kind = "torch"
        else:
            self.pp_kind = "native" if self.pipe_engine is not None else "none"
        if self.dp > 1:
            self.dp_kind = "native" if self.dp_engine is not None else "torch"
        else:
            self.dp_kind = "none"
        self.audit = None   # parallel/audit.CommAudit while a step is audited

    def _members(self, scope: str) -> list:
        """Global ranks of a scope's group (mesh layout: rank = dp_rank * pp + pp_rank)."""
        d, s = self.mesh.dp_rank, self.mesh.pp_rank
        if scope == "pp":
            return [d * self.pp + i for i in range(self.pp)]
        if scope == "embed":
            return sorted({d * self.pp, d * self.pp + self.pp - 1})
        return [i * self.pp + s for i in range(self.dp)]

    def _log(self, scope: str, op: str, t: torch.Tensor) -> None:
        if self.audit is not None:
            self.audit.coll(scope, self._members(scope), op, t)

    def _dp_native_wanted(self) -> bool:
        """This rank's own view: RCCL backend on a GPU and a native pipeline engine (or no
        pipeline) -- a pipeline whose pre-flight fell back to torch p2p has no engine."""
        return (os.environ.get("MIPIPE_COLL", "native") != "torch" and self.device.type == "cuda"
                and dist.is_initialized() and dist.get_backend(self.dp_group) == "nccl"
                and (self.pipe_engine is not None or self.pp == 1))

    def dp_transport_native(self, mesh) -> bool:
        """The DP transport, decided ALIKE on every rank: the pre-flight vote of a
        pipeline covers only that pipeline, so one replica may run native p2p while another
        fell back -- its DP peers would then never enter the engine's broadcast + blocking
        communicator init.  The native engine is used only if every rank of the world wants
        it (MIN vote over the world control group, gloo when the world is RCCL)."""
        want = self._dp_native_wanted()
        if not dist.is_initialized() or dist.get_world_size() <= 1:
            return want
        from .comm import agree
        return agree(want, getattr(mesh, "world_ctrl", None), self.device)

    @property
    def kind(self) -> str:
        return f"pp:{self.pp_kind},dp:{self.dp_kind}"

    def _size(self, scope: str) -> int:
        if scope == "embed":
            return dist.get_world_size(self.embed_group) if self.embed_group is not None else 1
        return self.pp if scope == "pp" else self.dp

    def _engine(self, scope: str):
        if scope == "pp":
            return self.pipe_engine, PIPE_COLL_CHANNEL
        if scope == "embed":
            return self.embed_engine, 0
        return self.dp_engine, 0

    def _group(self, scope: str):
        if scope == "embed":
            return self.embed_group
        return self.pp_group if scope == "pp" else self.dp_group

    # ------------------------------------------------------------------ issue
    def _native(self, scope: str, op: int, send: torch.Tensor, recv: torch.Tensor):
        from . import native_runner
        eng, ch = self._engine(scope)
        h = eng.coll(ch, op, send, recv)
        rec = native_runner.active()
        slot = -1
        if rec is not None:
            slot = rec.native_coll(eng, ch, op, send, recv, self._size(scope))
        return _EngineWork(eng, h, rec, slot)

    def _torch(self, issue):
        """Issue a torch.distributed collective (recorded as a CALL inside a recording step)."""
        from . import native_runner
        rec = native_runner.active()
        if rec is not None:
            return native_runner.record_issue(rec, lambda: [issue()])[0]
        return issue()

    def all_reduce(self, t: torch.Tensor, scope: str, op: str = "sum"):
        """In-place all-reduce (``op`` sum | max)."""
        if self._size(scope) <= 1:
            return _Done()
        self._log(scope, "all_reduce_" + op, t)
        eng, _ = self._engine(scope)
        if eng is not None:
            return self._native(scope, ALLREDUCE_SUM if op == "sum" else ALLREDUCE_MAX, t, t)
        rop = dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX
        return self._torch(lambda: dist.all_reduce(t, op=rop, group=self._group(scope), async_op=True))

    def reduce_scatter(self, full: torch.Tensor, scope: str) -> "tuple":
        """Sum ``full`` (1-D, numel divisible by the group size) over the group; this rank's
        block ``full[r*n:(r+1)*n]`` holds the result afterwards (in place).  Returns (work,
        shard view)."""
        n_ranks = self._size(scope)
        r = self.mesh.pp_rank if scope == "pp" else self.mesh.dp_rank
        n = full.numel() // n_ranks
        shard = full[r * n:(r + 1) * n]
        if n_ranks <= 1:
            return _Done(), shard
        self._log(scope, "reduce_scatter", full)
        eng, _ = self._engine(scope)
        if eng is not None:
            return self._native(scope, REDUCE_SCATTER_SUM, full, shard), shard
        g = self._group(scope)
        if dist.get_backend(g) == "gloo":
            # gloo has no reduce-scatter: all-reduce the whole buffer (CPU plumbing only)
            return self._torch(lambda: dist.all_reduce(full, group=g, async_op=True)), shard
        tmp = torch.empty_like(shard)

        def issue():
            return dist.reduce_scatter_tensor(tmp, full, group=g, async_op=True)
        return _Then(self._torch(issue), lambda: shard.copy_(tmp)), shard

    def all_gather(self, full: torch.Tensor, scope: str):
        """In-place all-gather: every rank's block ``full[r*n:(r+1)*n]`` is broadcast into
        the others' copies of ``full``."""
        n_ranks = self._size(scope)
        if n_ranks <= 1:
            return _Done()
        r = self.mesh.pp_rank if scope == "pp" else self.mesh.dp_rank
        n = full.numel() // n_ranks
        shard = full[r * n:(r + 1) * n]
        self._log(scope, "all_gather", full)
        eng, _ = self._engine(scope)
        if eng is not None:
            return self._native(scope, ALL_GATHER, shard, full)
        g = self._group(scope)
        if dist.get_backend(g) == "gloo":
            parts = [torch.empty_like(shard) for _ in range(n_ranks)]

            def fin():
                for i, p in enumerate(parts):
                    if i != r:
                        full[i * n:(i + 1) * n].copy_(p)
            return _Then(self._torch(lambda: dist.all_gather(parts, shard.clone(), group=g, async_op=True)), fin)
        return self._torch(lambda: dist.all_gather_into_tensor(full, shard.clone(), group=g, async_op=True))

    def close(self) -> None:
        for name in ("dp_engine", "embed_engine"):
            eng = getattr(self, name)
            if eng is not None:
                eng.close()
                setattr(self, name, None)
