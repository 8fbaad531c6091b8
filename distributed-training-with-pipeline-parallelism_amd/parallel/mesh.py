"""Process bootstrap and the DP x PP rank mesh.

One process per GPU (``torchrun``-style env: RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT).  Backend ``nccl`` is RCCL on ROCm; ``gloo`` is used on
CPU (the reference's plumbing config, helper:167-178).  Unlike the reference,
the process groups that are created are the ones actually used (the reference's
``pp_group = dist.new_group()`` is unused, helper:178).

Rank layout: ``global = dp_index * pp + pp_index`` -- a pipeline occupies
consecutive GPUs, so every stage boundary is a direct xGMI link (MI355X nodes are
fully connected, 7 links per GPU) and the DP all-reduce of a stage runs between
GPUs ``pp`` apart, also direct.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist


def init_distributed(backend: Optional[str] = None, timeout_s: Optional[float] = None) -> tuple:
    """Initialise the default process group from env; returns (rank, world, local_rank, device).

    ``timeout_s`` (default ``MIPIPE_PG_TIMEOUT_S`` or 300 s) bounds every collective and
    p2p wait of the process group -- well under a launcher's own limit, so a hung peer
    ends the job with an error instead of running into an external kill."""
    if timeout_s is None:
        timeout_s = float(os.environ.get("MIPIPE_PG_TIMEOUT_S", "300"))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    backend = backend or os.environ.get("MIPIPE_DIST_BACKEND") or None
    # MIPIPE_DIST_BACKEND=gloo on a GPU box: every rank computes on the GPU (ranks may
    # share one device) while gloo carries the traffic through host memory -- a test
    # mode for the multi-process GPU stack on a single-GPU machine
    gloo_on_gpu = backend == "gloo" and torch.cuda.is_available() and os.environ.get("MIPIPE_GLOO_GPU", "1") == "1"
    use_gpu = torch.cuda.is_available() and (backend != "gloo" or gloo_on_gpu)
    if use_gpu:
        dev_index = local_rank % torch.cuda.device_count() if gloo_on_gpu else local_rank
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    else:
        device = torch.device("cpu")
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = device  # eager RCCL communicator init
        dist.init_process_group(**kw)
    return rank, world, local_rank, device


@dataclass
class Mesh:
    rank: int
    world: int
    pp: int
    dp: int
    pp_rank: int
    dp_rank: int
    pipe_ranks: List[int]           # global ranks of my pipeline, by pipeline rank
    pp_group: Optional[object]
    dp_group: Optional[object]
    embed_group: Optional[object]   # first + last stage of my pipeline (tied embeddings)
    ctrl_group: Optional[object] = None   # gloo group of my pipeline: control-plane votes
    world_ctrl: Optional[object] = None   # gloo group of every rank (None: the world is gloo)

    @property
    def is_first(self) -> bool:
        return self.pp_rank == 0

    @property
    def is_last(self) -> bool:
        return self.pp_rank == self.pp - 1


def build_mesh(pp: int, dp: int = 1, backend_device: Optional[torch.device] = None) -> Mesh:
    if dist.is_initialized():
        rank, world = dist.get_rank(), dist.get_world_size()
    else:
        rank, world = 0, 1
    if pp * dp != world:
        raise ValueError(f"pp({pp}) x dp({dp}) != world size {world}")
    dp_rank, pp_rank = divmod(rank, pp)
    pp_group = dp_group = embed_group = ctrl_group = world_ctrl = None
    pipe_ranks = [dp_rank * pp + i for i in range(pp)]
    if world > 1:
        # host-side (gloo) group per pipeline for control-plane agreement (the native p2p
        # engine's pre-flight vote): it cannot be blocked by a wedged GPU communicator
        gloo_default = dist.get_backend() == "gloo"
        for d in range(dp):
            ranks = [d * pp + i for i in range(pp)]
            if gloo_default:
                g = None
            else:
                g = dist.new_group(ranks, backend="gloo") if pp > 1 else None
            if d == dp_rank:
                ctrl_group = g
        # world-wide control plane: decisions every rank must take alike (the DP transport,
        # the collective placement) are voted over it
        if not gloo_default:
            world_ctrl = dist.new_group(list(range(world)), backend="gloo")
        # every rank must create every group, in the same order
        for d in range(dp):
            ranks = [d * pp + i for i in range(pp)]
            g = dist.new_group(ranks) if pp < world else dist.group.WORLD
            if d == dp_rank:
                pp_group = g
        for i in range(pp):
            ranks = [d * pp + i for d in range(dp)]
            g = dist.new_group(ranks) if dp > 1 else None
            if i == pp_rank:
                dp_group = g
        for d in range(dp):
            ranks = sorted({d * pp, d * pp + pp - 1})
            g = dist.new_group(ranks) if len(ranks) > 1 else None
            if d == dp_rank and pp_rank in (0, pp - 1):
                embed_group = g
        # force communicator creation on every group (batch p2p requires an
        # initialised communicator before the first grouped call)
        dev = backend_device or (torch.device("cuda", torch.cuda.current_device())
                                 if dist.get_backend() == "nccl" else torch.device("cpu"))
        t = torch.zeros(1, device=dev)
        if pp_group is not None and pp > 1:
            dist.all_reduce(t, group=pp_group)
        if dp_group is not None:
            dist.all_reduce(t, group=dp_group)
        if embed_group is not None:
            dist.all_reduce(t, group=embed_group)
        if dev.type == "cuda":
            torch.cuda.synchronize()
    if ctrl_group is None and world > 1 and dist.get_backend() == "gloo":
        ctrl_group = pp_group
    return Mesh(rank, world, pp, dp, pp_rank, dp_rank, pipe_ranks, pp_group, dp_group, embed_group, ctrl_group,
                world_ctrl)
