"""Reference-compatible schedule classes.

The reference drives its pipeline through (helper:12, 215-220, 115-131)::

    ScheduleGPipe(stage, n_microbatches=4, loss_fn=...)
    Schedule1F1B(stage, n_microbatches=4, loss_fn=...)
    ScheduleInterleaved1F1B([stages], n_microbatches=4, loss_fn=...)
    schedule.step(x)                         # first stage
    schedule.step(target=y, losses=losses)   # last stage -> merged outputs
    schedule.step()                          # middle stages

These classes keep that API (plus ``eval`` and ``get_schedule_class`` /
``LoopedBFS`` / ``ZBH1``) on top of :class:`~.runtime.PipelineRuntime`.  Inputs and
targets are split into microbatches along dim 0 with ``tensor_split`` (dependency
microbatch.py:184-203) -- views, no copies -- and the last stage's outputs are
concatenated back (microbatch.py:423-544) only when ``return_outputs``.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Union

import torch
import torch.distributed as dist

from .comm import P2P
from .runtime import PipelineRuntime
from .schedules import SCHEDULES, canonical_name, interleave_params
from .stage import StageBase


def _split(t: torch.Tensor, m: int) -> List[torch.Tensor]:
    if t.shape[0] < m:
        raise ValueError(f"batch {t.shape[0]} smaller than n_microbatches {m}")
    return list(torch.tensor_split(t, m, dim=0))


class _PipelineSchedule:
    _name = "GPipe"

    def __init__(self, stages: Union[StageBase, Sequence[StageBase]], n_microbatches: int,
                 loss_fn: Optional[Callable] = None, scale_grads: bool = True, group=None,
                 pipe_ranks: Optional[Sequence[int]] = None, style: str = "loop", profile: bool = False,
                 copy_outputs: bool = True, p2p: Optional[P2P] = None):
        """``p2p``: an existing transport over the same group (a sweep building many schedules
        in one process group reuses one set of RCCL communicators).  ``copy_outputs`` (default, the reference's semantics): the last rank's ``step()``
        returns a fresh tensor, as the dependency's ``torch.cat`` merge does.  False: a
        zero-copy view of the native stage's persistent logits buffer -- valid only until the
        next ``step()``, which rewrites it in place (eager copy or graph replay)."""
        stages = [stages] if isinstance(stages, StageBase) else list(stages)
        self.copy_outputs = bool(copy_outputs)
        multi = SCHEDULES[self._name][2]
        if not multi and len(stages) != 1:
            raise ValueError(f"{self._name} takes exactly one stage per rank")
        self._stages = stages
        self._n_microbatches = n_microbatches
        self._loss_fn = loss_fn
        self.scale_grads = scale_grads
        num_stages = stages[0].num_stages
        if dist.is_initialized():
            group = group if group is not None else getattr(stages[0], "group", None)
            pp = dist.get_world_size(group)
            rank = dist.get_rank(group)
            if pipe_ranks is None:
                pipe_ranks = dist.get_process_group_ranks(group) if group is not None else list(range(pp))
        else:
            pp, rank, pipe_ranks = 1, 0, [0]
        if not multi and n_microbatches < num_stages:
            # torch schedules.py:578-583
            raise ValueError(f"{self._name} requires n_microbatches ({n_microbatches}) >= num_stages ({num_stages})")
        if self._name == "Interleaved1F1B":
            interleave_params(pp, n_microbatches)
        if p2p is None:
            p2p = P2P(group, pipe_ranks, stages[0].device)
        else:
            p2p.reset_channels()
        self._runtime = PipelineRuntime(stages, self._name, n_microbatches, rank, pp, p2p, loss_fn=loss_fn,
                                        scale_grads=scale_grads, style=style, profile=profile)
        self.pipeline_order = self._runtime.orders

    @property
    def runtime(self) -> PipelineRuntime:
        return self._runtime

    def step(self, *args, target: Optional[torch.Tensor] = None, losses: Optional[list] = None,
             return_outputs: bool = True, **kwargs):
        m = self._n_microbatches
        has_first = any(s.is_first for s in self._stages)
        has_last = any(s.is_last for s in self._stages)
        inputs = None
        if has_first:
            if not args:
                raise ValueError("the first-stage rank must pass inputs to step()")
            chunks = [_split(a, m) for a in args]
            inputs = [tuple(c[i] for c in chunks) for i in range(m)]
        targets = _split(target, m) if (has_last and target is not None) else None
        outs = self._runtime.step(inputs, targets, losses, return_outputs=return_outputs and has_last)
        if outs is None or not has_last:
            return None
        if len(outs[0]) == 1:
            return _merge([o[0] for o in outs], self.copy_outputs)   # merged last-stage outputs (logits)
        return tuple(_merge([o[i] for o in outs], self.copy_outputs) for i in range(len(outs[0])))

    def eval(self, *args, target=None, losses=None):
        """Forward-only pass (dependency schedules.py:402-420)."""
        with torch.no_grad():
            return self._run_forward_only(args, target, losses)

    def _run_forward_only(self, args, target, losses):
        from .ir import Op
        from .lower import lower
        rt = self._runtime
        orders = {r: [a for a in seq if a.op == Op.F] for r, seq in rt.orders.items()}
        prog = lower(orders, rt.pp, rt.v, rt.style, add_reduce_grad=False)
        ev = PipelineRuntime(list(rt.stages.values()), rt.schedule, rt.m, rt.rank, rt.pp, rt.p2p,
                             loss_fn=rt.loss_fn, scale_grads=False, style=rt.style, program=prog)
        ev._initialized = rt._initialized
        ev._recv_bufs = rt._recv_bufs
        m = self._n_microbatches
        inputs = None
        if any(s.is_first for s in self._stages):
            chunks = [_split(a, m) for a in args]
            inputs = [tuple(c[i] for c in chunks) for i in range(m)]
        targets = _split(target, m) if target is not None else None
        outs = ev.step(inputs, targets, losses)
        for st in rt.stages.values():
            st.clear_runtime_states()
        if not outs:
            return None
        return torch.cat([o[0] for o in outs], dim=0)


def _merge(parts, copy: bool = True):
    """torch.cat(parts, 0) -- or, when the parts are consecutive row blocks of one buffer (the
    native stage's persistent logits), the view of that buffer spanning them (``copy``: a
    clone of that view, so the result outlives the next step like the reference's)."""
    p0 = parts[0]
    if len(parts) > 1 and all(p.dim() == p0.dim() and p.shape[1:] == p0.shape[1:] and p.stride() == p0.stride()
                              and p.untyped_storage().data_ptr() == p0.untyped_storage().data_ptr()
                              for p in parts):
        step = p0.shape[0] * p0.stride(0)
        if all(p.shape[0] == p0.shape[0] and p.storage_offset() == p0.storage_offset() + i * step
               for i, p in enumerate(parts)):
            view = p0.as_strided((p0.shape[0] * len(parts),) + tuple(p0.shape[1:]), p0.stride(),
                                 p0.storage_offset())
            return view.clone() if copy else view
    return torch.cat(parts, dim=0)


class ScheduleGPipe(_PipelineSchedule):
    _name = "GPipe"


class Schedule1F1B(_PipelineSchedule):
    _name = "1F1B"


class ScheduleInterleaved1F1B(_PipelineSchedule):
    _name = "Interleaved1F1B"


class ScheduleLoopedBFS(_PipelineSchedule):
    _name = "LoopedBFS"


class ScheduleZBH1(_PipelineSchedule):
    _name = "ZBH1"


class ScheduleZBVZeroBubble(_PipelineSchedule):
    """Zero-bubble V schedule: two stages per rank in V placement (rank r holds stages
    r and 2P-1-r); stages must be built for ``style='v'``."""
    _name = "ZBV"

    def __init__(self, stages, n_microbatches, loss_fn=None, scale_grads=True, group=None, pipe_ranks=None,
                 style: str = "v", profile: bool = False, copy_outputs: bool = True, p2p=None):
        super().__init__(stages, n_microbatches, loss_fn, scale_grads, group, pipe_ranks, "v", profile, copy_outputs,
                         p2p)


_CLASSES = {"GPipe": ScheduleGPipe, "1F1B": Schedule1F1B, "Interleaved1F1B": ScheduleInterleaved1F1B,
            "LoopedBFS": ScheduleLoopedBFS, "ZBH1": ScheduleZBH1, "ZBV": ScheduleZBVZeroBubble}


def get_schedule_class(name: str):
    """Name registry (dependency schedules.py:3219-3243)."""
    return _CLASSES[canonical_name(name)]
