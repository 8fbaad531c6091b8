"""Pipeline stages: the per-(virtual)-stage compute objects the runtime drives.

Two implementations share one interface (:class:`StageBase`):

* :class:`PipelineStage` wraps an arbitrary ``nn.Module`` and runs its backward
  through torch autograd -- the reference-compatible manual frontend
  (``PipelineStage(submodule, stage_index, num_stages, device)``, used at
  helper:93; dependency stage.py:1321-1588 / 116-1013).
* ``mipipe.models.native.NativeStage`` runs our models with explicit per-layer
  backward on HIP kernels, a static activation stash and split dX/dW backward.

The runtime never looks inside a stage: it hands it microbatch inputs (or the
recv buffers), asks for outputs / input-grads, and calls ``reduce_grad`` at the
stage's REDUCE_GRAD action.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

Spec = Tuple[Tuple[int, ...], torch.dtype]


def _as_tuple(x) -> Tuple[torch.Tensor, ...]:
    if isinstance(x, torch.Tensor):
        return (x,)
    return tuple(x)


def specs_of(ts: Sequence[torch.Tensor]) -> List[Spec]:
    return [(tuple(t.shape), t.dtype) for t in ts]


class StageBase:
    """Interface between the pipeline runtime and one virtual stage."""

    stage_index: int
    num_stages: int
    device: torch.device
    input_specs: Optional[List[Spec]] = None    # per microbatch
    output_specs: Optional[List[Spec]] = None

    @property
    def is_first(self) -> bool:
        return self.stage_index == 0

    @property
    def is_last(self) -> bool:
        return self.stage_index == self.num_stages - 1

    # --- hooks --------------------------------------------------------------------
    def forward_mb(self, mb: int, args: Tuple[torch.Tensor, ...], target: Optional[torch.Tensor],
                   loss_fn: Optional[Callable], loss_scale: float) -> Tuple[Tuple[torch.Tensor, ...], Optional[torch.Tensor]]:
        raise NotImplementedError

    def backward_mb(self, mb: int, grad_outputs: Optional[Tuple[torch.Tensor, ...]]) -> Tuple[Optional[torch.Tensor], ...]:
        raise NotImplementedError

    def backward_input_mb(self, mb: int, grad_outputs):
        """Input-grad half of a split backward (I).  Default: full backward."""
        return self.backward_mb(mb, grad_outputs)

    def backward_weight_mb(self, mb: int) -> None:
        """Weight-grad half of a split backward (W).  Default: done by I."""
        return None

    def infer_output_specs(self, args: Tuple[torch.Tensor, ...]) -> List[Spec]:
        raise NotImplementedError

    def reduce_grad(self, n_microbatches: int, scaled_in_loss: bool):
        """Called once per step after this stage's last backward.  May return an
        async work handle (DP all-reduce) that the runtime waits for at step end."""
        return None

    def has_grad_reduction(self, scaled_in_loss: bool) -> bool:
        """Whether ``reduce_grad`` issues any work (a recorded native tape skips the CALL
        otherwise).  Conservative default: yes."""
        return True

    def clear_runtime_states(self) -> None:
        pass

    def post_step(self) -> None:
        """Called once after every microbatch and reduction of a step completed (e.g. tied
        embedding grad sync between the first and the last stage)."""
        return None


class PipelineStage(StageBase):
    """Autograd-driven stage around a user ``nn.Module`` (reference frontend).

    ``input_args``/``output_args`` (example tensors or specs) make shapes static;
    otherwise the runtime infers them once with a no-grad forward, chained stage
    by stage (dependency behavior stage.py:1410-1519, without pickled objects).
    """

    def __init__(self, submodule: nn.Module, stage_index: int, num_stages: int, device: torch.device,
                 input_args: Any = None, output_args: Any = None, group=None, dw_builder=None, *,
                 graphs: bool = False):
        if not 0 <= stage_index < num_stages:
            raise ValueError(f"stage_index {stage_index} out of range for {num_stages} stages")
        self.submod = submodule
        self.stage_index = stage_index
        self.num_stages = num_stages
        self.device = torch.device(device)
        self.group = group
        if input_args is not None:
            self.input_specs = specs_of(_as_tuple(input_args))
        if output_args is not None:
            self.output_specs = specs_of(_as_tuple(output_args))
        self._fwd_cache: Dict[int, Tuple[Tuple[torch.Tensor, ...], Tuple[torch.Tensor, ...]]] = {}
        self._loss_cache: Dict[int, torch.Tensor] = {}
        self.dp_group = None
        # HIP graphs for the user module (GPU only): one graphed forward/backward pair per
        # microbatch slot (torch.cuda.make_graphed_callables), so microbatches in flight
        # never share the static activation buffers.  Launch-bound short-token stages (the
        # reference's 1024-token microbatches: hundreds of small ATen kernels) replay each
        # direction as one graph.  Captured lazily on the first forward of each slot.
        self.graphs = bool(graphs)
        # make_graphed_callables synchronises the whole device while it captures, lazily, in
        # the middle of a step: with RCCL receives pending on the comm streams that is a
        # cross-rank wait.  Autograd-stage graphs stay for one process / gloo-staged runs;
        # NativeStage graphs (parallel/graphs.py capture) never synchronise
        import torch.distributed as dist
        if self.graphs and dist.is_initialized() and dist.get_world_size() > 1 and dist.get_backend() == "nccl":
            self.graphs = False
        self._graph_fns: Dict[int, Callable] = {}
        self._f32_kernels = False
        self._orig_forward: Optional[Callable] = None

    @property
    def f32_kernels(self) -> bool:
        """f32 modules on GPU: every linear / attention projection of the submodule on the
        f32 MFMA GEMM (ops.use_f32_kernels swaps the submodules' classes; nothing global is
        patched); off: ATen (hipBLASLt)."""
        return self._f32_kernels

    @f32_kernels.setter
    def f32_kernels(self, on: bool) -> None:
        on = bool(on)
        if on != self._f32_kernels:
            from ..ops.kernels import use_f32_kernels
            use_f32_kernels(self.submod, on)
            self._f32_kernels = on

    # reference-visible attributes
    @property
    def submod_parameters(self):
        return self.submod.parameters()

    def infer_output_specs(self, args):
        with torch.no_grad():
            out = _as_tuple(self.submod(*args))
        self.output_specs = specs_of(out)
        return self.output_specs

    def forward_mb(self, mb, args, target, loss_fn, loss_scale):
        inputs = []
        for a in args:
            if not self.is_first and a.is_floating_point():
                a = a.detach().requires_grad_(True)
            inputs.append(a)
        inputs = tuple(inputs)
        fwd = self._graphed_fn(mb, inputs) if self.graphs and self.device.type == "cuda" else self.submod
        with torch.enable_grad():
            out = _as_tuple(fwd(*inputs))
        loss = None
        if self.is_last and loss_fn is not None:
            loss = loss_fn(out[0] if len(out) == 1 else out, target)
            self._loss_cache[mb] = loss * loss_scale if loss_scale != 1.0 else loss
        self._fwd_cache[mb] = (inputs, out)
        return tuple(o.detach() for o in out), loss

    def _graphed_fn(self, mb: int, inputs: Tuple[torch.Tensor, ...]) -> Callable:
        fn = self._graph_fns.get(mb)
        if fn is None:
            mod = self.submod
            # make_graphed_callables patches module.forward with the graphed function:
            # keep the original for the next slot's capture and for eager calls
            if self._orig_forward is None:
                self._orig_forward = mod.forward
            mod.forward = self._orig_forward
            # the graphed backward hands its static grad buffers to AccumulateGrad, which
            # would adopt one as .grad (no copy) while .grad is None -- and the next replay
            # of that slot would overwrite it: give every parameter its own .grad first
            for p in mod.parameters():
                if p.requires_grad and p.grad is None:
                    p.grad = torch.zeros_like(p)
            sample = tuple(a.detach().clone().requires_grad_(a.requires_grad) for a in inputs)
            # warmup iterations use autograd.grad (no .grad accumulation); the module's
            # dropout draws from the graph-registered generator state on every replay
            torch.cuda.make_graphed_callables(mod, sample, num_warmup_iters=3)
            fn = mod.forward
            mod.forward = self._orig_forward
            self._graph_fns[mb] = fn
        return fn

    def backward_mb(self, mb, grad_outputs):
        inputs, out = self._fwd_cache.pop(mb)
        if self.is_last:
            if mb in self._loss_cache:
                torch.autograd.backward(self._loss_cache.pop(mb))
            else:
                raise RuntimeError("last stage backward without a loss (pass loss_fn to the schedule)")
        else:
            pairs = [(o, g) for o, g in zip(out, grad_outputs) if o.requires_grad and g is not None]
            if pairs:
                torch.autograd.backward([p[0] for p in pairs], grad_tensors=[p[1] for p in pairs])
        grads = tuple(x.grad if isinstance(x, torch.Tensor) and x.requires_grad else None for x in inputs)
        return grads

    def reduce_grad(self, n_microbatches, scaled_in_loss):
        if not scaled_in_loss:
            for p in self.submod.parameters():
                if p.grad is not None:
                    p.grad.div_(n_microbatches)
        if self.dp_group is not None:
            from .dp import allreduce_module_grads
            return allreduce_module_grads(self.submod, self.dp_group)
        return None

    def clear_runtime_states(self):
        self._fwd_cache.clear()
        self._loss_cache.clear()
