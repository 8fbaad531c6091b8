"""Adapter between :class:`~mipipe.models.native.NativeModel` and the pipeline runtime."""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.distributed as dist

from ..parallel.dp import allreduce_flat
from ..parallel.graphs import GraphCache
from ..parallel.stage import StageBase
from .config import NativeConfig
from .. import ops
from .native import MBContext, NativeModel, _seed


class NativeStage(StageBase):
    """One virtual pipeline stage of a native model.

    Static shapes (no runtime shape inference): stage 0 receives ``[mbs, S]`` int64
    tokens, every other stage ``[mbs*S, d_model]`` bf16 activations; the last stage
    emits the microbatch loss.  Gradients are already scaled by ``1/m`` through the loss
    scale; ``reduce_grad`` issues the async DP all-reduce on the flat grad arena and
    ``post_step`` sums tied-embedding grads between the first and last stage.
    """

    def __init__(self, model: NativeModel, mbs: int, seq_len: int, dp_group=None, embed_group=None,
                 seed: int = 1234, graphs: bool = False):
        self.model = model
        self.cfg: NativeConfig = model.cfg
        self.stage_index = model.stage_index
        self.num_stages = model.num_stages
        self.device = model.device
        self.mbs, self.S = mbs, seq_len
        self.dp_group = dp_group
        self.embed_group = embed_group
        self.seed = seed
        self.step_id = 0
        T = mbs * seq_len
        D = self.cfg.d_model
        if self.is_first:
            self.input_specs = [((mbs, seq_len), torch.int64)]
        else:
            self.input_specs = [((T, D), model.arena.dtype)]
        self.split_head = model.split_head
        if self.is_last and not self.split_head:
            self.output_specs = [((), torch.float32)]
        else:  # hidden states (the last stage's final-norm output with a distributed head)
            self.output_specs = [((T, D), model.arena.dtype)]
        self._ctx = {}
        # HIP graphs (parallel/graphs.py): step 1 runs eagerly (lazy kernel init), every
        # (op, microbatch) action is captured on its first later use and replayed after
        # (dropout stays graph-safe: kernels mix a device-side step counter into their
        # seeds, ops.set_dropout_step, so replays draw fresh masks)
        if graphs and model.device.type != "cuda":
            graphs = False
        self.graphs = GraphCache(str(self.stage_index)) if graphs else None
        self.want_outputs = False   # set per step by the runtime (step(return_outputs=...))
        self.n_microbatches = 1     # (likewise)
        # returned logits: microbatch mb's rows of one persistent [m * T, vocab_padded] buffer,
        # so the schedule hands back the merged [B, S, vocab] as a view (no concatenation)
        self._merged_logits: Optional[torch.Tensor] = None
        self._gctx = {}
        # activation-stash slot ring under HIP graphs (parallel/stash.py, set by the runtime):
        # mb -> (lane, slot); the graphs of a slot's microbatches share one memory pool
        self._slot_of: Dict[int, tuple] = {}
        self._last_reader: Dict[int, str] = {}
        self._pools: Dict[tuple, object] = {}
        self._released: set = set()

    def set_stash_plan(self, slot_of: Dict[int, tuple], last_reader: Dict[int, str]) -> None:
        """Slot of each microbatch's stash and the op that reads it last (B, or W after I)."""
        self._slot_of, self._last_reader = dict(slot_of), dict(last_reader)

    def stash_slots(self) -> int:
        return len(set(self._slot_of.values())) if self._slot_of else 0

    def _pool(self, mb: int):
        c = self._slot_of.get(mb)
        if c is None or self.model.device.type != "cuda":
            return None
        p = self._pools.get(c)
        if p is None:
            p = self._pools[c] = torch.cuda.graph_pool_handle()
        return p

    def _release_stash(self, mb: int, op: str) -> None:
        """After the capture of the stash's last reader: unpin it, so the slot's next
        forward capture reuses its blocks (replay order on the slot's lane = capture order)."""
        if self._last_reader.get(mb) != op or mb in self._released or mb not in self._slot_of:
            return
        self._released.add(mb)
        for key in (("F", mb), ("FL", mb), ("I", mb)):
            self.graphs.release(key)
        self._gctx.pop(mb, None)

    def _graphed(self) -> bool:
        return self.graphs is not None and self.step_id > 1

    @property
    def arena(self):
        return self.model.arena

    def clear_runtime_states(self):
        self._ctx.clear()
        self.step_id += 1
        if self.cfg.dropout > 0 and self.model.device.type == "cuda":
            ops.set_dropout_step(self.step_id, self.model.device)

    def forward_mb(self, mb, args, target, loss_fn, loss_scale):
        # compat step(return_outputs=True) on the last stage: also hand back the logits
        want_logits = self.is_last and not self.split_head and self.want_outputs and target is not None
        if self._graphed():
            return self._forward_graphed(mb, args, target, loss_scale, want_logits)
        # on the GPU the step enters through the device counter (set_dropout_step), so
        # eager and graph-replayed steps draw identical masks; the CPU ops see the seed only
        ctx = MBContext(mb, _seed(self.seed, 0 if self.model.device.type == "cuda" else self.step_id, mb))
        if want_logits:
            ctx.misc["logits_dst"] = self._logits_dst(mb)
        x = args[0]
        out = self.model.forward(x, ctx, self.mbs, self.S, target=target if self.is_last else None,
                                 loss_scale=loss_scale, keep_logits=want_logits)
        self._ctx[mb] = ctx
        if self.is_last and not self.split_head:
            if target is None:
                return (self._logits_view(out),), None
            if want_logits:
                # merged by the schedule into [B, S, vocab] like the reference's last-rank
                # step() return value (helper:128, schedules.py:646-652)
                return (self._logits_view(ctx.misc.pop("logits_out")),), out
            return (out.detach(),), out
        return (out,), None

    def _logits_dst(self, mb: int) -> torch.Tensor:
        T = self.mbs * self.S
        m = max(self.n_microbatches, mb + 1)
        buf = self._merged_logits
        if buf is None or buf.shape[0] < m * T:
            buf = self._merged_logits = torch.empty(m * T, self.cfg.vocab_padded, dtype=self.model.arena.dtype,
                                                    device=self.model.device)
        return buf[mb * T:(mb + 1) * T]

    def _logits_view(self, logits):
        """[T, vocab_padded] -> [mbs, S, vocab] (the reference's output shape)."""
        V = self.cfg.vocab_size
        return logits[:, :V].reshape(self.mbs, self.S, V)

    def _dy(self, grad_outputs):
        if (self.is_last and not self.split_head) or not grad_outputs:
            return None
        return grad_outputs[0]

    def backward_mb(self, mb, grad_outputs):
        if self._graphed():
            return self._backward_graphed("B", mb, grad_outputs, True)
        ctx = self._ctx.pop(mb)
        dy = self._dy(grad_outputs)
        dx = self.model.backward(dy, ctx, self.mbs, self.S, weight_grads=True)
        return (dx,) if dx is not None else ()

    def backward_input_mb(self, mb, grad_outputs):
        if self._graphed():
            return self._backward_graphed("I", mb, grad_outputs, False)
        ctx = self._ctx.pop(mb)
        dy = self._dy(grad_outputs)
        dx = self.model.backward(dy, ctx, self.mbs, self.S, weight_grads=False)
        return (dx,) if dx is not None else ()

    def backward_weight_mb(self, mb):
        if self._graphed():
            self.graphs.run(("W", mb), (), lambda ins: self.model.backward_weight(mb), pool=self._pool(mb))
            self._release_stash(mb, "W")
            return
        self.model.backward_weight(mb)

    # ------------------------------------------------------------------ HIP graphs
    def _forward_graphed(self, mb, args, target, loss_scale, want_logits=False):
        last_loss = self.is_last and not self.split_head and target is not None
        ins = (args[0],) + ((target,) if last_loss else ())

        def fn(ins):
            ctx = MBContext(mb, _seed(self.seed, 0, mb))
            if want_logits:
                ctx.misc["logits_dst"] = self._logits_dst(mb)
            out = self.model.forward(ins[0], ctx, self.mbs, self.S, target=ins[1] if last_loss else None,
                                     loss_scale=loss_scale, keep_logits=want_logits)
            self._gctx[mb] = ctx
            if want_logits:
                # the logits copy is a graph output: persistent, refreshed by every replay
                return out, self._logits_view(ctx.misc.pop("logits_out"))
            return out

        # the logits-returning forward (compat step(return_outputs=True)) is its own graph
        key = ("FL", mb) if want_logits else ("F", mb)
        out = self.graphs.run(key, ins, fn, keep=lambda: self._gctx[mb], pool=self._pool(mb))
        if want_logits:
            loss, logits = out
            return (logits,), loss
        if self.is_last and not self.split_head:
            if not last_loss:
                return (out,), None
            # the runtime copies it into a persistent loss slot (runtime._loss_slot)
            return (out.detach(),), out
        return (out,), None

    def _backward_graphed(self, op, mb, grad_outputs, weight_grads):
        dy = self._dy(grad_outputs)
        ins = (dy,) if dy is not None else ()

        def fn(ins):
            return self.model.backward(ins[0] if ins else None, self._gctx[mb], self.mbs, self.S,
                                       weight_grads=weight_grads)

        dx = self.graphs.run((op, mb), ins, fn, keep=lambda: self.model.defer_w.get(mb), pool=self._pool(mb))
        self._release_stash(mb, op)
        return (dx,) if dx is not None else ()

    def infer_output_specs(self, args):
        return self.output_specs

    # REDUCE_GRAD issues through parallel/collectives.py, which records its own native
    # COLL instruction (or CALL) on a recording step's tape
    records_own_collectives = True
    coll = None     # set by the trainer (engine.PipelineTrainer)

    def reduce_grad(self, n_microbatches, scaled_in_loss):
        if not scaled_in_loss:
            self.arena.grad.div_(n_microbatches)
        if self.dp_group is not None and dist.get_world_size(self.dp_group) > 1:
            # SUM: the 1/dp average is folded into the AdamW kernel (engine.FlatAdamW).  One
            # call over the flat arena: RCCL pipelines a large all-reduce internally
            if self.coll is not None:
                if self.arena.shard is not None and self.arena.shard_scope == "dp":
                    # ZeRO-1 over DP (engine.py): reduce-scatter -- this replica's block of
                    # the arena is summed; the optimizer updates it and all-gathers weights
                    if getattr(self.coll, "dp_reduce_dtype", torch.float32) == torch.bfloat16:
                        return self.coll.reduce_scatter(self._grad_bf16(), "dp")[0]
                    return self.coll.reduce_scatter(self.arena.grad, "dp")[0]
                return self.coll.all_reduce(self.arena.grad, "dp")
            return allreduce_flat(self.arena.grad, self.dp_group, average=False)
        return None

    def _grad_bf16(self) -> torch.Tensor:
        """MIPIPE_DP_REDUCE_DTYPE=bf16: the summed f32 gradient rounded into a bf16 staging
        buffer (half the bytes over the DP link); the optimizer widens this replica's reduced
        block back into the f32 gradient (engine.FlatAdamW).  The cast is captured as a graph
        of its own on graphed stages, so a recorded step replays it natively."""
        a = self.arena
        if getattr(a, "grad16", None) is None:
            a.grad16 = torch.empty(a.numel, dtype=torch.bfloat16, device=a.device)

        def cast(ins=()):
            ops.cast_f32_bf16(a.grad, a.grad16)
            return a.grad16
        if self._graphed():
            self.graphs.run(("C16", 0), (), cast)
        else:
            cast()
        return a.grad16

    def has_grad_reduction(self, scaled_in_loss):
        return (not scaled_in_loss) or (self.dp_group is not None and dist.get_world_size(self.dp_group) > 1)

    def post_step(self):
        if self.embed_group is not None and self.cfg.tie_embeddings and self.arena.has("tok_embeddings.weight"):
            g = self.arena.g("tok_embeddings.weight")
            if self.coll is not None:
                # parallel/collectives.py "embed" scope: the native 2-rank engine on GPUs (a
                # stream-ordered RCCL all-reduce, no host block), torch.distributed elsewhere
                self.coll.all_reduce(g, "embed").wait()
            else:
                dist.all_reduce(g, group=self.embed_group)


def build_reference_stage(args, stage_index: int, num_stages: int, device, mbs: int = 8, seq_len: int = 128,
                          seed: int = 0, dtype=torch.float32, graphs: Optional[bool] = None) -> NativeStage:
    """Reference architecture (helper:23-55) on the HIP path with the reference split rule.
    ``dtype``: the reference's own f32 by default -- on GPUs every op then runs on the f32
    kernels (gemm_f32.hip, attention_f32.hip, the f32 norm / CE / embedding builds); bf16
    is the fast path.  ``graphs`` (default: on with a GPU): per-microbatch HIP graphs, so
    the schedule replays its steps from the native tape (parallel/native_runner.py),
    including the last rank's merged-logits ``step()``."""
    cfg = NativeConfig.reference(n_layers=args.n_layers, n_heads=args.n_heads, dim=args.dim,
                                 vocab_size=args.vocab_size, dropout=getattr(args, "dropout", 0.1),
                                 dim_feedforward=getattr(args, "dim_feedforward", 2048))
    from .native import balanced_layer_ranges
    rng = balanced_layer_ranges(cfg, num_stages, reference_rule=True)[stage_index]
    model = NativeModel(cfg, stage_index, num_stages, device, layer_range=rng, seed=seed, dtype=dtype)
    if graphs is None:
        graphs = torch.device(device).type == "cuda"
    return NativeStage(model, mbs, seq_len, graphs=graphs)
