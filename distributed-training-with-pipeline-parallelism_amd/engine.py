"""High-level training engine: native model + pipeline schedule + DP + fused optimizer.

    trainer = PipelineTrainer(NativeConfig.gpt2("small"), pp=4, schedule="1F1B",
                              n_microbatches=8, mbs=8, seq_len=1024)
    loss = trainer.train_step(tokens, targets)   # tokens on pp-rank 0, targets on the last

One process per GPU (``torchrun``), RCCL over xGMI between pipeline ranks and between
DP replicas.  A training step = the lowered pipeline program (fwd/bwd of all
microbatches, p2p, per-stage DP all-reduce at REDUCE_GRAD, the distributed head's
gradient reduce-scatter at REDUCE_HEAD -- all on the native RCCL engines,
parallel/collectives.py) + tied-embedding sync + global grad-norm clip + one fused AdamW
launch per stage arena (the head: on this rank's shard only, then an all-gather of the
bf16 weights -- ZeRO-1 for the replicated head).
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from . import ops
from .models.config import NativeConfig
from .models.native import (HeadShard, NativeModel, ParamArena, balanced_layer_ranges, comm_units,
                            stage_cost_model)
from .models.stage import NativeStage
from .parallel.collectives import Collectives
from .parallel.comm import P2P
from .parallel.headsplit import HeadPlan, head_token_split, plan_head_schedule
from .parallel.mesh import Mesh, build_mesh
from .parallel.runtime import PipelineRuntime
from .parallel.ir import Op
from .parallel.schedules import (REQUIRED_STYLE, SCHEDULES, WARMUP_EXTRA, canonical_name, generate, rank_stages,
                                 stage_to_rank)


class FlatAdamW:
    """AdamW over flat stage arenas (one fused kernel launch per arena).

    Global grad-norm clipping sums the per-arena squared norms on device and, with PP,
    across the pipeline group (a 4-byte all-reduce) -- no host synchronisation."""

    def __init__(self, arenas: List[ParamArena], lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8,
                 weight_decay: float = 0.1, max_grad_norm: float = 1.0, pp_group=None, norm_skip=(),
                 norm_exclude=None, grad_scale: float = 1.0, coll=None, merged_norm: bool = True,
                 merged_norm_skip=()):
        self.arenas = arenas
        # parallel/collectives.py: the clip-norm sum over the pipeline group and the
        # all-gather of ZeRO-sharded arenas' updated bf16 weights
        self.coll = coll
        # arenas replicated across the pipeline group (distributed head) count in the
        # global grad norm on one rank only
        self.norm_skip = set(norm_skip)
        # {arena index: [(offset, numel), ...]}: slices left out of the norm (a tied
        # embedding's second copy on the last stage holds the same summed gradient)
        self.norm_exclude = {i: sorted(r) for i, r in (norm_exclude or {}).items()}
        # gradients arrive DP-summed (the all-reduces skip a separate divide pass); the
        # 1/dp factor is applied inside the AdamW kernel (and to the clip norm)
        self.grad_scale = float(grad_scale)
        # the fused lane merge's sum of squares is the clipping norm only when nothing
        # reduces the gradient after the merge (no DP all-reduce in between)
        self.merged_norm = bool(merged_norm)
        # arenas whose gradient is reduced further after the merge even without DP (a
        # replicated head all-reduced over the pipeline, stage 0's tied-embedding copy
        # summed with the last stage's): their norm is taken from the reduced gradient
        self.merged_norm_skip = set(merged_norm_skip)
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.max_norm = max_grad_norm
        self.pp_group = pp_group
        self.step_count = 0
        # moments over what the optimizer updates (this rank's range of a sharded arena)
        self.m = [torch.zeros_like(a.opt_views()[0]) for a in arenas]
        self.v = [torch.zeros_like(a.opt_views()[0]) for a in arenas]
        dev = arenas[0].device if arenas else torch.device("cpu")
        self.sumsq = torch.zeros(1, device=dev, dtype=torch.float32)
        # partial sum of squares of the arenas ZeRO-sharded over DP replicas: each replica
        # holds a disjoint block, so it is summed over DP before joining the rest
        self.dp_sharded = any(a.shard is not None and a.shard_scope == "dp" for a in arenas)
        self.sumsq_dp = torch.zeros(1, device=dev, dtype=torch.float32)

    def step(self, lr: Optional[float] = None) -> None:
        self.step_count += 1
        lr = self.lr if lr is None else lr
        for a in self.arenas:
            g16 = getattr(a, "grad16", None)
            if g16 is not None and a.shard is not None and a.shard_scope == "dp":
                lo, hi, _ = a.shard        # bf16 DP reduce-scatter: widen this replica's block
                a.grad[lo:hi].copy_(g16[lo:hi])
        use_clip = self.max_norm and self.max_norm > 0
        if use_clip:
            self.sumsq.zero_()
            if self.dp_sharded:
                self.sumsq_dp.zero_()
            for i, a in enumerate(self.arenas):
                if i in self.norm_skip:
                    continue
                if a.shard is not None:     # this rank's (reduced) range of a sharded arena
                    ops.sumsq(a.opt_views()[1], self.sumsq_dp if a.shard_scope == "dp" else self.sumsq)
                    continue
                if (self.merged_norm and len(a.grad_lanes) > 1 and a.merged_sumsq is not None
                        and i not in self.norm_exclude and i not in self.merged_norm_skip):
                    self.sumsq.add_(a.merged_sumsq)     # computed by the fused lane merge
                    continue
                lo = 0
                for off, n in self.norm_exclude.get(i, ()):
                    if off > lo:
                        ops.sumsq(a.grad[lo:off], self.sumsq)
                    lo = max(lo, off + n)
                if lo < a.grad.numel():
                    ops.sumsq(a.grad[lo:] if lo else a.grad, self.sumsq)
            if self.dp_sharded:
                self.coll.all_reduce(self.sumsq_dp, "dp").wait()
                self.sumsq.add_(self.sumsq_dp)
            if self.coll is not None:
                self.coll.all_reduce(self.sumsq, "pp").wait()
            elif self.pp_group is not None and dist.get_world_size(self.pp_group) > 1:
                dist.all_reduce(self.sumsq, group=self.pp_group)
        for a, m, v in zip(self.arenas, self.m, self.v):
            master, g, w16, n_decay = a.opt_views()
            ops.adamw_(master, g, m, v, w16, n_decay, lr, self.betas[0], self.betas[1], self.eps, self.wd,
                       self.step_count, self.sumsq if use_clip else None, self.max_norm if use_clip else 0.0,
                       self.grad_scale, zero_grad=True)
            if a.shard is not None:
                lo, hi, _ = a.shard
                a.grad[:lo].zero_()
                a.grad[hi:].zero_()
                self.coll.all_gather(a.w16, a.shard_scope).wait()
            a.refresh_transposes()

    def state_dict(self):
        return {"step": self.step_count, "m": [t.clone() for t in self.m], "v": [t.clone() for t in self.v]}

    def load_state_dict(self, sd):
        self.step_count = sd["step"]
        for dst, src in zip(self.m, sd["m"]):
            dst.copy_(src)
        for dst, src in zip(self.v, sd["v"]):
            dst.copy_(src)


def max_inflight_microbatches(order, stages) -> int:
    """Largest number of microbatches a rank holds forward activations for at once
    (forwards done, backwards not yet) over its stages, from its compute order."""
    live, peak = 0, 0
    for a in order:
        if a is None or a.stage not in stages:
            continue
        if a.op == Op.F:
            live += 1
        elif a.op in (Op.B, Op.I):
            live -= 1
        peak = max(peak, live)
    return max(peak, 1)


def plan_recompute(cfg: NativeConfig, layer_ranges, my_stages, order, mbs: int, seq_len: int, device,
                   head_tokens: int = 0, budget_frac: float = 0.85, head_shards: int = 1,
                   stage_shards: int = 1, dtype=torch.bfloat16, graphs: bool = False, lanes: int = 1,
                   hbm: Optional[float] = None, head_split: Optional[bool] = None) -> dict:
    """HBM plan of one pipeline rank and the recompute decision of ``recompute="auto"``:
    recompute only if the activation stash would not fit ``budget_frac`` of the device.

    bytes = parameters x 20 (bf16 weights + bf16 W^T copies + f32 master, grad, Adam m, v)
            + an f32 gradient per extra microbatch lane
          + per stash slot: local layers x per-layer stash (config.stash_bytes_per_layer),
            + the deferred weight-gradient inputs with a split backward (ZBH1 / ZBV:
            config.wgrad_stash_bytes_per_layer, held from I to W)
          + the last stage's logits per stash slot (kept from F to B, the gradient written
            in place; one token chunk with MIPIPE_HEAD_CHUNK > 0)
          + a distributed head's chunk logits: a transient of each captured head graph, so
            one per microbatch with HIP graphs (each keeps a private pool), one eager
          + backward temporaries: ~1.3 layer stashes per memory pool that holds them -- each
            stash slot's graph pool with HIP graphs (a pool keeps its freed blocks reserved),
            one set eager -- + 0.5 GB of workspace.
    Reconciled with the RESERVED peak of the caching allocator (what the device actually
    holds) on one MI355X (profiles/r6_hbm_reserved.md, tests/test_native_runner_gpu.py).
    The distributed head with ZeRO-1 (``head_shards`` = PP) keeps its f32 master and Adam
    moments (12 of the 20 bytes) for 1 / head_shards of the matrix: ``head_optimizer_bytes``
    is that per-rank optimizer state, ``head_state_bytes`` all of the head's.  ZeRO-1 over DP
    (``stage_shards`` = DP) does the same for the stage parameters: 8 + 12 / dp bytes each.
    f32 arenas (the reference's precision): the f32 weights ARE the master, so sharding
    leaves them whole and splits only the Adam moments -- 12 + 8 / shards bytes per
    parameter (head: 12 + 8 / head_shards).
    The stash is counted per stage from the slot plan of the rank's order
    (parallel/stash.py): the in-flight microbatches of each stage -- also with HIP graphs,
    whose captures share one pool per stash slot (``lanes``: slots are per microbatch lane;
    MIPIPE_STASH_RING=0 restores one private pool per graph, i.e. all m stashes).
    ``hbm``: the device's bytes (default: the device's own; unbounded off the GPU).
    ``head_split``: whether ``head_tokens`` is a distributed head's chunk (default: inferred)."""
    T = mbs * seq_len
    from .parallel.stash import stash_slots_per_stage
    layers_of = {s: layer_ranges[s][1] - layer_ranges[s][0] for s in my_stages}
    nlayers = sum(layers_of.values())
    emb = cfg.vocab_padded * cfg.d_model
    nparams = cfg.layer_params() * nlayers + (emb if 0 in my_stages else 0)
    f32 = dtype == torch.float32
    fixed_b, shard_b = (12.0, 8.0) if f32 else (8.0, 12.0)
    head_opt = shard_b * emb / max(1, head_shards) if head_tokens else 0.0
    head_state = (fixed_b * emb if head_tokens else 0.0) + head_opt
    slots = stash_slots_per_stage(order, my_stages, lanes if graphs else 1)
    n_mb = len({a.mb for a in order if a is not None and a.stage in set(my_stages) and a.op == Op.F})
    if graphs and os.environ.get("MIPIPE_STASH_RING", "1") == "0":
        slots = {s: n_mb for s in my_stages}
    split = any(a is not None and a.op == Op.I and a.stage in set(my_stages) for a in order)
    stash_layers = sum(slots.get(s, 1) * layers_of[s] for s in my_stages)   # stash-layer units
    inflight = max(slots.values(), default=1)
    from .models.native import _HEAD_CHUNK
    last = len(layer_ranges) - 1
    logit_b = 4.0 if f32 else 2.0
    act_b = 2.0 if f32 else 1.0       # stash formulas count bf16 bytes
    per_layer = act_b * cfg.stash_bytes_per_layer(T, recompute=False)
    per_layer_rc = act_b * cfg.stash_bytes_per_layer(T, recompute=True)
    wgrad = act_b * cfg.wgrad_stash_bytes_per_layer(T) if split else 0.0
    logits = 0.0
    if head_split is None:       # a distributed head's chunk is not the whole microbatch
        head_split = bool(head_tokens) and (head_tokens != T or last not in my_stages)
    if last in my_stages and not head_split:
        rows = min(T, _HEAD_CHUNK) if _HEAD_CHUNK > 0 else T
        logits = logit_b * rows * cfg.vocab_padded * slots.get(last, 1)
    elif head_tokens:
        rows = min(head_tokens, _HEAD_CHUNK) if _HEAD_CHUNK > 0 else head_tokens
        logits = logit_b * rows * cfg.vocab_padded * (max(1, n_mb) if graphs else 1)
    pools = sum(slots.get(s, 1) for s in my_stages) if graphs else 1
    temps = 1.3 * per_layer * pools + 0.5e9
    fixed = (fixed_b + shard_b / max(1, stage_shards)) * nparams + head_state + \
        4.0 * nparams * (max(1, lanes) - 1 if graphs else 0) + logits + temps
    full = fixed + stash_layers * (per_layer + wgrad)
    rec = fixed + stash_layers * (per_layer_rc + wgrad) + per_layer

    def selective(k: int) -> float:
        """bytes with the first ``k`` local layers of every stage recomputed (their stash is
        the layer input; one layer's full stash is rebuilt at a time in the backward)."""
        if k <= 0:
            return full
        kept = sum(slots.get(s_, 1) * max(0, layers_of[s_] - k) for s_ in my_stages)
        rc = sum(slots.get(s_, 1) * min(k, layers_of[s_]) for s_ in my_stages)
        return fixed + kept * (per_layer + wgrad) + rc * (per_layer_rc + wgrad) + per_layer
    # selective recompute: the fewest recomputed layers per stage whose plan
    # fits the budget -- 0 if the whole stash fits, every layer if nothing less does
    max_layers = max(layers_of.values(), default=0)
    total_ = float(hbm) if hbm is not None else (torch.cuda.get_device_properties(device).total_memory
                                                 if device.type == "cuda" else float("inf"))
    k_fit = next((k for k in range(max_layers + 1) if selective(k) <= budget_frac * total_), max_layers)
    if hbm is not None:
        total = float(hbm)
    else:
        total = torch.cuda.get_device_properties(device).total_memory if device.type == "cuda" else float("inf")
    return dict(inflight=inflight, stash_slots=slots, layers=nlayers, bytes_no_recompute=full, bytes_recompute=rec,
                hbm=total,
                recompute=bool(full > budget_frac * total), head_state_bytes=head_state,
                head_optimizer_bytes=head_opt, recompute_layers=k_fit, bytes_selective=selective(k_fit),
                max_stage_layers=max_layers, selective_fn=selective)


# HBM the planners assume off the GPU (CPU tests, the supervisor's plan child): one MI355X
MI355X_HBM_BYTES = 288 * 2 ** 30


def plan_rank_memory(cfg: NativeConfig, pp: int, v: int, style: str, layer_ranges, chunks, orders, mbs: int,
                     seq_len: int, dtype=torch.bfloat16, graphs: bool = True, lanes: int = 2, head_zero: bool = True,
                     dp: int = 1, dp_zero: bool = False, hbm: Optional[float] = None) -> Dict[int, dict]:
    """:func:`plan_recompute` of every pipeline rank for one set of compute orders, without a
    device (``hbm``: default one MI355X) -- what a schedule's warmup depth (its head lag)
    costs in stash slots and bytes on each rank.  ``chunks``: the distributed head's token
    chunk per rank (None: the head on the last stage)."""
    out = {}
    S = pp * v
    for r in range(pp):
        my = rank_stages(r, pp, v, style)
        ht = chunks[r] if chunks is not None else (mbs * seq_len if (S - 1) in my else 0)
        out[r] = plan_recompute(cfg, layer_ranges, my, orders.get(r, []), mbs, seq_len, torch.device("cpu"),
                                head_tokens=ht,
                                head_shards=pp if (head_zero and pp > 1 and chunks is not None) else 1,
                                stage_shards=dp if dp_zero else 1, dtype=dtype, graphs=graphs, lanes=lanes,
                                hbm=MI355X_HBM_BYTES if hbm is None else hbm, head_split=chunks is not None)
    return out


def resolve_v(cfg: NativeConfig, schedule: str, pp: int, v: Optional[int], seq_len: int,
              head_on_last: bool = False) -> int:
    """Virtual stages per rank.  Given explicitly: that (1 for single-chunk schedules).
    Defaulted: the schedule's default only if the cost-balanced split over ``pp * v``
    stages leaves no stage empty -- otherwise 1, the reference's own fallback when the
    layers do not divide over 2P chunks (helper:181-183; VERDICT r4: GPT-2 small at P = 8
    would otherwise build 16 virtual stages for 12 layers)."""
    schedule = canonical_name(schedule)
    if not SCHEDULES[schedule][2]:
        return 1
    if v is not None:
        return int(v)
    v = SCHEDULES[schedule][1]
    if v > 1 and pp > 1:
        rng = balanced_layer_ranges(cfg, pp * v, seq_len, head_on_last=head_on_last, ranks=pp)
        if cfg.n_layers < pp * v or any(r1 <= r0 for r0, r1 in rng):
            return 1
    return v


def plan_head_pipeline(cfg: NativeConfig, pp: int, schedule: str, m: int, mbs: int, seq_len: int,
                       v: Optional[int] = None, style: str = "loop", layer_ranges=None,
                       head_align: Optional[int] = None, max_lag: Optional[int] = None,
                       mem_bound: Optional[dict] = None) -> dict:
    """The distributed-head pipeline plan of one schedule (what PipelineTrainer runs at
    PP > 1): layer split, per-stage costs (stage_cost_model units), water-filled head token
    chunks, and the head-aware compute orders with their simulated makespan
    (headsplit.plan_head_schedule).  ``ideal`` is the no-bubble time in the same units, so
    ideal / makespan is the planned pipeline efficiency.

    ``max_lag``: cap on the head lag, the extra warmup forwards every rank runs (0: the
    schedule's own warmup, e.g. torch 1F1B's P - s).  ``mem_bound``: keyword arguments of
    :func:`plan_rank_memory` plus ``budget_frac`` (default 0.85) and ``recompute``: a lag
    whose HBM plan exceeds ``budget_frac`` of the device on any rank is not a candidate
    (a deep lag turns 1F1B's and ZBH1's stash into GPipe's).  ``memory`` in
    the result: the chosen orders' per-rank plan (with a bound)."""
    schedule = canonical_name(schedule)
    style = REQUIRED_STYLE.get(schedule, style)
    v = resolve_v(cfg, schedule, pp, v, seq_len) if layer_ranges is None else \
        (v if v is not None and SCHEDULES[schedule][2] else (len(layer_ranges) // pp))
    S = pp * v
    if layer_ranges is None:
        layer_ranges = balanced_layer_ranges(cfg, S, seq_len, head_on_last=False, ranks=pp)
    lc, head_units, ec = stage_cost_model(cfg, seq_len)
    stage_costs = [(r1 - r0) * lc + (ec if s == 0 else 0.0) + (0.1 if s == S - 1 else 0.0)
                   for s, (r0, r1) in enumerate(layer_ranges)]
    rank_load = [sum(stage_costs[s] for s in range(S) if stage_to_rank(s, pp, style) == r) for r in range(pp)]
    T = mbs * seq_len
    align = head_align or next(a for a in (256, 128, 64, 32, 16, 8, 1) if T % a == 0)
    chunks = head_token_split(T, rank_load, head_units, align=align)
    head_costs = {r: 3.0 * head_units * chunks[r] / T for r in range(pp) if chunks[r] > 0}
    base = generate(schedule, pp, m, v, style)
    regen = ((lambda lag: generate(schedule, pp, m, v, style, warmup_extra=lag)) if schedule in WARMUP_EXTRA
             else None)
    comm = comm_units(cfg, seq_len, tokens=T)
    fits = None
    mb_kw = {}
    if mem_bound is not None:
        mb_kw = {k: x for k, x in mem_bound.items() if k not in ("budget_frac", "recompute")}
        frac = float(mem_bound.get("budget_frac", 0.85))
        key = "bytes_recompute" if mem_bound.get("recompute") is True else "bytes_no_recompute"

        def fits(o):
            plans = plan_rank_memory(cfg, pp, v, style, layer_ranges, chunks, o, mbs, seq_len, **mb_kw)
            return all(p[key] <= frac * p["hbm"] for p in plans.values())
    orders, lag, makespan = plan_head_schedule(base, pp, v, style, head_costs, stage_costs, regen=regen, comm=comm,
                                               max_lag=max_lag, fits=fits)
    memory = None
    if mem_bound is not None:
        memory = plan_rank_memory(cfg, pp, v, style, layer_ranges, chunks, orders, mbs, seq_len, **mb_kw)
    # no-bubble time in the same units (F = 1, B = 2 per stage-cost unit)
    ideal = (3.0 * sum(stage_costs) + sum(head_costs.values())) * m / pp
    return dict(schedule=schedule, v=v, style=style, layer_ranges=layer_ranges, stage_costs=stage_costs, comm=comm,
                chunks=chunks, head_costs=head_costs, orders=orders, lag=lag, makespan=makespan, ideal=ideal,
                efficiency=ideal / makespan if makespan > 0 else 0.0, memory=memory)


def pick_schedule(cfg: NativeConfig, pp: int, m: int, mbs: int, seq_len: int,
                  candidates=("GPipe", "1F1B", "Interleaved1F1B", "ZBH1"),
                  margin: float = 0.03, v: Optional[int] = None, style: str = "loop", layer_ranges=None,
                  head_align: Optional[int] = None, same_traffic_margin: float = 0.01,
                  mem_bound: Optional[dict] = None, details: Optional[dict] = None) -> Tuple[str, Dict[str, float]]:
    """``schedule="auto"``: 1F1B unless another candidate's head-aware plan is more
    efficient by more than ``margin`` (relative) -- the plan's p2p model is an estimate, and
    an interleaved rank sends twice the activations (1F1B at PP = 1, where every schedule is
    bubble-free and 1F1B keeps one stage per rank).  ZBH1 (zero-bubble: the input-gradient
    and weight-gradient halves of each backward scheduled apart) is a candidate: its I / W
    split costs nothing per GPU (one GPU, 128 sequences: 969K vs 959K tok/s at 4 x 32,
    931K vs 925K at 8 x 16, profiles/r4_zbh1_vs_1f1b_1gpu.json) and it fills the bubble
    with W work -- GPT-2 small plans 0.959 vs 0.904 at P = 2.  Returns (name, {name: planned
    efficiency}).  ``v`` / ``style`` / ``layer_ranges`` / ``head_align``: the caller's own
    configuration -- a candidate it cannot run as given (a layer split sized for
    another stage count) is skipped.  ``margin`` guards the p2p estimate, so it applies in
    full only to a candidate that sends MORE than 1F1B (interleaved with v > 1). GPipe,
    ZBH1 and v = 1 interleaved send exactly 1F1B's messages and need only
    ``same_traffic_margin``.  GPT-2 small at P = 8, 16-sequence microbatches: ZBH1 plans
    0.906 vs 0.8825, which a 3 % margin would throw away.

    Every candidate is planned under ``mem_bound`` (plan_head_pipeline; default: bf16 with HIP
    graphs and 2 lanes on one MI355X): its head lag is the smallest within the lag tolerance
    of its best plan AND whose stash fits the HBM budget on every rank.
    ``details`` (a dict, filled): per candidate its planned efficiency, v, the head lag it
    assumed, the largest per-rank stash slot count and planned GB."""
    if pp == 1:
        return "1F1B", {}
    eff = {}
    vs: Dict[str, int] = {}
    mem_bound = {} if mem_bound is None else mem_bound
    for c in candidates:
        try:
            cv = v if SCHEDULES[canonical_name(c)][2] else 1
            rng = layer_ranges
            if rng is not None and len(rng) != pp * (cv if cv is not None else SCHEDULES[canonical_name(c)][1]):
                continue
            plan = plan_head_pipeline(cfg, pp, c, m, mbs, seq_len, v=cv, style=style, layer_ranges=rng,
                                      head_align=head_align, mem_bound=mem_bound)
            eff[c], vs[c] = plan["efficiency"], int(plan["v"])
            if details is not None:
                mem = plan["memory"] or {}
                details[c] = {"efficiency": round(plan["efficiency"], 4), "v": int(plan["v"]), "head_lag": plan["lag"],
                              "stash_slots_max": max((sum(p["stash_slots"].values()) for p in mem.values()), default=None),
                              "planned_gb_max": round(max((p["bytes_no_recompute"] for p in mem.values()), default=0.0)
                                                      / 1e9, 1)}
        except (ValueError, RuntimeError, KeyError):
            continue
    if "1F1B" not in eff:
        return max(eff, key=lambda k: eff[k]), eff
    # each candidate must beat 1F1B by its own margin; among those that do, the best plan
    ok = [c for c in eff if c != "1F1B" and
          eff[c] >= eff["1F1B"] * (1.0 + (margin if vs.get(c, 1) > 1 else same_traffic_margin))]
    best = max(ok, key=lambda k: eff[k]) if ok else "1F1B"
    return best, eff


# Per-GPU training throughput vs tokens per microbatch (GEMM M), relative to 32K tokens:
# GPT-2 small, 128 x 1024 tokens per step, 2 microbatch lanes, one MI355X
# (profiles/r4_bench_1gpu_mbs_sweep.json: 973K / 947K / 907K / 750K tok/s at 64K / 32K /
# 16K / 8K tokens).  Smaller microbatches shrink the pipeline bubble but run each kernel
# on fewer rows.
MICROBATCH_RATE = ((65536, 1.027), (32768, 1.0), (16384, 0.958), (8192, 0.79))


def microbatch_rate(tokens: int) -> float:
    """MICROBATCH_RATE interpolated in log2(tokens), clamped at the ends."""
    import math
    pts = sorted(MICROBATCH_RATE)
    if tokens <= pts[0][0]:
        return pts[0][1]
    if tokens >= pts[-1][0]:
        return pts[-1][1]
    for (t0, r0), (t1, r1) in zip(pts, pts[1:]):
        if t0 <= tokens <= t1:
            f = (math.log2(tokens) - math.log2(t0)) / (math.log2(t1) - math.log2(t0))
            return r0 + f * (r1 - r0)
    return 1.0


def rate_probe_config(cfg: NativeConfig, pp: int) -> NativeConfig:
    """The per-rank work of a ``pp``-stage pipeline of ``cfg`` as a one-GPU model: L / pp of
    its layers (same shapes) and a vocabulary of V / pp (the distributed head spreads the
    head's token chunks evenly over the ranks, parallel/headsplit.py) -- what bench.py's
    microbatch-rate probe times at each candidate microbatch size (``rates`` of
    :func:`pick_microbatch`)."""
    import dataclasses
    v = max(128, (cfg.vocab_size // max(1, pp) + 127) // 128 * 128)
    return dataclasses.replace(cfg, n_layers=max(1, cfg.n_layers // max(1, pp)), vocab_size=v, vocab_padded=0)


def pick_microbatch(cfg: NativeConfig, pp: int, seq_len: int, seqs_per_replica: int,
                    candidates=(32, 16), margin: float = 0.02,
                    rates: Optional[Dict[int, float]] = None) -> Tuple[int, int, Dict[int, dict]]:
    """``--mbs auto`` at PP > 1 with a fixed batch per pipeline replica (weak scaling): for
    each candidate microbatch size the schedule ``pick_schedule`` would run and its planned
    efficiency (bubble + distributed head + p2p), times the per-GPU kernel rate at that
    microbatch size.  ``rates`` ({mbs: tokens/s}): measured for THIS model's per-rank shapes
    (bench.py's rate probe, :func:`rate_probe_config`); without it the
    GPT-2-small table ``microbatch_rate``.  The first candidate (the larger microbatch) is
    kept unless another scores more than ``margin`` better.  Returns (mbs, microbatches,
    {mbs: detail})."""
    scores = {}
    base = None
    if rates:
        rates = {int(k): float(v) for k, v in rates.items() if v}
        base = next((rates[c] for c in candidates if c in rates), None)
    for mbs in candidates:
        if seqs_per_replica % mbs:
            continue
        m = seqs_per_replica // mbs
        sched, eff = pick_schedule(cfg, pp, m, mbs, seq_len)
        e = eff.get(sched, 1.0 if pp == 1 else 0.0)
        if base and mbs in rates:
            rate, src = rates[mbs] / base, "measured"
        else:
            rate, src = microbatch_rate(mbs * seq_len), "gpt2-small table"
        scores[mbs] = {"microbatches": m, "schedule": sched, "planned_efficiency": round(e, 4),
                       "kernel_rate": round(rate, 4), "rate_source": src, "score": round(e * rate, 4)}
    if not scores:
        raise ValueError(f"no candidate microbatch size divides {seqs_per_replica} sequences")
    first = next(iter(scores))
    best = max(scores, key=lambda k: scores[k]["score"])
    if scores[best]["score"] < scores[first]["score"] * (1.0 + margin):
        best = first
    return best, scores[best]["microbatches"], scores


def auto_lanes(cfg: NativeConfig, pp: int, v: int, graphs: bool, device, m: int, tokens: int, params: int,
               layers: int, recompute: bool = False) -> int:
    """Microbatch lanes (PipelineRuntime.set_lanes) at PP = 1 with HIP graphs: up to 4 for
    <= 4096-token microbatches, 2 above, if the extra per lane (an f32 gradient buffer + one
    more microbatch's activation stash in flight) stays within 20 % of HBM.  Measured on one
    MI355X (profiles/r2_lanes_ab.txt): reference model L8H8 (1024-token microbatches,
    m = 4) 311K tok/s with 1 lane, 495K with 2, 456K with 3 (a lane on the compute
    stream's hardware queue: fixed by the queue probe, parallel/runtime.py), 594K with 4;
    GPT-2 small (16K-token microbatches, m = 2) 850K -> 888K with 2."""
    device = torch.device(device)
    if not (graphs and device.type == "cuda" and m >= 2):
        return 1
    if pp > 1 and os.environ.get("MIPIPE_PP_LANES", "1") == "0":
        return 1
    lanes = min(m, 4 if tokens <= 4096 else 2)
    if pp > 1:
        lanes = min(lanes, 2)   # a pipeline rank has at most F(i+w) and B(i) ready at once
    per_lane = 4.0 * params + layers * cfg.stash_bytes_per_layer(tokens, recompute=recompute)
    hbm = torch.cuda.get_device_properties(device).total_memory
    while lanes > 1 and (lanes - 1) * per_lane > 0.2 * hbm:
        lanes -= 1
    return lanes


class PipelineTrainer:
    def __init__(self, cfg: NativeConfig, pp: int = 1, dp: int = 1, schedule: str = "1F1B",
                 n_microbatches: int = 8, mbs: int = 8, seq_len: int = 1024, v: Optional[int] = None,
                 device=None, lr: float = 3e-4, weight_decay: float = 0.1, max_grad_norm: float = 1.0,
                 recompute: bool = False, profile: bool = False, seed: int = 0, style: str = "loop",
                 mesh: Optional[Mesh] = None, layer_ranges=None, dtype=torch.bfloat16,
                 split_head: Optional[bool] = None, head_align: Optional[int] = None, graphs: bool = False,
                 adam_eps: float = 1e-8, head_max_lag: Optional[int] = None):
        """``head_max_lag``: cap on the distributed head's lag (extra warmup forwards; 0 = the
        schedule's own depth, e.g. 1F1B's P - s).  Whatever the cap, the lag is bounded by
        the HBM plan (``self.mem_bound``)."""
        self.cfg = cfg
        # schedule="auto": the best head-aware plan (pick_schedule; 1F1B at PP = 1)
        self.schedule_choice = None
        if str(schedule).lower() == "auto":
            if split_head is not None and not split_head:
                # the plans are head-aware (distributed head); without it: 1F1B
                schedule, self.schedule_choice = "1F1B", {}
            else:
                schedule, self.schedule_choice = pick_schedule(cfg, pp, n_microbatches, mbs, seq_len, v=v,
                                                               style=style, layer_ranges=layer_ranges,
                                                               head_align=head_align)
        self.schedule = canonical_name(schedule)
        style = REQUIRED_STYLE.get(self.schedule, style)
        self.style = style
        if layer_ranges is not None and v is None and SCHEDULES[self.schedule][2]:
            v = len(layer_ranges) // pp
        v = resolve_v(cfg, self.schedule, pp, v, seq_len,
                      head_on_last=not (pp > 1 if split_head is None else (bool(split_head) and pp > 1)))
        self.v = v
        self.m, self.mbs, self.S = n_microbatches, mbs, seq_len
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else \
                torch.device("cpu")
        self.device = torch.device(device)
        self.mesh = mesh if mesh is not None else build_mesh(pp, dp, self.device)
        num_stages = pp * v
        # distributed LM head (parallel/headsplit.py): default on whenever there is a pipeline
        self.split_head = pp > 1 if split_head is None else (bool(split_head) and pp > 1)
        if layer_ranges is None:
            layer_ranges = balanced_layer_ranges(cfg, num_stages, seq_len, head_on_last=not self.split_head,
                                                  ranks=pp if style == "loop" else None)
        self.layer_ranges = layer_ranges
        my_stages = rank_stages(self.mesh.pp_rank, pp, v, style)
        tied_pp = cfg.tie_embeddings and num_stages > 1 and not self.split_head
        # V placement puts the first and the last stage on rank 0: tie them locally
        self._tie_local = tied_pp and 0 in my_stages and (num_stages - 1) in my_stages
        if self._tie_local:
            tied_pp = False
        self.head: Optional[HeadShard] = None
        orders = head_plan = head_costs = stage_costs = None
        self.head_chunks = None
        self.head_lag = None
        # ZeRO-1 for the replicated head: master / Adam moments sharded over the pipeline
        # group (MIPIPE_HEAD_ZERO=0: fully replicated, gradient all-reduced)
        self.head_zero = self.split_head and os.environ.get("MIPIPE_HEAD_ZERO", "1") != "0"
        # ZeRO-1 over DP replicas (see below): known before the HBM plan
        self.dp_zero = (self.mesh.dp > 1 and os.environ.get("MIPIPE_DP_ZERO", "1") != "0"
                        and not (tied_pp or self._tie_local))
        graphed = bool(graphs) and self.device.type == "cuda"
        # microbatch lanes (PipelineRuntime.set_lanes), decided BEFORE the HBM plan: slots of
        # the stash ring are per lane (the plan used to assume 2).  MIPIPE_LANES=
        # auto|1 (off)|n.  Not with plain GEMMs on hipBLASLt (MIPIPE_GEMM=blas|auto): its
        # stream-K kernels synchronise their workgroups and assume all of them resident; a
        # second lane's kernels holding CUs left a Llama-3 1B step hung in that mode
        # (profiles/r3_model_families_1gpu.txt)
        from .ops.kernels import GEMM_BACKEND
        my_layers = sum(layer_ranges[st][1] - layer_ranges[st][0] for st in my_stages)
        params_est = (cfg.layer_params() * my_layers + (cfg.vocab_padded * cfg.d_model if 0 in my_stages else 0)
                      + (cfg.vocab_padded * cfg.d_model if self.split_head else 0))
        if os.environ.get("MIPIPE_LANES", "auto") == "auto":
            self.planned_lanes = auto_lanes(cfg, pp, v, graphs, self.device, n_microbatches, mbs * seq_len,
                                            params_est, my_layers, recompute is True)
        else:
            self.planned_lanes = max(1, int(os.environ["MIPIPE_LANES"]))
        if GEMM_BACKEND != "hip":
            self.planned_lanes = 1
        hbm = torch.cuda.get_device_properties(self.device).total_memory if self.device.type == "cuda" \
            else MI355X_HBM_BYTES
        # the head lag's memory bound (plan_head_pipeline): every rank's stash within 85 % of HBM
        self.mem_bound = dict(dtype=dtype, graphs=graphed, lanes=self.planned_lanes if graphed else 1,
                              head_zero=self.head_zero, dp=self.mesh.dp, dp_zero=self.dp_zero, hbm=hbm,
                              budget_frac=0.85, recompute=recompute)
        if self.split_head:
            self.head = HeadShard(cfg, self.device, seed=seed, dtype=dtype, shards=pp if self.head_zero else 1)
            plan = plan_head_pipeline(cfg, pp, self.schedule, n_microbatches, mbs, seq_len, v, style, layer_ranges,
                                      head_align, max_lag=head_max_lag, mem_bound=self.mem_bound)
            orders, self.head_lag, self.planned_makespan = plan["orders"], plan["lag"], plan["makespan"]
            stage_costs, head_costs, chunks = plan["stage_costs"], plan["head_costs"], plan["chunks"]
            self.planned_ideal = plan["ideal"]
            head_plan = HeadPlan(chunks, cfg.d_model, runner=self.head.run, dtype=dtype)
            head_plan.arena = self.head.arena   # per-lane head gradients (PipelineRuntime.set_lanes)
            if graphs and self.device.type == "cuda":
                from .parallel.graphs import GraphCache
                head_plan.graphs = GraphCache(f"{self.mesh.pp_rank}")
            self.head_chunks = chunks
        # recompute="auto": HBM plan from the schedule's in-flight microbatches (288 GB per
        # MI355X usually holds the whole stash, and recompute costs a forward per layer).
        # The plan is made (and reported: bench.py's config.memory_plan) whatever the
        # setting; recompute="auto" acts on it
        self._order = (orders if orders is not None else
                       generate(self.schedule, pp, n_microbatches, v, style)).get(self.mesh.pp_rank, [])
        self._my_stages = my_stages
        self.memory_plan = self._plan_memory(self.planned_lanes if graphed else 1)
        self.recompute_requested = recompute
        max_layers = self.memory_plan["max_stage_layers"]
        if recompute == "auto":
            # selective: the fewest recomputed layers per stage that fit the HBM budget
            k = self.memory_plan["recompute_layers"]
        elif recompute is True:
            k = max_layers
        elif recompute is False or recompute is None:
            k = 0
        else:
            k = max(0, min(int(recompute), max_layers))
        self.recompute_layers = k
        recompute = k > 0
        self.recompute = bool(recompute)
        # ZeRO-1 over DP replicas (MIPIPE_DP_ZERO=0: replicated master / moments, gradient
        # all-reduced): each replica owns 1/dp of every stage arena -- its f32 master and Adam
        # moments; REDUCE_GRAD reduce-scatters the gradient into that block and the step
        # all-gathers the updated weights.  Not with a tied embedding copied across stages
        # (its two copies' gradients are summed after the DP reduction).  self.dp_zero: above.
        self.stages: List[NativeStage] = []
        for s in my_stages:
            model = NativeModel(cfg, s, num_stages, self.device, layer_range=layer_ranges[s], seed=seed,
                                recompute=self.recompute_layers, mbs=mbs, seq_len=seq_len, dtype=dtype, head=self.head,
                                arena_multiple=8 * self.mesh.dp if self.dp_zero else 8)
            egroup = self.mesh.embed_group if (tied_pp and (s == 0 or s == num_stages - 1)) else None
            self.stages.append(NativeStage(model, mbs, seq_len, dp_group=self.mesh.dp_group, embed_group=egroup,
                                           seed=seed + 1000 * self.mesh.dp_rank, graphs=graphs))
        p2p = P2P(self.mesh.pp_group, self.mesh.pipe_ranks, self.device, ctrl_group=self.mesh.ctrl_group)
        # every collective of the step (DP all-reduce, head reduction, clip norm, losses)
        self.coll = Collectives(self.mesh, self.device, pipe_engine=p2p.engine, embed=tied_pp)
        for st in self.stages:
            st.coll = self.coll
        self.runtime = PipelineRuntime(self.stages, self.schedule, n_microbatches, self.mesh.pp_rank, pp, p2p,
                                       scale_grads=True, style=style, profile=profile, orders=orders,
                                       head=head_plan, head_costs=head_costs, stage_costs=stage_costs,
                                       dp=self.mesh.dp, head_reduce_after_stage0=bool(cfg.tie_embeddings),
                                       vote_group=self.mesh.world_ctrl)
        # microbatch lanes (PipelineRuntime.set_lanes): MIPIPE_LANES=auto|1 (off)|n.  Not with
        # plain GEMMs on hipBLASLt (MIPIPE_GEMM=blas|auto): its stream-K kernels synchronise
        # their workgroups and assume all of them resident; a second lane's kernels holding
        # CUs left a Llama-3 1B step hung in that mode (profiles/r3_model_families_1gpu.txt)
        self.lanes = self.runtime.set_lanes(self.planned_lanes)
        if graphed and self.lanes != self.planned_lanes:
            # the runtime took fewer lanes than planned: re-plan with the real count
            self.memory_plan = self._plan_memory(self.lanes)
            if self.recompute_requested == "auto" and self.memory_plan["recompute_layers"] != self.recompute_layers:
                raise RuntimeError(f"recompute='auto' planned with {self.planned_lanes} microbatch lanes, but the "
                                   f"runtime runs {self.lanes}: the HBM plan's decision changes "
                                   f"({self.recompute_layers} -> {self.memory_plan['recompute_layers']} recomputed "
                                   f"layers per stage); set MIPIPE_LANES")
        arenas = [st.arena for st in self.stages]
        if self.dp_zero:
            dp, dr = self.mesh.dp, self.mesh.dp_rank
            for a in arenas:
                n = a.numel // dp

                def gather_dp(shard, numel=a.numel, lo=dr * n, n=n):
                    full = torch.empty(numel, dtype=shard.dtype, device=shard.device)
                    full[lo:lo + n].copy_(shard)
                    self.coll.all_gather(full, "dp").wait()
                    return full
                a.shard_master(dr * n, dr * n + n, gather_dp, scope="dp")
        norm_skip = []
        norm_exclude = {}
        merged_skip = set()
        if tied_pp or self._tie_local:
            # stage 0's embedding gradient is summed with the last stage's copy after the
            # lane merge (post_step / train_step)
            merged_skip.update(i for i, st in enumerate(self.stages) if st.stage_index == 0)
        if (tied_pp or self._tie_local) and (num_stages - 1) in my_stages:
            # the last stage's copy of the tied embedding holds the same (summed) gradient
            # as stage 0's after post_step: count it once in the global norm
            i = [st.stage_index for st in self.stages].index(num_stages - 1)
            a = self.stages[i].arena
            g = a.g("tok_embeddings.weight")
            norm_exclude[i] = [(g.storage_offset() - a.grad.storage_offset(), g.numel())]
        if self.head is not None:
            ha = self.head.arena
            if self.head_zero and pp > 1:
                # this pipeline rank owns block pp_rank of the head arena: its f32 master and
                # Adam moments; the gradient is reduce-scattered into that block
                n = ha.numel // pp
                lo = self.mesh.pp_rank * n

                def gather(shard, numel=ha.numel, lo=lo, n=n):
                    full = torch.empty(numel, dtype=shard.dtype, device=shard.device)
                    full[lo:lo + n].copy_(shard)
                    self.coll.all_gather(full, "pp").wait()
                    return full
                ha.shard_master(lo, lo + n, gather)
            else:
                if self.mesh.pp_rank != 0:
                    norm_skip.append(len(arenas))
                if pp > 1:
                    merged_skip.add(len(arenas))    # all-reduced over the pipeline after the merge
            arenas.append(ha)
            if self.mesh.world > 1:
                self.runtime.head_reduce = self._head_reduce
        self.optimizer = FlatAdamW(arenas, lr=lr, eps=adam_eps, weight_decay=weight_decay, max_grad_norm=max_grad_norm,
                                   pp_group=self.mesh.pp_group if pp > 1 else None, norm_skip=norm_skip,
                                   norm_exclude=norm_exclude, grad_scale=1.0 / self.mesh.dp, coll=self.coll,
                                   merged_norm=self.mesh.dp == 1,
                                   # (MIPIPE_MERGED_NORM_SKIP=0: the pre-fix behaviour, for A/B tests only)
                                   merged_norm_skip=merged_skip if os.environ.get("MIPIPE_MERGED_NORM_SKIP", "1") != "0"
                                   else ())
        self.last_losses: List[torch.Tensor] = []

    def _head_reduce(self) -> list:
        """REDUCE_HEAD: sum the replicated head's gradient over the pipeline x DP ranks --
        ZeRO-1: reduce-scatter over the pipeline group (this rank's block is summed), then
        all-reduce of that block over DP; replicated: all-reduce of the whole gradient over
        the pipeline group, then over DP.  On the native engines both run on the one
        collective stream (FIFO: the DP step follows the pipeline step without a stream
        wait); through torch.distributed the second waits for the first."""
        g = self.head.arena.grad
        if self.head_zero and self.mesh.pp > 1:
            w1, part = self.coll.reduce_scatter(g, "pp")
        else:
            w1, part = self.coll.all_reduce(g, "pp"), g
        if self.mesh.dp == 1:
            return [w1]
        if self.coll.pp_kind == "native" and self.coll.dp_kind == "native":
            return [w1, self.coll.all_reduce(part, "dp")]
        # through torch.distributed the DP step needs the pipeline step's result, i.e. a
        # wait -- taken when the runtime drains its reductions at the step end, not here: a
        # host block at REDUCE_HEAD would hold this rank's remaining flush hostage to the
        # other pipeline ranks reaching theirs (a hang with the overlapped placement)
        coll = self.coll

        class _Chain:
            def wait(self):
                w1.wait()
                coll.all_reduce(part, "dp").wait()
                return True
        return [_Chain()]

    def _plan_memory(self, lanes: int) -> dict:
        """This rank's HBM plan (plan_recompute) for its compute order with ``lanes`` lanes."""
        head_tokens = (self.head_chunks[self.mesh.pp_rank] if self.head_chunks is not None else
                       (self.mbs * self.S if (len(self.layer_ranges) - 1) in self._my_stages else 0))
        mb = self.mem_bound
        return plan_recompute(self.cfg, self.layer_ranges, self._my_stages, self._order, self.mbs, self.S,
                              self.device, head_tokens=head_tokens,
                              head_shards=self.mesh.pp if (self.head_zero and self.mesh.pp > 1) else 1,
                              stage_shards=self.mesh.dp if self.dp_zero else 1, dtype=mb["dtype"],
                              graphs=mb["graphs"], lanes=lanes, hbm=mb["hbm"],
                              head_split=self.head_chunks is not None)

    def _auto_lanes(self, pp: int, v: int, graphs: bool, m: int, mbs: int, seq_len: int) -> int:
        layers = sum(self.layer_ranges[st.stage_index][1] - self.layer_ranges[st.stage_index][0]
                     for st in self.stages)
        params = sum(st.arena.numel for st in self.stages) + (self.head.arena.numel if self.head is not None else 0)
        return auto_lanes(self.cfg, pp, v, graphs, self.device, m, mbs * seq_len, params, layers, self.recompute)

    @property
    def is_first(self) -> bool:
        return any(st.is_first for st in self.stages)

    @property
    def is_last(self) -> bool:
        """Holds the loss (every rank with a distributed head)."""
        return self.head is not None or any(st.is_last for st in self.stages)

    def num_params_local(self) -> int:
        return sum(st.arena.numel for st in self.stages)

    def train_step(self, tokens: Optional[torch.Tensor] = None, targets: Optional[torch.Tensor] = None,
                   lr: Optional[float] = None) -> Optional[torch.Tensor]:
        """tokens/targets: [m*mbs, S] int64 (tokens needed on the first stage's rank,
        targets on the last).  Returns the mean loss tensor on the last-stage rank."""
        inputs = None
        if self.is_first:
            inputs = [(c,) for c in torch.tensor_split(tokens, self.m, dim=0)]
        tg = list(torch.tensor_split(targets, self.m, dim=0)) if self.is_last else None
        losses: List[torch.Tensor] = []
        audit = self._begin_comm_audit()
        try:
            self.runtime.step(inputs, tg, losses, return_outputs=False)
        except BaseException:
            if audit is not None:     # a failed step leaves no logger attached
                self.runtime.p2p.audit = None
                if self.coll is not None:
                    self.coll.audit = None
            raise
        if self._tie_local:
            by_idx = {st.stage_index: st for st in self.stages}
            g0 = by_idx[0].arena.g("tok_embeddings.weight")
            gl = by_idx[len(self.layer_ranges) - 1].arena.g("tok_embeddings.weight")
            g0.add_(gl)      # both copies were already DP-reduced with their stage arenas
            gl.copy_(g0)
        if self.head is not None:
            # (the head gradient all-reduce was issued and waited on inside the step)
            parts = torch.stack([self.runtime.head_losses.get(i, torch.zeros((), device=self.device))
                                 for i in range(self.m)]).float()
            self.coll.all_reduce(parts, "pp").wait()
            losses = list(parts / (self.mbs * self.S))
        self.optimizer.step(lr)
        if audit is not None:
            self._end_comm_audit(audit)
        self.last_losses = losses
        if losses:
            return torch.stack(losses).mean()
        return None

    # ------------------------------------------------------------------ comm audit
    comm_audit: Optional[dict] = None

    def _begin_comm_audit(self):
        """First training step of a multi-rank job (MIPIPE_COMM_AUDIT=0: never): log every
        p2p post and collective this rank issues (parallel/audit.py)."""
        if (self.comm_audit is not None or self.mesh.world <= 1 or not dist.is_initialized()
                or os.environ.get("MIPIPE_COMM_AUDIT", "1") == "0"):
            return None
        from .parallel.audit import CommAudit
        audit = CommAudit(self.mesh.rank)
        self.runtime.p2p.audit = audit
        if self.coll is not None:
            self.coll.audit = audit
        return audit

    def _end_comm_audit(self, audit) -> None:
        """Exchange the logs over the gloo control group and check p2p order per pair and
        channel and collective sequences per group; raise on the first divergence."""
        from .parallel.audit import gather_and_check
        self.runtime.p2p.audit = None
        if self.coll is not None:
            self.coll.audit = None
        ok, problems, n = gather_and_check(audit, self.mesh.world_ctrl)
        # whether this rank's log held its pipeline p2p (an eager step) or only collectives
        # (a step replayed from the native tape issues p2p from C++, unlogged)
        p2p_logged = any(e[0] == "p2p" for e in audit.entries)
        self.comm_audit = {"ok": ok, "entries": n, "problems": problems,
                           "p2p": "audited" if (p2p_logged or self.mesh.pp == 1) else "not covered (native replay)"}
        if not ok:
            raise RuntimeError("communication issued by the ranks does not match (would hang under RCCL):\n  "
                               + "\n  ".join(problems))

    def describe(self) -> str:
        """Hang report (utils/metrics.Watchdog): the runtime's program grid plus, for every
        native RCCL engine of this rank, the issued groups that have not completed."""
        from .parallel.comm import comm_progress_report
        eng = {"p2p": getattr(self.runtime.p2p, "engine", None),
               "dp": getattr(self.coll, "dp_engine", None), "embed": getattr(self.coll, "embed_engine", None)}
        out = self.runtime.describe() + "\n" + comm_progress_report(eng)
        audit = getattr(self.runtime.p2p, "audit", None)
        if audit is not None:
            # stalled inside the audited first step: what this rank issued so far, in order
            # (compare across the ranks' reports: the first entry without a partner blocks)
            tail = audit.entries[-8:]
            out += f"\n[comm audit] {len(audit.entries)} issued this step; last {len(tail)}:\n" + \
                "\n".join(f"[comm audit]   {e}" for e in tail)
        return out

    def capture_graphs(self, tokens: Optional[torch.Tensor] = None, targets: Optional[torch.Tensor] = None) -> None:
        """Setup, not training: run the pipeline program twice without an optimizer step
        (eager lazy-init, then HIP-graph capture of every per-microbatch action) and
        discard the gradients.  Later ``train_step`` calls replay the graphs."""
        if not any(st.graphs is not None for st in self.stages):
            return
        inputs = [(c,) for c in torch.tensor_split(tokens, self.m, dim=0)] if self.is_first else None
        tg = list(torch.tensor_split(targets, self.m, dim=0)) if self.is_last else None
        first = True
        while min(st.step_id for st in self.stages) < 2:
            if not first and self.device.type == "cuda":
                # the eager step's activations went back to the caching allocator's default
                # pool; return them to the device before the graphs take their own pools, or
                # the device holds both (113.8 vs 58.5 GB reserved on GPT-2 small, 2 x 64K
                # tokens: profiles/r6_hbm_reserved.md)
                torch.cuda.empty_cache()
            first = False
            # the first (eager) step issues every p2p post through Python: audit it here --
            # the first train_step after capture replays the native tape, where only the
            # collectives would be seen
            audit = self._begin_comm_audit()
            try:
                self.runtime.step(inputs, tg, [], return_outputs=False)
            except BaseException:
                if audit is not None:
                    self.runtime.p2p.audit = None
                    if self.coll is not None:
                        self.coll.audit = None
                raise
            if audit is not None:
                self._end_comm_audit(audit)
        for a in self.optimizer.arenas:
            a.grad.zero_()
        if self.device.type == "cuda":
            torch.cuda.empty_cache()

    def bubble(self) -> float:
        return self.runtime.bubble()

    # ------------------------------------------------------------------ checkpoint
    def save_checkpoint(self, path: str, extra: Optional[dict] = None) -> None:
        """Per-pipeline-rank safetensors shards keyed by global FQNs + JSON manifest
        (collective; see utils/checkpoint.py)."""
        from .utils.checkpoint import save_checkpoint
        save_checkpoint(self, path, extra=extra)

    def load_checkpoint(self, path: str, load_optimizer: bool = True) -> dict:
        """Resume from a checkpoint written at any PP degree (re-split by FQN)."""
        from .utils.checkpoint import load_checkpoint
        return load_checkpoint(self, path, load_optimizer=load_optimizer)

    def state_dict(self):
        sd = {}
        for st in self.stages:
            sd.update(st.arena.state_dict())
        if self.head is not None:
            sd.update(self.head.arena.state_dict())
        return sd
