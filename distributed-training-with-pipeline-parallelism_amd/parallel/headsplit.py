"""Distributed LM head: spread the vocabulary projection + loss over every pipeline rank.

With a 50k vocabulary the head of GPT-2 small costs as much as ~5 transformer layers,
so at PP=8 the last stage alone would bound the pipeline to ~40 % of ideal
(12 layers + head cannot be split evenly when the head is one indivisible block).
The reference has no answer to this (its last stage simply owns the head,
helper:23-55 / helper:70-75); here the head becomes a set of ``H`` actions:

* the last stage's forward stops at the final norm; its output rows (tokens) are cut
  into per-rank chunks and sent to every rank (``SEND_H``);
* rank r runs ``rH m`` on its chunk: logits = h W^T, fused softmax-CE forward+backward,
  dh = dlogits W, dW += dlogits^T h, and sends dh back (``SEND_D``); softmax is over the
  full vocabulary, so chunks need no cross-rank statistics;
* the last stage's backward starts from the gathered dh.

Every rank holds the (tied) head weight; its gradient is all-reduced once per step and
the replicated AdamW update keeps the copies bit-identical.  Chunk sizes are chosen by
water-filling so that (stage layers + head chunk) is level across ranks, and the ``H``
actions are placed into each rank's compute order by a list-scheduling simulation
(``insert_head_ops``), after which the normal lowering/deadlock check applies.
"""
from __future__ import annotations

import os

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

from .ir import Action, Op
from .schedules import stage_to_rank
from .simulate import DEFAULT_COSTS, action_rank, in_messages, simulate, uses_split_backward


def head_token_split(T: int, rank_load: Sequence[float], head_load: float, align: int = 128) -> List[int]:
    """Token chunk per rank so that ``rank_load[r] + head_load * tokens_r / T`` is as
    level as possible (water-filling), in multiples of ``align`` tokens, summing to T."""
    P = len(rank_load)
    units = T // align
    if units * align != T:
        raise ValueError(f"{T} tokens are not a multiple of the chunk alignment {align}")
    per_unit = head_load / units
    # water level L: sum_r max(0, L - load_r) = head_load
    loads = sorted(rank_load)
    level = loads[0]
    rem = head_load
    for i in range(P):
        nxt = loads[i + 1] if i + 1 < P else float("inf")
        cap = (nxt - loads[i]) * (i + 1)
        if rem <= cap:
            level = loads[i] + rem / (i + 1)
            break
        rem -= cap
    share = [max(0.0, level - x) / per_unit for x in rank_load]
    cnt = [int(s) for s in share]
    # largest remainders get the leftover units
    left = units - sum(cnt)
    order = sorted(range(P), key=lambda r: -(share[r] - cnt[r]))
    for r in order[:left]:
        cnt[r] += 1
    return [c * align for c in cnt]


def _lag_last_stage(order: List[Action], last, lag: int) -> List[Action]:
    """Delay the backward (B/I/W) of microbatch i of stage(s) ``last`` (an index or a set)
    until after that stage's forward of i+lag (the slack that lets the other ranks fit
    their head chunks in).  A stable re-sort: relative orders of forwards and of
    backwards are unchanged."""
    if lag <= 0:
        return list(order)
    stages = {last} if isinstance(last, int) else set(last)
    fpos = {(a.stage, a.mb): i for i, a in enumerate(order) if a.stage in stages and a.op == Op.F}
    if not fpos:
        return list(order)
    flast = {}
    for (st, _), i in fpos.items():
        flast[st] = max(flast.get(st, -1), i)
    keys = []
    for i, a in enumerate(order):
        k = float(i)
        if a.stage in stages and a.op in (Op.B, Op.I, Op.W):
            k = max(k, fpos.get((a.stage, a.mb + lag), flast[a.stage]) + 0.5)
        keys.append(k)
    return [a for _, a in sorted(zip(keys, order), key=lambda t: t[0])]


def insert_head_ops(orders: Dict[int, Sequence[Optional[Action]]], pp: int, v: int, style: str,
                    head_costs: Dict[int, float], stage_costs: Optional[Sequence[float]] = None,
                    lag: int = 1, comm: float = 0.05, costs: Optional[Dict[Op, float]] = None,
                    policy: str = "head_first") -> Dict[int, List[Action]]:
    """Insert ``rH m`` actions (ranks with a non-zero ``head_costs[r]``) into per-rank
    compute orders by list scheduling: whenever a rank is free it runs whichever is
    startable first -- its next scheduled action or its next head chunk (ties go to
    the head chunk, which the last stage is waiting for)."""
    costs = {**DEFAULT_COSTS, **(costs or {})}
    S = pp * v
    s2r = [stage_to_rank(s, pp, style) for s in range(S)]
    base = {r: [a for a in orders.get(r, []) if a is not None and a.op.is_compute] for r in range(pp)}
    split = uses_split_backward(base)
    last_rank = s2r[S - 1]
    if lag > 0:
        # every stage gets `lag` more warmup forwards (delaying only the last stage's
        # backwards would starve the upstream ranks' steady state); with several
        # virtual stages per rank, each of them does
        for r in range(pp):
            base[r] = _lag_last_stage(base[r], {s for s in range(S) if s2r[s] == r}, lag)
    head = tuple(r for r in range(pp) if head_costs.get(r, 0.0) > 0.0)
    mbs = sorted({a.mb for a in base[last_rank] if a.op == Op.F and a.stage == S - 1})

    def cost(a: Action) -> float:
        if a.op == Op.H:
            return costs[Op.H] * head_costs[a.stage]
        return costs[a.op] * (stage_costs[a.stage] if stage_costs is not None else 1.0)

    ptr = {r: 0 for r in range(pp)}
    hptr = {r: 0 for r in range(pp)}
    avail = {r: 0.0 for r in range(pp)}
    end: Dict[Action, float] = {}
    out: Dict[int, List[Action]] = {r: [] for r in range(pp)}
    total = sum(len(b) for b in base.values()) + len(head) * len(mbs)

    deps: Dict[Action, list] = {}

    def ready_time(a: Action, r: int) -> Optional[float]:
        dl = deps.get(a)
        if dl is None:
            dl = deps[a] = [(d, action_rank(d, s2r) != r) for d, _ in in_messages(a, S, split, head)]
        t = avail[r]
        for d, remote in dl:
            e = end.get(d)
            if e is None:
                waiters.setdefault(d, []).append(r)
                return None
            t = max(t, e + comm) if remote else max(t, e)
        return t

    # a rank's candidates change only when it runs an action (its ``avail``) or when an
    # input one of them waits for is scheduled: otherwise they are reused (same result)
    cached: Dict[int, list] = {}
    waiters: Dict[Action, List[int]] = {}
    done = 0
    while done < total:
        best = None  # (start, tie, rank, action, is_head)
        for r in range(pp):
            if r in cached:
                for c in cached[r]:
                    if best is None or (c[0], c[1], c[2]) < (best[0], best[1], best[2]):
                        best = c
                continue
            cands = []
            if r in head and hptr[r] < len(mbs):
                h = Action(r, Op.H, mbs[hptr[r]])
                t = ready_time(h, r)
                if t is not None:
                    cands.append((t, 0, r, h, True))
            if ptr[r] < len(base[r]):
                a = base[r][ptr[r]]
                t = ready_time(a, r)
                if t is not None:
                    cands.append((t, 1, r, a, False))
            if policy == "fill" and len(cands) == 2 and cands[1][0] <= avail[r] + 1e-9:
                cands = cands[1:]   # the scheduled action can start now: head chunks only fill gaps
            elif policy == "fill" and len(cands) == 2:
                cands = [cands[0]] if cands[0][0] <= cands[1][0] else [cands[1]]
            cached[r] = cands
            for c in cands:
                if best is None or (c[0], c[1], c[2]) < (best[0], best[1], best[2]):
                    best = c
        if best is None:
            stuck = {r: str(base[r][ptr[r]]) for r in range(pp) if ptr[r] < len(base[r])}
            raise RuntimeError(f"head placement deadlocks; stuck at {stuck}")
        t, _, r, a, is_head = best
        end[a] = t + cost(a)
        avail[r] = end[a]
        cached.pop(r, None)
        for w in waiters.pop(a, ()):
            cached.pop(w, None)
        out[r].append(a)
        if is_head:
            hptr[r] += 1
        else:
            ptr[r] += 1
        done += 1
    return out


def plan_head_schedule(orders: Dict[int, Sequence[Optional[Action]]], pp: int, v: int, style: str,
                       head_costs: Dict[int, float], stage_costs: Optional[Sequence[float]] = None,
                       comm: float = 0.05, lags: Sequence[int] = (0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32),
                       policies: Sequence[str] = ("head_first", "fill"),
                       regen: Optional[Callable[[int], Dict[int, Sequence[Optional[Action]]]]] = None,
                       lag_tol: Optional[float] = None, max_lag: Optional[int] = None,
                       fits: Optional[Callable[[Dict[int, List[Action]]], bool]] = None
                       ) -> Tuple[Dict[int, List[Action]], int, float]:
    """Best of ``insert_head_ops`` over the candidate last-stage lags (simulated
    makespan).  Returns (orders, lag, makespan).

    Deep lags matter with 1F1B: the last stage's B(i) waits for every rank's H(i), which
    waits for its F(i) -- a round trip on the critical cycle unless the last stage has
    `lag` more forwards to run meanwhile.  GPT-2 small, PP=2, m=8: lag <= 2 planned 0.755
    of ideal, lag 8 0.912; each unit of lag stashes one more microbatch per stage
    (hundreds of MB at GPT-2 scale, cheap next to 288 GB of HBM) -- but not free: a lag of m
    turns 1F1B's stash into GPipe's.  So the plan takes the SMALLEST lag whose makespan is
    within ``lag_tol`` (default 1 %, ``MIPIPE_HEAD_LAG_TOL``) of the best, and never more than
    ``max_lag`` (``MIPIPE_HEAD_MAX_LAG``).  ``fits(orders)``: the memory bound -- a placement
    with a positive lag whose orders it rejects (engine.plan_head_pipeline: the HBM plan of
    every rank's stash slots over its budget) is not a candidate; lag 0 (the schedule's own
    warmup depth) always is.

    ``regen(lag)``: the schedule regenerated with ``lag`` extra warmup forwards on every
    rank (schedules.generate(..., warmup_extra=lag)).  Tried next to the re-sort of
    ``_lag_last_stage``, which deadlocks for interleaved orders (it moves one chunk's
    backwards past the other chunk's forwards): with it, GPT-2 small Interleaved1F1B (v=2,
    m=4P) plans 0.952 / 0.935 / 0.894 of ideal at P=2/4/8 instead of 0.845 / 0.927 / 0.773."""
    if lag_tol is None:
        lag_tol = float(os.environ.get("MIPIPE_HEAD_LAG_TOL", "0.01"))
    if max_lag is None and os.environ.get("MIPIPE_HEAD_MAX_LAG"):
        max_lag = int(os.environ["MIPIPE_HEAD_MAX_LAG"])
    cands = []
    nmb = 1 + max((a.mb for es in orders.values() for a in es if a is not None), default=0)
    # up to a full-depth warmup (lag m: every forward first, GPipe's order): at P = 8 with
    # GPT-2 small's 16-sequence microbatches a hop costs about a layer forward and 1F1B
    # plans 0.79 at lag 32 but 0.88 at lag m = 64
    lags = sorted(set(lags) | {l for l in (48, 64, 96, 128) if l < nmb * max(1, v)} | {nmb * max(1, v)})
    for lag in lags:
        if lag > nmb * max(1, v) or (max_lag is not None and lag > max_lag):
            continue
        cands.append((lag, orders, lag))
        if regen is not None and lag > 0:
            cands.append((lag, None, 0))
    found = []
    regen_cache: Dict[int, Dict[int, Sequence[Optional[Action]]]] = {}
    for pol in policies:
        for lag, base, ins_lag in cands:
            try:
                if base is None:
                    if lag not in regen_cache:
                        regen_cache[lag] = regen(lag)
                    base = regen_cache[lag]
                o = insert_head_ops(base, pp, v, style, head_costs, stage_costs, lag=ins_lag, comm=comm, policy=pol)
                if lag > 0 and fits is not None and not fits(o):
                    continue
                res = simulate(o, pp, v, style, comm_latency=comm, stage_costs=stage_costs, head_costs=head_costs)
            except (RuntimeError, ValueError):
                continue
            found.append((o, lag, res.makespan))
    if not found:
        raise RuntimeError("no feasible head placement")
    fastest = min(f[2] for f in found)
    # first (policy order) of the smallest lags that stay within the tolerance
    return min((f for f in found if f[2] <= fastest * (1.0 + lag_tol) + 1e-9), key=lambda f: f[1])


@dataclass
class HeadPlan:
    """Runtime description of a distributed head.

    ``chunks[r]``: tokens of every microbatch that rank r processes (rows
    ``offsets[r] : offsets[r] + chunks[r]`` of the last stage's [T, D] output);
    ``runner(h, target, dh_out, grad_scale) -> loss_sum`` runs this rank's chunk."""
    chunks: List[int]
    d_model: int
    runner: Optional[Callable] = None
    dtype: object = None
    offsets: List[int] = field(default_factory=list)
    graphs: object = None   # GraphCache: chunks replayed as HIP graphs after the first step
    arena: object = None    # the head's ParamArena (per-lane gradients with microbatch lanes)

    def __post_init__(self):
        self.offsets = [sum(self.chunks[:r]) for r in range(len(self.chunks))]

    @property
    def tokens(self) -> int:
        return sum(self.chunks)

    @property
    def ranks(self) -> Tuple[int, ...]:
        return tuple(r for r, c in enumerate(self.chunks) if c > 0)

    def rows(self, r: int) -> slice:
        return slice(self.offsets[r], self.offsets[r] + self.chunks[r])
