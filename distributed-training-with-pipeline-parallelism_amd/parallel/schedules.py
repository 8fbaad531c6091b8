"""Microbatch schedule generators (compute order per rank).

Each generator returns ``{rank: [Action, ...]}`` -- the order in which a rank runs
its forward / backward work.  Communication is added later by :mod:`.lower`.

Behavior parity with the reference dependency (torch pipelining, used by
/root/reference/LLMsDistributedTrainingHelper.py:12,215-220):

* GPipe (schedules.py:727-843): all m forwards, then all m backwards.
* 1F1B (schedules.py:846-994): ``P-s-1`` warmup forwards, steady 1F1B, cooldown.
  (torch counts one more "warmup" forward and then runs 1B1F -- the resulting
  op order is identical.)
* Interleaved 1F1B (schedules.py:2493-2611): ``rounds = max(1, m // P)``,
  ``mpr = m // rounds``, warmup ``min((v-1)*mpr + 2*(P-1-r), m*v)``; forward
  chunk ``(k // mpr) % v``, backward chunk reversed.  Reproduces the golden IR in
  SURVEY.md Appendix A exactly (see tests/test_schedules.py).
* Looped BFS (schedules.py:2287-2350): every local stage runs all m forwards,
  backwards in reverse stage order.
* ZB-H1 (zero-bubble, split backward): a list-scheduled 1F1B in which the weight
  gradient ``W`` is deferred into what would otherwise be cooldown bubbles; memory
  bound identical to 1F1B.  Built by :func:`_greedy_schedule`, a small list
  scheduler that is also usable for custom policies.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

from .ir import Action, Op

# ----------------------------------------------------------------------------------------
# placement
# ----------------------------------------------------------------------------------------


def stage_to_rank(stage: int, pp: int, style: str = "loop") -> int:
    """Map a (virtual) stage to its pipeline rank.

    ``loop``: stage k -> k % pp (reference helper:208 ``stage_idx = rank + world_size*i``).
    ``v``: zig-zag, chunk c runs forward on even c, backward on odd c (torch _utils.py:91-122).
    """
    if style == "loop":
        return stage % pp
    if style == "v":
        c, i = divmod(stage, pp)
        return i if c % 2 == 0 else pp - 1 - i
    raise ValueError(f"unknown placement style {style!r}")


def rank_stages(rank: int, pp: int, v: int, style: str = "loop") -> List[int]:
    return [s for s in range(pp * v) if stage_to_rank(s, pp, style) == rank]


# ----------------------------------------------------------------------------------------
# generators
# ----------------------------------------------------------------------------------------


def gen_gpipe(pp: int, m: int, v: int = 1, style: str = "loop", warmup_extra: int = 0) -> Dict[int, List[Action]]:
    if v != 1:
        raise ValueError("GPipe runs one stage per rank (use LoopedBFS for v>1)")
    return {r: [Action(r, Op.F, i) for i in range(m)] + [Action(r, Op.B, i) for i in range(m)] for r in range(pp)}


def gen_1f1b(pp: int, m: int, v: int = 1, style: str = "loop", warmup_extra: int = 0) -> Dict[int, List[Action]]:
    """``warmup_extra``: forwards added to every rank's warmup (deeper 1F1B; m - 1 or more
    is GPipe).  The distributed head's planner uses it to give the last stage slack."""
    if v != 1:
        raise ValueError("1F1B runs one stage per rank (use Interleaved1F1B for v>1)")
    out = {}
    for r in range(pp):
        w = min(pp - r - 1 + max(0, warmup_extra), m)
        ops = [Action(r, Op.F, i) for i in range(w)]
        for i in range(m - w):
            ops.append(Action(r, Op.F, w + i))
            ops.append(Action(r, Op.B, i))
        ops += [Action(r, Op.B, i) for i in range(m - w, m)]
        out[r] = ops
    return out


def interleave_params(pp: int, m: int) -> Tuple[int, int]:
    """(rounds, microbatches_per_round) of the interleaved schedule (torch schedules.py:2535-2542)."""
    rounds = max(1, m // pp)
    if m % rounds != 0:
        raise ValueError(f"Interleaved1F1B needs n_microbatches ({m}) divisible by rounds ({rounds})")
    return rounds, m // rounds


def gen_interleaved_1f1b(pp: int, m: int, v: int = 2, style: str = "loop",
                         warmup_extra: int = 0) -> Dict[int, List[Action]]:
    """torch's interleaved order; ``warmup_extra`` forwards are added to every rank's warmup
    (0 = torch's).  A uniformly deeper warmup keeps the order valid and deadlock-free (the
    limit is all-forwards-first) and is how the distributed head's planner buys the last
    stage slack without re-sorting chunks against each other (headsplit.plan_head_schedule)."""
    if style != "loop":
        raise ValueError("Interleaved1F1B's warmup formula assumes loop placement (use LoopedBFS/ZBH1 for 'v')")
    _, mpr = interleave_params(pp, m)
    out = {}
    for r in range(pp):
        stages = rank_stages(r, pp, v, style)  # chunk order
        total = m * v
        warm = min((v - 1) * mpr + 2 * (pp - 1 - r) + max(0, warmup_extra), total)
        fwd_next = [0] * v
        bwd_next = [0] * v
        ops: List[Action] = []

        def f(k):
            c = (k // mpr) % v
            ops.append(Action(stages[c], Op.F, fwd_next[c]))
            fwd_next[c] += 1

        def b(k):
            c = v - 1 - (k // mpr) % v
            ops.append(Action(stages[c], Op.B, bwd_next[c]))
            bwd_next[c] += 1

        for k in range(warm):
            f(k)
        for k in range(total - warm):
            f(warm + k)
            b(k)
        for k in range(total - warm, total):
            b(k)
        out[r] = ops
    return out


def gen_looped_bfs(pp: int, m: int, v: int = 2, style: str = "loop") -> Dict[int, List[Action]]:
    out = {}
    for r in range(pp):
        stages = rank_stages(r, pp, v, style)
        ops = [Action(s, Op.F, i) for s in stages for i in range(m)]
        ops += [Action(s, Op.B, i) for s in reversed(stages) for i in range(m)]
        out[r] = ops
    return out


def _greedy_schedule(pp: int, m: int, v: int, style: str, costs: Dict[Op, float],
                     max_inflight: Callable[[int], int], split_backward: bool,
                     comm: float = 0.0) -> Dict[int, List[Action]]:
    """Event-driven list scheduler.

    Each rank, whenever idle, picks the ready action with the highest priority:
    backward-input (I/B) > forward (if the activation stash has room) > weight-grad W.
    W only runs when nothing else is ready, which is what removes the cooldown
    bubbles (zero-bubble ZB-H1 idea).  ``max_inflight(rank)`` bounds the number of
    microbatches whose activations are stashed on that rank (1F1B memory bound).
    """
    S = pp * v
    s2r = [stage_to_rank(s, pp, style) for s in range(S)]
    bwd_op = Op.I if split_backward else Op.B
    done: Dict[Action, float] = {}
    rank_time = [0.0] * pp
    order: Dict[int, List[Action]] = {r: [] for r in range(pp)}
    pending_w: Dict[int, List[Action]] = {r: [] for r in range(pp)}
    fwd_next = {s: 0 for s in range(S)}
    bwd_next = {s: 0 for s in range(S)}
    inflight = [0] * pp
    total = sum(m * 2 + (m if split_backward else 0) for _ in range(S))
    n_done = 0

    def ready_time(a: Action) -> Optional[float]:
        if a.op == Op.F:
            if a.stage == 0:
                return 0.0
            dep = Action(a.stage - 1, Op.F, a.mb)
            if dep not in done:
                return None
            return done[dep] + (comm if s2r[a.stage - 1] != s2r[a.stage] else 0.0)
        if a.op in (Op.B, Op.I):
            own = Action(a.stage, Op.F, a.mb)
            if own not in done:
                return None
            if a.stage == S - 1:
                return done[own]
            dep = Action(a.stage + 1, bwd_op, a.mb)
            if dep not in done:
                return None
            return max(done[own], done[dep] + (comm if s2r[a.stage + 1] != s2r[a.stage] else 0.0))
        if a.op == Op.W:
            dep = Action(a.stage, Op.I, a.mb)
            return done.get(dep)
        raise AssertionError(a)

    guard = 0
    while n_done < total:
        guard += 1
        if guard > 100 * total + 1000:
            raise RuntimeError("greedy scheduler did not converge")
        # pick the rank that becomes free earliest and has something ready
        best = None
        for r in range(pp):
            cands = []
            for s in [s for s in range(S) if s2r[s] == r]:
                if bwd_next[s] < m:
                    a = Action(s, bwd_op, bwd_next[s])
                    t = ready_time(a)
                    if t is not None:
                        cands.append((0, t, -s, a))
                # the stash bound gates only the rank's entry chunk: later chunks' forwards
                # are what drains the stash (multi-chunk V placement)
                entry = s == min(x for x in range(S) if s2r[x] == r)
                if fwd_next[s] < m and (inflight[r] < max_inflight(r) or not entry):
                    a = Action(s, Op.F, fwd_next[s])
                    t = ready_time(a)
                    if t is not None:
                        cands.append((1, t, s, a))
            for a in pending_w[r]:
                cands.append((2, done[Action(a.stage, Op.I, a.mb)], 0, a))
            if not cands:
                continue
            start = max(rank_time[r], min(c[1] for c in cands))
            # among candidates ready by `start`, take highest priority
            avail = [c for c in cands if c[1] <= start]
            avail.sort(key=lambda c: (c[0], c[2], c[1]))
            pick = avail[0]
            # a W only runs if no higher-priority op becomes ready before it would finish
            key = (start, r)
            if best is None or key < best[0]:
                best = (key, r, pick)
        if best is None:
            raise RuntimeError("greedy scheduler deadlocked")
        (start, r), _, pick = best[0], best[1], best[2]
        a = pick[3]
        end = start + costs[a.op]
        done[a] = end
        rank_time[r] = end
        order[r].append(a)
        n_done += 1
        # stash accounting in chunk units: +1 per forward, -1 when the chunk's activations
        # are released (after B, or after W with a split backward)
        if a.op == Op.F:
            fwd_next[a.stage] += 1
            inflight[r] += 1
        elif a.op in (Op.B, Op.I):
            bwd_next[a.stage] += 1
            if a.op == Op.I:
                pending_w[r].append(Action(a.stage, Op.W, a.mb))
            else:
                inflight[r] -= 1
        elif a.op == Op.W:
            pending_w[r].remove(a)
            inflight[r] -= 1
    return order


def gen_zb_h1(pp: int, m: int, v: int = 1, style: str = "loop") -> Dict[int, List[Action]]:
    if v != 1:
        raise ValueError("ZBH1 runs one stage per rank")
    # one chunk more in flight than 1F1B's P - r lets W fill the bubble at P > 1; at P = 1
    # there is no bubble to fill, and the extra chunk (a whole microbatch's activations plus
    # its deferred weight-gradient inputs) only cost HBM: 72.4 vs 52.9 GB on GPT-2 small
    # (BENCH_r04) -- there ZBH1 is F I W per microbatch, 1F1B's memory
    extra = 1 if pp > 1 else 0
    return _greedy_schedule(pp, m, 1, style, {Op.F: 1.0, Op.I: 1.0, Op.W: 1.0, Op.B: 2.0},
                            max_inflight=lambda r: pp - r + extra, split_backward=True)


def gen_zbv(pp: int, m: int, v: int = 2, style: str = "v") -> Dict[int, List[Action]]:
    """Zero-bubble V schedule (ZB-V; the dependency's ScheduleZBVZeroBubble, torch
    schedules.py:2287-3216 family): two chunks per rank in V placement (rank r holds
    stages r and 2P-1-r, so the last chunk's output returns to rank 0's neighbour for
    free), split backward with weight-grad fill, 1F1B-level activation memory
    (2P half-size chunks in flight per rank)."""
    if v != 2:
        raise ValueError("ZBV runs two stages per rank")
    if style != "v":
        raise ValueError("ZBV needs the 'v' stage placement")
    return _greedy_schedule(pp, m, 2, "v", {Op.F: 1.0, Op.I: 1.0, Op.W: 1.0, Op.B: 2.0},
                            max_inflight=lambda r: 2 * pp, split_backward=True)


# ----------------------------------------------------------------------------------------
# registry
# ----------------------------------------------------------------------------------------

# name -> (generator, default v, multi-stage-per-rank?)
SCHEDULES: Dict[str, Tuple[Callable[..., Dict[int, List[Action]]], int, bool]] = {
    "GPipe": (gen_gpipe, 1, False),
    "1F1B": (gen_1f1b, 1, False),
    "Interleaved1F1B": (gen_interleaved_1f1b, 2, True),
    "LoopedBFS": (gen_looped_bfs, 2, True),
    "ZBH1": (gen_zb_h1, 1, False),
    "ZBV": (gen_zbv, 2, True),
}
# schedules that only exist for one stage placement
REQUIRED_STYLE: Dict[str, str] = {"ZBV": "v"}

_ALIASES = {k.lower(): k for k in SCHEDULES}
_ALIASES.update({"gpipe": "GPipe", "1f1b": "1F1B", "interleaved": "Interleaved1F1B",
                 "interleaved1f1b": "Interleaved1F1B", "loopedbfs": "LoopedBFS", "bfs": "LoopedBFS",
                 "zbh1": "ZBH1", "zb": "ZBH1", "zerobubble": "ZBH1", "zbv": "ZBV",
                 "zbvzerobubble": "ZBV"})


def canonical_name(name: str) -> str:
    key = name.replace("_", "").replace("-", "").lower()
    if key not in _ALIASES:
        raise ValueError(f"unknown schedule {name!r}; known: {sorted(SCHEDULES)}")
    return _ALIASES[key]


# generators that take a ``warmup_extra`` (deeper warmup) argument
WARMUP_EXTRA = ("GPipe", "1F1B", "Interleaved1F1B")


def generate(name: str, pp: int, m: int, v: Optional[int] = None, style: str = "loop",
             warmup_extra: int = 0) -> Dict[int, List[Action]]:
    name = canonical_name(name)
    gen, dv, multi = SCHEDULES[name]
    v = dv if v is None else v
    if not multi and v != 1:
        raise ValueError(f"{name} supports one stage per rank")
    if m < 1 or pp < 1 or v < 1:
        raise ValueError("pp, m, v must be >= 1")
    if warmup_extra:
        if name not in WARMUP_EXTRA:
            raise ValueError(f"{name} has no warmup_extra")
        return gen(pp, m, v, style, warmup_extra=warmup_extra)
    return gen(pp, m, v, style)


def analytic_bubble(name: str, pp: int, m: int, v: int = 1) -> float:
    """Idle fraction of an ideal pipeline with uniform stages and B = 2F.

    GPipe/1F1B: (P-1)/(m+P-1).  Interleaved: (P-1)/(v*m+P-1) (Narayanan et al. 2021).
    Zero-bubble ZB-H1 is measured by :mod:`.simulate` rather than a closed form.
    """
    name = canonical_name(name)
    if name in ("GPipe", "1F1B"):
        return (pp - 1) / (m + pp - 1)
    if name in ("Interleaved1F1B", "LoopedBFS"):
        return (pp - 1) / (v * m + pp - 1)
    from .simulate import simulate
    style = REQUIRED_STYLE.get(name, "loop")
    return simulate(generate(name, pp, m, v, style), pp, v, style).bubble
