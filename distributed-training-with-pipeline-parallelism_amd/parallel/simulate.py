"""Schedule simulators: timing/bubble model and RCCL-semantics deadlock checker.

* :func:`simulate` replays per-rank compute orders with per-op costs and a p2p
  latency, honouring cross-stage dependencies, and reports makespan, per-rank busy
  time and the bubble fraction ``1 - busy / (P * makespan)``.  It plays the role of
  the dependency's ``_simulate_comms_compute`` (torch schedules.py:3246-3376) but
  also produces *time stamps*, which :mod:`.lower` uses to build a globally
  consistent p2p order.
* :func:`check_lowered` models the executor on a GPU: per rank one in-order compute
  stream and one in-order comm stream per engine channel (1, or 2 = one per traffic
  direction); a comm group starts after the previous group of its stream completed and
  after every compute issued before it; a message completes when both endpoint groups
  have started; a compute waits for the groups that carry its inputs.  A fixpoint that
  does not finish means the lowered program can hang.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from .ir import Action, CommGroup, Entry, Op
from .schedules import stage_to_rank

DEFAULT_COSTS = {Op.F: 1.0, Op.B: 2.0, Op.I: 1.0, Op.W: 1.0, Op.H: 1.0, Op.REDUCE_GRAD: 0.0}


@dataclass
class SimResult:
    start: Dict[Action, float]
    end: Dict[Action, float]
    rank_of: Dict[Action, int]
    makespan: float
    busy: Dict[int, float]
    bubble: float
    per_rank_bubble: Dict[int, float] = field(default_factory=dict)

    def chrome_trace(self) -> dict:
        ev = []
        for a, t0 in self.start.items():
            ev.append({"name": str(a), "ph": "X", "pid": self.rank_of[a], "tid": 0,
                       "ts": t0 * 1000.0, "dur": (self.end[a] - t0) * 1000.0,
                       "args": {"stage": a.stage, "mb": a.mb, "op": a.op.value}})
        return {"traceEvents": ev, "displayTimeUnit": "ms"}

    def dump_chrome_trace(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(self.chrome_trace(), f)


def head_ranks_of(orders) -> Tuple[int, ...]:
    """Ranks that run a chunk of the distributed LM head (``H`` actions)."""
    return tuple(sorted({a.stage for v in orders.values() for a in v if a is not None and a.op == Op.H}))


def action_rank(a: Action, s2r: Sequence[int]) -> int:
    """Rank executing an action: ``H`` actions carry their rank in the stage field."""
    return a.stage if a.op == Op.H else s2r[a.stage]


def in_messages(a: Action, num_stages: int, split: bool, head: Sequence[int] = ()) -> List[Tuple[Action, Optional[tuple]]]:
    """Data inputs of a compute action: ``(producer, message key)``; the key is None for
    state that never leaves the stage (a backward's own forward activations).

    Keys: ``('F', s, m)`` activation into stage s, ``('B', s, m)`` gradient into stage s,
    ``('H', r, m)`` head chunk r's hidden states, ``('D', r, m)`` head chunk r's input
    gradient.  With a distributed head (``head`` = chunk ranks) the last stage's
    backward consumes the ``D`` messages of every chunk."""
    bwd = Op.I if split else Op.B
    if a.op == Op.F:
        return [] if a.stage == 0 else [(Action(a.stage - 1, Op.F, a.mb), ("F", a.stage, a.mb))]
    if a.op in (Op.B, Op.I):
        out: List[Tuple[Action, Optional[tuple]]] = [(Action(a.stage, Op.F, a.mb), None)]
        if a.stage < num_stages - 1:
            out.append((Action(a.stage + 1, bwd, a.mb), ("B", a.stage, a.mb)))
        else:
            out += [(Action(r, Op.H, a.mb), ("D", r, a.mb)) for r in head]
        return out
    if a.op == Op.W:
        return [(Action(a.stage, Op.I, a.mb), None)]
    if a.op == Op.H:
        return [(Action(num_stages - 1, Op.F, a.mb), ("H", a.stage, a.mb))]
    return []


def _deps(a: Action, num_stages: int, split: bool, head: Sequence[int] = ()) -> List[Action]:
    """Cross-stage data dependencies of a compute action."""
    return [d for d, _ in in_messages(a, num_stages, split, head)]


def uses_split_backward(orders: Dict[int, Sequence[Optional[Action]]]) -> bool:
    return any(a is not None and a.op in (Op.I, Op.W) for v in orders.values() for a in v)


def simulate(orders: Dict[int, Sequence[Optional[Action]]], pp: int, v: int = 1, style: str = "loop",
             costs: Optional[Dict[Op, float]] = None, comm_latency: float = 0.0,
             stage_costs: Optional[Sequence[float]] = None,
             head_costs: Optional[Dict[int, float]] = None) -> SimResult:
    """Time a per-rank compute order.  ``stage_costs`` scales each stage's op costs
    (non-uniform partitions); ``head_costs[r]`` is the cost of rank r's head chunk."""
    costs = dict(DEFAULT_COSTS, **(costs or {}))
    S = pp * v
    split = uses_split_backward(orders)
    head = head_ranks_of(orders)
    s2r = [stage_to_rank(s, pp, style) for s in range(S)]
    seq = {r: [a for a in orders[r] if a is not None and a.op.is_compute] for r in orders}
    ptr = {r: 0 for r in seq}
    t_rank = {r: 0.0 for r in seq}
    start: Dict[Action, float] = {}
    end: Dict[Action, float] = {}
    remaining = sum(len(v_) for v_ in seq.values())
    while remaining:
        progressed = False
        for r in seq:
            while ptr[r] < len(seq[r]):
                a = seq[r][ptr[r]]
                ready = t_rank[r]
                ok = True
                for d in _deps(a, S, split, head):
                    if d not in end:
                        ok = False
                        break
                    lat = comm_latency if action_rank(d, s2r) != action_rank(a, s2r) else 0.0
                    ready = max(ready, end[d] + lat)
                if not ok:
                    break
                if a.op == Op.H:
                    c = costs[Op.H] * (head_costs.get(a.stage, 1.0) if head_costs else 1.0)
                else:
                    c = costs[a.op] * (stage_costs[a.stage] if stage_costs is not None else 1.0)
                start[a] = ready
                end[a] = ready + c
                t_rank[r] = end[a]
                ptr[r] += 1
                remaining -= 1
                progressed = True
        if not progressed:
            stuck = {r: str(seq[r][ptr[r]]) for r in seq if ptr[r] < len(seq[r])}
            raise RuntimeError(f"schedule deadlocks (compute dependencies); stuck at {stuck}")
    makespan = max(end.values()) if end else 0.0
    busy = {r: sum(end[a] - start[a] for a in seq[r]) for r in seq}
    bubble = 1.0 - sum(busy.values()) / (len(seq) * makespan) if makespan > 0 else 0.0
    prb = {r: 1.0 - busy[r] / makespan if makespan > 0 else 0.0 for r in seq}
    rank_of = {a: r for r in seq for a in seq[r]}
    return SimResult(start, end, rank_of, makespan, busy, bubble, prb)


def to_grid(res: SimResult, pp: int) -> Dict[int, List[Optional[Action]]]:
    """Unit-time grid (for printing) from a simulation with integer costs."""
    grid: Dict[int, List[Optional[Action]]] = {r: [] for r in range(pp)}
    for a, t0 in sorted(res.start.items(), key=lambda kv: kv[1]):
        r = res.rank_of[a]
        slot = int(round(t0))
        while len(grid[r]) < slot:
            grid[r].append(None)
        grid[r].append(a)
    return grid


# ----------------------------------------------------------------------------------------
# deadlock check of a lowered program
# ----------------------------------------------------------------------------------------


def message_channel(key: tuple) -> int:
    """Engine channel of a message: 0 = activations down the pipeline (F, H), 1 =
    gradients back up (B, D) -- one RCCL communicator + stream each (csrc/comm/rccl_p2p.h)."""
    return 0 if key[0] in ("F", "H") else 1


def check_lowered(program: Dict[int, List[Entry]], num_stages: int, channels: int = 1) -> None:
    """Raise RuntimeError if the lowered program can hang under RCCL semantics.

    Model: per rank one in-order compute stream and ``channels`` in-order comm streams
    (``channels=2``: each CommGroup is split by :func:`message_channel` and every part goes
    to its direction's stream, as the native engine posts it).  A posted group starts
    after the previous group of its stream completed and after every compute issued
    before it; a message completes when both endpoint groups have started; a group
    completes when all its messages have; a compute waits for the groups carrying its
    inputs.  A fixpoint that does not finish means the program can hang."""
    comp_orders = {r: [e for e in es if isinstance(e, Action)] for r, es in program.items()}
    split = uses_split_backward(comp_orders)
    head = head_ranks_of(comp_orders)
    ranks = sorted(program)
    chan = (lambda key: 0) if channels <= 1 else message_channel
    # posted (sub)groups per rank: (channel, ops, index of the last compute issued before it)
    posts: Dict[int, List[Tuple[int, List, int]]] = {}
    comp_list: Dict[int, List[Action]] = {}
    for r in ranks:
        posts[r], comp_list[r] = [], []
        for e in program[r]:
            if isinstance(e, CommGroup):
                by_ch: Dict[int, List] = {}
                for op in e.ops:
                    by_ch.setdefault(chan(op.key), []).append(op)
                for ch in sorted(by_ch):
                    posts[r].append((ch, by_ch[ch], len(comp_list[r]) - 1))
            else:
                comp_list[r].append(e)
    msg_groups: Dict[tuple, List[Tuple[int, int]]] = {}
    recv_group_of: Dict[tuple, Tuple[int, int]] = {}
    queues: Dict[Tuple[int, int], List[int]] = {}       # (rank, channel) -> post indices in order
    for r in ranks:
        for gi, (ch, ops, _) in enumerate(posts[r]):
            queues.setdefault((r, ch), []).append(gi)
            for op in ops:
                msg_groups.setdefault(op.key, []).append((r, gi))
                if op.action.op.is_recv:
                    recv_group_of[(r,) + op.key] = (r, gi)
    for k, gs in msg_groups.items():
        if len(gs) != 2:
            raise RuntimeError(f"message {k} has {len(gs)} endpoints (expected send+recv)")
    comp_waits: Dict[Tuple[int, int], List[Tuple[int, int]]] = {}
    for r in ranks:
        for ci, a in enumerate(comp_list[r]):
            comp_waits[(r, ci)] = [recv_group_of[(r,) + key] for _, key in in_messages(a, num_stages, split, head)
                                   if key is not None and (r,) + key in recv_group_of]
    comp_done: Dict[Tuple[int, int], bool] = {}
    grp_started: Dict[Tuple[int, int], bool] = {}
    grp_done: Dict[Tuple[int, int], bool] = {}
    cptr = {r: 0 for r in ranks}
    qptr = {q: 0 for q in queues}
    ncomp = {r: len(comp_list[r]) for r in ranks}
    changed = True
    while changed:
        changed = False
        for r in ranks:
            while cptr[r] < ncomp[r] and all(grp_done.get(g, False) for g in comp_waits[(r, cptr[r])]):
                comp_done[(r, cptr[r])] = True
                cptr[r] += 1
                changed = True
        for q, lst in queues.items():
            r = q[0]
            # retire completed heads, then start the next group if its computes are done
            while qptr[q] < len(lst) and grp_done.get((r, lst[qptr[q]]), False):
                qptr[q] += 1
                changed = True
            if qptr[q] < len(lst):
                gi = lst[qptr[q]]
                if (r, gi) not in grp_started:
                    last_c = posts[r][gi][2]
                    if last_c < 0 or comp_done.get((r, last_c), False):
                        grp_started[(r, gi)] = True
                        changed = True
        for (r, gi) in list(grp_started):
            if grp_done.get((r, gi)):
                continue
            if all(all(grp_started.get(x, False) for x in msg_groups[op.key]) for op in posts[r][gi][1]):
                grp_done[(r, gi)] = True
                changed = True
    stuck = {r for r in ranks if cptr[r] < ncomp[r]} | {q[0] for q, lst in queues.items() if qptr[q] < len(lst)}
    if stuck:
        detail = {r: (str(comp_list[r][cptr[r]]) if cptr[r] < ncomp[r] else "-") for r in sorted(stuck)}
        raise RuntimeError(f"lowered schedule can deadlock ({channels} comm channel(s)); stuck computes: {detail}")
