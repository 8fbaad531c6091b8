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
    costs = {**DEFAULT_COSTS, **(costs or {})}
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
    gradients back up (B, D) -- one RCCL communicator + stream each (csrc/comm/rccl_engine.h)."""
    return 0 if key[0] in ("F", "H") else 1


def check_lowered(program: Dict[int, List[Entry]], num_stages: int, channels: int = 1, serial: bool = False,
                  dp: int = 1, lanes: int = 1, recv_early: bool = False) -> None:
    """Raise RuntimeError if the lowered program can hang under RCCL semantics.

    Queues of a rank (each a FIFO in host issue order = program order):

    * independent model (``serial=False``, every stream on a hardware queue of its own):
      one compute queue; ``channels`` p2p queues (``channels=2``: each CommGroup is split
      by :func:`message_channel`, one part per direction stream, as the native engine posts
      it); one collective queue (``REDUCE_GRAD`` with ``dp > 1`` -- the stage's DP
      all-reduce -- and ``REDUCE_HEAD`` -- the pipeline-wide head reduction);
    * serial model (``serial=True``): ONE queue holding every entry -- the worst case of
      hardware-queue sharing (GPU_MAX_HW_QUEUES streams per priority, a blocked RCCL kernel
      holds its queue).  Any real stream -> queue mapping only removes ordering edges from
      this model, so a program proven here cannot hang whatever the mapping.

    Rules: an entry starts when it is at the head of its queue and the previous entry of
    the queue has COMPLETED; a comm group or collective also waits for every compute
    issued before it (the engine orders its stream after the compute stream); a compute
    waits for the groups carrying its inputs (stream-event waits).  A compute completes
    when it starts; a p2p group when every message in it has both endpoint groups started;
    a collective when every member has started it (``REDUCE_HEAD``: every rank of the
    program; ``REDUCE_GRAD``: the same stage of the DP replicas, which run this program
    symmetrically).  A fixpoint that does not drain every queue means a possible hang.

    ``lanes`` (independent model): microbatch lanes (PipelineRuntime.set_lanes) -- the
    compute of microbatch mb is a FIFO of its own per lane ``mb % lanes`` (the lane streams
    have hardware queues of their own, probed); a comm group or collective still waits for
    every compute issued before it (the runtime orders a post after the lanes whose output
    it sends, a reduction after all of them).  Splitting the compute FIFO only removes
    ordering edges, so a program proven with ``lanes=1`` is safe with any lane count; the
    parameter lets the runtime prove the exact program it runs.

    ``recv_early`` (independent model): a channel part of a comm group that only RECEIVES does
    not wait for the compute issued before it -- the native stage runner orders such a post
    after the start of the step instead (RcclEngine::post_raw ``after``), so
    it starts at post time; it still waits for the entries before it on its channel queue."""
    comp_orders = {r: [e for e in es if isinstance(e, Action) and e.op.is_compute] for r, es in program.items()}
    split = uses_split_backward(comp_orders)
    head = head_ranks_of(comp_orders)
    ranks = sorted(program)
    chan = (lambda key: 0) if channels <= 1 else message_channel
    # items per rank: (queue, kind, payload, index of the last compute issued before it)
    #   kind 'c': compute Action; 'g': list of CommOps; 'x': collective key
    items: Dict[int, List[Tuple[object, str, object, int]]] = {}
    for r in ranks:
        lst = []
        ncomp = 0
        for e in program[r]:
            if isinstance(e, CommGroup):
                by_ch: Dict[int, List] = {}
                for op in e.ops:
                    by_ch.setdefault(chan(op.key), []).append(op)
                for ch in sorted(by_ch):
                    only_recv = all(op.action.op.is_recv for op in by_ch[ch])
                    lst.append((0 if serial else ("p", ch), "g", by_ch[ch],
                                -1 if (recv_early and not serial and only_recv) else ncomp - 1))
            elif e.op.is_compute:
                cq = "c" if (lanes <= 1 or e.mb is None) else ("c", e.mb % lanes)
                lst.append((0 if serial else cq, "c", e, ncomp - 1))
                ncomp += 1
            elif e.op == Op.REDUCE_HEAD:
                lst.append((0 if serial else "x", "x", ("RH",), ncomp - 1))
            elif e.op == Op.REDUCE_GRAD and dp > 1:
                lst.append((0 if serial else "x", "x", ("RG", e.stage, r), ncomp - 1))
        items[r] = lst
    # message -> the (rank, item) endpoints; collective key -> members
    msg_items: Dict[tuple, List[Tuple[int, int]]] = {}
    recv_item_of: Dict[tuple, Tuple[int, int]] = {}
    coll_items: Dict[tuple, List[Tuple[int, int]]] = {}
    comp_index: Dict[Tuple[int, int], int] = {}
    for r in ranks:
        ci = 0
        for ii, (q, kind, pl, _) in enumerate(items[r]):
            if kind == "g":
                for op in pl:
                    msg_items.setdefault(op.key, []).append((r, ii))
                    if op.action.op.is_recv:
                        recv_item_of[(r,) + op.key] = (r, ii)
            elif kind == "x":
                coll_items.setdefault(pl, []).append((r, ii))
            else:
                comp_index[(r, ci)] = ii
                ci += 1
    for k, gs in msg_items.items():
        if len(gs) != 2:
            raise RuntimeError(f"message {k} has {len(gs)} endpoints (expected send+recv)")
    n_rh = len(coll_items.get(("RH",), []))
    if n_rh and n_rh != len(ranks):
        raise RuntimeError(f"REDUCE_HEAD issued by {n_rh} of {len(ranks)} ranks")
    waits: Dict[Tuple[int, int], List[Tuple[int, int]]] = {}
    for r in ranks:
        for ii, (q, kind, pl, _) in enumerate(items[r]):
            if kind == "c":
                waits[(r, ii)] = [recv_item_of[(r,) + key] for _, key in in_messages(pl, num_stages, split, head)
                                  if key is not None and (r,) + key in recv_item_of]
    queues: Dict[Tuple[int, object], List[int]] = {}
    for r in ranks:
        for ii, (q, _, _, _) in enumerate(items[r]):
            queues.setdefault((r, q), []).append(ii)
    started: Dict[Tuple[int, int], bool] = {}
    done: Dict[Tuple[int, int], bool] = {}
    qptr = {q: 0 for q in queues}
    changed = True
    while changed:
        changed = False
        for q, lst in queues.items():
            r = q[0]
            while qptr[q] < len(lst) and done.get((r, lst[qptr[q]]), False):
                qptr[q] += 1
                changed = True
            if qptr[q] >= len(lst):
                continue
            ii = lst[qptr[q]]
            if (r, ii) in started:
                continue
            _, kind, pl, last_c = items[r][ii]
            if kind == "c":
                ok = all(done.get(g, False) for g in waits[(r, ii)])
            else:
                ok = last_c < 0 or done.get((r, comp_index[(r, last_c)]), False)
            if ok:
                started[(r, ii)] = True
                if kind == "c":
                    done[(r, ii)] = True
                changed = True
        for (r, ii) in list(started):
            if done.get((r, ii)):
                continue
            _, kind, pl, _ = items[r][ii]
            if kind == "g":
                fin = all(all(started.get(x, False) for x in msg_items[op.key]) for op in pl)
            else:
                fin = all(started.get(x, False) for x in coll_items[pl])
            if fin:
                done[(r, ii)] = True
                changed = True
    stuck = sorted({q[0] for q, lst in queues.items() if qptr[q] < len(lst)})
    if stuck:
        detail = {}
        for r in stuck:
            heads = [str(items[r][lst[qptr[q]]][2]) for q, lst in queues.items() if q[0] == r and qptr[q] < len(lst)]
            detail[r] = heads
        model = "serial (one queue per rank)" if serial else f"{channels} comm channel(s)"
        raise RuntimeError(f"lowered schedule can deadlock ({model}); stuck queue heads: {detail}")
