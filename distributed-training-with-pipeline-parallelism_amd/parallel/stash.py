"""Activation-stash slots: how many microbatches' forward activations a rank holds at once.

A stage keeps a microbatch's forward activations (its stash) from ``F(mb)`` to the last
action that reads them: ``B(mb)``, or ``W(mb)`` when the backward is split into input and
weight halves (ZBH1 / ZBV, the W half re-reads layer inputs).  With HIP graphs every
captured forward owns the memory it allocates, so without a plan a rank would hold the
stash of ALL m microbatches whatever the schedule.  The plan replays the rank's compute
order and gives each forward the lowest free slot of its stage; the graphs of all
microbatches sharing a slot capture into ONE memory pool (parallel/graphs.py), and the
slot's previous occupant releases its stash references once its last reader is captured,
so the pool hands the same blocks to the next occupant: a rank holds ``slots`` stashes
per stage -- 1F1B's ``P - s`` (+1 for the steady-state forward issued before its
backward), GPipe's ``m`` -- as the schedule intends (SURVEY D2 "activation stash in a slot
ring"; torch's Schedule1F1B warmup ``min(m, P - s)``, schedules.py:873-876).

Microbatch lanes: microbatch ``mb`` runs on lane ``mb % lanes``; a slot is never shared
across lanes (its occupants' graphs then replay in order on ONE stream, so a forward can
never overwrite a stash a backward on another stream is still reading).
"""
from __future__ import annotations

import heapq
from collections import defaultdict
from typing import Dict, Iterable, Optional, Sequence, Tuple

from .ir import Action, Op


def plan_stash_slots(order: Sequence[Optional[Action]], stages: Iterable[int], lanes: int = 1
                     ) -> Tuple[Dict[Tuple[int, int], Tuple[int, int]], Dict[Tuple[int, int], str],
                                Dict[Tuple[int, int], int]]:
    """Slot of every (stage, mb) forward in ``order`` (one rank's compute order).

    Returns ``(slot, last, count)``: ``slot[(stage, mb)] = (lane, index)``; ``last[(stage,
    mb)]`` = the op name ("B" / "I" / "W") of the stash's last reader; ``count[(stage,
    lane)]`` = slots that lane of that stage uses (its peak of stashes alive)."""
    stages = set(stages)
    lanes = max(1, int(lanes))
    last_i: Dict[Tuple[int, int], int] = {}
    for i, a in enumerate(order):
        if a is not None and a.stage in stages and a.op in (Op.B, Op.I, Op.W):
            last_i[(a.stage, a.mb)] = i
    free: Dict[Tuple[int, int], list] = defaultdict(list)
    count: Dict[Tuple[int, int], int] = defaultdict(int)
    slot: Dict[Tuple[int, int], Tuple[int, int]] = {}
    last: Dict[Tuple[int, int], str] = {}
    for i, a in enumerate(order):
        if a is None or a.stage not in stages or a.mb is None:
            continue
        key = (a.stage, a.mb)
        cls = (a.stage, a.mb % lanes)
        if a.op == Op.F and key not in slot:
            k = heapq.heappop(free[cls]) if free[cls] else count[cls]
            if k == count[cls]:
                count[cls] += 1
            slot[key] = (a.mb % lanes, k)
        if last_i.get(key) == i and key in slot:
            last[key] = a.op.value
            heapq.heappush(free[cls], slot[key][1])
    return slot, last, dict(count)


def stash_slots_per_stage(order: Sequence[Optional[Action]], stages: Iterable[int], lanes: int = 1) -> Dict[int, int]:
    """Stashes a stage holds at its peak under the slot plan (summed over lanes)."""
    _, _, count = plan_stash_slots(order, stages, lanes)
    out: Dict[int, int] = defaultdict(int)
    for (s, _), n in count.items():
        out[s] += n
    return dict(out)
