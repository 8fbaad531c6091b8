"""Static checks of a compute schedule (parity with torch schedules.py:1339-1459).

* every stage runs exactly ``m`` forwards and ``m`` backwards (``B``, or ``I`` + ``W``);
* per microbatch, ``F`` precedes its backward and ``I`` precedes ``W`` on the rank;
* every action sits on the rank the placement assigns to its stage;
* no action appears twice;
* distributed-head actions ``rH m`` sit on rank r, and each head rank runs every
  microbatch's chunk exactly once, in microbatch order.
"""
from __future__ import annotations

from collections import Counter
from typing import Dict, Optional, Sequence

from .ir import Action, Op
from .schedules import stage_to_rank


class ScheduleError(ValueError):
    pass


def validate(orders: Dict[int, Sequence[Optional[Action]]], pp: int, v: int, m: int, style: str = "loop") -> None:
    S = pp * v
    seen = Counter()
    for r, seq in orders.items():
        pos: Dict[Action, int] = {}
        for i, a in enumerate(seq):
            if a is None or not a.op.is_compute:
                continue
            if a.op == Op.H:
                if a.stage != r:
                    raise ScheduleError(f"rank {r}: head chunk {a} belongs to rank {a.stage}")
                if a.mb is None or not 0 <= a.mb < m:
                    raise ScheduleError(f"rank {r}: {a} microbatch out of range")
                if a in pos:
                    raise ScheduleError(f"rank {r}: {a} scheduled twice")
                pos[a] = i
                seen[("H", r)] += 1
                continue
            if not 0 <= a.stage < S:
                raise ScheduleError(f"rank {r}: stage {a.stage} out of range")
            if stage_to_rank(a.stage, pp, style) != r:
                raise ScheduleError(f"rank {r}: {a} belongs to rank {stage_to_rank(a.stage, pp, style)}")
            if a.mb is None or not 0 <= a.mb < m:
                raise ScheduleError(f"rank {r}: {a} microbatch out of range")
            if a in pos:
                raise ScheduleError(f"rank {r}: {a} scheduled twice")
            pos[a] = i
            seen[(a.stage, a.op)] += 1
        for a, i in pos.items():
            if a.op in (Op.B, Op.I):
                f = Action(a.stage, Op.F, a.mb)
                if f not in pos or pos[f] > i:
                    raise ScheduleError(f"rank {r}: {a} before its forward")
            if a.op == Op.W:
                ib = Action(a.stage, Op.I, a.mb)
                if ib not in pos or pos[ib] > i:
                    raise ScheduleError(f"rank {r}: {a} before its input-grad backward")
    for r, seq in orders.items():
        hs = [a.mb for a in seq if a is not None and a.op == Op.H]
        if hs and (len(hs) != m or hs != sorted(hs)):
            raise ScheduleError(f"rank {r}: head chunks {hs} must cover all {m} microbatches in order")
    for s in range(S):
        if seen[(s, Op.F)] != m:
            raise ScheduleError(f"stage {s}: {seen[(s, Op.F)]} forwards, expected {m}")
        nb, ni, nw = seen[(s, Op.B)], seen[(s, Op.I)], seen[(s, Op.W)]
        if not ((nb == m and ni == nw == 0) or (nb == 0 and ni == nw == m)):
            raise ScheduleError(f"stage {s}: backward counts B={nb} I={ni} W={nw}, expected m={m}")
