"""Measured pipeline timelines: Chrome traces and bubble accounting.

The runtime (``profile=True``) brackets every compute action with HIP events on the
compute stream; this module turns those intervals into a Chrome trace (one process per
rank) and into the bubble fraction ``1 - busy / step`` that is compared with the
analytic ``(P-1)/(v*m+P-1)``."""
from __future__ import annotations

import json
from typing import Dict, List, Sequence, Tuple

Interval = Tuple[str, float, float]  # (action, start_ms, end_ms)


def timeline_to_chrome(timeline: Sequence[Interval], path: str, rank: int = 0) -> None:
    ev = [{"name": a, "ph": "X", "pid": rank, "tid": 0, "ts": s * 1000.0, "dur": (e - s) * 1000.0,
           "cat": "F" if "F" in a else "B"} for a, s, e in timeline]
    with open(path, "w") as f:
        json.dump({"traceEvents": ev, "displayTimeUnit": "ms"}, f)


def merge_chrome(paths: Sequence[str], out: str) -> None:
    evs = []
    for p in paths:
        with open(p) as f:
            evs += json.load(f)["traceEvents"]
    with open(out, "w") as f:
        json.dump({"traceEvents": evs, "displayTimeUnit": "ms"}, f)


def bubble_fraction(timelines: Dict[int, Sequence[Interval]], step_ms: Dict[int, float]) -> float:
    """Pipeline-wide bubble: 1 - sum(busy) / (ranks * max step time)."""
    if not timelines:
        return float("nan")
    span = max(step_ms.values())
    busy = sum(sum(e - s for _, s, e in tl) for tl in timelines.values())
    return max(0.0, 1.0 - busy / (len(timelines) * span))


def summarize(timeline: Sequence[Interval]) -> Dict[str, float]:
    out: Dict[str, List[float]] = {}
    for a, s, e in timeline:
        kind = "F" if "F" in a and "REDUCE" not in a else ("W" if a.rstrip("0123456789").endswith("W") else "B")
        out.setdefault(kind, []).append(e - s)
    return {k: sum(v) / len(v) for k, v in out.items()}
