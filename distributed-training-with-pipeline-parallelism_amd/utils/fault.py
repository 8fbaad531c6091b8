"""Fault injection for the hang-detection tests.

``MIPIPE_FAULT_STALL="rank:step[:attempt]"`` makes that rank block forever at the start of
that training step (only in that benchmark attempt, if given) -- a stand-in for a peer that
stops answering.  The watchdog (utils/metrics.py) must turn it into a diagnosable non-zero
exit, and bench.py's supervisor into a retry.  Unset: no effect, no cost.
"""
from __future__ import annotations

import os
import time


def _spec():
    s = os.environ.get("MIPIPE_FAULT_STALL", "")
    if not s:
        return None
    parts = [int(x) for x in s.split(":")]
    return parts[0], parts[1], (parts[2] if len(parts) > 2 else None)


def maybe_stall(rank: int, step: int, attempt: int = 0) -> None:
    sp = _spec()
    if sp is None:
        return
    r, st, att = sp
    if r == rank and st == step and (att is None or att == attempt):
        while True:        # a hung rank: never returns (the watchdog ends the process)
            time.sleep(3600)
