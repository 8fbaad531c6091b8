"""Runtime dependency checker (debug builds of the stage runner).

Enabled with ``MIPIPE_DEBUG=1`` (or ``PipelineRuntime(debug=True)``).  Every buffer a
compute action reads must have a recorded producer: a received message must have been
posted AND waited (its RCCL work joined into the compute stream) before it is read; a
message must be produced before it is sent; at the end of a step nothing may be left
posted-but-unread, produced-but-unsent, or handed-off-but-unconsumed.  Optionally
(``MIPIPE_DEBUG=2``) every activation / gradient crossing a stage boundary is checked
for NaN/Inf, naming the action that produced it.

The dependency's equivalents are runtime asserts in ``_PipelineScheduleRuntime``
(double recv, compute before recv: torch schedules.py:2095-2111, :2145-2150); here the
check is by message key, so it also covers distributed-head H/D traffic.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, Optional, Set

import torch


class DependencyError(RuntimeError):
    pass


def debug_level() -> int:
    try:
        return int(os.environ.get("MIPIPE_DEBUG", "0"))
    except ValueError:
        return 0


class DepTracker:
    def __init__(self, rank: int, level: int = 1):
        self.rank = rank
        self.level = level
        self.reset()

    def reset(self) -> None:
        self.posted: Set[tuple] = set()
        self.waited: Set[tuple] = set()
        self.consumed: Set[tuple] = set()
        self.produced: Dict[tuple, str] = {}

    # -------------------------------------------------------------- receives
    def on_post_recv(self, key: tuple) -> None:
        if key in self.posted:
            raise DependencyError(f"rank {self.rank}: receive {key} posted twice in one step")
        self.posted.add(key)

    def on_wait(self, key: tuple) -> None:
        if key not in self.posted:
            raise DependencyError(f"rank {self.rank}: waiting on {key} that was never posted")
        self.waited.add(key)

    def on_read(self, key: tuple, action) -> None:
        if key not in self.posted:
            raise DependencyError(f"rank {self.rank}: {action} reads {key} but no receive was posted")
        if key not in self.waited:
            raise DependencyError(f"rank {self.rank}: {action} reads {key} before its receive completed")
        if key in self.consumed and key[0] != "D":
            raise DependencyError(f"rank {self.rank}: {key} read twice")
        self.consumed.add(key)

    # -------------------------------------------------------------- sends
    def on_produce(self, key: tuple, action, tensors: Optional[Iterable[torch.Tensor]] = None) -> None:
        self.produced[key] = str(action)
        if self.level >= 2 and tensors is not None:
            for t in tensors:
                if t.is_floating_point() and not bool(torch.isfinite(t).all()):
                    raise DependencyError(f"rank {self.rank}: {action} produced non-finite values for {key}")

    def on_send(self, key: tuple, pending: Dict[tuple, object]) -> None:
        if key not in pending:
            raise DependencyError(f"rank {self.rank}: send of {key} posted before its producer ran")

    # -------------------------------------------------------------- step end
    def finish(self, pending_sends: Dict[tuple, object], handoff: Dict[tuple, object]) -> None:
        unread = self.posted - self.consumed
        if unread:
            raise DependencyError(f"rank {self.rank}: received but never read: {sorted(unread)[:6]}")
        if pending_sends:
            raise DependencyError(f"rank {self.rank}: produced but never sent: {sorted(pending_sends)[:6]}")
        if handoff:
            raise DependencyError(f"rank {self.rank}: same-rank hand-offs never consumed: {sorted(handoff)[:6]}")
        self.reset()
