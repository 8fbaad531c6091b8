"""Pipeline schedule IR.

An :class:`Action` is one unit of work a rank executes for one (virtual) stage and
one microbatch: a forward (``F``), a full backward (``B``), a split backward
(input-grad ``I`` / weight-grad ``W``), a point-to-point transfer (``SEND_F``,
``RECV_F``, ``SEND_B``, ``RECV_B``) or a per-stage gradient reduction
(``REDUCE_GRAD``).  The string form matches the reference dependency's
(``"2F0"``, ``"1SEND_B3"``, ``"0REDUCE_GRAD"``; torch pipelining
schedules.py:44-215) so schedules can be compared and dumped to CSV/JSON.

Unlike the reference dependency, communication is not a per-op property that the
executor discovers at run time: the lowering pass (:mod:`.lower`) groups comm
actions into :class:`CommGroup` entries whose per-peer order is globally
consistent, which is what RCCL's in-order per-communicator semantics require.
"""
from __future__ import annotations

import enum
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Union


class Op(enum.Enum):
    F = "F"
    B = "B"           # full backward (input + weight grads)
    I = "I"           # backward, input grads only
    W = "W"           # backward, weight grads only
    SEND_F = "SEND_F"
    RECV_F = "RECV_F"
    SEND_B = "SEND_B"
    RECV_B = "RECV_B"
    REDUCE_GRAD = "REDUCE_GRAD"
    # distributed LM head: ``rREDUCE_HEAD`` = rank r issues the reduction of the replicated
    # head's gradient (reduce-scatter over the pipeline, then all-reduce of its shard over
    # DP) -- a collective of the whole pipeline group, placed by :func:`.lower.add_head_reduce`
    REDUCE_HEAD = "REDUCE_HEAD"
    # distributed LM head (see :mod:`.headsplit`): ``rH m`` = rank r's token chunk of
    # microbatch m through the head + loss (fwd and bwd fused); the last stage sends the
    # chunk's final hidden states (SEND_H) and receives its input gradient (RECV_D)
    H = "H"
    SEND_H = "SEND_H"
    RECV_H = "RECV_H"
    SEND_D = "SEND_D"
    RECV_D = "RECV_D"

    @property
    def is_compute(self) -> bool:
        return self in (Op.F, Op.B, Op.I, Op.W, Op.H)

    @property
    def is_collective(self) -> bool:
        return self in (Op.REDUCE_GRAD, Op.REDUCE_HEAD)

    @property
    def is_comm(self) -> bool:
        return self.is_send or self.is_recv

    @property
    def is_send(self) -> bool:
        return self in (Op.SEND_F, Op.SEND_B, Op.SEND_H, Op.SEND_D)

    @property
    def is_recv(self) -> bool:
        return self in (Op.RECV_F, Op.RECV_B, Op.RECV_H, Op.RECV_D)


# message kind -> (send op, recv op)
MSG_OPS = {"F": (Op.SEND_F, Op.RECV_F), "B": (Op.SEND_B, Op.RECV_B), "H": (Op.SEND_H, Op.RECV_H),
           "D": (Op.SEND_D, Op.RECV_D)}

_ACTION_RE = re.compile(r"^(\d+)(SEND_F|RECV_F|SEND_B|RECV_B|SEND_H|RECV_H|SEND_D|RECV_D|REDUCE_GRAD|REDUCE_HEAD|F|B|I|W|H)(\d*)$")


@dataclass(frozen=True)
class Action:
    stage: int
    op: Op
    mb: Optional[int] = None

    def __str__(self) -> str:
        return f"{self.stage}{self.op.value}{'' if self.mb is None else self.mb}"

    __repr__ = __str__

    @staticmethod
    def parse(s: str) -> "Action":
        m = _ACTION_RE.match(s.strip())
        if not m:
            raise ValueError(f"cannot parse action {s!r}")
        stage, op, mb = m.groups()
        return Action(int(stage), Op(op), int(mb) if mb != "" else None)


@dataclass
class CommOp:
    """One half of a point-to-point transfer as seen by one rank."""
    action: Action          # SEND_F / RECV_F / SEND_B / RECV_B
    peer: int               # peer rank
    key: tuple              # global message key, identical on sender and receiver

    def __str__(self) -> str:
        return f"{self.action}@{self.peer}"


@dataclass
class CommGroup:
    """A batch of comm ops issued together (one ``batch_isend_irecv`` / RCCL group)."""
    ops: List[CommOp]

    def __str__(self) -> str:
        return "{" + " ".join(str(o) for o in self.ops) + "}"

    __repr__ = __str__


Entry = Union[Action, CommGroup]


def format_compute_grid(per_rank: Dict[int, Sequence[Optional[Action]]], error_step: Optional[int] = None,
                        error_rank: Optional[int] = None) -> str:
    """Step x rank grid like the dependency's pretty printer (schedules.py:222-282).

    ``None`` entries are bubbles.  When ``error_step``/``error_rank`` are given the
    failing cell is marked (failure reporting).
    """
    ranks = sorted(per_rank)
    n = max((len(v) for v in per_rank.values()), default=0)
    width = max([6] + [len(str(a)) + 2 for v in per_rank.values() for a in v if a is not None])
    lines = ["        " + "".join(f"Rank {r}".ljust(width) for r in ranks)]
    for i in range(n):
        cells = []
        for r in ranks:
            a = per_rank[r][i] if i < len(per_rank[r]) else None
            txt = "" if a is None else str(a)
            if error_step == i and error_rank == r:
                txt += " <-- ERROR HERE"
            cells.append(txt.ljust(width))
        lines.append(f"Step {i:02d}: " + "".join(cells))
    return "\n".join(lines)


def to_csv(per_rank: Dict[int, Sequence[Optional[Action]]]) -> str:
    """One row per rank, comma-separated action strings (blank = bubble)."""
    return "\n".join(",".join("" if a is None else str(a) for a in per_rank[r]) for r in sorted(per_rank))


def from_csv(text: str) -> Dict[int, List[Optional[Action]]]:
    out: Dict[int, List[Optional[Action]]] = {}
    for r, line in enumerate(l for l in text.splitlines() if l.strip()):
        out[r] = [Action.parse(c) if c.strip() else None for c in line.split(",")]
    return out
