"""Lowering: compute order -> executable per-rank program with grouped p2p.

RCCL (like NCCL) executes the point-to-point operations a rank posts on one
communicator strictly in order, and a send of a large message completes only when
the peer's matching receive runs.  A per-rank program is therefore safe only if
every pair of ranks posts its shared messages in one consistent order.  The
reference dependency reaches that with per-peer sorted batching
(schedules.py:508-532) and a topological SEND/RECV placement
(schedules.py:1223-1336).  Here the order is derived once, globally:

1. :func:`.simulate.simulate` times the compute order (F=1, B=2, p2p latency
   ``comm``), giving every message a send time stamp.
2. All messages are sorted by (time, src rank, dst rank, kind, stage, mb); each
   rank posts its own sends/receives in that global order.  A receive is posted
   no later than right before its consumer; a send right after its producer.
3. Comm ops posted at the same point form one :class:`~.ir.CommGroup`
   (one ``batch_isend_irecv`` = one RCCL group), so bidirectional traffic on a
   link (1F1B steady state, interleaved wrap-around P-1 -> 0) runs concurrently.
4. ``REDUCE_GRAD`` is placed right after each stage's last backward
   (schedules.py:1069-1099 semantics) so the DP all-reduce of that stage can
   overlap the rest of the flush.

:func:`.simulate.check_lowered` then proves the program cannot hang.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from .ir import MSG_OPS, Action, CommGroup, CommOp, Entry, Op
from .schedules import stage_to_rank
from .simulate import action_rank, check_lowered, head_ranks_of, in_messages, simulate, uses_split_backward


@dataclass
class Message:
    key: tuple            # (kind 'F'|'B'|'H'|'D', dst stage (or head rank), mb)
    src: int
    dst: int
    t: float
    producer: Action
    consumer: Action

    def order_key(self):
        kind, stage, mb = self.key
        return (self.t, self.src, self.dst, kind, stage, mb)


def lower(orders: Dict[int, Sequence[Optional[Action]]], pp: int, v: int = 1, style: str = "loop",
          comm: float = 0.05, add_reduce_grad: bool = True, check: bool = True,
          costs: Optional[Dict[Op, float]] = None, head_costs: Optional[Dict[int, float]] = None,
          stage_costs: Optional[Sequence[float]] = None) -> Dict[int, List[Entry]]:
    S = pp * v
    s2r = [stage_to_rank(s, pp, style) for s in range(S)]
    seq = {r: [a for a in orders.get(r, []) if a is not None and a.op.is_compute] for r in range(pp)}
    split = uses_split_backward(seq)
    head = head_ranks_of(seq)
    sim = simulate(seq, pp, v, style, comm_latency=comm, costs=costs, head_costs=head_costs,
                   stage_costs=stage_costs)

    # every cross-rank input of every compute is one message (same-rank inputs are
    # hand-offs); stamped with the producer's simulated end time
    msgs: List[Message] = []
    for r in range(pp):
        for a in seq[r]:
            for prod, key in in_messages(a, S, split, head):
                if key is None:
                    continue
                src = action_rank(prod, s2r)
                if src == r:
                    continue
                msgs.append(Message(key, src, r, sim.end[prod], prod, a))
    msgs.sort(key=Message.order_key)

    program: Dict[int, List[Entry]] = {}
    for r in range(pp):
        mine = [mm for mm in msgs if mm.src == r or mm.dst == r]
        # index of consumer compute for each recv / producer compute for each send
        pos = {a: i for i, a in enumerate(seq[r])}

        ops_ordered: List[Tuple[CommOp, int, bool]] = []  # (op, anchor compute idx, is_send)
        for mm in mine:
            kind, st, mb = mm.key
            send_op, recv_op = MSG_OPS[kind]
            if mm.src == r:
                act = Action(mm.producer.stage, send_op, mb)
                ops_ordered.append((CommOp(act, mm.dst, mm.key), pos[mm.producer], True))
            else:
                act = Action(st, recv_op, mb)
                ops_ordered.append((CommOp(act, mm.src, mm.key), pos[mm.consumer], False))

        # slot p = "posted right before compute p".  Walk the global order; each op goes
        # at max(previous op's slot, earliest allowed): sends after their producer,
        # receives as early as the order allows (RCCL streams wait on the compute
        # issued before a post, so early receives overlap the transfer with compute).
        n = len(ops_ordered)
        slots = []
        cur = 0
        for op, anchor, is_send in ops_ordered:
            earliest = anchor + 1 if is_send else 0
            s_ = max(cur, earliest)
            if not is_send and s_ > anchor:
                raise RuntimeError(f"rank {r}: cannot post {op} before its consumer (order conflict)")
            slots.append(s_)
            cur = s_
        # Group contiguous ops posted at the same point, but never put receives for two
        # different consumer computes in one group: a coalesced RCCL group completes as
        # a unit, so a compute waiting on it would also wait for the other transfers.
        entries: List[Entry] = []
        k = 0
        for p in range(len(seq[r]) + 1):
            grp: List[CommOp] = []
            grp_consumer = None
            while k < n and slots[k] == p:
                op, anchor, is_send = ops_ordered[k]
                if not is_send:
                    if grp_consumer is not None and anchor != grp_consumer:
                        entries.append(CommGroup(grp))
                        grp = []
                    grp_consumer = anchor
                grp.append(op)
                k += 1
            if grp:
                entries.append(CommGroup(grp))
            if p < len(seq[r]):
                entries.append(seq[r][p])
        program[r] = entries

    if add_reduce_grad:
        for r in range(pp):
            last_bwd: Dict[int, int] = {}
            for i, e in enumerate(program[r]):
                if isinstance(e, Action) and e.op in (Op.B, Op.W):
                    last_bwd[e.stage] = i
            # insert after the last backward and the comm groups that directly follow it
            # (its sends), in descending index order, so a blocking grad reduction can
            # never hold back the send its peer is waiting for
            for st, i in sorted(last_bwd.items(), key=lambda kv: -kv[1]):
                program[r].insert(_after_sends(program[r], i), Action(st, Op.REDUCE_GRAD))
    if check:
        check_lowered(program, S)
    return program


def _after_sends(prog: List[Entry], i: int) -> int:
    """Index right after entry ``i`` and the send-only comm groups that directly follow it
    (a collective placed there never holds back the send its peer waits for)."""
    j = i + 1
    while j < len(prog) and isinstance(prog[j], CommGroup) and all(op.action.op.is_send for op in prog[j].ops):
        j += 1
    return j


def add_head_reduce(program: Dict[int, List[Entry]], after_stage0: bool = False) -> Dict[int, List[Entry]]:
    """Insert ``rREDUCE_HEAD`` into every rank's program, right after the rank's last write
    to the replicated head arena -- its last ``H`` (with tied embeddings also stage 0's last
    backward, whose embedding gradient lands in the head arena) and the sends that follow
    it -- so the head-gradient reduction overlaps the rest of the flush.  Every rank of the
    pipeline issues exactly one (a collective of the whole group)."""
    out = {}
    for r, prog in program.items():
        last = -1
        for i, e in enumerate(prog):
            if isinstance(e, Action) and (e.op == Op.H or (after_stage0 and e.stage == 0 and
                                                            e.op in (Op.B, Op.I, Op.W))):
                last = i
        j = _after_sends(prog, last) if last >= 0 else len(prog)
        out[r] = list(prog[:j]) + [Action(r, Op.REDUCE_HEAD)] + list(prog[j:])
    return out


def defer_collectives(program: Dict[int, List[Entry]]) -> Dict[int, List[Entry]]:
    """Move every collective (``REDUCE_GRAD``, ``REDUCE_HEAD``) to the end of its rank's
    program, keeping their relative order: all point-to-point traffic of the step is
    issued before the first collective.  The safe placement when comm streams may share a
    hardware queue with compute (see :func:`.simulate.check_lowered` ``serial``)."""
    out = {}
    for r, prog in program.items():
        coll = [e for e in prog if isinstance(e, Action) and e.op.is_collective]
        out[r] = [e for e in prog if not (isinstance(e, Action) and e.op.is_collective)] + coll
    return out


def format_program(program: Dict[int, List[Entry]]) -> str:
    return "\n".join(f"rank {r}: " + " ".join(str(e) for e in program[r]) for r in sorted(program))
