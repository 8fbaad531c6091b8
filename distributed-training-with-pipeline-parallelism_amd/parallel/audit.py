"""Cross-rank audit of the communication a step actually issued.

The lowered program is proven hang-free before it runs (``simulate.check_lowered``), but
the proof covers the program's p2p and its placed collectives only.  Some collectives are
issued from other places: the clip-norm sum, the head reductions and the tied-embedding
sum.  On the first step every rank therefore logs what it issues: each grouped p2p post
(channel, peers, sizes) and each collective (group members, op, size).  The logs are
exchanged over the gloo control group and checked against the two rules that keep RCCL
from hanging:

* **p2p**: on every channel, the sends from rank a to rank b, in a's issue order, must equal
  the receives at b from a, in b's issue order (count, sizes, dtypes).  RCCL matches a
  pair's p2p operations on one communicator in order.
* **collectives**: every member of a group must issue the same sequence of collectives on
  it (op, size, dtype).

A mismatch raises before the step that would hang runs again, naming the first divergence.
This is the runtime counterpart of torch's schedule validation and its "recv twice" /
"compute before recv" asserts (torch:distributed/pipelining/schedules.py:2095-2111,
:2145-2150).
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, List, Sequence, Tuple

import torch


class CommAudit:
    """One rank's log of issued communication (entries are plain tuples: picklable)."""

    def __init__(self, rank: int):
        self.rank = rank
        self.entries: List[tuple] = []

    @staticmethod
    def _desc(t: torch.Tensor) -> Tuple[int, str]:
        return int(t.numel()), str(t.dtype).replace("torch.", "")

    def p2p(self, channel: int, sends: Sequence[Tuple[torch.Tensor, int]],
            recvs: Sequence[Tuple[torch.Tensor, int]]) -> None:
        """One grouped post; peers are GLOBAL ranks."""
        self.entries.append(("p2p", int(channel), tuple((int(p),) + self._desc(t) for t, p in sends),
                             tuple((int(p),) + self._desc(t) for t, p in recvs)))

    def coll(self, scope: str, members: Sequence[int], op: str, t: torch.Tensor) -> None:
        self.entries.append(("coll", scope, tuple(int(m) for m in members), op) + self._desc(t))


def check(logs: Dict[int, List[tuple]], limit: int = 5) -> List[str]:
    """Problems found in the gathered logs (global rank -> entries); [] if consistent."""
    problems: List[str] = []
    sends: Dict[tuple, list] = defaultdict(list)
    recvs: Dict[tuple, list] = defaultdict(list)
    colls: Dict[tuple, Dict[int, list]] = defaultdict(lambda: defaultdict(list))
    for r, entries in logs.items():
        for e in entries:
            if e[0] == "p2p":
                _, ch, ss, rr = e
                for peer, n, dt in ss:
                    sends[(r, peer, ch)].append((n, dt))
                for peer, n, dt in rr:
                    recvs[(peer, r, ch)].append((n, dt))
            elif e[0] == "coll":
                _, scope, members, op, n, dt = e
                colls[(scope, members)][r].append((op, n, dt))
    for key in sorted(set(sends) | set(recvs)):
        a, b, ch = key
        s, q = sends.get(key, []), recvs.get(key, [])
        if s != q:
            i = next((k for k in range(min(len(s), len(q))) if s[k] != q[k]), min(len(s), len(q)))
            problems.append(f"p2p {a}->{b} channel {ch}: {len(s)} sends vs {len(q)} receives; first difference "
                            f"at #{i}: send {s[i] if i < len(s) else None} / recv {q[i] if i < len(q) else None}")
    for (scope, members), per in sorted(colls.items()):
        missing = [m for m in members if m not in per]
        seqs = {m: per.get(m, []) for m in members}
        ref_rank = min(per)
        ref = per[ref_rank]
        for m, seq in seqs.items():
            if m in missing and ref:
                problems.append(f"{scope} collectives over {list(members)}: rank {m} issued none, "
                                f"rank {ref_rank} issued {len(ref)}")
            elif seq != ref:
                i = next((k for k in range(min(len(seq), len(ref))) if seq[k] != ref[k]), min(len(seq), len(ref)))
                problems.append(f"{scope} collectives over {list(members)}: rank {m} differs from rank {ref_rank} "
                                f"at #{i}: {seq[i] if i < len(seq) else None} vs {ref[i] if i < len(ref) else None}")
    return problems[:limit] if limit else problems


def gather_and_check(audit: CommAudit, group=None) -> Tuple[bool, List[str], int]:
    """all_gather_object the logs over ``group`` (gloo: host objects) and check them on every
    rank.  Returns (consistent, problems, entries on this rank)."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if group is not None else dist.get_world_size()
    allv: List = [None] * world
    dist.all_gather_object(allv, (audit.rank, audit.entries), group=group)
    logs = {r: e for r, e in allv}
    problems = check(logs)
    return not problems, problems, len(audit.entries)
