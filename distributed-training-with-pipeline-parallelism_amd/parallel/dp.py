"""Data parallelism across pipeline replicas (DP x PP).

The reference has no DP; BASELINE config 5 needs it.  Each
pipeline stage all-reduces its gradients with the same stage of the other
replicas right at the stage's REDUCE_GRAD action (after its last backward), so
the all-reduce of late stages overlaps the flush of earlier ones.

Native stages keep every gradient in one flat fp32 buffer, so the all-reduce is
issued on contiguous bucket views (no pack/unpack copies).  Bucket size is
chosen for point-to-point xGMI: a ring between DP peers is bound by one link
(~153 GB/s), so a few large buckets (default 256 MiB) amortise launch latency
while still letting the first bucket start before the last grads are final.
For ``nn.Module`` stages (autograd path) grads are packed into flat buckets.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 256 << 20


class _Multi:
    def __init__(self, works, finish=None):
        self.works = works
        self.finish = finish

    def wait(self):
        for w in self.works:
            w.wait()
        if self.finish is not None:
            self.finish()
            self.finish = None
        return True


def allreduce_flat(flat: torch.Tensor, group, bucket_bytes: int = DEFAULT_BUCKET_BYTES, average: bool = True):
    """Async all-reduce of a flat buffer in contiguous bucket views."""
    n = flat.numel()
    per = max(1, bucket_bytes // flat.element_size())
    works = []
    ws = dist.get_world_size(group)
    for i in range(0, n, per):
        view = flat[i: i + per]
        if average and ws > 1:
            view.div_(ws)
        works.append(dist.all_reduce(view, group=group, async_op=True))
    return _Multi(works)


def allreduce_module_grads(module: torch.nn.Module, group, bucket_bytes: int = DEFAULT_BUCKET_BYTES):
    grads = [p.grad for p in module.parameters() if p.grad is not None]
    if not grads:
        return None
    ws = dist.get_world_size(group)
    buckets: List[List[torch.Tensor]] = [[]]
    size = 0
    for g in grads:
        if size and size + g.numel() * g.element_size() > bucket_bytes:
            buckets.append([])
            size = 0
        buckets[-1].append(g)
        size += g.numel() * g.element_size()
    works, packs = [], []
    for b in buckets:
        flat = torch.cat([g.reshape(-1) for g in b]).div_(ws)
        packs.append((flat, b))
        works.append(dist.all_reduce(flat, group=group, async_op=True))

    def finish():
        for flat, b in packs:
            off = 0
            for g in b:
                g.copy_(flat[off: off + g.numel()].view_as(g))
                off += g.numel()

    return _Multi(works, finish)
