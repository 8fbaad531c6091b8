"""Attention forward / backward on the reference model's shape (B 8, S 128, H 8, D 96,
full) with and without dropout 0.1: the cost of regenerating the mask in-kernel.

    python tools/attn_drop_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe import ops  # noqa: E402


def t(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for (B, S, H, D, causal) in [(8, 128, 8, 96, False), (16, 1024, 12, 64, True)]:
    T = B * S
    qkv = torch.randn(T, 3 * H * D, device="cuda").to(torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(T, H * D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device="cuda")
    do = torch.randn_like(o)
    d = torch.empty_like(qkv)
    for p in (0.0, 0.1):
        f = t(lambda: ops.attn_fwd(q, k, v, o, lse, B, S, S, H, H, D, causal, p_drop=p, seed=7))
        b = t(lambda: ops.attn_bwd(q, k, v, o, do, lse, d[:, :H * D], d[:, H * D:2 * H * D], d[:, 2 * H * D:], B, S, S,
                                   H, H, D, causal, p_drop=p, seed=7))
        print(f"B{B} S{S} H{H} D{D} causal={causal} p={p}: fwd {f:.1f} us, bwd {b:.1f} us", flush=True)
