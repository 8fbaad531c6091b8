"""Attention backward on a few shapes, for rocprofv3 per-kernel timing (dq vs dkdv,
causal vs full, sequence length).  python tools/attn_bwd_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe import ops  # noqa: E402

for (B, S, H, D, causal) in [(16, 1024, 12, 64, True), (16, 1024, 12, 64, False), (4, 4096, 12, 64, True),
                             (1, 8192, 32, 128, True)]:
    T = B * S
    qkv = torch.randn(T, 3 * H * D, device="cuda").to(torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    o = torch.empty(T, H * D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H * S, device="cuda")
    do = torch.randn_like(o)
    d = torch.empty_like(qkv)
    ops.attn_fwd(q, k, v, o, lse, B, S, S, H, H, D, causal)
    for _ in range(5):
        ops.attn_bwd(q, k, v, o, do, lse, d[:, :H * D], d[:, H * D:2 * H * D], d[:, 2 * H * D:], B, S, S, H, H, D,
                     causal)
    torch.cuda.synchronize()
print("ok")
