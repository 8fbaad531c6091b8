"""How far is the short-sequence attention (the reference's shape: B 8, S 128, H 8, d 96,
non-causal, bf16) from the latency floor of ANY kernel that touches its bytes?  Times, per
launch over 500 back-to-back launches on one stream: our attention forward and backward,
a 1-element fill (launch floor), a copy of q -> o (the output bytes), q + k -> o (two
reads and a write of the same sizes), and one graph-replayed forward (launch overhead
removed).  python tools/probes/attn_short_floor.py"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.ops import kernels as K  # noqa: E402

B, S, H, D = 8, 128, 8, 96
T = B * S
dev = "cuda"
qkv = torch.randn(T, 3 * H * D, device=dev, dtype=torch.bfloat16)
q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
o = torch.empty(T, H * D, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B * H * S, device=dev, dtype=torch.float32)
do = torch.randn_like(o)
dqkv = torch.empty_like(qkv)
dq, dk, dv = dqkv[:, :H * D], dqkv[:, H * D:2 * H * D], dqkv[:, 2 * H * D:]
one = torch.empty(1, device=dev)
qc, kc = q.contiguous(), k.contiguous()


def t(fn, it=500):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


fwd = lambda: K.attn_fwd(q, k, v, o, lse, B, S, S, H, H, D, False)   # noqa: E731
fwd()
bwd = lambda: K.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, S, S, H, H, D, False)   # noqa: E731
g = torch.cuda.CUDAGraph()
st = torch.cuda.Stream()
st.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(st):
    for _ in range(3):
        fwd()
    torch.cuda.synchronize()
    g.capture_begin()
    for _ in range(10):
        fwd()
    g.capture_end()
torch.cuda.synchronize()
fl_f = 4.0 * B * H * S * S * D
res = {}
for rep in range(2):
    for name, fn, n in (("attn fwd", fwd, 1), ("attn bwd", bwd, 1), ("fill 1 elem", lambda: one.fill_(1.0), 1),
                        ("copy q->o", lambda: o.copy_(qc), 1), ("q+k->o", lambda: torch.add(qc, kc, out=o), 1),
                        ("attn fwd x10 in one graph", g.replay, 10)):
        us = t(fn) / n
        res[name] = min(res.get(name, 1e9), us)
for name, us in res.items():
    extra = ""
    if name.startswith("attn fwd"):
        extra = f"  {fl_f / us / 1e6:.0f} TF"
    if name == "attn bwd":
        extra = f"  {2.5 * fl_f / us / 1e6:.0f} TF"
    print(f"{name:28s} {us:7.2f} us{extra}", flush=True)
