"""Time the fused norm backward on the GPT-2 / Llama shapes (LayerNorm + dres + bias-grad
colsums as used by GPT-2's residual points; RMSNorm at D=4096)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe import ops  # noqa: E402


def t(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


TOK = int(os.environ.get("NORM_PROBE_T", "16384"))
for kind, T, D, cols in [("layernorm", TOK, 768, True), ("layernorm", TOK, 768, False), ("rmsnorm", 8192, 4096, False)]:
    dy = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    s_ = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    dres = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    w = torch.randn(D, device="cuda").to(torch.bfloat16)
    mean, rstd = torch.zeros(T, device="cuda"), torch.ones(T, device="cuda")
    dw = torch.zeros(D, device="cuda")
    db = torch.zeros(D, device="cuda") if kind == "layernorm" else None
    c1 = torch.zeros(D, device="cuda") if cols else None
    c2 = torch.zeros(D, device="cuda") if cols else None
    ds = torch.empty_like(dy)
    us = t(lambda: ops.norm_bwd(dy, s_, w, mean, rstd, kind, dres=dres, dw=dw, dbias=db, ds=ds, colsum_dres=c1,
                                colsum_ds=c2))
    nbytes = 4 * T * D * 2
    print(f"norm_bwd {kind} {T}x{D} cols={cols}: {us:.1f} us, {nbytes / us / 1e6:.2f} TB/s", flush=True)

for T, D in [(16384, 768), (1024, 768), (8192, 3072), (1024, 2048)]:
    x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    db = torch.zeros(D, device="cuda")
    us = t(lambda: ops.colsum(x, db))
    print(f"colsum {T}x{D}: {us:.1f} us, {T * D * 2 / us / 1e6:.2f} TB/s", flush=True)

for T, D, branch in [(16384, 768, True), (16384, 768, False), (8192, 4096, True), (1024, 768, True)]:
    x = torch.randn(T, D, device="cuda").to(torch.bfloat16)
    br = torch.randn(T, D, device="cuda").to(torch.bfloat16) if branch else None
    w = torch.randn(D, device="cuda").to(torch.bfloat16)
    b = torch.randn(D, device="cuda").to(torch.bfloat16)
    us = t(lambda: ops.norm_fwd(x, w, b, branch=br))
    nbytes = (4 if branch else 2) * T * D * 2
    print(f"norm_fwd {T}x{D} branch={branch}: {us:.1f} us, {nbytes / us / 1e6:.2f} TB/s", flush=True)
