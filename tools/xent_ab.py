"""Fused softmax-CE kernel timing on the GPT-2 head shape (bf16 logits [T, 50304], V = 50257),
for the occupancy variants of xent_reg_kernel (MIPIPE_XENT = '' | occ3 | t1024, read once
per process).  Prints one JSON line: us per call, effective TB/s (logits read + gradient
written), and the max abs difference of loss / gradient vs the default kernel's output
saved by the first run (numerics must be identical up to summation order).

    MIPIPE_XENT=occ3 python tools/xent_ab.py [--tokens 16384]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import mipipe  # noqa: F401
from mipipe import ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    T, V, Vp = a.tokens, 50257, 50304
    g = torch.Generator(device="cuda").manual_seed(0)
    base = (torch.randn(T, Vp, device="cuda", generator=g) * 3).to(torch.bfloat16)
    tgt = torch.randint(0, V, (T,), device="cuda", generator=g)
    x = base.clone()
    loss = ops.xent_fwd_bwd(x, tgt, V, 1.0 / T)
    ref = torch.empty(T, Vp, device="cuda", dtype=torch.bfloat16)
    ref.copy_(base)
    # reference numerics: f32 softmax-CE
    lf = base.float()[:, :V]
    lse = torch.logsumexp(lf, 1)
    ref_loss = lse - lf.gather(1, tgt[:, None])[:, 0]
    err_loss = float((loss - ref_loss).abs().max())
    p = torch.softmax(lf, 1)
    p[torch.arange(T, device="cuda"), tgt] -= 1.0
    err_grad = float((x.float()[:, :V] - p / T).abs().max()) * T
    del lf, p
    bufs = [base.clone() for _ in range(2)]
    for i in range(3):
        ops.xent_fwd_bwd(bufs[i % 2], tgt, V, 1.0 / T)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(a.iters):
        ops.xent_fwd_bwd(bufs[i % 2], tgt, V, 1.0 / T)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / a.iters * 1e3
    print(json.dumps({"variant": os.environ.get("MIPIPE_XENT", "default"), "tokens": T, "us": round(us, 1),
                      "tb_s": round(2 * T * Vp * 2 / us / 1e6, 2), "max_err_loss": err_loss,
                      "max_err_grad_x_T": err_grad}), flush=True)


if __name__ == "__main__":
    main()
