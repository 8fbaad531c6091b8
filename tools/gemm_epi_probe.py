"""Cost of the fused GEMM epilogues at the GPT-2 small headline shapes (64K-token microbatch):
the same GEMM timed with each epilogue the step uses, so an epilogue that stalls the store
loop (a global load per 8 outputs: residual, pre-activation) shows against the plain store.

    python tools/gemm_epi_probe.py [--m 65536] [--graph]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.ops import kernels as K_  # noqa: E402


def timed(fn, graph, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    reps = 1
    if graph:
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            g.capture_begin()
            for _ in range(it):
                fn()
            g.capture_end()
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        fn, reps, it = g.replay, it, 3
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=65536)
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    M, D, F = a.m, 768, 3072
    dev = "cuda"
    bf = torch.bfloat16
    r = lambda *s: torch.randn(*s, device=dev, dtype=bf)
    x, x3 = r(M, D), r(M, F)
    w1, w2, wo = r(F, D) * D ** -0.5, r(D, F) * F ** -0.5, r(D, D) * D ** -0.5
    w1t, w2t, wot = w1.t().contiguous(), w2.t().contiguous(), wo.t().contiguous()
    b1, bo = r(F), r(D)
    res = r(M, D)
    pre = r(M, F)
    cs = torch.zeros(F, device=dev, dtype=torch.float32)
    y3, y = torch.empty(M, F, device=dev, dtype=bf), torch.empty(M, D, device=dev, dtype=bf)
    aux = torch.empty(M, F, device=dev, dtype=bf)
    cases = {
        # FC1 shape: [M, 3072] = [M, 768] W1^T
        "fc1 plain": lambda: K_._gemm(x, w1, y3),
        "fc1 bias+gelu (fwd)": lambda: K_.linear(x, w1, b1, act="gelu", out=y3, aux=aux),
        "dGELU dX (no colsum)": lambda: K_.linear_dx(x, w2, act_input=pre, act="gelu", out=y3, wt=w2t),
        "dGELU dX + colsum": lambda: K_.linear_dx(x, w2, act_input=pre, act="gelu", out=y3, wt=w2t, colsum=cs),
        "dX plain (same shape)": lambda: K_.linear_dx(x, w2, out=y3, wt=w2t),
        "dReLU dX": lambda: K_.linear_dx(x, w2, act_input=pre, act="relu", out=y3, wt=w2t),
        "fc1 bias+relu": lambda: K_.linear(x, w1, b1, act="relu", out=y3, aux=aux),
        "fc1 bias": lambda: K_.linear(x, w1, b1, out=y3),
        # out-proj shape: [M, 768] = [M, 768] Wo^T
        "out-proj plain": lambda: K_._gemm(x, wo, y),
        "out-proj bias": lambda: K_.linear(x, wo, bo, out=y),
        "out-proj bias+res (fwd)": lambda: K_.linear(x, wo, bo, residual=res, out=y),
        # FC2 shape: [M, 768] = [M, 3072] W2^T
        "fc2 plain": lambda: K_._gemm(x3, w2, y),
        "fc2 bias+res (fwd)": lambda: K_.linear(x3, w2, bo, residual=res, out=y),
    }
    out = {}
    for name, fn in cases.items():
        us = timed(fn, a.graph)
        tf = (2 * M * D * D if name.startswith("out") else 2 * M * F * D) / us / 1e6
        out[name] = {"us": round(us, 1), "tf": round(tf, 1)}
        print(f"{name:28s} {us:8.1f} us  {tf:7.1f} TF", flush=True)
    print(json.dumps({"m": M, "graph": a.graph, "cases": out}))


if __name__ == "__main__":
    main()
