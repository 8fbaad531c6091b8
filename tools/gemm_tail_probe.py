"""Tile-wave quantisation of the N = 768 GEMMs at 32K-token microbatches (the PP > 1 bench
microbatch): 256x256 tiles are 384 = 1.5 waves of 256 CUs; 256x192 tiles are 512 = 2 waves.
Times forced configs (gemm2 cfg 1 = 256x192, cfg 2 = 256x128, -1 = the planner's choice,
i.e. the ping-pong 256x256 engine) and hipBLASLt, interleaved.  python tools/gemm_tail_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.ops import kernels as _k  # noqa: E402


def t(fn, it=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


for M in (32768, 65536):
    for N, K in ((768, 768), (768, 2304), (768, 3072), (2304, 768), (3072, 768)):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * K ** -0.5
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        res = {}
        for rep in range(2):
            for cfg in (-1, 1, 2):
                us = t(lambda: _k._gemm(x, w, y, cfg=cfg))
                res[cfg] = min(res.get(cfg, 1e9), us)
            us = t(lambda: torch.mm(x, w.t(), out=y))
            res["lib"] = min(res.get("lib", 1e9), us)
        fl = 2.0 * M * N * K
        print(f"M={M} N={N} K={K} " + " ".join(f"{k}:{v:.1f}us/{fl / v / 1e6:.0f}TF" for k, v in res.items()),
              flush=True)
