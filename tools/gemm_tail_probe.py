"""Tile-wave quantisation of the N = 768 GEMMs at 32K-token microbatches (the PP > 1 bench
microbatch): 256x256 tiles are 384 = 1.5 waves of 256 CUs; 256x192 tiles are 512 = 2 waves.
Times forced configs (5 = the ping-pong 256x256 engine gemm3, 9 = the ping-pong 256x192
engine gemm6, 1 = gemm2's 2-stage 256x192, -1 = the planner's choice) and hipBLASLt,
interleaved.  python tools/gemm_tail_probe.py [--ms 8192,32768,65536] [--cfgs=-1,5,9,1] [--graph]
(14 = the split-tail engine gemm7)"""
import argparse
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
    if GRAPH:   # the in-step condition: launches replayed from one HIP graph
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
        fn = g.replay
        it_ = it
        it = 3
    else:
        it_ = 1
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it / it_ * 1e3


ap = argparse.ArgumentParser()
ap.add_argument("--ms", default="32768,65536")
ap.add_argument("--cfgs", default="-1,5,9,1")
ap.add_argument("--graph", action="store_true", help="time 20 launches replayed from one HIP graph")
a = ap.parse_args()
GRAPH = a.graph
CFGS = [int(c) for c in a.cfgs.split(",")]
for M in [int(m) for m in a.ms.split(",")]:
    for N, K in ((768, 768), (768, 2304), (768, 3072), (2304, 768), (3072, 768)):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * K ** -0.5
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        res = {}
        for rep in range(2):
            for cfg in CFGS:
                us = t(lambda: _k._gemm(x, w, y, cfg=cfg))
                res[cfg] = min(res.get(cfg, 1e9), us)
            us = t(lambda: torch.mm(x, w.t(), out=y))
            res["lib"] = min(res.get("lib", 1e9), us)
        fl = 2.0 * M * N * K
        print(f"M={M} N={N} K={K} " + " ".join(f"{k}:{v:.1f}us/{fl / v / 1e6:.0f}TF" for k, v in res.items()),
              flush=True)
