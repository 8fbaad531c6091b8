"""Fixed (per-tile) vs per-K-tile cost of the big NT GEMM engine.

For M = 16384, N = 3072 (768 tiles of 256x256 = 3 full waves of 256 CUs) time the GEMM
at K = 64 .. 3072 and fit t(K) = a + b * K / 64: `a` is the prologue + epilogue + launch
cost of a tile wave, `b` the main-loop cost of one K-tile.  Same for hipBLASLt (torch.mm).

    python tools/gemm_overhead_probe.py [--cfg N]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.ops import kernels as _k  # noqa: E402


def timeit(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=-1)
    ap.add_argument("--M", type=int, default=16384)
    ap.add_argument("--N", type=int, default=3072)
    a = ap.parse_args()
    M, N = a.M, a.N
    rows = []
    for K in (64, 128, 256, 512, 768, 1536, 3072):
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * K ** -0.5).to(torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        wt = w.t()
        ours = min(timeit(lambda: _k._gemm(x, w, y, cfg=a.cfg)) for _ in range(3))
        lib = min(timeit(lambda: torch.mm(x, wt, out=y)) for _ in range(3))
        r = {"K": K, "ours_us": round(ours, 2), "lib_us": round(lib, 2),
             "ours_tf": round(2 * M * N * K / ours / 1e6, 1), "lib_tf": round(2 * M * N * K / lib / 1e6, 1)}
        rows.append(r)
        print(json.dumps(r), flush=True)
    kt = np.array([r["K"] / 64 for r in rows])
    for key in ("ours_us", "lib_us"):
        t = np.array([r[key] for r in rows])
        b, a0 = np.polyfit(kt, t, 1)
        print(json.dumps({"fit": key, "fixed_us": round(float(a0), 2), "per_ktile_us": round(float(b), 3),
                          "fixed_share_at_K768": round(float(a0 / (a0 + 12 * b)), 3)}), flush=True)


if __name__ == "__main__":
    main()
