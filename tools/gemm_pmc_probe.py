"""One NT GEMM shape on each engine, launched eagerly a few times, for rocprofv3 --pmc:
gemm3 (cfg 5), gemm8 (cfg 15) and hipBLASLt (torch.mm).

    python tools/gemm_pmc_probe.py [--m 65536 --n 768 --k 3072 --reps 5]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.ops import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=65536)
ap.add_argument("--n", type=int, default=768)
ap.add_argument("--k", type=int, default=3072)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--cfgs", default="5,15,lib")
a = ap.parse_args()
x = torch.randn(a.m, a.k, device="cuda", dtype=torch.bfloat16)
w = (torch.randn(a.n, a.k, device="cuda") * a.k ** -0.5).to(torch.bfloat16)
y = torch.empty(a.m, a.n, device="cuda", dtype=torch.bfloat16)
for c in a.cfgs.split(","):
    for _ in range(a.reps):
        if c == "lib":
            torch.mm(x, w.t(), out=y)
        else:
            K._gemm(x, w, y, cfg=int(c))
    torch.cuda.synchronize()
print("done", flush=True)
