"""Tiny GEMM workload for rocprofv3 --pmc passes: the big NT engine on GPT-2's fc1 shape
(16384 x 3072 x 768) and the small-tile engines on the reference model's 1024-token q
projection (NT, 1024 x 768 x 768) and its dW (TT, 768 x 768 over 1024 tokens).

    rocprofv3 --pmc <counters> --kernel-include-regex gemm -- python3 tools/gemm_pmc_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.ops import kernels as _k  # noqa: E402


def rnd(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)


x, w, y = rnd(16384, 768), rnd(3072, 768), torch.empty(16384, 3072, device="cuda", dtype=torch.bfloat16)
xs, ws, ys = rnd(1024, 768), rnd(768, 768), torch.empty(1024, 768, device="cuda", dtype=torch.bfloat16)
dy, xx, g = rnd(1024, 768), rnd(1024, 768), torch.zeros(768, 768, device="cuda")
for _ in range(10):
    _k._gemm(x, w, y)
for _ in range(10):
    _k._gemm(xs, ws, ys)
for _ in range(10):
    _k._gemm(dy, xx, g, transA=True, transB=True, accum=True)
torch.cuda.synchronize()
print("ok")
