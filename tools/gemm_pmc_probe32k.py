"""GEMM workload for rocprofv3 --pmc passes at the 32K-token microbatch of a PP > 1 rank:
the planner's NT engine (gemm3 ping-pong 256x256) on N = 768 K = 3072 (fwd fc2 / dX fc1),
N = 768 K = 768 (fwd / dX wo) and N = 2304 K = 768 (fwd qkv), 10 dispatches each, in that
order (the counter CSV rows are matched by dispatch order and grid size).

    rocprofv3 --pmc <counters> --kernel-include-regex gemm -- python3 tools/gemm_pmc_probe32k.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.ops import kernels as _k  # noqa: E402


def rnd(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).to(torch.bfloat16)


M = 32768
for N, K in ((768, 3072), (768, 768), (2304, 768)):
    x, w = rnd(M, K), rnd(N, K) * K ** -0.5
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(10):
        _k._gemm(x, w, y)
    torch.cuda.synchronize()
print("ok")
