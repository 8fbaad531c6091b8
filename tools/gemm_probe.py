"""Run one GEMM shape a few times (for rocprofv3 --pmc counter collection).

    python tools/gemm_probe.py M N K [cfg] [layout: nt|ntacc|tt] [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.ops import kernels as _k  # noqa: E402

M, N, K = (int(x) for x in sys.argv[1:4])
cfg = int(sys.argv[4]) if len(sys.argv) > 4 else -1
layout = sys.argv[5] if len(sys.argv) > 5 else "nt"
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 5
if layout == "nt":
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    fn = lambda: _k._gemm(a, b, c, cfg=cfg)
elif layout == "ntacc":   # the dW problem with both operands K-contiguous (f32 accumulate, split-K)
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    c = torch.zeros(M, N, device="cuda", dtype=torch.float32)
    fn = lambda: _k._gemm(a, b, c, accum=True, cfg=cfg)
else:
    a = torch.randn(K, M, device="cuda").to(torch.bfloat16)
    b = torch.randn(K, N, device="cuda").to(torch.bfloat16)
    c = torch.zeros(M, N, device="cuda", dtype=torch.float32)
    fn = lambda: _k._gemm(a, b, c, transA=True, transB=True, accum=True, cfg=cfg)
for _ in range(iters):
    fn()
torch.cuda.synchronize()
print("ok", M, N, K, cfg, layout)
