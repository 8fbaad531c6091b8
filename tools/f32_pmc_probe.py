"""f32 workload for rocprofv3 --pmc passes: gemm_f32 on the reference's LM head (forward,
1024 x 10000 x 768: 2512 tiles, main-loop bound), the qkv projection (1024 x 2304 x 768)
and its dW (2304 x 768 over 1024 tokens, both operands outer-contiguous), and the f32
attention forward / backward at B 8, S 128, H 8, d_h 96 with dropout.

    rocprofv3 --pmc <counters> --kernel-include-regex "gemm_f32|af32" -- python3 tools/f32_pmc_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe import ops  # noqa: E402

K_ = ops.kernels
dev = "cuda"
T = 1024
x, wh, yh = torch.randn(T, 768, device=dev), torch.randn(10000, 768, device=dev), torch.empty(T, 10000, device=dev)
wq, yq = torch.randn(2304, 768, device=dev), torch.empty(T, 2304, device=dev)
dyq, dwq = torch.randn(T, 2304, device=dev), torch.zeros(2304, 768, device=dev)
for _ in range(10):
    K_._gemm_f32(x, wh.t(), yh)
for _ in range(10):
    K_._gemm_f32(x, wq.t(), yq)
for _ in range(10):
    K_._gemm_f32(dyq.t(), x, dwq, accumulate=True)
# dX of linear1 (1024 x 768 over K = 2048: 192 tiles, 32 K-tile pairs), no split: one
# workgroup per CU, the main loop at 2 waves per SIMD
dy1, w1, dx1 = torch.randn(T, 2048, device=dev), torch.randn(2048, 768, device=dev), torch.empty(T, 768, device=dev)
ext = ops.load_ext()
for _ in range(10):
    ext.gemm_f32_ex(dy1, w1, dx1, None, None, None, 0, 1.0, False, 0.0, 0, 1)
B, S, H, D = 8, 128, 8, 96
qkv = torch.randn(B * S, 3 * H * D, device=dev)
q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
o, lse = torch.empty(B * S, H * D, device=dev), torch.empty(B * H * S, device=dev)
do, dqkv = torch.randn(B * S, H * D, device=dev), torch.empty_like(qkv)
ops.set_dropout_step(1)
for _ in range(10):
    ops.attn_fwd(q, k, v, o, lse, B, S, S, H, H, D, False, p_drop=0.1, seed=3)
    ops.attn_bwd(q, k, v, o, do, lse, dqkv[:, :H * D], dqkv[:, H * D:2 * H * D], dqkv[:, 2 * H * D:], B, S, S, H, H,
                 D, False, p_drop=0.1, seed=3)
torch.cuda.synchronize()
print("ok")
