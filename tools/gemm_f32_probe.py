"""f32 MFMA GEMM (gemm_f32.hip) vs ATen f32 (hipBLASLt, TF32 off) on the reference
model's linear shapes (1024-token microbatches, d 768, FFN 2048, vocab 10000) and a
large square.  One MI355X."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mipipe  # noqa: F401
from mipipe import ops

torch.backends.cuda.matmul.allow_tf32 = False
SH = [("qkv fwd", 1024, 2304, 768), ("out fwd", 1024, 768, 768), ("ffn1 fwd", 1024, 2048, 768),
      ("ffn2 fwd", 1024, 768, 2048), ("head fwd", 1024, 10000, 768), ("qkv dW", 2304, 768, 1024),
      ("square", 4096, 4096, 4096)]


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


ext = ops.load_ext()
for name, M, N, K in SH:
    a = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda")
    c = torch.empty(M, N, device="cuda")
    ours = t(lambda: ext.gemm_f32(a, w.t(), c, None, 1.0, False))
    lib = t(lambda: torch.mm(a, w.t()))
    fl = 2.0 * M * N * K
    print(f"{name:10s} {M}x{N}x{K}: gemm_f32 {ours:8.1f} us ({fl / ours / 1e6:6.1f} TF)  ATen f32 {lib:8.1f} us "
          f"({fl / lib / 1e6:6.1f} TF)", flush=True)
