"""Is torch.mm f32 on this ROCm build exact f32?  Error vs an f64 reference of torch.mm (hipBLASLt)
and of the framework's gemm_f32 (v_mfma_f32_32x32x2_f32: bit-for-bit fma chains), plus their
times, on the reference's 1024-token shapes.  python tools/probes/f32_exactness.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.ops import kernels as _k  # noqa: E402


def t(fn, it=50):
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


print("allow_tf32:", torch.backends.cuda.matmul.allow_tf32, "float32_matmul_precision:",
      torch.get_float32_matmul_precision())
torch.manual_seed(0)
for M, N, K in ((1024, 768, 3072), (1024, 3072, 768), (1024, 2304, 768)):
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(K, N, device="cuda")
    ref = (a.double().cpu() @ b.double().cpu())
    scale = (a.double().cpu().abs() @ b.double().cpu().abs())
    c_lib = torch.mm(a, b)
    c_our = torch.empty(M, N, device="cuda")
    _k._gemm_f32(a, b, c_our)
    torch.cuda.synchronize()
    e_lib = ((c_lib.double().cpu() - ref).abs() / scale).max().item()
    e_our = ((c_our.double().cpu() - ref).abs() / scale).max().item()
    us_lib = t(lambda: torch.mm(a, b, out=c_lib))
    us_our = t(lambda: _k._gemm_f32(a, b, c_our))
    fl = 2.0 * M * N * K
    print(f"M={M} N={N} K={K}  max |err|/sum|a*b|: lib {e_lib:.2e}  ours {e_our:.2e}   "
          f"lib {us_lib:.1f}us {fl / us_lib / 1e6:.0f}TF  ours {us_our:.1f}us {fl / us_our / 1e6:.0f}TF", flush=True)
