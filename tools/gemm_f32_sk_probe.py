"""Stream-K vs split-K for the f32 GEMM (gemm_f32.hip) on the reference model's 1024-token
shapes (fwd, dX = K-contiguous dY x N-contiguous W, dW = both outer-contiguous), every
layout the f32 path runs: force_ks -2 = stream-K, 1..8 = split-K, 0 = the planner; torch.mm
f32 (hipBLASLt) for scale.  Interleaved x2, best.  python tools/gemm_f32_sk_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.ops import kernels as _k  # noqa: E402

V = 10000
T = 1024
# (name, A builder, B builder): A [M,K], B [K,N] views as the native f32 model passes them
SH = []
for nm, n_out, n_in in (("qkv", 2304, 768), ("out_proj", 768, 768), ("linear1", 2048, 768), ("linear2", 768, 2048),
                        ("head", V, 768)):
    SH.append((f"fwd {nm}", (T, n_in, "kc"), (n_in, n_out, "w_t")))      # x @ W^T
    SH.append((f"dx {nm}", (T, n_out, "kc"), (n_out, n_in, "w")))        # dy @ W
    SH.append((f"dw {nm}", (n_out, T, "t"), (T, n_in, "nc")))            # dy^T @ x


def make(spec):
    r, c, kind = spec
    if kind == "kc" or kind == "nc" or kind == "w":
        return torch.randn(r, c, device="cuda")
    if kind == "w_t":
        return torch.randn(c, r, device="cuda").t()
    return torch.randn(c, r, device="cuda").t()       # "t": transposed view of [K, M]


def t(fn, it=30):
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


e = _k._ext()
print("shape            auto    sk(-2)   s1      s2      s4    | aten    (us)")
for name, sa, sb in SH:
    A, B = make(sa), make(sb)
    M, N, K = A.shape[0], B.shape[1], A.shape[1]
    C = torch.empty(M, N, device="cuda")
    res = {}
    for rep in range(2):
        for fk in (0, -2, 1, 2, 4):
            us = t(lambda: e.gemm_f32_ex(A, B, C, None, None, None, 0, 1.0, False, 0.0, 0, fk))
            res[fk] = min(res.get(fk, 1e9), us)
        us = t(lambda: torch.mm(A, B, out=C))
        res["lib"] = min(res.get("lib", 1e9), us)
    fl = 2.0 * M * N * K
    print(f"{name:14s} " + " ".join(f"{res[k]:7.1f}" for k in (0, -2, 1, 2, 4)) + f" | {res['lib']:7.1f}   "
          f"auto {fl / res[0] / 1e6:.0f} TF, sk {fl / res[-2] / 1e6:.0f} TF, aten {fl / res['lib'] / 1e6:.0f} TF",
          flush=True)
