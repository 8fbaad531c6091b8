"""gemm4 (persistent, deferred C stores), gemm5 (4 waves, one per SIMD) vs gemm3 (cfg 5) vs hipBLASLt on the NT shapes it
takes by default (plain / bias GEMMs of more than 256 256x256 tiles).  One MI355X."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mipipe  # noqa: F401
from mipipe.ops import kernels as _k

SHAPES = [("fwd_qkv", 16384, 2304, 768, 1), ("fwd_fc1(plain)", 16384, 3072, 768, 0), ("fwd_head", 16384, 50304, 768, 0),
          ("dx_fc1", 16384, 768, 3072, 0), ("dx_qkv", 16384, 768, 2304, 0), ("l_qkv", 16384, 6144, 4096, 0),
          ("l_w2", 16384, 4096, 14336, 0), ("l_w13", 16384, 28672, 4096, 0)]


def bench(fn, it=20):
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


for name, M, N, K, bias in SHAPES:
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16) if bias else None
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y3 = torch.empty_like(y)
    res = {}
    y5 = torch.empty_like(y)
    for tag, cfg, out in (("g3", 5, y3), ("g4", 7, y), ("g5", 8, y5)):
        res[tag] = bench(lambda: _k._gemm(x, w, out, bias=b, epi=bias, cfg=cfg))
    res["lib"] = bench(lambda: torch.nn.functional.linear(x, w, b))
    err = (y.float() - y3.float()).abs().max().item()
    err5 = (y5.float() - y3.float()).abs().max().item()
    fl = 2.0 * M * N * K
    print(f"{name:16s} M={M} N={N} K={K}: gemm3 {res['g3']:8.1f} us ({fl / res['g3'] / 1e6:6.0f} TF)  "
          f"gemm4 {res['g4']:8.1f} us ({fl / res['g4'] / 1e6:6.0f} TF)  hipBLASLt {res['lib']:8.1f} us "
          f"({fl / res['lib'] / 1e6:6.0f} TF)  gemm5 {res['g5']:8.1f} us ({fl / res['g5'] / 1e6:6.0f} TF)  "
          f"max|g4-g3| {err:.3g} max|g5-g3| {err5:.3g}", flush=True)
