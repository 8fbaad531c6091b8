"""The reference model's 1024-token GEMM shapes (batch 8 x seq 128 microbatches, d 768,
FFN 2048, vocab 10000): the small-tile engine (cfg 10/11/12), the planner's default and
the big-tile split-K plan (MIPIPE_GEMM_SMALL=0 path, cfg -2 here) vs hipBLASLt (torch.mm).

    python tools/gemm_small_bench.py      (GPU; one JSON line per shape)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.ops import kernels as _k  # noqa: E402


def timeit(fn, iters=50, warm=10):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


T, d, f, V = 1024, 768, 2048, 10048
SHAPES = [("qkv", T, 3 * d, d), ("q", T, d, d), ("kv", T, 2 * d, d), ("wo", T, d, d), ("ff1", T, f, d),
          ("ff2", T, d, f), ("dx_qkv", T, d, 3 * d), ("dx_ff1", T, d, f), ("dx_ff2", T, f, d), ("head", T, V, d),
          ("dx_head", T, d, V)]
for name, M, N, K in SHAPES:
    a = (torch.randn(M, K, device="cuda") * 0.1).to(torch.bfloat16)
    b = (torch.randn(N, K, device="cuda") * 0.1).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    row = {"shape": name, "M": M, "N": N, "K": K}
    for cfg in (10, 11, 12, -1):
        us = timeit(lambda: _k._gemm(a, b, c, cfg=cfg))
        row[f"cfg{cfg}_us"] = round(us, 2)
    bt = b.t()
    row["blas_us"] = round(timeit(lambda: torch.mm(a, bt, out=c)), 2)
    fl = 2.0 * M * N * K
    row["best_ours_tf"] = round(fl / min(row[f"cfg{c_}_us"] for c_ in (10, 11, 12, -1)) / 1e6, 1)
    row["blas_tf"] = round(fl / row["blas_us"] / 1e6, 1)
    print(json.dumps(row), flush=True)
# dW (TT): dw[N, K] += dy^T x with K = 1024 tokens (f32 accumulate)
for name, N_, K_ in [("dw_qkv", 3 * d, d), ("dw_q", d, d), ("dw_kv", 2 * d, d), ("dw_ff1", f, d), ("dw_ff2", d, f)]:
    dy = (torch.randn(T, N_, device="cuda") * 0.1).to(torch.bfloat16)
    x = (torch.randn(T, K_, device="cuda") * 0.1).to(torch.bfloat16)
    g = torch.zeros(N_, K_, device="cuda")
    row = {"shape": name, "M": N_, "N": K_, "K": T}
    for cfg in (13, -1, 2, 6):
        row[f"cfg{cfg}_us"] = round(timeit(lambda: _k._gemm(dy, x, g, transA=True, transB=True, accum=True, cfg=cfg)), 2)
    dyt = dy.t()
    row["blas_us"] = round(timeit(lambda: g.add_(torch.mm(dyt, x, out_dtype=torch.float32))), 2)
    fl = 2.0 * N_ * K_ * T
    row["best_ours_tf"] = round(fl / min(row[f"cfg{c_}_us"] for c_ in (13, -1, 2, 6)) / 1e6, 1)
    print(json.dumps(row), flush=True)
