"""Kernel microbenchmarks on the transformer's real shapes: our HIP kernels vs the
vendor libraries (hipBLASLt via torch.mm, flash attention via torch SDPA).

    python tools/bench_kernels.py [--json out.json]

Interleaved A/B timing in one process (cdna guide §5.4 rule 24), random operands."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe import ops  # noqa: E402
from mipipe.ops import kernels as _k  # noqa: E402


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def timeit_graph(fn, iters=20):
    """GPU time per call of ``fn`` replayed from one HIP graph of ``iters`` back-to-back calls
    -- how the training step runs its kernels (no host launch / Python overhead between
    them; an eager loop of microsecond kernels measures the launches instead)."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / iters * 1e-3
        best = t if best is None else min(best, t)
    return best


def gemm_cases(T=16384):
    d, f, V = 768, 3072, 50304
    out = []
    for name, N, K in [("qkv", 3 * d, d), ("wo", d, d), ("fc1", f, d), ("fc2", d, f), ("head", V, d)]:
        out.append((f"fwd_{name}", "fwd", T, N, K))
        out.append((f"dx_{name}", "dx", T, K, N))
        out.append((f"dw_{name}", "dw", N, K, T))
    out.append(("fwdgelu_fc1", "fwdgelu", T, f, d))
    out.append(("dxdgelu_fc2", "dxdgelu", T, f, d))
    for name, N, K in [("l_qkv", 6144, 4096), ("l_w13", 28672, 4096), ("l_w2", 4096, 14336)]:
        out.append((f"fwd_{name}", "fwd", T, N, K))
        out.append((f"dw_{name}", "dw", N, K, T))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None)
    ap.add_argument("--cfg", type=int, default=-1, help="force a gemm2 tile config (4 = ping-pong 256x256)")
    a = ap.parse_args()
    dev = "cuda"
    res = {}
    torch.manual_seed(0)
    for tag, kind, M, N, K in gemm_cases():
        if a.only and a.only not in tag:
            continue
        fl = 2.0 * M * N * K
        if kind == "fwd":   # y[M,N] = x[M,K] w[N,K]^T
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * K ** -0.5
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ours = lambda: _k._gemm(x, w, y, cfg=a.cfg)
            lib = lambda: torch.mm(x, w.t(), out=y)
        elif kind == "fwdgelu":  # a = x w^T + b; y = gelu(a)   (fused epilogue vs addmm + gelu)
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * K ** -0.5
            b = torch.randn(N, device=dev, dtype=torch.bfloat16)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            aux = torch.empty_like(y)
            ours = lambda: _k._gemm(x, w, y, bias=b, aux=aux, epi=_k.EPI_BIAS_GELU, cfg=a.cfg)
            lib = lambda: F.gelu(torch.addmm(b, x, w.t(), out=aux), approximate="tanh")
        elif kind == "dxdgelu":  # da = (dy W) * gelu'(a)
            dy = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            wt = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * K ** -0.5
            aux = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ours = lambda: _k._gemm(dy, wt, y, aux=aux, epi=_k.EPI_DGELU, cfg=a.cfg)
            lib = lambda: torch.mm(dy, wt.t(), out=y).mul_(aux)
        elif kind == "dx":  # dx[M,N] = dy[M,K] w[K,N]
            dy = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(K, N, device=dev, dtype=torch.bfloat16) * K ** -0.5
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            wt = w.t().contiguous()   # the arena keeps W^T: dX runs as an NT GEMM
            ours = lambda: _k._gemm(dy, wt, y, cfg=a.cfg)
            lib = lambda: torch.mm(dy, w, out=y)
        else:               # dw[M,N] += dy[K,M]^T x[K,N]  (f32 accumulate)
            dy = torch.randn(K, M, device=dev, dtype=torch.bfloat16)
            xx = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
            g = torch.zeros(M, N, device=dev, dtype=torch.float32)
            ours = lambda: _k._gemm(dy, xx, g, transA=True, transB=True, accum=True)
            lib = lambda: g.add_(torch.mm(dy.t(), xx, out_dtype=torch.float32))
        to, tl = [], []
        for _ in range(3):
            to.append(timeit(ours))
            tl.append(timeit(lib))
        res[tag] = dict(M=M, N=N, K=K, ours_tflops=round(fl / min(to) / 1e12, 1),
                        lib_tflops=round(fl / min(tl) / 1e12, 1), ours_us=round(min(to) * 1e6, 1),
                        lib_us=round(min(tl) * 1e6, 1))
        print(tag, res[tag], flush=True)
    # attention: GPT-2 small / Llama-3 8B shapes
    for (B, S, H, KV, D, causal) in [(8, 1024, 12, 12, 64, True), (16, 1024, 12, 12, 64, True),
                                     (1, 8192, 32, 8, 128, True),
                                     (8, 128, 8, 8, 96, False)]:
        tag = f"attn_B{B}S{S}H{H}KV{KV}D{D}c{int(causal)}"
        if a.only and a.only not in tag:
            continue
        T = B * S
        qkv = torch.randn(T, (H + 2 * KV) * D, device=dev, dtype=torch.bfloat16)
        q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + KV) * D], qkv[:, (H + KV) * D:]
        o = torch.empty(T, H * D, device=dev, dtype=torch.bfloat16)
        lse = torch.empty(B * H * S, device=dev)
        do = torch.randn_like(o)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = dqkv[:, :H * D], dqkv[:, H * D:(H + KV) * D], dqkv[:, (H + KV) * D:]
        f_ours = lambda: ops.attn_fwd(q, k, v, o, lse, B, S, S, H, KV, D, causal)
        b_ours = lambda: ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, S, S, H, KV, D, causal)
        Q = q.reshape(B, S, H, D).transpose(1, 2).contiguous().requires_grad_()
        Kt = k.reshape(B, S, KV, D).transpose(1, 2).contiguous().requires_grad_()
        Vt = v.reshape(B, S, KV, D).transpose(1, 2).contiguous().requires_grad_()
        gqa = dict(enable_gqa=True) if KV != H else {}
        f_lib = lambda: F.scaled_dot_product_attention(Q, Kt, Vt, is_causal=causal, **gqa)
        ol = f_lib()
        gl = torch.randn_like(ol)
        b_lib = lambda: torch.autograd.grad(f_lib(), (Q, Kt, Vt), gl)
        fl = 4.0 * B * H * S * S * D * (0.5 if causal else 1.0)
        tf, tb, lf, lb = [], [], [], []
        for _ in range(3):
            tf.append(timeit(f_ours))
            tb.append(timeit(b_ours))
            lf.append(timeit(f_lib))
            lb.append(timeit(b_lib) - min(lf))
        gf, gb = timeit_graph(f_ours), timeit_graph(b_ours)
        res[tag] = dict(ours_fwd_tflops=round(fl / min(tf) / 1e12, 1), ours_bwd_tflops=round(2.5 * fl / min(tb) / 1e12, 1),
                        lib_fwd_tflops=round(fl / min(lf) / 1e12, 1), lib_bwd_tflops=round(2.5 * fl / min(lb) / 1e12, 1),
                        ours_fwd_us=round(min(tf) * 1e6, 1), ours_bwd_us=round(min(tb) * 1e6, 1),
                        # the same kernels replayed from a HIP graph (as in the training step)
                        ours_fwd_graph_us=round(gf * 1e6, 1), ours_bwd_graph_us=round(gb * 1e6, 1),
                        ours_fwd_graph_tflops=round(fl / gf / 1e12, 1),
                        ours_bwd_graph_tflops=round(2.5 * fl / gb / 1e12, 1))
        print(tag, res[tag], flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
