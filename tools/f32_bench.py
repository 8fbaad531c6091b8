"""f32 kernels vs ATen f32 on the reference model's shapes (one MI355X).

    python tools/f32_bench.py [--json out.json]

GEMMs: gemm_f32_ex (csrc/kernels/gemm_f32.hip) vs torch.mm f32 (hipBLASLt, TF32 off) for
the forward (x W^T), dX (dy W) and dW (dy^T x) products of every linear of the reference
block at its 1024-token microbatch (d 768, FFN 2048, vocab 10000) and a 4096^3 square.
Attention: attention_f32.hip forward / backward vs ATen SDPA f32 (math) at B 8, S 128,
d_h 64 / 96 / 192, non-causal, dropout 0.1."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

import mipipe  # noqa: F401
from mipipe import ops

torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False
K_ = ops.kernels


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    out = {"gemm": [], "attention": []}
    dev = "cuda"
    lin = [("qkv", 2304, 768), ("out_proj", 768, 768), ("q_cross", 768, 768), ("kv_cross", 1536, 768),
           ("linear1", 2048, 768), ("linear2", 768, 2048), ("head", 10000, 768)]
    T = 1024
    for name, N, Kd in lin:
        x = torch.randn(T, Kd, device=dev)
        w = torch.randn(N, Kd, device=dev)
        dy = torch.randn(T, N, device=dev)
        y = torch.empty(T, N, device=dev)
        dx = torch.empty(T, Kd, device=dev)
        dw = torch.zeros(N, Kd, device=dev)
        for kind, ours, lib, fl in (
                ("fwd", lambda: K_._gemm_f32(x, w.t(), y), lambda: torch.mm(x, w.t()), 2.0 * T * N * Kd),
                ("dx", lambda: K_._gemm_f32(dy, w, dx), lambda: torch.mm(dy, w), 2.0 * T * N * Kd),
                ("dw", lambda: K_._gemm_f32(dy.t(), x, dw, accumulate=True), lambda: dw.addmm_(dy.t(), x),
                 2.0 * T * N * Kd)):
            to, tl = t(ours), t(lib)
            r = dict(shape=f"{kind} {name}", M=T if kind != "dw" else N, N=N if kind == "fwd" else Kd,
                     K=Kd if kind == "fwd" else (N if kind == "dx" else T), ours_us=round(to, 1),
                     aten_us=round(tl, 1), ours_tf=round(fl / to / 1e6, 1), aten_tf=round(fl / tl / 1e6, 1),
                     ratio=round(tl / to, 3))
            out["gemm"].append(r)
            print(json.dumps(r), flush=True)
    n = 4096
    A, B, C = torch.randn(n, n, device=dev), torch.randn(n, n, device=dev), torch.empty(n, n, device=dev)
    to, tl = t(lambda: K_._gemm_f32(A, B.t(), C), 5), t(lambda: torch.mm(A, B.t()), 5)
    r = dict(shape="square 4096", ours_tf=round(2 * n ** 3 / to / 1e6, 1), aten_tf=round(2 * n ** 3 / tl / 1e6, 1),
             ratio=round(tl / to, 3))
    out["gemm"].append(r)
    print(json.dumps(r), flush=True)
    Bb, S, Dm = 8, 128, 768
    for H in (4, 8, 12):
        D = Dm // H
        qkv = torch.randn(Bb * S, 3 * Dm, device=dev)
        q, k, v = qkv[:, :Dm], qkv[:, Dm:2 * Dm], qkv[:, 2 * Dm:]
        o = torch.empty(Bb * S, Dm, device=dev)
        lse = torch.empty(Bb * H * S, device=dev)
        do = torch.randn(Bb * S, Dm, device=dev)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = dqkv[:, :Dm], dqkv[:, Dm:2 * Dm], dqkv[:, 2 * Dm:]
        ops.set_dropout_step(1)
        f_ours = t(lambda: ops.attn_fwd(q, k, v, o, lse, Bb, S, S, H, H, D, False, p_drop=0.1, seed=3))
        b_ours = t(lambda: ops.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, Bb, S, S, H, H, D, False, p_drop=0.1, seed=3))
        qh = q.reshape(Bb, S, H, D).transpose(1, 2).contiguous().requires_grad_()
        kh = k.reshape(Bb, S, H, D).transpose(1, 2).contiguous().requires_grad_()
        vh = v.reshape(Bb, S, H, D).transpose(1, 2).contiguous().requires_grad_()
        doh = do.reshape(Bb, S, H, D).transpose(1, 2).contiguous()

        def aten_f():
            with torch.no_grad():
                return F.scaled_dot_product_attention(qh, kh, vh, dropout_p=0.1)

        def aten_fb():
            oo = F.scaled_dot_product_attention(qh, kh, vh, dropout_p=0.1)
            oo.backward(doh)
        f_lib = t(aten_f)
        fb_lib = t(aten_fb)
        fl_f = 4.0 * Bb * H * S * S * D
        r = dict(shape=f"attn B{Bb} S{S} H{H} D{D} drop0.1", fwd_us=round(f_ours, 1), bwd_us=round(b_ours, 1),
                 fwd_tf=round(fl_f / f_ours / 1e6, 1), bwd_tf=round(2.5 * fl_f / b_ours / 1e6, 1),
                 aten_fwd_us=round(f_lib, 1), aten_fwd_bwd_us=round(fb_lib, 1),
                 ratio_fwd_bwd=round(fb_lib / (f_ours + b_ours), 3))
        out["attention"].append(r)
        print(json.dumps(r), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
