"""Every GEMM of one GPT-2 training microbatch, ours vs hipBLASLt, shape by shape.

For T tokens per microbatch: the forward NT GEMMs with their fused epilogues (qkv +bias,
attention-out +bias +residual, fc1 +bias +GELU, fc2 +bias +residual, LM head), the dX GEMMs
(both operands K-contiguous: the arena keeps W^T; fc1's with the dGELU epilogue) and the f32
dW accumulates (TT + split-K).  The library arm is torch.mm (hipBLASLt) on the same
operands without epilogues (bf16 out; dW: f32 out), i.e. a lower bound on what the library
would cost for our fused op.  Times are per launch, replayed from one HIP graph (the in-step
condition), interleaved ours / lib per shape.

    python tools/gemm_step_shapes.py [--tokens 65536,16384] [--model gpt2-small] [--out f.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.models.config import NativeConfig  # noqa: E402
from mipipe.ops import kernels as K  # noqa: E402


def graph_time(fn, it=10, rounds=3):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g.capture_begin()
        for _ in range(it):
            fn()
        g.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    best = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best.append(a.elapsed_time(b) / it * 1e3)
    return sorted(best)[len(best) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="65536,16384")
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--only", default="", help="comma list of op names to run")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cfg = NativeConfig.by_name(a.model)
    D, F, V, Q = cfg.d_model, cfg.d_ff, cfg.vocab_padded, cfg.qkv_dim
    dev = torch.device("cuda")
    bf = torch.bfloat16
    rows = []
    only = set(x for x in a.only.split(",") if x)
    for T in [int(t) for t in a.tokens.split(",")]:
        # (name, N, K, kind, epilogue)
        specs = [("fwd_qkv", Q, D, "fwd", "bias"), ("fwd_proj", D, D, "fwd", "bias_res"),
                 ("fwd_fc1", F, D, "fwd", "gelu"), ("fwd_fc2", D, F, "fwd", "bias_res"),
                 ("fwd_head", V, D, "fwd", "none"),
                 ("dx_qkv", D, Q, "dx", "none"), ("dx_proj", D, D, "dx", "none"), ("dx_fc1", D, F, "dx", "none"),
                 ("dx_fc2", F, D, "dx", "dgelu"), ("dx_head", D, V, "dx", "none"),
                 ("dw_qkv", Q, D, "dw", ""), ("dw_proj", D, D, "dw", ""), ("dw_fc1", F, D, "dw", ""),
                 ("dw_fc2", D, F, "dw", ""), ("dw_head", V, D, "dw", "")]
        for name, N, Kd, kind, epi in specs:
            if only and name not in only:
                continue
            g = torch.Generator(device=dev).manual_seed(1)
            if kind == "fwd":
                x = torch.randn(T, Kd, device=dev, dtype=bf, generator=g)
                w = (torch.randn(N, Kd, device=dev, generator=g) * Kd ** -0.5).to(bf)
                bias = torch.randn(N, device=dev, dtype=bf, generator=g) * 0.1
                res = torch.randn(T, N, device=dev, dtype=bf, generator=g) if epi == "bias_res" else None
                out = torch.empty(T, N, device=dev, dtype=bf)
                aux = torch.empty(T, N, device=dev, dtype=bf) if epi == "gelu" else None
                act = "gelu_tanh" if epi == "gelu" else "none"
                b_ = bias if epi != "none" else None

                def ours():
                    K.linear(x, w, b_, act=act, residual=res, out=out, aux=aux)

                def lib():
                    torch.mm(x, w.t(), out=out)
            elif kind == "dx":
                dy = torch.randn(T, Kd, device=dev, dtype=bf, generator=g)      # [T, N_layer_out]
                w = (torch.randn(Kd, N, device=dev, generator=g) * Kd ** -0.5).to(bf)   # [N_out, K_in]
                wt = w.t().contiguous()
                out = torch.empty(T, N, device=dev, dtype=bf)
                ai = torch.rand(T, N, device=dev, dtype=bf, generator=g) if epi == "dgelu" else None
                act = "gelu_tanh" if epi == "dgelu" else "none"

                def ours():
                    K.linear_dx(dy, w, act_input=ai, act=act, out=out, wt=wt)

                def lib():
                    torch.mm(dy, w, out=out)
            else:
                dy = torch.randn(T, N, device=dev, dtype=bf, generator=g)
                x = torch.randn(T, Kd, device=dev, dtype=bf, generator=g)
                dw = torch.zeros(N, Kd, device=dev, dtype=torch.float32)
                tmp = torch.empty(N, Kd, device=dev, dtype=torch.float32)

                def ours():
                    K.linear_dw(dy, x, dw)

                def lib():
                    torch.mm(dy.t(), x, out_dtype=torch.float32, out=tmp)
            flop = 2.0 * T * N * Kd
            t_o = graph_time(ours)
            t_l = graph_time(lib)
            t_o2 = graph_time(ours)
            t_o = min(t_o, t_o2)
            r = {"T": T, "op": name, "M": T if kind != "dw" else N, "N": N if kind != "dw" else Kd,
                 "K": Kd if kind != "dw" else T, "ours_us": round(t_o, 1), "lib_us": round(t_l, 1),
                 "ours_tf": round(flop / t_o / 1e6, 0), "lib_tf": round(flop / t_l / 1e6, 0),
                 "ratio_lib_over_ours": round(t_l / t_o, 3)}
            rows.append(r)
            print(json.dumps(r), flush=True)
            del ours, lib
            torch.cuda.empty_cache()
        tot_o = sum(r["ours_us"] for r in rows if r["T"] == T)
        tot_l = sum(r["lib_us"] for r in rows if r["T"] == T)
        print(json.dumps({"T": T, "sum_ours_us": round(tot_o, 1), "sum_lib_us": round(tot_l, 1)}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
