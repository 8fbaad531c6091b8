"""Weight-gradient GEMMs (dW += dY^T X, both operands token-major: the split-K TT engine)
at the GPT-2 small headline shapes, timed as the step runs them (HIP graph of 20 launches).
Run twice to A/B the split-K XCD mapping:

    python tools/gemm_dw_probe.py [--m 65536]
    MIPIPE_G3_SPLIT_REMAP=0 python tools/gemm_dw_probe.py"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.ops import kernels as K_  # noqa: E402
from tools.gemm_epi_probe import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=65536)
    a = ap.parse_args()
    T = a.m
    out = {}
    # (name, N_out, K_in): qkv, out-proj, fc1, fc2, LM head
    for name, n, k in (("qkv", 2304, 768), ("out-proj", 768, 768), ("fc1", 3072, 768), ("fc2", 768, 3072),
                       ("head", 50304, 768)):
        dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(T, k, device="cuda", dtype=torch.bfloat16)
        dw = torch.zeros(n, k, device="cuda", dtype=torch.float32)
        us = timed(lambda: K_.linear_dw(dy, x, dw), True, it=10 if name == "head" else 20)
        tf = 2 * T * n * k / us / 1e6
        out[name] = {"us": round(us, 1), "tf": round(tf, 1)}
        print(f"{name:10s} [{n} x {k}] over {T} tokens  {us:9.1f} us  {tf:7.1f} TF", flush=True)
        del dy, x, dw
    print(json.dumps({"m": T, "split_remap": os.environ.get("MIPIPE_G3_SPLIT_REMAP", "1"), "cases": out}))


if __name__ == "__main__":
    main()
