"""gemm_f32_ex split-K sweep on the reference's 1024-token shapes (one MI355X).

    python tools/f32_gemm_sweep.py [--json out.json]

For each linear of the reference block (fwd / dX / dW) times gemm_f32_ex at forced split
factors 1..8 against torch.mm f32 (hipBLASLt, TF32 off), so pick_split can be checked
against the measured best."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import mipipe  # noqa: F401
from mipipe import ops

torch.backends.cuda.matmul.allow_tf32 = False


def t(fn, it=30):
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
    ext = ops.load_ext()
    dev = "cuda"
    T = 1024
    out = []
    for name, N, Kd in (("qkv", 2304, 768), ("out_proj", 768, 768), ("linear1", 2048, 768),
                        ("linear2", 768, 2048), ("head", 10000, 768)):
        x, w, dy = torch.randn(T, Kd, device=dev), torch.randn(N, Kd, device=dev), torch.randn(T, N, device=dev)
        y, dx, dw = torch.empty(T, N, device=dev), torch.empty(T, Kd, device=dev), torch.zeros(N, Kd, device=dev)
        for kind, args, lib in (("fwd", (x, w.t(), y), lambda: torch.mm(x, w.t())),
                                ("dx", (dy, w, dx), lambda: torch.mm(dy, w)),
                                ("dw", (dy.t(), x, dw), lambda: torch.mm(dy.t(), x))):
            fl = 2.0 * T * N * Kd
            row = dict(shape=f"{kind} {name}", aten_us=round(t(lib), 1))
            for s in (1, 2, 3, 4, 6, 8):
                us = t(lambda: ext.gemm_f32_ex(*args, None, None, None, 0, 1.0, False, 0.0, 0, s))
                row[f"s{s}"] = round(us, 1)
            us = t(lambda: ext.gemm_f32_ex(*args, None, None, None, 0, 1.0, False, 0.0, 0, 0))
            row["auto"] = round(us, 1)
            row["auto_tf"] = round(fl / us / 1e6, 1)
            row["aten_tf"] = round(fl / row["aten_us"] / 1e6, 1)
            out.append(row)
            print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
