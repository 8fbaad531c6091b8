"""gemm8 (four-wave register-staged 256x192 NT engine, force cfg 15) vs gemm3 (cfg 5, the
ping-pong 256x256 engine) vs hipBLASLt: numerics against an f32 reference on edge shapes
first, then per-launch times replayed from one HIP graph, interleaved.

    python tools/gemm8_probe.py [--ms 65536,16384] [--check-only]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
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
    out = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) / it * 1e3)
    return sorted(out)[len(out) // 2]


def check(M, N, Kd, epi, dev, cfgs=(5, 15)):
    g = torch.Generator(device=dev).manual_seed(M + N + Kd)
    x = torch.randn(M, Kd, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, Kd, device=dev, generator=g) * Kd ** -0.5).to(torch.bfloat16)
    b = (torch.randn(N, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    r = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    kw = {}
    if epi == "bias":
        ref = ref + b.float()
        kw = dict(bias=b, epi=K.EPI_BIAS)
    elif epi == "bias_res":
        ref = ref + b.float() + r.float()
        kw = dict(bias=b, residual=r, epi=K.EPI_BIAS_RES)
    outs = {}
    for cfg in cfgs:
        y = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        K._gemm(x, w, y, cfg=cfg, **kw)
        torch.cuda.synchronize()
        err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
        outs[cfg] = (err, y)
    ok = all(outs[c][0] < 2e-2 and not torch.isnan(outs[c][1]).any().item() for c in cfgs)
    print(f"check M={M} N={N} K={Kd} {epi}: " + " ".join(f"cfg{c} {outs[c][0]:.2e}" for c in cfgs)
          + f" {'OK' if ok else 'FAIL'}", flush=True)
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="65536,16384")
    ap.add_argument("--check-only", action="store_true")
    ap.add_argument("--cfgs", default="5,15,16")
    ap.add_argument("--shapes", default="2304x768,768x768,3072x768,768x3072,768x2304,50304x768")
    a = ap.parse_args()
    dev = torch.device("cuda")
    ok = True
    for (M, N, Kd, epi) in ((256, 192, 64, "none"), (512, 384, 128, "bias"), (1000, 200, 192, "none"),
                            (300, 776, 640, "bias_res"), (4096, 768, 768, "bias"), (8192, 2304, 768, "none"),
                            (2048, 768, 3072, "bias_res"), (1024, 50304, 768, "none")):
        ok &= check(M, N, Kd, epi, dev, [int(c) for c in a.cfgs.split(',')])
    if not ok:
        print("NUMERICS FAIL", flush=True)
        sys.exit(1)
    if a.check_only:
        return
    for M in [int(m) for m in a.ms.split(",")]:
        for N, Kd in [tuple(int(v) for v in x.split("x")) for x in a.shapes.split(",")]:
            x = torch.randn(M, Kd, device=dev, dtype=torch.bfloat16)
            w = (torch.randn(N, Kd, device=dev) * Kd ** -0.5).to(torch.bfloat16)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            res = {}
            for _ in range(2):
                for cfg in [int(c) for c in a.cfgs.split(",")]:
                    res[cfg] = min(res.get(cfg, 1e9), graph_time(lambda: K._gemm(x, w, y, cfg=cfg)))
                res["lib"] = min(res.get("lib", 1e9), graph_time(lambda: torch.mm(x, w.t(), out=y)))
            fl = 2.0 * M * N * Kd
            print(f"M={M} N={N} K={Kd} " + " ".join(f"{k}:{v:.1f}us/{fl / v / 1e6:.0f}TF" for k, v in res.items())
                  + "  " + " ".join(f"g3/{c} {res[5] / res[c]:.3f}" for c in res if c not in (5, "lib")) + f"  lib/best {res['lib'] / min(v for k, v in res.items() if k != 'lib'):.3f}", flush=True)
            del x, w, y
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
