"""Llama-3 8B training steps on ONE GPU (PP=1, activation recompute, bf16 HIP kernels):
exercises the 8B shapes (D=4096 RMSNorm, GQA D=128 flash attention, SwiGLU 14336,
128K-vocab fused CE) end to end.  Prints one JSON line.

    python tools/llama8b_step.py [--seq 8192] [--mbs 1] [--m 2] [--steps 3]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mbs", type=int, default=1)
    ap.add_argument("--m", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--layers", type=int, default=None, help="override n_layers (smaller probe)")
    ap.add_argument("--no-recompute", action="store_true")
    ap.add_argument("--recompute", default="auto",
                    help="auto: the trainer's HBM plan picks the fewest recomputed layers (engine.plan_recompute); "
                         "1: every layer; 0: none; k: the first k layers")
    ap.add_argument("--schedule", default="1F1B")
    ap.add_argument("--graphs", type=int, default=0)
    a = ap.parse_args()
    import torch
    import mipipe  # noqa: F401
    from mipipe.engine import PipelineTrainer
    from mipipe.models.config import NativeConfig
    kw = {} if a.layers is None else dict(n_layers=a.layers)
    cfg = NativeConfig.llama3("8b", **kw)
    t0 = time.time()
    rc = {"auto": "auto", "1": True, "0": False}.get(a.recompute)
    if rc is None:
        rc = int(a.recompute)
    tr = PipelineTrainer(cfg, pp=1, n_microbatches=a.m, mbs=a.mbs, seq_len=a.seq, device=torch.device("cuda", 0),
                         recompute=False if a.no_recompute else rc, lr=1e-4, schedule=a.schedule,
                         graphs=bool(a.graphs))
    if a.graphs:
        g0 = torch.Generator(device="cuda").manual_seed(0)
        xc = torch.randint(0, cfg.vocab_size, (a.m * a.mbs, a.seq), device="cuda", generator=g0)
        tr.capture_graphs(xc, xc)
        torch.cuda.reset_peak_memory_stats()
    init_s = time.time() - t0
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randint(0, cfg.vocab_size, (a.m * a.mbs, a.seq), device="cuda", generator=g)
    y = torch.randint(0, cfg.vocab_size, (a.m * a.mbs, a.seq), device="cuda", generator=g)
    losses, times = [], []
    for i in range(a.steps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        loss = tr.train_step(x, y)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t)
        losses.append(float(loss))
        print(f"step {i} loss {losses[-1]:.4f} {times[-1]:.3f}s", flush=True)
    best = min(times[1:]) if len(times) > 1 else times[0]
    tok = a.m * a.mbs * a.seq
    flops = cfg.flops_per_token(a.seq) * tok
    print(json.dumps({"model": "llama3-8b" + (f"-L{a.layers}" if a.layers else ""), "params": cfg.n_params(),
                      "seq": a.seq, "tokens_per_step": tok, "step_s": round(best, 4),
                      "tokens_per_s": round(tok / best, 1), "model_tflops": round(flops / best / 1e12, 1),
                      "recompute": tr.recompute, "recompute_layers": tr.recompute_layers, "schedule": tr.schedule,
                      "m": a.m, "memory_plan_gb": None if tr.memory_plan is None else
                      {k: round(v / 1e9, 1) for k, v in tr.memory_plan.items() if k.startswith("bytes")},
                      "losses": [round(v, 4) for v in losses],
                      "hbm_reserved_peak_gb": round(torch.cuda.max_memory_reserved() / 1e9, 1),
                      "hbm_allocated_peak_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1),
                      "init_s": round(init_s, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
