#!/usr/bin/env python3
"""Flagship benchmark: GPT-2 pipeline-parallel training throughput on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model gpt2-small]
                    [--schedule 1F1B] [--mbs 8] [--seq 1024] [--microbatches M]

N GPUs = N pipeline stages (PP=N, one process per GPU, RCCL p2p over xGMI); for N>1 the
driver launches it with torch.distributed.run (if launched without it, this script
re-launches itself under torch.distributed.run).  Work per GPU is fixed as N grows:
``microbatches = 2*N`` (8 at PP=4, BASELINE config 2), microbatch = ``mbs`` sequences
of ``seq`` tokens, so the global batch grows with N ("weak" scaling).  Each timed step
is a full training step: all microbatch forwards/backwards through the lowered 1F1B
program, p2p of activations/grads, grad-norm clip and the fused AdamW update.

Prints ONE JSON line on rank 0 (value = whole-job tokens/s, max elapsed over ranks).
Random-init weights, synthetic uniform tokens (no dataset / checkpoint access).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = ("tokens/sec/node + pipeline bubble fraction, GPT-2 PP=1/2/4/8 (GPipe vs 1F1B vs interleaved)")
# Best published reference throughput (nb:683: L4 H4 P4 1F1B, CPU/gloo).
BASELINE_TOK_S = 3722.89


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--schedule", default="1F1B")
    ap.add_argument("--mbs", type=int, default=16)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--microbatches", type=int, default=None)
    ap.add_argument("--dp", type=int, default=1)
    # (not "--v": torch.distributed.run's argparse would take it for an abbreviation of
    # its --virtual-local-rank even after the script name)
    ap.add_argument("--vstages", type=int, default=None, help="virtual stages per rank (interleaved)")
    ap.add_argument("--recompute", nargs="?", const="1", default="0", choices=["0", "1", "auto"],
                    help="activation recompute: 1 (on), 0 (off), auto (HBM plan: only if the stash does not fit)")
    ap.add_argument("--graphs", type=int, default=None,
                    help="replay per-microbatch stage compute as HIP graphs (default: on for 1 GPU)")
    ap.add_argument("--no-split-head", action="store_true",
                    help="keep the LM head on the last stage (default with PP>1: distributed head)")
    ap.add_argument("--no-bubble", action="store_true", help="skip the profiled bubble-measurement step")
    ap.add_argument("--trace", default=None, help="write a Chrome trace of the profiled step (per rank)")
    return ap.parse_args()


def main():
    a = parse()
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    n = a.gpus if a.gpus is not None else world_env
    if n > 1 and world_env == 1 and "RANK" not in os.environ:
        # not launched by torch.distributed.run: launch ourselves (before touching the GPU)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", os.environ.get("MASTER_PORT", "29533"),
               os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    import torch
    import torch.distributed as dist
    import mipipe  # noqa: F401
    from mipipe.engine import PipelineTrainer
    from mipipe.models.config import NativeConfig
    from mipipe.parallel.mesh import init_distributed
    from mipipe.parallel.schedules import analytic_bubble

    rank, world, local_rank, device = init_distributed()
    if n != world:
        raise SystemExit(f"--gpus {n} but WORLD_SIZE={world}")
    dp = a.dp
    pp = world // dp
    m = a.microbatches if a.microbatches is not None else max(2, 2 * pp)
    cfg = NativeConfig.by_name(a.model)
    if a.graphs is None:
        a.graphs = 1 if world == 1 else 0
    trainer = PipelineTrainer(cfg, pp=pp, dp=dp, schedule=a.schedule if pp > 1 else "1F1B", n_microbatches=m,
                              mbs=a.mbs, seq_len=a.seq, v=a.vstages, device=device, recompute=a.recompute if a.recompute == "auto" else a.recompute == "1", seed=0,
                              split_head=False if a.no_split_head else None, graphs=bool(a.graphs))
    gb = dp * m * a.mbs
    g = torch.Generator(device=device).manual_seed(1234 + trainer.mesh.dp_rank)
    tokens = torch.randint(0, cfg.vocab_size, (m * a.mbs, a.seq), device=device, generator=g)
    targets = torch.randint(0, cfg.vocab_size, (m * a.mbs, a.seq), device=device, generator=g)

    if a.graphs:
        trainer.capture_graphs(tokens, targets)   # setup: capture per-microbatch HIP graphs

    def sync():
        if world > 1:
            dist.barrier()
        if device.type == "cuda":
            torch.cuda.synchronize()

    for _ in range(a.warmup):
        trainer.train_step(tokens, targets)
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = trainer.train_step(tokens, targets)
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    tokens_per_step = gb * a.seq
    value = tokens_per_step * a.steps / elapsed
    ms = elapsed / a.steps * 1e3

    # one extra profiled step: measured bubble = 1 - busy/step, max over ranks
    bubble = None
    if not a.no_bubble:
        trainer.runtime.profile = True
        trainer.train_step(tokens, targets)
        trainer.runtime.profile = False
        b = trainer.bubble()
        bt = torch.tensor([b], device=device, dtype=torch.float64)
        if world > 1:
            dist.all_reduce(bt, op=dist.ReduceOp.MAX)
        bubble = float(bt.item())
        if a.trace:
            from mipipe.utils.profiling import timeline_to_chrome
            timeline_to_chrome(trainer.runtime.last_timeline, f"{a.trace}.rank{rank}.json", rank)
    loss_val = None
    if trainer.is_last and loss is not None:
        loss_val = float(loss.item())
    flops = cfg.flops_per_token(a.seq) * value
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / BASELINE_TOK_S, 2),
        "baseline_ref": "BASELINE.md Table 1 best run 3722.89 tok/s (nb:683, reference toy model on CPU/gloo)",
        "dtype": "bf16",
        "data": "synthetic uniform tokens, random-init weights",
        "bubble_fraction": None if bubble is None else round(bubble, 4),
        "analytic_bubble": round(analytic_bubble(trainer.schedule, pp, m, trainer.v), 4),
        "model_tflops_per_gpu": round(flops / world / 1e12, 1),
        "config": {"model": a.model, "params": cfg.n_params(), "global_batch": gb, "seq_len": a.seq,
                   "micro_batch": a.mbs, "microbatches": m, "schedule": trainer.schedule, "v": trainer.v,
                   "parallelism": f"pp{pp}" + (f"_dp{dp}" if dp > 1 else ""),
                   "layer_split": trainer.layer_ranges, "optimizer": "AdamW(fused, clip 1.0)",
                   "hip_graphs": bool(a.graphs),
                   "recompute": trainer.recompute,
                   "native_runner": trainer.runtime.native_runner is not None,
                   "head": ("distributed, token chunks " + str(trainer.head_chunks)) if trainer.head is not None
                   else "last stage",
                   "head_lag": getattr(trainer, "head_lag", None),
                   "planned_efficiency": None if getattr(trainer, "planned_makespan", None) is None else
                   round(trainer.planned_ideal / trainer.planned_makespan, 3)},
    }
    if loss_val is not None:
        out["last_loss"] = round(loss_val, 4)
    # the loss lives on the last pipeline rank; rank 0 prints
    if world > 1 and trainer.head is None:
        lv = torch.tensor([loss_val if loss_val is not None else 0.0], device=device, dtype=torch.float64)
        dist.all_reduce(lv, op=dist.ReduceOp.SUM)
        out["last_loss"] = round(float(lv.item()) / dp, 4)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
