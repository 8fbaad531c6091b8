#!/usr/bin/env python3
"""Training entry point: one process per GPU (torchrun), config from YAML/JSON + overrides.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py --config configs/gpt2_small_pp8.yaml \
        train.steps=200 train.ckpt_dir=/data/ckpt train.ckpt_every=50

    python train.py --reference-compat --pp 2          # the reference's experiment, CPU/gloo ok

Features: PP x DP mesh, any schedule, distributed head, warmup+cosine LR, grad-norm
clipping, JSONL metrics, periodic checkpoints (FQN-keyed shards) and resume at any
PP degree, fail-fast watchdog.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=None, help="YAML or JSON run config")
    ap.add_argument("--reference-compat", action="store_true", help="reference defaults (helper.py / notebook)")
    ap.add_argument("--pp", type=int, default=None, help="shortcut for parallel.pp")
    ap.add_argument("--dump-config", default=None, help="write the resolved config and exit")
    ap.add_argument("overrides", nargs="*", help="section.field=value")
    return ap.parse_args()


class TokenData:
    """Synthetic uniform tokens, a learnable synthetic stream (``pattern[:K]``: every
    sequence walks a fixed random permutation of K tokens, x[t+1] = perm[x[t]], from a
    random start -- a model that learns the K-entry successor table drives the loss to 0),
    or random windows of a memory-mapped token file (uint16 ``.bin`` / int32 ``.i32``);
    deterministic in (step, dp rank)."""

    def __init__(self, spec: str, vocab: int, n_seq: int, seq: int, device, dp_rank: int, seed: int):
        import numpy as np
        self.spec, self.vocab, self.n, self.S = spec, vocab, n_seq, seq
        self.device, self.dp_rank, self.seed = device, dp_rank, seed
        self.mm = None
        self.perm = None
        if spec.startswith("pattern"):
            import torch
            k = int(spec.split(":")[1]) if ":" in spec else min(vocab, 4096)
            g = torch.Generator().manual_seed(seed + 7)
            self.perm = torch.randperm(min(k, vocab), generator=g).to(device)
        elif spec != "synthetic":
            dt = np.int32 if spec.endswith(".i32") else np.uint16
            self.mm = np.memmap(spec, dtype=dt, mode="r")

    def batch(self, step: int):
        import numpy as np
        import torch
        if self.perm is not None:
            g = torch.Generator(device=self.device).manual_seed(self.seed * 1000003 + step * 131 + self.dp_rank)
            cur = torch.randint(0, self.perm.numel(), (self.n,), device=self.device, generator=g)
            cols = [cur]
            for _ in range(self.S):
                cur = self.perm[cur]
                cols.append(cur)
            x = torch.stack(cols, 1)
        elif self.mm is None:
            g = torch.Generator(device=self.device).manual_seed(self.seed * 1000003 + step * 131 + self.dp_rank)
            x = torch.randint(0, self.vocab, (self.n, self.S + 1), device=self.device, generator=g)
        else:
            rng = np.random.default_rng(self.seed * 1000003 + step * 131 + self.dp_rank)
            starts = rng.integers(0, len(self.mm) - self.S - 1, self.n)
            x = torch.from_numpy(np.stack([np.asarray(self.mm[s: s + self.S + 1], dtype=np.int64) for s in starts]))
            x = x.to(self.device)
        return x[:, :-1].contiguous(), x[:, 1:].contiguous()


def main():
    a = parse()
    import torch
    import mipipe  # noqa: F401
    from mipipe.config import RunConfig, lr_at
    from mipipe.engine import PipelineTrainer
    from mipipe.parallel.mesh import init_distributed
    from mipipe.utils.metrics import MetricsLogger, Watchdog

    ov = list(a.overrides) + ([f"parallel.pp={a.pp}"] if a.pp else [])
    if a.reference_compat:
        cfg = RunConfig.reference_compat(pp=a.pp or 2)
        for o in a.overrides:
            cfg.set(o)
    else:
        cfg = RunConfig.load(a.config, ov)
    if a.dump_config:
        cfg.save(a.dump_config)
        return
    rank, world, local_rank, device = init_distributed()
    p, t = cfg.parallel, cfg.train
    if p.pp * p.dp != world:
        raise SystemExit(f"parallel.pp*dp = {p.pp * p.dp} but WORLD_SIZE = {world}")
    ncfg = cfg.native_config()
    m = cfg.microbatches
    trainer = PipelineTrainer(ncfg, pp=p.pp, dp=p.dp, schedule=p.schedule, n_microbatches=m, mbs=t.micro_batch,
                              seq_len=t.seq_len, v=p.v, device=device, lr=t.lr, weight_decay=t.weight_decay,
                              max_grad_norm=t.max_grad_norm, recompute=t.recompute, seed=t.seed, style=p.style,
                              layer_ranges=[tuple(r) for r in p.layer_ranges] if p.layer_ranges else None,
                              split_head=p.split_head,
                              dtype=torch.bfloat16 if device.type == "cuda" else torch.float32,
                              graphs=(device.type == "cuda") if t.graphs is None else bool(t.graphs))
    start = 0
    if t.resume:
        man = trainer.load_checkpoint(t.resume)
        start = int(man["step"])
        if rank == 0:
            print(f"resumed from {t.resume} at step {start} (saved at pp={man['pp']})", flush=True)
    data = TokenData(t.data, ncfg.vocab_size, m * t.micro_batch, t.seq_len, device, trainer.mesh.dp_rank, t.seed)
    if start < t.steps:
        # HIP graphs: two setup passes on the first batch capture every per-microbatch
        # action (gradients discarded, weights untouched); later steps replay them, from
        # the native stage runner once one step has been recorded
        trainer.capture_graphs(*data.batch(start))
    log = MetricsLogger(t.metrics_file, rank, device)
    wd = Watchdog(t.watchdog_s, describe=trainer.describe)
    tokens_per_step = p.dp * m * t.micro_batch * t.seq_len
    for step in range(start, t.steps):
        x, y = data.batch(step)
        lr = lr_at(step, t)
        t0 = time.perf_counter()
        with wd.step():
            loss = trainer.train_step(x, y, lr=lr)
            if device.type == "cuda":
                torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if (step + 1) % t.log_every == 0 or step == t.steps - 1:
            gn = (float(trainer.optimizer.sumsq.sqrt().item()) * trainer.optimizer.grad_scale  # un-scaled sums (1/dp folded)
                  if t.max_grad_norm else None)
            rec = log.log(step + 1, tokens_per_step, dt, loss=None if loss is None else float(loss), lr=lr,
                          grad_norm=gn)
            if rank == 0:
                print(f"step {step + 1:6d} loss {rec['loss']} lr {lr:.2e} {rec['tokens_per_s']:.0f} tok/s "
                      f"{rec['step_ms']:.1f} ms", flush=True)
        if t.ckpt_dir and t.ckpt_every and (step + 1) % t.ckpt_every == 0:
            trainer.save_checkpoint(os.path.join(t.ckpt_dir, f"step{step + 1:07d}"))
    wd.close()
    log.close()
    import torch.distributed as dist
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
