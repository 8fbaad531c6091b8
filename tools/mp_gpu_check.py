"""Multi-rank pipeline training check on GPU (ranks may share one GPU with
MIPIPE_DIST_BACKEND=gloo).  Prints the per-step losses as one JSON line on rank 0.

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/mp_gpu_check.py --schedule 1F1B [--graphs 1]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--schedule", default="1F1B")
    ap.add_argument("--graphs", type=int, default=0)
    ap.add_argument("--split-head", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--dp", type=int, default=1, help="data-parallel replicas (pp = world / dp)")
    ap.add_argument("--vstages", type=int, default=None, help="virtual stages per rank (Interleaved1F1B)")
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--microbatches", type=int, default=8, help="microbatches per replica x dp (same data for every world)")
    ap.add_argument("--mem", type=int, default=0, help="report every rank's HBM peak above its post-init level")
    ap.add_argument("--clip", type=float, default=1.0, help="max grad norm (the reported norms are pre-clip)")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    import mipipe  # noqa: F401
    from mipipe.engine import PipelineTrainer
    from mipipe.models.config import NativeConfig
    from mipipe.parallel.mesh import init_distributed
    rank, world, _, device = init_distributed()
    cfg = NativeConfig.gpt2("tiny", vocab_size=1000, d_model=256, n_layers=a.layers, n_heads=4, d_ff=1024, max_seq_len=256)
    m, mbs, S = a.microbatches, 2, 256   # same data for every world size
    dp = a.dp
    pp = world // dp
    if a.mem:
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(device)
    tr = PipelineTrainer(cfg, pp=pp, dp=dp, schedule=a.schedule if pp > 1 else "1F1B", n_microbatches=m // dp,
                         mbs=mbs,
                         seq_len=S, device=device, seed=3, graphs=bool(a.graphs),
                         split_head=bool(a.split_head), lr=1e-3, v=a.vstages if pp > 1 else None,
                         max_grad_norm=a.clip)
    g = torch.Generator(device=device).manual_seed(11)
    x = torch.randint(0, cfg.vocab_size, (m * mbs, S), device=device, generator=g)
    y = torch.randint(0, cfg.vocab_size, (m * mbs, S), device=device, generator=g)
    if dp > 1:   # each replica trains on its shard of the same global batch
        n = x.shape[0] // dp
        r = tr.mesh.dp_rank
        x, y = x[r * n:(r + 1) * n].contiguous(), y[r * n:(r + 1) * n].contiguous()
    if a.mem:
        torch.cuda.empty_cache()
    base = torch.cuda.memory_reserved(device) if a.mem else 0
    if a.graphs:
        tr.capture_graphs(x, y)
    if a.mem:
        # the steady state: what the device holds for the training steps (reserved: graph
        # pools keep their freed blocks), not the setup's eager step
        torch.cuda.reset_peak_memory_stats(device)
    losses, norms = [], []
    for _ in range(a.steps):
        loss = tr.train_step(x, y)
        norms.append(float(tr.optimizer.sumsq.sqrt()) if a.clip > 0 else None)
        v = torch.tensor([float(loss) if loss is not None else 0.0], dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(v)
            # the loss lives on one rank per replica (last stage) or on every rank (distributed head)
            v /= dp * (pp if tr.head is not None else 1)
        losses.append(float(v.item()))
    mem = None
    if a.mem:
        torch.cuda.synchronize()
        mine = torch.tensor([torch.cuda.max_memory_reserved(device) - base,
                             float(sum(st.stash_slots() for st in tr.stages))], dtype=torch.float64, device=device)
        allv = [torch.zeros_like(mine) for _ in range(world)] if world > 1 else [mine]
        if world > 1:
            dist.all_gather(allv, mine)
        mem = {"peak_above_init": [float(v[0]) for v in allv], "stash_slots": [int(v[1]) for v in allv]}
    if rank == 0:
        print(json.dumps({"world": world, "schedule": a.schedule, "losses": losses, "mem": mem, "norms": norms,
                          "native_runner": tr.runtime.native_runner is not None,
                          "native_reason": tr.runtime.native_reason,
                          "p2p": getattr(tr.runtime.p2p, "kind", None), "lanes": tr.runtime.lanes,
                          "placement": tr.runtime.coll_placement}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
