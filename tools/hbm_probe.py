"""Physical HBM of one training configuration vs the engine's HBM plan.

Builds a PipelineTrainer on one GPU (HIP graphs, lanes as the trainer picks them), captures,
runs --steps steps, and prints one JSON line: the caching allocator's allocated and reserved
peaks, the device's used bytes (mem_get_info) at the end, the plan's bytes with and without
recompute, and the planned stash slots.  One configuration per process (peaks and graph
pools are per process).

    python tools/hbm_probe.py --schedule 1F1B --mbs 64 --microbatches 2 [--model gpt2-small]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: E402,F401
from mipipe.engine import PipelineTrainer  # noqa: E402
from mipipe.models.config import NativeConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--schedule", default="1F1B")
    ap.add_argument("--mbs", type=int, default=64)
    ap.add_argument("--microbatches", type=int, default=2)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--recompute", default="0")
    ap.add_argument("--pools", action="store_true", help="also report reserved / allocated bytes per allocator pool")
    a = ap.parse_args()
    cfg = NativeConfig.by_name(a.model)
    dev = torch.device("cuda", 0)
    free0, total = torch.cuda.mem_get_info(dev)
    rc = {"0": False, "1": True}.get(a.recompute, a.recompute)
    tr = PipelineTrainer(cfg, pp=1, schedule=a.schedule, n_microbatches=a.microbatches, mbs=a.mbs, seq_len=a.seq,
                         device=dev, graphs=True, recompute=rc)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randint(0, cfg.vocab_size, (a.microbatches * a.mbs, a.seq), device=dev, generator=g)
    y = torch.randint(0, cfg.vocab_size, (a.microbatches * a.mbs, a.seq), device=dev, generator=g)
    tr.capture_graphs(x, y)
    torch.cuda.reset_peak_memory_stats(dev)      # the steady state: training steps after setup
    for _ in range(a.steps):
        tr.train_step(x, y)
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info(dev)
    p = tr.memory_plan
    gb = 1e9
    out = {"model": a.model, "schedule": tr.schedule, "mbs": a.mbs, "microbatches": a.microbatches,
           "lanes": tr.lanes, "recompute": tr.recompute, "stash_slots": {str(k): v for k, v in p["stash_slots"].items()},
           "allocated_peak_gb": round(torch.cuda.max_memory_allocated(dev) / gb, 2),
           "reserved_peak_gb": round(torch.cuda.max_memory_reserved(dev) / gb, 2),
           "reserved_now_gb": round(torch.cuda.memory_reserved(dev) / gb, 2),
           "device_used_gb": round((total - free1) / gb, 2),
           "device_used_by_process_gb": round((free0 - free1) / gb, 2),
           "planned_gb": round((p["bytes_recompute"] if tr.recompute else p["bytes_no_recompute"]) / gb, 2),
           "planned_gb_no_recompute": round(p["bytes_no_recompute"] / gb, 2),
           "planned_gb_recompute": round(p["bytes_recompute"] / gb, 2),
           "stash_ring": os.environ.get("MIPIPE_STASH_RING", "1")}
    out["plan_over_reserved"] = round(out["planned_gb"] / out["reserved_peak_gb"], 3)
    if a.pools:
        # reserved vs allocated bytes per allocator pool (graph pools: the stash slots' and the
        # head's; (0, 0) is the default pool), and the largest blocks still allocated
        pools = {}
        for seg in torch.cuda.memory_snapshot():
            key = str(tuple(seg.get("segment_pool_id", (0, 0))))
            d = pools.setdefault(key, {"segments": 0, "reserved_gb": 0.0, "allocated_gb": 0.0})
            d["segments"] += 1
            d["reserved_gb"] += seg["total_size"] / gb
            d["allocated_gb"] += seg["allocated_size"] / gb
        out["pools"] = {k: {kk: (round(vv, 2) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in sorted(pools.items(), key=lambda kv: -kv[1]["reserved_gb"])}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
