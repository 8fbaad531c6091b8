#!/usr/bin/env python3
"""Where does a schedule's step time go?  Measured per-action costs replayed in the simulator.

For one reference config (L, H, P; batch 32 x 128, m = 4, fwd+bwd, the compat API, helper:
150-235) and each of GPipe / 1F1B / Interleaved1F1B this runs P ranks (CPU/gloo, or
``--device cuda`` with MIPIPE_DIST_BACKEND=gloo: all ranks time-sharing ONE GPU), times
``--steps`` steps, then one profiled step whose per-action intervals (HIP events on GPU,
perf_counter on CPU; parallel/runtime.py) are gathered from every rank.  It reports:

* ``measured_ms``: the slowest rank's step time (max over ranks);
* ``sim_ms``: the same schedule's compute order replayed by :func:`parallel.simulate.simulate`
  with each rank's measured mean F / B duration per stage and zero transfer latency -- what
  the schedule costs with these kernels and perfect transport;
* ``transport_ms`` = measured - sim: p2p latency on the critical path (gloo host staging on
  GPU) plus any effect the simulator does not model (time-sharing of one device);
* ``busy_sum / step``: > 1 means the ranks' intervals overlap in time (they share the
  device: each action's measured duration is inflated by the other rank's concurrent work).

    python tools/schedule_attrib.py --layers 8 --heads 8 --procs 2 [--device cuda] [--out profiles/x.json]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _worker(rank, world, L, H, sched, device, steps, port, q, precision):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    try:
        import mipipe  # noqa: F401
        from mipipe.bench.compat import native_reference_schedule, stages_per_worker
        from mipipe.models.ref_transformer import ModelArgs, Transformer, manual_model_split, tokenwise_loss_fn
        from mipipe.parallel.api import get_schedule_class
        if device == "cuda":
            torch.cuda.set_device(0)
            dev = torch.device("cuda", 0)
        else:
            torch.set_num_threads(max(1, (os.cpu_count() or 2) // world))
            dev = torch.device("cpu")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.manual_seed(rank)
        args = ModelArgs(n_layers=L, n_heads=H)
        B, S, m = 32, 128, 4
        x = torch.randint(0, args.vocab_size, (B, S), device=dev)
        y = torch.randint(0, args.vocab_size, (B, S), device=dev)
        if device == "cuda":
            schedule = native_reference_schedule(args, sched, rank, world, B, S, m, dev, precision=precision,
                                                 lanes=1)
        else:
            spw = stages_per_worker(sched, L, world)
            stages = [manual_model_split(Transformer(args), rank + world * i, world * spw, dev) for i in range(spw)]
            cls = get_schedule_class(sched)
            schedule = cls(stages if spw > 1 or sched == "Interleaved1F1B" else stages[0], n_microbatches=m,
                           loss_fn=tokenwise_loss_fn(args.vocab_size))
        rt = schedule.runtime

        def one():
            first, last = rank == 0, rank == world - 1
            if first and last:
                schedule.step(x, target=y, losses=[])
            elif first:
                schedule.step(x)
            elif last:
                schedule.step(target=y, losses=[])
            else:
                schedule.step()

        def sync():
            dist.barrier()
            if device == "cuda":
                torch.cuda.synchronize()
        for _ in range(3):
            one()
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            one()
        sync()
        el = (time.perf_counter() - t0) / steps * 1e3
        rt.profile = True
        sync()
        one()
        rt.profile = False
        rec = {"rank": rank, "step_ms_timed": el, "timeline": rt.last_timeline, "step_ms": rt.last_step_ms,
               "orders": {str(r): [str(a) for a in acts] for r, acts in rt.orders.items()}, "v": rt.v}
        out = [None] * world
        dist.all_gather_object(out, rec)
        if rank == 0:
            q.put(out)
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback
        traceback.print_exc()
        q.put({"error": f"rank {rank}: {e}"})


def analyse(recs, P):
    from mipipe.parallel.ir import Action
    from mipipe.parallel.simulate import simulate
    v = recs[0]["v"]
    orders = {int(r): [Action.parse(a) for a in acts] for r, acts in recs[0]["orders"].items()}
    dur = {}
    busy = []
    import re
    lab = re.compile(r"^(\d+)(FL|F|B|I|W|H|M|C16)(\d+)$")   # native-tape graph labels (graphs.py)
    for rec in recs:
        b = 0.0
        for label, s, e in rec["timeline"]:
            b += e - s
            mt = lab.match(label)
            if mt is None:
                continue
            op = "F" if mt.group(2) == "FL" else mt.group(2)
            if op in ("F", "B"):
                dur.setdefault((int(mt.group(1)), op), []).append(e - s)
        busy.append(b)
    S = P * v
    # per-stage F and B costs (ms); the simulator takes op costs x per-stage scale: F = 1 x
    # fwd_ms[stage] via stage_costs, B cost ratio from the measured means
    fwd = [statistics.mean(dur.get((s, "F"), [0.0])) for s in range(S)]
    bwd = [statistics.mean(dur.get((s, "B"), [0.0])) for s in range(S)]
    from mipipe.parallel.ir import Op
    # one simulation with per-stage costs: F costs fwd[s]; B costs bwd[s] (stage_costs scales
    # both by the same factor, so express B as ratio x fwd and use the mean ratio per stage)
    ratio = statistics.mean(b / f for f, b in zip(fwd, bwd) if f > 0) if any(fwd) else 2.0
    sim = simulate(orders, P, v, "loop", costs={Op.F: 1.0, Op.B: ratio}, stage_costs=fwd)
    measured = max(r["step_ms"] for r in recs)
    timed = max(r["step_ms_timed"] for r in recs)
    return {"measured_ms": round(measured, 3), "timed_ms_per_step": round(timed, 3), "sim_ms": round(sim.makespan, 3),
            "transport_ms": round(measured - sim.makespan, 3), "sim_bubble": round(sim.bubble, 4),
            "measured_bubble": round(1 - sum(busy) / (P * measured), 4) if measured > 0 else None,
            "busy_sum_over_step": round(sum(busy) / measured, 3) if measured > 0 else None,
            "fwd_ms_per_stage": [round(x, 3) for x in fwd], "bwd_ms_per_stage": [round(x, 3) for x in bwd]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--heads", type=int, default=8)
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--schedules", default="GPipe,1F1B,Interleaved1F1B")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch.multiprocessing as mp
    from mipipe.bench.compat import _free_port
    out = {}
    for sched in a.schedules.split(","):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        ps = [ctx.Process(target=_worker, args=(r, a.procs, a.layers, a.heads, sched, a.device, a.steps, port, q,
                                                a.precision)) for r in range(a.procs)]
        for p in ps:
            p.start()
        recs = q.get(timeout=900)
        for p in ps:
            p.join(60)
        if isinstance(recs, dict):
            out[sched] = recs
        else:
            out[sched] = analyse(recs, a.procs)
        print(sched, json.dumps(out[sched]), flush=True)
    g = out.get("GPipe", {}).get("timed_ms_per_step")
    for s, r in out.items():
        if g and "timed_ms_per_step" in r:
            r["speedup_vs_gpipe"] = round(g / r["timed_ms_per_step"], 4)
    res = {"config": {"layers": a.layers, "heads": a.heads, "procs": a.procs, "device": a.device,
                      "precision": a.precision, "batch": 32, "seq": 128, "m": 4}, "schedules": out}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
