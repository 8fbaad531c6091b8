#!/usr/bin/env python3
"""The reference's own hardware class: CPU processes over gloo, its 9 (L, H) configs at
P = 2 (and optionally 4), its three schedules -- run with

* ``reference``: the reference's helper unchanged (torch.distributed.pipelining +
  nn.TransformerDecoderLayer autograd; /root/reference/LLMsDistributedTrainingHelper.py
  worker_process, imported read-only), when the file is present;
* ``torch``: this framework's runtime (lowered schedule, executor, gloo p2p) around the
  same nn.Module stages (bench/compat.py engine='torch');
* ``native``: this framework's runtime around the explicit-backward NativeModel (f32).

Same batch 32 x seq 128, m = 4, 2 warmup + 5 timed steps (nb:306, nb:372, helper:113).
Writes a JSON with every row and a markdown table with the per-engine speedup vs GPipe
next to the published one (nb:802-837), answering whether 1F1B >= GPipe here.

    python tools/cpu_gloo_table.py --out profiles/r4_cpu_gloo_table [--procs 2] [--engines reference,torch,native]
"""
import argparse
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = "/root/reference/LLMsDistributedTrainingHelper.py"

# published throughput: (L, H, P, schedule) -> tok/s
from mipipe.bench.published import PUBLISHED as PUB, SCHEDULES as SCHEDS  # noqa: E402


def _ref_worker(rank, world, L, H, sched, B, S, iters, q, port):
    """Runs the reference's worker_process in a spawned process (its own env setup uses a
    fixed port; ours is set first and it overwrites MASTER_PORT with 29500 -- runs are
    sequential, so that is safe)."""
    spec = importlib.util.spec_from_file_location("ref_helper", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.worker_process(rank, world, L, H, sched, B, S, iters, q)


def run_reference(L, H, P, sched, B=32, S=128, iters=5, timeout=600):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_ref_worker, args=(r, P, L, H, sched, B, S, iters, q, 29500)) for r in range(P)]
    for p in ps:
        p.start()
    try:
        res = q.get(timeout=timeout)
    except Exception:
        res = {"error": "no result"}
    for p in ps:
        p.join(30)
        if p.is_alive():
            p.terminate()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="profiles/r4_cpu_gloo_table")
    ap.add_argument("--procs", default="2")
    ap.add_argument("--engines", default="reference,torch,native")
    ap.add_argument("--layers", default="4,8,12")
    ap.add_argument("--heads", default="4,8,12")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--reps", type=int, default=1, help="repetitions per (config, engine), interleaved; md = median")
    ap.add_argument("--append", default=None, help="earlier rows (JSON) to merge in as repetitions")
    a = ap.parse_args()
    from mipipe.bench import compat
    engines = [e for e in a.engines.split(",") if e and (e != "reference" or os.path.exists(REF))]
    rows = []
    if a.append:
        with open(os.path.join(ROOT, a.append)) as f:
            rows = [dict(r, rep=r.get("rep", 0)) for r in json.load(f)]
    rep0 = 1 + max((r["rep"] for r in rows), default=-1)
    path_json = os.path.join(ROOT, a.out + ".json")
    for L in [int(x) for x in a.layers.split(",")]:
        for H in [int(x) for x in a.heads.split(",")]:
            for P in [int(x) for x in a.procs.split(",")]:
                for rep in range(rep0, rep0 + a.reps):
                    for sched in SCHEDS:
                        for eng in engines:
                            t0 = time.time()
                            if eng == "reference":
                                m = run_reference(L, H, P, sched, iters=a.iters)
                            else:
                                m = compat.run_one_experiment(L, H, P, sched, batch_size=32, seq_length=128,
                                                              num_iterations=a.iters, device="cpu", engine=eng,
                                                              timeout=900)
                            row = dict(n_layers=L, n_heads=H, num_processes=P, schedule=sched, engine=eng, rep=rep,
                                       wall_s=round(time.time() - t0, 1), published=PUB.get((L, H, P, sched)))
                            row.update({k: v for k, v in m.items()
                                        if isinstance(v, (int, float, str, bool)) or v is None})
                            rows.append(row)
                            print(json.dumps(row), flush=True)
                            with open(path_json, "w") as f:
                                json.dump(rows, f, indent=1)
    write_md(rows, os.path.join(ROOT, a.out + ".md"), engines)


def write_md(rows, path, engines):
    import statistics
    grp = {}
    for r in rows:
        if r.get("throughput"):
            grp.setdefault((r["n_layers"], r["n_heads"], r["num_processes"], r["schedule"], r["engine"]),
                           []).append(r["throughput"])
    # median over repetitions
    by = {k: {"throughput": statistics.median(v), "n": len(v)} for k, v in grp.items()}
    nrep = max((v["n"] for v in by.values()), default=1)
    lines = ["# CPU/gloo, the reference's configs (batch 32 x 128, m = 4, 5 timed steps), this container's 8 CPUs",
             "", f"tok/s per engine (median of up to {nrep} interleaved repetitions); "
             "speedup = tok/s / GPipe tok/s of the same engine and (L, H, P); "
             "`pub` = the notebook's published speedup (nb:802-837, 10-core CPU).", ""]
    hdr = "| L | H | P | schedule | " + " | ".join(f"{e} tok/s | {e} speedup" for e in engines) + " | pub tok/s | pub speedup |"
    lines += [hdr, "|" + "---|" * (hdr.count("|") - 1)]
    keys = sorted({k[:4] for k in by})
    for L, H, P, s in keys:
        cells = []
        for e in engines:
            r = by.get((L, H, P, s, e), {})
            g = by.get((L, H, P, "GPipe", e), {})
            t, tg = r.get("throughput"), g.get("throughput")
            cells.append(f"{t:.1f}" if t else "err")
            cells.append(f"{t / tg:.3f}" if (t and tg) else "-")
        pub, pubg = PUB.get((L, H, P, s)), PUB.get((L, H, P, "GPipe"))
        tail = f" | {pub} | {pub / pubg:.3f} |" if (pub and pubg) else " | - | - |"
        lines.append(f"| {L} | {H} | {P} | {s} | " + " | ".join(cells) + tail)
    # mean speedups
    lines += ["", "Mean speedup vs GPipe over the (L, H) configs:", ""]
    for e in engines + ["published"]:
        for P in sorted({k[2] for k in keys}):
            for s in SCHEDS[1:]:
                sp = []
                for L, H in sorted({(k[0], k[1]) for k in keys}):
                    if e == "published":
                        a_, b_ = PUB.get((L, H, P, s)), PUB.get((L, H, P, "GPipe"))
                    else:
                        a_ = by.get((L, H, P, s, e), {}).get("throughput")
                        b_ = by.get((L, H, P, "GPipe", e), {}).get("throughput")
                    if a_ and b_:
                        sp.append(a_ / b_)
                if sp:
                    lines.append(f"- {e}, P={P}, {s}: {sum(sp) / len(sp):.3f} "
                                 f"(min {min(sp):.3f}, max {max(sp):.3f}, {sum(1 for x in sp if x >= 1.0)}/{len(sp)} >= 1)")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
