"""Step timeline from a rocprofv3 kernel trace (csv): for the last complete training step
(AdamW kernel to AdamW kernel) report wall time, GPU-busy time (union of all kernel
intervals), idle gaps, per-stream busy time, and per-kernel time split into "alone"
(the only kernel running) vs "overlapped".

    python tools/timeline_stats.py gpurun_out/prof_ref/kernel_trace.csv [--steps 1]"""
import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        stream = r.get("Stream_Id") or r.get("Queue_Id") or "0"
        ks.append((s, e, r["Kernel_Name"], stream))
    ks.sort()
    ends = [e for s, e, n, _ in ks if n.startswith("adamw_kernel")]
    if len(ends) < a.steps + 1:
        raise SystemExit(f"need {a.steps + 1} AdamW kernels, found {len(ends)}")
    t0, t1 = ends[-1 - a.steps], ends[-1]
    win = [(max(s, t0), min(e, t1), n, st) for s, e, n, st in ks if e > t0 and s < t1]
    # sweep: busy union and per-kernel alone / overlapped time
    ev = []
    for i, (s, e, n, st) in enumerate(win):
        ev.append((s, 1, i))
        ev.append((e, -1, i))
    ev.sort()
    active = set()
    last = t0
    busy = 0
    alone = defaultdict(float)
    over = defaultdict(float)
    gaps = []
    for t, kind, i in ev:
        dt = t - last
        if dt > 0:
            if active:
                busy += dt
                for j in active:
                    (alone if len(active) == 1 else over)[win[j][2]] += dt / len(active)
            else:
                gaps.append(dt)
        last = t
        if kind == 1:
            active.add(i)
        else:
            active.discard(i)
    if t1 > last:
        gaps.append(t1 - last)
    wall = t1 - t0
    per_stream = defaultdict(int)
    for s, e, n, st in win:
        per_stream[st] += e - s

    def short(n):
        return n.split("(")[0].replace("void ", "")[:70]
    tot = defaultdict(float)
    for n in set(alone) | set(over):
        tot[short(n)] += alone.get(n, 0) + over.get(n, 0)
    al = defaultdict(float)
    for n, v in alone.items():
        al[short(n)] += v
    top = sorted(tot.items(), key=lambda x: -x[1])[: a.top]
    out = {"steps": a.steps, "wall_ms": wall / 1e6 / a.steps, "busy_ms": busy / 1e6 / a.steps,
           "idle_ms": sum(gaps) / 1e6 / a.steps, "n_gaps": len(gaps) // a.steps,
           "gaps_over_5us": sum(1 for g in gaps if g > 5000) // a.steps,
           "kernels_per_step": len(win) // a.steps,
           "per_stream_kernel_ms": {k: round(v / 1e6 / a.steps, 3) for k, v in per_stream.items()},
           "top_kernels_ms (share of busy time; alone)": [
               (n, round(v / 1e6 / a.steps, 3), round(al.get(n, 0) / 1e6 / a.steps, 3)) for n, v in top]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
