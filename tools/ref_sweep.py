"""The reference's 54-run experiment sweep on this framework, in BASELINE.md's table format.

The notebook sweeps layers {4,8,12} x heads {4,8,12} x processes {2,4} x {GPipe, 1F1B,
Interleaved1F1B} with ``run_one_experiment(..., batch_size=32, seq_length=128,
num_iterations=5)`` (nb:345-392) and derives speedup vs GPipe and "efficiency" =
speedup / P x 100 (nb:402-433).  This runs exactly that through the reference-compatible
API (``mipipe.bench.compat``: same worker, same timed loop, same interleave rule, same
m=4), one process per GPU (RCCL) -- or on CPU/gloo -- and writes

* a markdown table with one row per run: our tok/s next to the reference's published
  number (parsed), the ratio, the measured and analytic bubble;
* the speedup / efficiency table next to the reference's;
* the raw rows as JSON.

    python tools/ref_sweep.py --device cuda --out profiles/ref_sweep      # needs >= 4 GPUs
    python tools/ref_sweep.py --device cpu --layers 4 --heads 4 ...       # CPU plumbing run
    MIPIPE_DIST_BACKEND=gloo python tools/ref_sweep.py --device cuda ...  # ranks share 1 GPU
                                                                          # (timings meaningless)

Precision: ``--engine native`` runs the HIP kernels at ``--precision`` (default fp32, the
reference's precision: f32 MFMA GEMMs, f32 flash attention, ...); ``--engine torch`` runs the
reference's own nn.Module graph in f32 on ATen.
"""
import argparse
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def reference_tables():
    """Table 1 {(L,H,P,sched): tok/s}, Table 2 {(L,H,P,sched): (speedup, eff)}."""
    thr, spd = {}, {}
    p1 = re.compile(r"^\| tokens/s \| (\d+) \| (\d+) \| (\d+) \| (\w+) \| \d+ \| ([\d,\.]+) \|")
    p2 = re.compile(r"^\| speedup \| (\d+) \| (\d+) \| (\d+) \| (\w+) \| \d+ \| ([\d\.]+) \| ([\d\.]+) \|")
    with open(os.path.join(ROOT, "BASELINE.md")) as f:
        for line in f:
            m = p1.match(line)
            if m:
                L, H, P, s, v = m.groups()
                thr[(int(L), int(H), int(P), s)] = float(v.replace(",", ""))
            m = p2.match(line)
            if m:
                L, H, P, s, sp, ef = m.groups()
                spd[(int(L), int(H), int(P), s)] = (float(sp), float(ef))
    return thr, spd


def fmt_table(df, eff, ref_thr, ref_spd, header: str) -> str:
    lines = [header, "",
             "| L | H | P | schedule | tok/s (this) | tok/s (reference, nb) | x | bubble measured | bubble analytic |",
             "|---|---|---|---|---|---|---|---|---|"]
    for _, r in df.sort_values(["n_layers", "n_heads", "num_processes", "schedule"]).iterrows():
        key = (int(r.n_layers), int(r.n_heads), int(r.num_processes), r.schedule)
        ref = ref_thr.get(key)
        b = r.get("bubble_fraction")
        a = r.get("analytic_bubble")
        lines.append(f"| {key[0]} | {key[1]} | {key[2]} | {key[3]} | {r.throughput:,.1f} | "
                     f"{'' if ref is None else f'{ref:,.2f}'} | {'' if ref is None else f'{r.throughput / ref:.1f}'} | "
                     f"{'' if b is None or b != b else f'{b:.3f}'} | {'' if a is None or a != a else f'{a:.3f}'} |")
    lines += ["", "| L | H | P | schedule | speedup vs GPipe (this) | efficiency % (this) | speedup (reference) | "
                  "efficiency % (reference) |", "|---|---|---|---|---|---|---|---|"]
    for _, r in eff.sort_values(["n_layers", "n_heads", "num_processes", "schedule"]).iterrows():
        key = (int(r.n_layers), int(r.n_heads), int(r.num_processes), r.schedule)
        rs = ref_spd.get(key)
        lines.append(f"| {key[0]} | {key[1]} | {key[2]} | {key[3]} | {r.speedup:.4f} | {r.efficiency:.2f} | "
                     f"{'' if rs is None else f'{rs[0]:.4f}'} | {'' if rs is None else f'{rs[1]:.2f}'} |")
    return "\n".join(lines) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default=None, choices=["cuda", "cpu"])
    ap.add_argument("--engine", default="auto", choices=["auto", "native", "torch"])
    ap.add_argument("--layers", type=int, nargs="+", default=[4, 8, 12])
    ap.add_argument("--heads", type=int, nargs="+", default=[4, 8, 12])
    ap.add_argument("--procs", type=int, nargs="+", default=[2, 4])
    ap.add_argument("--schedules", nargs="+", default=["GPipe", "1F1B", "Interleaved1F1B"])
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--timeout", type=float, default=600.0)
    ap.add_argument("--precision", default="fp32", choices=["fp32", "bf16"],
                    help="native engine compute precision (fp32 = the reference's)")
    ap.add_argument("--out", default=None, help="path prefix: writes <out>.md and <out>.json")
    a = ap.parse_args()
    import torch
    import mipipe  # noqa: F401
    from mipipe.bench import compat

    dev = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    df = compat.run_all_experiments(n_heads_list=tuple(a.heads), n_layers_list=tuple(a.layers),
                                    num_processes_list=tuple(a.procs), schedules=tuple(a.schedules),
                                    num_iterations=a.iters, batch_size=a.batch, seq_length=a.seq, device=dev,
                                    engine=a.engine, timeout=a.timeout, precision=a.precision)
    eff = compat.compute_speedup_and_efficiency(df) if len(df) else df
    ref_thr, ref_spd = reference_tables()
    engine = a.engine if a.engine != "auto" else ("native" if dev == "cuda" else "torch")
    header = (f"## Reference sweep on this framework: device={dev}, engine={engine} "
              f"({a.precision + ' HIP kernels' if engine == 'native' and dev == 'cuda' else 'f32 ATen'}), batch {a.batch} x seq "
              f"{a.seq}, m=4, {a.iters} timed iterations after 2 warmup (nb:345-392)"
              + (", all P ranks sharing ONE GPU, p2p staged through host memory by gloo (a lower bound for P GPUs)"
                 if os.environ.get("MIPIPE_DIST_BACKEND") == "gloo" and dev == "cuda" else ""))
    text = fmt_table(df, eff, ref_thr, ref_spd, header) if len(df) else header + "\n(no successful runs)\n"
    print(text)
    if a.out:
        with open(a.out + ".md", "w") as f:
            f.write(text)
        with open(a.out + ".json", "w") as f:
            json.dump({"device": dev, "engine": engine, "rows": df.to_dict(orient="records")}, f, indent=1)


if __name__ == "__main__":
    main()
