"""Planned pipeline efficiency of every schedule for a model, from the list-scheduled
lowered program and the stage cost model (models/native.py stage_cost_model: per-layer
and LM-head costs from measured kernel rates).  Efficiency = no-bubble time / simulated
makespan, so it includes the bubble, stage imbalance and the distributed head placement.

    python tools/schedule_table.py [--model gpt2-small] [--seq 1024] [--mbs 16]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--mbs", type=int, default=16)
    a = ap.parse_args()
    import mipipe  # noqa: F401
    from mipipe.models.config import NativeConfig
    from mipipe.models.native import balanced_layer_ranges, stage_cost_model
    from mipipe.parallel.headsplit import head_token_split, plan_head_schedule
    from mipipe.parallel.schedules import SCHEDULES, analytic_bubble, canonical_name, generate, stage_to_rank
    from mipipe.parallel.schedules import REQUIRED_STYLE
    cfg = NativeConfig.by_name(a.model)
    lc, hu, ec = stage_cost_model(cfg, a.seq)
    T = a.mbs * a.seq
    print(f"# {a.model}: layer cost {lc:.2f}, LM head {hu:.2f} layer units, embedding {ec:.2f}; mbs {a.mbs} x seq {a.seq}")
    print("| schedule | PP | v | m | layer split | head chunks | head lag | analytic bubble | planned efficiency |")
    print("|---|---|---|---|---|---|---|---|---|")
    for sched in ("GPipe", "1F1B", "Interleaved1F1B", "ZBH1", "ZBV"):
        name = canonical_name(sched)
        for pp in (2, 4, 8):
            v = SCHEDULES[name][1] if SCHEDULES[name][2] else 1
            S = pp * v
            if S > cfg.n_layers + 1:
                continue
            style = REQUIRED_STYLE.get(name, "loop")
            for m in (2 * pp, 4 * pp):
                lr = balanced_layer_ranges(cfg, S, a.seq, head_on_last=False)
                sc = [(r1 - r0) * lc + (ec if s == 0 else 0.0) + (0.1 if s == S - 1 else 0.0)
                      for s, (r0, r1) in enumerate(lr)]
                load = [sum(sc[s] for s in range(S) if stage_to_rank(s, pp, style) == r) for r in range(pp)]
                ch = head_token_split(T, load, hu, align=256)
                hc = {r: 3.0 * hu * ch[r] / T for r in range(pp) if ch[r] > 0}
                try:
                    base = generate(name, pp, m, v, style)
                    _, lag, mk = plan_head_schedule(base, pp, v, style, hc, sc)
                except Exception as e:  # noqa: BLE001
                    print(f"| {sched} | {pp} | {v} | {m} | - | - | - | - | n/a ({type(e).__name__}) |")
                    continue
                ideal = (3.0 * sum(sc) + sum(hc.values())) * m / pp
                print(f"| {sched} | {pp} | {v} | {m} | {[r1 - r0 for r0, r1 in lr]} | {ch} | {lag} | "
                      f"{analytic_bubble(name, pp, m, v):.3f} | {ideal / mk:.3f} |")


if __name__ == "__main__":
    main()
