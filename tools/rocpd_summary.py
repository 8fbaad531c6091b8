"""Summarise a rocprofv3 rocpd database (run_results.db): per-kernel totals and the GPU's
busy fraction (union of kernel intervals over all streams) in a time window.

    python tools/rocpd_summary.py DB [--last-frac 0.3] [--top 25]"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-frac", type=float, default=0.3, help="window = the last fraction of the trace")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, stream_id, grid_x, grid_y, grid_z, workgroup_x from kernels "
                     "order by start").fetchall()
    t0, t1 = rows[0][1], max(r[2] for r in rows)
    w0 = t1 - (t1 - t0) * a.last_frac
    rows = [r for r in rows if r[1] >= w0]
    busy, cur_s, cur_e = 0, None, None
    for r in rows:
        s, e = r[1], r[2]
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = rows[-1][2] - rows[0][1]
    tot = defaultdict(lambda: [0, 0, set()])
    for name, s, e, st, gx, gy, gz, wx in rows:
        k = name.split("(")[0][:90]
        tot[k][0] += 1
        tot[k][1] += e - s
        tot[k][2].add((gx // max(wx, 1), gy, gz))
    summ = sum(v[1] for v in tot.values())
    streams = len({r[3] for r in rows})
    print(f"window {span / 1e6:.1f} ms, {len(rows)} kernels on {streams} streams, busy (union) "
          f"{busy / span * 100:.1f} %, summed kernel time {summ / span * 100:.1f} % of the window")
    print(f"{'kernel':90s} {'calls':>6s} {'total ms':>9s} {'avg us':>8s} {'%':>5s}  grids(wg)")
    for k, (n, d, g) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:a.top]:
        gs = sorted(g)[:3]
        print(f"{k:90s} {n:6d} {d / 1e6:9.2f} {d / n / 1e3:8.1f} {d / summ * 100:5.1f}  {gs}")


if __name__ == "__main__":
    main()
