"""Per-kernel statistics from a rocprofv3 SQLite output (``run_results.db``), in the
column layout of rocprofv3's kernel_stats.csv (Name, Calls, TotalDurationNs, AverageNs,
Percentage, MinNs, MaxNs), plus a flag for kernels that are not this framework's own
(ATen / hipBLASLt / MIOpen / rocBLAS / Tensile).

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db [--csv out.csv]"""
import argparse
import csv
import re
import sqlite3
import sys

FOREIGN = re.compile(r"at::|native::|Cijk_|hipblaslt|miopen|MIOpen|rocblas|Tensile|elementwise_kernel|"
                     r"vectorized_|cutlass|ck::", re.I)


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), min(duration), max(duration) from kernels group by name")
    out = []
    for name, n, tot, mn, mx in rows:
        out.append(dict(Name=name, Calls=n, TotalDurationNs=tot, AverageNs=tot / n, MinNs=mn, MaxNs=mx))
    total = sum(r["TotalDurationNs"] for r in out) or 1
    for r in out:
        r["Percentage"] = 100.0 * r["TotalDurationNs"] / total
        r["Foreign"] = bool(FOREIGN.search(r["Name"]))
    out.sort(key=lambda r: -r["TotalDurationNs"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    out = stats(a.db)
    keys = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "Foreign"]
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=keys)
            w.writeheader()
            w.writerows(out)
    for r in out[:25]:
        print(f"{r['Percentage']:6.2f}% {r['Calls']:6d} {r['AverageNs'] / 1e3:9.1f}us {'FOREIGN ' if r['Foreign'] else ''}"
              f"{r['Name'][:100]}")
    fr = [r for r in out if r["Foreign"]]
    print(f"foreign kernels: {len(fr)} names, {sum(r['Percentage'] for r in fr):.2f}% of kernel time", file=sys.stderr)


if __name__ == "__main__":
    main()
