"""Summarise rocprofv3 counter_collection.csv files per kernel (sum over dispatches):
python tools/pmc_summary.py gpurun_out/gpmc"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(int)
for f in glob.glob(f"{d}/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:70]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k)
    for c in sorted(v):
        print(f"   {c:28s} {v[c]:.4g}")
    b = v.get("SQ_BUSY_CYCLES")
    if v.get("SQ_VALU_MFMA_BUSY_CYCLES") and v.get("GRBM_GUI_ACTIVE"):
        print(f"   -> MFMA busy per SIMD: {v['SQ_VALU_MFMA_BUSY_CYCLES'] / (v['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
    if v.get("SQ_WAIT_ANY") and v.get("SQ_WAVE_CYCLES"):
        print(f"   -> wait fraction: {v['SQ_WAIT_ANY'] / v['SQ_WAVE_CYCLES']:.3f}")
