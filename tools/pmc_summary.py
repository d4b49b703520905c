"""Summarise rocprofv3 --pmc CSVs: mean counter value per kernel (per dispatch)."""
import csv
import glob
import os
import sys

root = sys.argv[1]
agg = {}
for f in glob.glob(os.path.join(root, "**", "run_counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, d in agg.items():
    if not any(x in k for x in ("pass_kernel", "extend_kernel", "shade_kernel")):
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:32s} n={len(v):3d} mean={sum(v) / len(v):.6g}")
