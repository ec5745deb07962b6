"""Summarise scripts/pmc_trace.sh output: per kernel, counter totals over the
dispatches and the derived issue / wait / VALU-utilisation ratios.
    python scripts/pmc_report.py gpurun_out/pmc_<tag> [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

src = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else ""
tot = defaultdict(lambda: defaultdict(float))
for f in sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if want and want not in k:
            continue
        key = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:48]
        tot[key][row["Counter_Name"]] += float(row["Counter_Value"])
for k, c in tot.items():
    print(k)
    for n in sorted(c):
        print(f"   {n:28s} {c[n]:.4g}")
    wc = c.get("SQ_WAVE_CYCLES", 0)
    if wc:
        for n in ("SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if n in c:
                print(f"   {n + ' / wave cycles':40s} {c[n] / wc:.3f}")
    if c.get("SQ_ACTIVE_INST_VALU") and c.get("SQ_THREAD_CYCLES_VALU"):
        print(f"   VALU lane utilisation                    {c['SQ_THREAD_CYCLES_VALU'] / (64 * c['SQ_ACTIVE_INST_VALU']):.3f}")
    if c.get("SQ_WAVES"):
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH"):
            if n in c:
                print(f"   {n + ' per wave':40s} {c[n] / c['SQ_WAVES']:.1f}")
