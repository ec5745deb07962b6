#!/usr/bin/env python3
"""Path-state HBM traffic of the vertex kernels (SURVEY 8(d) B_state), from the
FETCH_SIZE / WRITE_SIZE passes of scripts/pmc_trace.sh (serial, WR_PIPES=1).

    python scripts/state_traffic.py gpurun_out/pmc_bd gpurun_out/pmc_pt > profiles/r1/state_traffic.json

Per kernel: dispatches, HBM bytes read / written per dispatch (MI355X_MICROARCH.md
"HBM [CDNA4]": FETCH_SIZE and WRITE_SIZE in KiB, FETCH_SIZE counting half the
bytes on gfx950), mean dispatch duration in those passes, and the rate.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def kernel(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def main():
    out = {}
    for d in sys.argv[1:]:
        acc = defaultdict(lambda: defaultdict(list))
        for f in sorted(glob.glob(d + "/p*/run_counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] not in ("FETCH_SIZE", "WRITE_SIZE"):
                    continue
                k = kernel(r["Kernel_Name"])
                dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                acc[k][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"]), dur))
        for k, c in acc.items():
            if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
                continue
            n = len(c["FETCH_SIZE"])
            rd = 2 * 1024 * sum(v for _, v, _ in c["FETCH_SIZE"]) / n
            wr = 1024 * sum(v for _, v, _ in c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
            dur = sum(t for _, _, t in c["FETCH_SIZE"]) / n
            out[k] = {"source": d, "dispatches": n, "read_bytes_per_dispatch": round(rd),
                      "write_bytes_per_dispatch": round(wr), "mean_dispatch_ms": round(dur * 1e3, 4),
                      "hbm_gbs": round((rd + wr) / dur / 1e9, 1) if dur > 0 else None}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
