#!/usr/bin/env python3
"""Reproduce the bench line's roofline fraction from a rocprofv3 kernel trace.

The line's `roofline.frac` prices the step's algorithmic bytes over the union
of the traversal launches' intervals, which bench.py measures with HIP events
on every pipeline's stream (`trace_wall_ms`).  This script takes the same
union from the rocprofv3 kernel trace of the same command -- the intervals of
the timed (non-counting) traversal kernels: k_trace_fast, k_fast_resolve,
k_fast_hard and the KD walk k_trace -- and recomputes achieved / peak with the
line's own algorithmic bytes.  The warm-up and the counting replay run the
counting builds (`<true, ...>`) and are excluded by name; the trace pass runs
with --no-compare so that no other timed traversal is in the trace.

    python scripts/trace_union.py <rocprof out dir> <file holding the bench line> [--out profiles/r6/trace_union_c2.json]
"""
import argparse
import csv
import glob
import json
import os
import re

TIMED = re.compile(r"k_trace_fast<false|k_fast_resolve<false|k_fast_hard<false|k_trace<false")


def union_ns(iv):
    iv.sort()
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("line_file")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *kernel_trace.csv under {a.trace_dir}")
    iv, names = [], {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "")
                if not TIMED.search(k):
                    continue
                s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
                iv.append((s, e))
                short = k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
                names[short] = names.get(short, 0) + 1
    line = None
    with open(a.line_file) as f:
        for ln in f:
            if ln.startswith("{"):
                line = json.loads(ln)
    if line is None or not line.get("roofline"):
        raise SystemExit("no bench line with a roofline in " + a.line_file)
    r = line["roofline"]
    u_ms = union_ns(iv) / 1e6
    span_ms = (max(e for _, e in iv) - min(s for s, _ in iv)) / 1e6 if iv else 0.0
    total_bytes = r["algorithmic_bytes_per_step"] * line["steps"]
    achieved = total_bytes / (u_ms / 1e3) / 1e9
    frac = achieved / r["peak"]
    out = {"source": os.path.relpath(a.trace_dir), "launches": len(iv), "kernels": names,
           "union_ms": round(u_ms, 3), "span_ms": round(span_ms, 3),
           "line_trace_wall_ms": r["trace_wall_ms"], "union_over_line": round(u_ms / r["trace_wall_ms"], 4),
           "algorithmic_bytes_per_step": r["algorithmic_bytes_per_step"], "steps": line["steps"],
           "achieved_gbs": round(achieved, 1), "peak_gbs": r["peak"], "frac_from_trace": round(frac, 4),
           "line_frac": r["frac"], "frac_over_line": round(frac / r["frac"], 4),
           "line_frac_step": r.get("frac_step"), "line_ms_per_step": line["ms_per_step"],
           "frac_step_recomputed": round(r["algorithmic_bytes_per_step"] / (line["ms_per_step"] / 1e3) / 1e9
                                         / r["peak"], 4),
           "lib": line.get("lib_sha")}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
