#!/usr/bin/env python3
"""Condense a scripts/profile_round.sh output directory into profiles/<tag>/.

    python scripts/summarize_profile.py gpurun_out/prof_<tag> profiles/<tag>

Writes
  kernel_stats.csv  rocprofv3 --kernel-trace --stats summary (copied as is)
  pmc_summary.json  per kernel: dispatches and the per-dispatch mean of every
                    PMC counter collected in the separate --pmc passes
  traffic.json      HBM bytes per k_trace launch, per MI355X_MICROARCH.md
                    "HBM [CDNA4]": FETCH_SIZE / WRITE_SIZE are in KiB, and on
                    gfx950 FETCH_SIZE counts half the bytes of a read, so
                    traffic = 2 * 1024 * FETCH_SIZE + 1024 * WRITE_SIZE.
                    bench.py reports it as roofline.traffic.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

DOMINANT = "k_trace"


def short(name):
    """'void (anonymous namespace)::k_trace<false, false>(...)' -> 'k_trace<false, false>'"""
    base = name
    for part in name.replace("void ", "").split("::"):
        if part.startswith("k_"):
            base = part
            break
    return base.split("(")[0].strip()


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values (one per dispatch)
    for f in sorted(glob.glob(os.path.join(src, "pmc*", "run_counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                per[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    summary = {}
    for k, counters in per.items():
        summary[k] = {c: {"dispatches": len(v), "mean": sum(v) / len(v)} for c, v in counters.items()}
    with open(os.path.join(dst, "pmc_summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1, sort_keys=True)

    tr = [k for k in summary if k.startswith(DOMINANT)]
    out = {"kernel": DOMINANT, "variants": tr}
    if tr:
        def mean_of(counter):
            vals = [v for k in tr for v in per[k].get(counter, [])]
            return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)
        fetch, nf = mean_of("FETCH_SIZE")
        write, nw = mean_of("WRITE_SIZE")
        hit, _ = mean_of("TCC_HIT_sum")
        miss, _ = mean_of("TCC_MISS_sum")
        out.update({"fetch_kib_per_launch": fetch, "write_kib_per_launch": write, "launches": nf,
                    "hbm_bytes_per_launch": (2 * 1024 * fetch + 1024 * write)
                    if fetch is not None and write is not None else None,
                    "l2_hit_rate": hit / (hit + miss) if hit is not None and miss else None})
    with open(os.path.join(dst, "traffic.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))

    # the trace pass's bench line beside rocprof's own k_trace durations (the
    # warm-up runs the counting build, so k_trace<false, ...> = the timed launches)
    line = None
    log = os.path.join(src, "trace.log")
    if os.path.exists(log):
        with open(log) as fh:
            lines = [l for l in fh if l.startswith('{"metric"')]
        line = json.loads(lines[-1]) if lines else None
    if line and os.path.exists(stats):
        with open(os.path.join(dst, "bench_c2_profiled_run.json"), "w") as fh:
            fh.write(json.dumps(line) + "\n")
        rows = [r for r in csv.DictReader(open(stats)) if short(r["Name"]).startswith(DOMINANT + "<false")]
        calls = sum(int(r["Calls"]) for r in rows)
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        r = line["roofline"]
        cmp_ = {"rocprof_kernel": [short(r_["Name"]) for r_ in rows],
                "rocprof_calls": calls, "rocprof_avg_ms": round(tot / max(1, calls) / 1e6, 4),
                "bench_launches": r["launches"], "bench_event_avg_ms": r["avg_launch_ms"],
                "ratio_events_over_rocprof": round(r["avg_launch_ms"] / (tot / max(1, calls) / 1e6), 3)}
        with open(os.path.join(dst, "duration_check.json"), "w") as fh:
            json.dump(cmp_, fh, indent=1)
        print(json.dumps(cmp_))


if __name__ == "__main__":
    main()
