#!/usr/bin/env python3
"""Condense a scripts/profile_round.sh output directory into profiles/<tag>/.

    python scripts/summarize_profile.py gpurun_out/prof_<tag> profiles/<tag> [config]

Writes
  kernel_stats_<config>.csv  rocprofv3 --kernel-trace --stats summary (copied as is)
  pmc_summary_<config>.json  per kernel: dispatches and the per-dispatch mean of every
                    PMC counter collected in the separate --pmc passes
  traffic_<config>.json (config c2 when not given)
                    HBM bytes per traversal step (k_trace, or the BVH mode's
                    three kernels), per MI355X_MICROARCH.md
                    "HBM [CDNA4]": FETCH_SIZE / WRITE_SIZE are in KiB, and on
                    gfx950 FETCH_SIZE counts half the bytes of a read, so
                    traffic = 2 * 1024 * FETCH_SIZE + 1024 * WRITE_SIZE.
                    bench.py reports it as roofline.traffic.  Beside it the
                    path-state kernels' bytes (gen, vertex and resolve kernels:
                    everything but the traversal) per traversal step, and per
                    kernel -- bench.py's roofline.state_hbm -- and the sha256
                    prefix of the library the passes ran (lib.sha).
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
    config = sys.argv[3] if len(sys.argv) > 3 else "c2"
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, f"kernel_stats_{config}.csv"))
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values (one per dispatch)
    for f in sorted(glob.glob(os.path.join(src, "pmc*", "run_counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                per[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    summary = {}
    for k, counters in per.items():
        summary[k] = {c: {"dispatches": len(v), "mean": sum(v) / len(v)} for c, v in counters.items()}
    with open(os.path.join(dst, f"pmc_summary_{config}.json"), "w") as fh:
        json.dump(summary, fh, indent=1, sort_keys=True)

    # one traversal step = k_trace (reference mode) or k_trace_fast +
    # k_fast_resolve + k_fast_hard (BVH mode); per-step means over the dispatches
    bvh = any(k.startswith("k_trace_fast") for k in summary)
    fam = ("k_trace_fast", "k_fast_resolve", "k_fast_hard") if bvh else (DOMINANT,)
    lead = fam[0]
    tr = [k for k in summary if k.startswith(fam) and not k.startswith("k_trace_fast") or k.startswith(lead)]
    tr = [k for k in summary if any(k.startswith(f + "<") or k == f for f in fam)]
    out = {"kernel": " + ".join(fam), "variants": tr, "config": config}
    try:  # the build the counters describe (run here, after the box's files are pulled)
        import subprocess
        out["head"] = subprocess.run(["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True,
                                     cwd=os.path.dirname(os.path.abspath(__file__))).stdout.strip() or None
    except OSError:
        out["head"] = None
    if tr:
        steps = len([v for k in tr if k.startswith(lead + "<") or k == lead for v in per[k].get("FETCH_SIZE", [])])

        def per_step(counter):
            vals = [v for k in tr for v in per[k].get(counter, [])]
            return (sum(vals) / steps, steps) if vals and steps else (None, 0)
        fetch, nf = per_step("FETCH_SIZE")
        write, nw = per_step("WRITE_SIZE")
        hit, _ = per_step("TCC_HIT_sum")
        miss, _ = per_step("TCC_MISS_sum")
        out.update({"fetch_kib_per_launch": fetch, "write_kib_per_launch": write, "launches": nf,
                    "hbm_bytes_per_launch": (2 * 1024 * fetch + 1024 * write)
                    if fetch is not None and write is not None else None,
                    "l2_hit_rate": hit / (hit + miss) if hit is not None and miss else None})
        # every other kernel of the render (path state: gen, vertex / resolve
        # kernels, film clears) per traversal step, by kernel
        state = {}
        for k, cs in per.items():
            if k in tr or "true" in k.split("<", 1)[-1].split(",", 1)[0]:  # (the counting build: warm-up only)
                continue
            f, w = cs.get("FETCH_SIZE"), cs.get("WRITE_SIZE")
            if f and w and steps:
                state[k] = {"dispatches": len(f), "bytes_per_step": (2 * 1024 * sum(f) + 1024 * sum(w)) / steps}
        if state:
            out["state_kernels"] = state
            out["state_bytes_per_launch"] = sum(v["bytes_per_step"] for v in state.values())
    sha = os.path.join(src, "lib.sha")
    out["lib_sha"] = open(sha).read().strip() if os.path.exists(sha) else None
    with open(os.path.join(dst, f"traffic_{config}.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))

    # the trace pass's bench line beside rocprof's own durations of the timed
    # traversal steps (the warm-up runs the counting build, <true ...>; the
    # comparison leg in the other mode is skipped in profiled runs)
    line = None
    log = os.path.join(src, "trace.log")
    if os.path.exists(log):
        with open(log) as fh:
            lines = [l for l in fh if l.startswith('{"metric"')]
        line = json.loads(lines[-1]) if lines else None
    if line and os.path.exists(stats):
        with open(os.path.join(dst, f"bench_profiled_run_{config}.json"), "w") as fh:
            fh.write(json.dumps(line) + "\n")
        rows = [r for r in csv.DictReader(open(stats))
                if any(short(r["Name"]).startswith(f + "<false") for f in fam)]
        calls = sum(int(r["Calls"]) for r in rows if short(r["Name"]).startswith(lead + "<false"))
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        r = line["roofline"]
        cmp_ = {"rocprof_kernels": [short(r_["Name"]) for r_ in rows],
                "rocprof_steps": calls, "rocprof_avg_ms_per_step": round(tot / max(1, calls) / 1e6, 4),
                "bench_launches": r["launches"], "bench_event_avg_ms": r["avg_launch_ms"],
                "ratio_events_over_rocprof": round(r["avg_launch_ms"] / (tot / max(1, calls) / 1e6), 3)}
        with open(os.path.join(dst, f"duration_check_{config}.json"), "w") as fh:
            json.dump(cmp_, fh, indent=1)
        print(json.dumps(cmp_))


if __name__ == "__main__":
    main()
