#!/usr/bin/env python3
"""Wait, VALU lane utilisation, SALU share and L2 hit rate per kernel from a
pmc_summary_<config>.json (scripts/summarize_profile.py): per-dispatch means.
    python scripts/pmc_ratios.py profiles/r6/pmc_summary_c2.json [kernel-prefix ...]"""
import json
import sys

d = json.load(open(sys.argv[1]))
want = sys.argv[2:] or ["k_trace_fast<false", "k_fast_resolve<false", "k_fast_hard<false", "k_camera_step", "k_light_shade"]
out = {}
for k, v in d.items():
    if not any(k.startswith(w) for w in want):
        continue
    m = {n: x["mean"] for n, x in v.items() if isinstance(x, dict) and "mean" in x}
    try:
        r = {"wait": m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"],
             "valu_lane_util": m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"]),
             "salu_over_valu": m["SQ_INSTS_SALU"] / m["SQ_INSTS_VALU"],
             "l2_hit": m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]),
             "wave_cycles_per_dispatch": m["SQ_WAVE_CYCLES"]}
    except (KeyError, ZeroDivisionError):
        continue
    out[k] = {a: round(b, 4) for a, b in r.items()}
print(json.dumps(out, indent=1))
