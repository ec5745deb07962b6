#!/usr/bin/env python3
"""Timeline of the last render in a rocprofv3 kernel trace: per queue, the
sequence of kernels of the timed render with durations and the idle gaps
between them; plus the fraction of wall time each kernel kind is running on
at least one queue.

    python scripts/timeline.py <run_kernel_trace.csv> [--from-kernel k_light_gen --nth -1]
"""
import csv
import sys
from collections import defaultdict


def short(n):
    for part in n.replace("void ", "").split("::"):
        if part.startswith("k_"):
            return part.split("(")[0]
    return n.split("(")[0]


rows = list(csv.DictReader(open(sys.argv[1])))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), short(r["Kernel_Name"]),
       int(r["VGPR_Count"]), int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))) for r in rows]
ks.sort()
# the timed render: the light-gen launches of the last render call (time_kernels run).  A render starts
# with k_light_gen on every pipeline; find the last cluster of them.
gens = [k for k in ks if k[3] == "k_light_gen" or k[3] == "k_camera_gen"]
lg = [k for k in ks if k[3] == "k_light_gen"]
# clusters separated by > 5 ms
clusters, cur = [], [lg[0]]
for k in lg[1:]:
    if k[0] - cur[-1][0] > 5e6:
        clusters.append(cur)
        cur = [k]
    else:
        cur.append(k)
clusters.append(cur)
nth = int(sys.argv[sys.argv.index("--nth") + 1]) if "--nth" in sys.argv else -1
start = clusters[nth][0][0]
end_next = clusters[nth + 1][0][0] if nth != -1 and nth + 1 < len(clusters) else float("inf")
sel = [k for k in ks if start <= k[0] < end_next]
# stop at the last kernel before a gap > 20 ms (the count replay etc.)
out = [sel[0]]
for k in sel[1:]:
    if k[0] - max(x[1] for x in out) > 20e6:
        break
    out.append(k)
t0, t1 = out[0][0], max(k[1] for k in out)
print(f"render: {len(out)} kernels over {(t1 - t0) / 1e6:.3f} ms, queues {sorted(set(k[2] for k in out))}")
busy = defaultdict(list)
for k in out:
    busy[k[3]].append((k[0], k[1]))
def union(iv):
    iv = sorted(iv)
    tot, lo, hi = 0, None, None
    for a, b in iv:
        if hi is None or a > hi:
            if hi is not None:
                tot += hi - lo
            lo, hi = a, b
        else:
            hi = max(hi, b)
    return tot + (hi - lo if hi is not None else 0)
print("kernel            launches  sum_ms   union_ms  share_of_wall  vgpr  max_grid")
for name, iv in sorted(busy.items(), key=lambda x: -union(x[1])):
    vg = max(k[4] for k in out if k[3] == name)
    gr = max(k[5] for k in out if k[3] == name)
    print(f"{name:18s} {len(iv):6d} {sum(b - a for a, b in iv) / 1e6:9.3f} {union(iv) / 1e6:9.3f} {union(iv) / (t1 - t0):10.3f}  {vg:5d} {gr:8d}")
print(f"any kernel running: {union([(k[0], k[1]) for k in out]) / (t1 - t0):.3f} of the wall")
q = sorted(set(k[2] for k in out))[0]
print(f"\nqueue {q} sequence (kernel, start_ms, dur_us, gap_before_us):")
prev = None
for k in [k for k in out if k[2] == q][:120]:
    gap = (k[0] - prev) / 1e3 if prev else 0
    print(f"  {k[3]:16s} {(k[0] - t0) / 1e6:8.3f} {(k[1] - k[0]) / 1e3:9.1f} {gap:8.1f}")
    prev = k[1]
