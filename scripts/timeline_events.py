#!/usr/bin/env python3
"""One render's launch timeline from the library's own HIP events
(WR_TIMELINE=<file>, no profiler): C2 torus at 1920x1080, `iterations`
iterations on 16 pipelines.  Prints each pipeline's start / end, the
concurrency over time, and per-category sums.

    python scripts/timeline_events.py <iterations> [out.csv]
"""
import os
import sys
import tempfile

os.environ["GPU_MAX_HW_QUEUES"] = "16"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402

import _scenes  # noqa: E402
from winmad_rt import native  # noqa: E402

it = int(sys.argv[1])
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(tempfile.mkdtemp(), "tl.csv")
W, H = 1920, 1080
c = native.Context(native.Scene(_scenes.torus(W, H)), 0)
c.set_trace_mode(native.TRACE_BVH)
c.render_bdpt(W, H, iterations=2, seed=5489, iter_begin=1 << 20, time_kernels=1)  # warm-up
os.environ["WR_TIMELINE"] = out
_, st = c.render_bdpt(W, H, iterations=it, seed=5489, time_kernels=1)
del os.environ["WR_TIMELINE"]
rays = st.closest_rays + st.shadow_rays
rows = np.loadtxt(out, delimiter=",", ndmin=2)
names = {0: "trace", 1: "shade", 2: "resolve", 3: "gen", 4: "other"}
print(f"{it} iterations: {st.seconds * 1e3:.2f} ms host, {rays / st.seconds / 1e6:.0f} Mrays/s, "
      f"trace union {st.trace_wall_ms:.2f} ms")
end = rows[:, 3].max()
for p in sorted(set(rows[:, 0].astype(int))):
    r = rows[rows[:, 0] == p]
    busy = (r[:, 3] - r[:, 2]).sum()
    print(f"  pipe {p:2d}: {int(len(r)):4d} launches  first {r[:, 2].min():7.2f}  last {r[:, 3].max():7.2f} ms  "
          f"sum of launch spans {busy:7.2f}")
for cat in sorted(set(rows[:, 1].astype(int))):
    r = rows[rows[:, 1] == cat]
    print(f"  {names.get(cat, cat):8s} launches {len(r):5d}  mean span {np.mean(r[:, 3] - r[:, 2]) * 1e3:8.1f} us")
edges = np.linspace(0, end, 21)
conc = [int(((rows[:, 2] < b) & (rows[:, 3] > a)).sum()) for a, b in zip(edges[:-1], edges[1:])]
print("  pipelines with a launch in flight, per 5 % of the render:", conc)
