#!/usr/bin/env python3
"""Per-launch trace log (WR_TRACE_LOG=1: every launch synchronised, rays and
search / resolve / hard durations) of single-iteration C2 renders, to find
slow hard-ray launches.  Usage: python scripts/slow_iter_probe.py [iter ...]"""
import os
import sys

os.environ["GPU_MAX_HW_QUEUES"] = "16"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import _scenes  # noqa: E402
from winmad_rt import native  # noqa: E402

W, H = 1920, 1080
c = native.Context(native.Scene(_scenes.torus(W, H)), 0)
c.set_trace_mode(native.TRACE_BVH)
c.render_bdpt(W, H, iterations=32, seed=5489, iter_begin=1 << 20)  # warm-up
for it in [int(a) for a in sys.argv[1:]] or [0, 64]:
    _, st = c.render_bdpt(W, H, iterations=1, seed=5489, iter_begin=it)
    print(f"iteration {it}: {st.seconds * 1e3:.2f} ms (untraced)", file=sys.stderr, flush=True)
os.environ["WR_TRACE_LOG"] = "1"
c2 = native.Context(native.Scene(_scenes.torus(W, H)), 0)
c2.set_trace_mode(native.TRACE_BVH)
for it in [int(a) for a in sys.argv[1:]] or [0, 64]:
    print(f"== iteration {it}", file=sys.stderr, flush=True)
    _, st = c2.render_bdpt(W, H, iterations=1, seed=5489, iter_begin=it)
