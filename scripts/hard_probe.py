#!/usr/bin/env python3
"""Per-launch search / resolve / hard timing and the hard rays' kinds for one
C2 iteration (WR_TRACE_LOG=1 prints every launch; count_work=1 adds the
latency and walk counters).  Diagnostics (GPU box).

    WR_TRACE_LOG=1 python scripts/hard_probe.py [iterations] [count]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import _scenes  # noqa: E402
from winmad_rt import native  # noqa: E402

it = int(sys.argv[1]) if len(sys.argv) > 1 else 1
count = int(sys.argv[2]) if len(sys.argv) > 2 else 1
c = native.Context(native.Scene(_scenes.torus(1920, 1080)), 0)
c.render_bdpt(1920, 1080, iterations=1, seed=7, iter_begin=1000)  # warm-up
print("---- timed", flush=True)
f, st = c.render_bdpt(1920, 1080, iterations=it, seed=5489, count_work=count)
print("rays", st.closest_rays + st.shadow_rays, "fallback", st.fallback_rays, "seconds", st.seconds, flush=True)
