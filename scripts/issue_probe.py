#!/usr/bin/env python3
"""Host issue time against render time (WR_ISSUE_LOG): C2 torus 1080p,
BVH mode, 16 pipelines, for a few iteration counts, with and without the
per-launch timing events.  Shows whether a short render is bound by the
host's launch calls.

    python scripts/issue_probe.py
"""
import os
import sys

os.environ["GPU_MAX_HW_QUEUES"] = "16"
os.environ["WR_ISSUE_LOG"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import _scenes  # noqa: E402
from winmad_rt import native  # noqa: E402

W, H = 1920, 1080
c = native.Context(native.Scene(_scenes.torus(W, H)), 0)
c.set_trace_mode(native.TRACE_BVH)
c.render_bdpt(W, H, iterations=32, seed=5489, iter_begin=1 << 20)  # warm-up (buffers for 16 pipelines)
for it in [int(a) for a in sys.argv[1:]] or [1, 2, 4, 20]:
    for tk in (0,) if os.environ.get("WR_ISSUE_THREADS") else (0, 1):
        for rep in range(2):
            _, st = c.render_bdpt(W, H, iterations=it, seed=5489, iter_begin=rep * 64, time_kernels=tk)
            rays = st.closest_rays + st.shadow_rays
            print(f"iterations {it:3d} timing {tk}: {st.seconds * 1e3:8.2f} ms  {rays / st.seconds / 1e6:7.1f} Mrays/s",
                  file=sys.stderr, flush=True)
