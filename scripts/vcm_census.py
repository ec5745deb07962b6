#!/usr/bin/env python3
"""VCM light-vertex census, GPU vs oracle: with a merge radius covering the
whole scene every query finds every light vertex, so vm_found / vm_queries is
the number of light vertices of the iteration (per maximum path length)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import _oracle  # noqa: E402
import _scenes  # noqa: E402
from winmad_rt import native  # noqa: E402

for W, H, seed in ((16, 16, 3), (32, 32, 5)):
    path = _scenes.torus(W, H)
    c = native.Context(native.Scene(path), 0)
    o = _oracle.Scene(path)
    for hi in (2, 3, 4, 10):
        _, st = c.render_vcm(W, H, iterations=1, seed=seed, radius_factor=10.0, min_path_length=0, max_path_length=hi)
        _, rs = o.vcm(W, H, 1, seed, mode=1, radius_factor=10.0, min_len=0, max_len=hi)
        print(json.dumps({"film": [W, H], "maxlen": hi, "gpu_q_found": [int(st.vm_queries), int(st.vm_found)],
                          "orc_q_found": [int(rs.vm_queries), int(rs.vm_found)],
                          "gpu_nv": st.vm_found / max(1, st.vm_queries), "orc_nv": rs.vm_found / max(1, rs.vm_queries),
                          "closest": [int(st.closest_rays), int(rs.closest_rays)],
                          "emitter_first_orc": int(rs.vm_emitter_first)}), flush=True)
