#!/usr/bin/env python3
"""VCM GPU vs oracle bias, strategy by strategy: path-length windows and a
merge radius at its EPS floor (no merges) separate vertex merging from the
other strategies."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402

import _oracle  # noqa: E402
import _scenes  # noqa: E402
from winmad_rt import native  # noqa: E402

path = _scenes.torus(64, 64)
c = native.Context(native.Scene(path), 0)
o = _oracle.Scene(path)
for rf in (0.05, 1e-9):
    for lo, hi in ((0, 10), (2, 2), (3, 3), (4, 4), (5, 5), (3, 5)):
        film, st = c.render_vcm(64, 64, iterations=3, seed=3, radius_factor=rf, min_path_length=lo, max_path_length=hi)
        ref, rst = o.vcm(64, 64, 3, 3, mode=1, radius_factor=rf, min_len=lo, max_len=hi)
        a, b = film.astype(np.float64), ref.astype(np.float64)
        d = a - b
        s = max(b.sum(), 1e-30)
        rel = np.abs(d) / np.maximum(np.abs(b), 1e-3 * np.abs(b).mean() + 1e-30)
        bad = rel > 1e-4
        print(json.dumps({"rf": rf, "len": [lo, hi], "bias": float(d.sum() / s), "sum_ref": float(b.sum()),
                          "bad_neg": int((bad & (d < 0)).sum()), "bad_pos": int((bad & (d > 0)).sum()),
                          "merged": [int(st.vm_merged), int(rst.vm_merged)], "found": [int(st.vm_found), int(rst.vm_found)],
                          "shadow": [int(st.shadow_rays), int(rst.shadow_rays)]}), flush=True)
