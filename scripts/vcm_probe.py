#!/usr/bin/env python3
"""VCM GPU vs oracle (counter RNG): merge counts and the sign of the film
differences on the pixels that differ by more than 1e-4 -- a symmetric spread
means merges flipping at the radius by an ulp of position, a one-sided one a
systematic difference."""
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

CASES = [("torus64_rf05", _scenes.torus, 64, 64, 3, 3, 0.05, 0, 10), ("torus64_win35", _scenes.torus, 64, 64, 2, 5, 0.05, 3, 5),
         ("torus256_ref", _scenes.torus, 256, 256, 2, 5489, 0.003, 0, 10), ("tent64", _scenes.tent, 64, 64, 2, 3, 0.05, 0, 10)]
for name, mk, W, H, it, seed, rf, lo, hi in CASES:
    path = mk(W, H)
    c = native.Context(native.Scene(path), 0)
    film, st = c.render_vcm(W, H, iterations=it, seed=seed, radius_factor=rf, min_path_length=lo, max_path_length=hi)
    ref, rst = _oracle.Scene(path).vcm(W, H, it, seed, mode=1, radius_factor=rf, min_len=lo, max_len=hi)
    a, b = film.astype(np.float64), ref.astype(np.float64)
    d = a - b
    rel = np.abs(d) / np.maximum(np.abs(b), 1e-3 * np.abs(b).mean())
    bad = rel > 1e-4
    r = {"case": name, "found": [int(st.vm_found), int(rst.vm_found)], "merged": [int(st.vm_merged), int(rst.vm_merged)],
         "queries": [int(st.vm_queries), int(rst.vm_queries)], "closest": [int(st.closest_rays), int(rst.closest_rays)],
         "bad_values": int(bad.sum()), "bad_neg": int((bad & (d < 0)).sum()), "bad_pos": int((bad & (d > 0)).sum()),
         "sum_d_bad": float(d[bad].sum()), "sum_ref": float(b.sum()), "bias": float(d.sum() / b.sum())}
    print(json.dumps(r), flush=True)
