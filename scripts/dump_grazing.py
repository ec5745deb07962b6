#!/usr/bin/env python3
"""Dump tests/test_gpu_bvh.py's plane-grazing corpus for one scene (same seed
and size as the test) with the reference mode's answers, for CPU analysis
(tests/native/cell_filter_check.cpp RAYS mode).

    python scripts/dump_grazing.py cbox gpurun_out/grazing_cbox.npz
"""
import os
import sys

import numpy as np

_REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(_REPO, "tests"))
sys.path.insert(0, os.path.join(_REPO, "winmad-s-raytracer-v1.0_amd"))
import _scenes  # noqa: E402
import test_gpu_bvh as T  # noqa: E402
from winmad_rt import native  # noqa: E402

name, out = sys.argv[1], sys.argv[2]
maker = dict(T.SCENES + [("torus1m", lambda: T.big_torus(64, 64))])[name]
ref, fast = T.pair(maker())
n = 600_000 if name != "torus1m" else 200_000
rays = T._plane_grazing_rays(ref, n, 99)
a = ref.trace_closest(rays)
b = fast.trace_closest(rays)
bad = np.nonzero(~T._same_hits(a, b))[0]
print(name, rays.shape, "mismatches", bad[:20])
np.savez(out, rays=rays, prim=a["prim"], t=a["t"], fprim=b["prim"], ft=b["t"], bad=bad)
