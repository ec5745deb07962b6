#!/usr/bin/env python3
"""The plane-grazing probe's mismatching rays (tests/test_gpu_bvh.py), dumped
for analysis: each ray, the KD walk's and the BVH mode's (prim, t), and the
geometry of both triangles.  GPU box:  python scripts/graze_mismatch.py [scene]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "winmad-s-raytracer-v1.0_amd"))
import _scenes  # noqa: E402
from test_gpu_bvh import _plane_grazing_rays, _same_hits, big_torus, pair  # noqa: E402
from winmad_rt import native  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "torus"
path = {"torus": lambda: _scenes.torus(256, 256), "cbox": lambda: _scenes.cbox(256, 192),
        "torus1m": lambda: big_torus(64, 64)}[name]()
ref, fast = pair(path)
n = 600_000 if name != "torus1m" else 200_000
seeds = [int(x) for x in (sys.argv[2:] or ["99"])]
out = []
sc = native.Scene(path)
dump = sc.dump(os.path.join("/tmp", f"graze_{name}.txt"))
tris = [l.split() for l in dump.splitlines() if l.startswith("tri ")]
for seed in seeds:
    rays = _plane_grazing_rays(ref, n, seed)
    a = ref.trace_closest(rays)
    b = fast.trace_closest(rays)
    ok = _same_hits(a, b)
    for k in np.nonzero(~ok)[0]:
        rec = {"seed": seed, "k": int(k), "ray": [float.hex(float(x)) for x in rays[k]],
               "kd": [int(a["prim"][k]), float.hex(float(a["t"][k]))],
               "bvh": [int(b["prim"][k]), float.hex(float(b["t"][k]))]}
        for tag, p in (("kd_tri", a["prim"][k]), ("bvh_tri", b["prim"][k])):
            if p >= 0:
                rec[tag] = tris[int(p)][2:11]
        out.append(rec)
    print(name, seed, rays.shape[0], "rays", int((~ok).sum()), "mismatches", flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", f"graze_mm_{name}.json"), "w") as f:
    json.dump(out, f, indent=1)
