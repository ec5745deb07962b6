#!/usr/bin/env python3
"""Where do GPU BDPT films still split from the oracle's?  (debugging, GPU box)

For one case: the oracle renders with its traversal log on (every closest /
shadow query: ray and answer); the GPU traces the same rays through the C ABI
in both traversal modes and the answers are compared bit for bit; then both
films are rendered and the split pixels listed.

  python scripts/split_probe.py torus 100 60 3 21 [ctl]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import _oracle  # noqa: E402
import _scenes  # noqa: E402
from _parity import film_stats  # noqa: E402
from winmad_rt import native  # noqa: E402

scene, W, H, it, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
ctl = int(sys.argv[6]) if len(sys.argv) > 6 else 3
path = getattr(_scenes, scene)(W, H)

L = _oracle.lib()
L.cr_set_ray_log.argtypes = [C.POINTER(C.c_float), C.c_int64]
L.cr_ray_log_count.restype = C.c_int64
cap = W * H * it * 12 + 1024
log = np.zeros((cap, 8), np.float32)
L.cr_set_ray_log(log.ctypes.data_as(C.POINTER(C.c_float)), cap)
ref, rst = _oracle.Scene(path).bdpt(W, H, it, seed, mode=1, control_length=ctl)
n = L.cr_ray_log_count()
L.cr_set_ray_log(None, 0)
log = log[:n]
print(f"oracle: {n} traversal queries (closest {rst.closest_rays}, shadow {rst.shadow_rays})", flush=True)

rays = np.zeros((n, 8), np.float32)
rays[:, :6] = log[:, :6]
rays[:, 7] = 1e7
ref_prim = log[:, 7].copy().view(np.int32)
ref_t = log[:, 6]
ctx = native.Context(native.Scene(path), 0)
out = {"case": f"{scene}{W}x{H}_i{it}_s{seed}_ctl{ctl}", "queries": int(n)}
for name, mode in (("bvh", native.TRACE_BVH), ("kd", native.TRACE_REFERENCE)):
    ctx.set_trace_mode(mode)
    h = ctx.trace_closest(rays)
    dp = np.nonzero(h["prim"] != ref_prim)[0]
    hit = (h["prim"] >= 0) & (ref_prim >= 0)
    dt = np.nonzero(hit & (h["t"].view(np.int32) != ref_t.view(np.int32)))[0]
    out[name] = {"prim_diff": int(dp.size), "t_diff": int(dt.size)}
    for k in dp[:8]:
        print(f"  {name} prim diff q{k}: ray {rays[k, :6].tolist()} oracle {ref_prim[k]} t {ref_t[k]!r} "
              f"gpu {h['prim'][k]} t {h['t'][k]!r}", flush=True)
ctx.set_trace_mode(native.TRACE_BVH)
film, st = ctx.render_bdpt(W, H, iterations=it, seed=seed, control_length=ctl)
s = film_stats(film, ref)
a, b = film.astype(np.float64), ref.astype(np.float64)
bad = np.argwhere((np.abs(a - b) / np.maximum(np.abs(b), 1e-3 * np.abs(b).mean() + 1e-30) > 1e-4).any(-1))
out["bad_pixels"] = int(s["bad_pixels"])
out["bias"] = s["bias"]
out["rays"] = [int(st.closest_rays), int(st.shadow_rays), int(rst.closest_rays), int(rst.shadow_rays)]
out["bad_list"] = [[int(i), int(j), a[i, j].tolist(), b[i, j].tolist()] for i, j in bad[:12]]
print(json.dumps(out), flush=True)
