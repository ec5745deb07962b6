import os, sys
sys.path.insert(0, "winmad-s-raytracer-v1.0_amd"); sys.path.insert(0, "tests")
import numpy as np
os.environ["WR_BVH_DIAG"] = "4"
from winmad_rt import native
import _scenes
s = native.Scene(_scenes.torus(256, 256)); c = native.Context(s, 0); c.set_trace_mode(native.TRACE_BVH)
rays = np.load("scripts/_dbg_bad_rays.npy")
h = c.trace_closest(rays)
for i in range(5):
    p = int(h["prim"][i])
    if p <= -2:
        dbg = -2 - p
        print(i, "n", dbg & 0xff, "r0", (dbg >> 8) & 1, "r1", (dbg >> 9) & 1, "0before1", (dbg >> 10) & 1, "off1", dbg >> 12)
    else:
        print(i, "prim", p, "t", float(h["t"][i]))
