#!/usr/bin/env python3
"""Speed of the KD walks of k_fast_hard: every ray to the walk
(WR_BVH_DIAG=256) through wr_trace_closest (one ray per wave), the wave-wide
walk (kd_walk_wave) against the serial one (WR_WALK_WAVE=0), on the 1M-triangle
torus and torus.scene.  Prints one JSON line per (scene, mode).

    python scripts/walk_speed.py [nrays]
"""
import json
import os
import subprocess
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def child(scene_name, n):
    sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "winmad-s-raytracer-v1.0_amd")]
    import numpy as np
    import test_gpu_bvh as T
    import _scenes
    from winmad_rt import native
    path = T.big_torus(64, 64) if scene_name == "torus1m" else _scenes.torus(256, 256)
    s = native.Scene(path)
    c = native.Context(s, 0, trace=native.TRACE_BVH)
    rays, _ = T._corpus(c, n, 5)
    rays = rays[:n]
    c.trace_closest(rays[:1024])
    t0 = time.perf_counter()
    h = c.trace_closest(rays)
    dt = time.perf_counter() - t0
    print(json.dumps({"scene": scene_name, "walk_wave": os.environ.get("WR_WALK_WAVE", "1"), "rays": int(rays.shape[0]),
                      "seconds": round(dt, 4), "us_per_ray_wave": round(dt / rays.shape[0] * 1e6, 3),
                      "hits": int((h["prim"] >= 0).sum())}))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]))
        sys.exit(0)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    for scene in ("torus", "torus1m"):
        for ww in ("1", "0"):
            env = dict(os.environ, WR_BVH_DIAG="256", WR_WALK_WAVE=ww)
            r = subprocess.run([sys.executable, __file__, "--child", scene, str(n)], env=env, timeout=300)
            if r.returncode:
                sys.exit(r.returncode)
