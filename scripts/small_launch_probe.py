"""What sets the duration of a small search launch?

Traces subsets of n rays (primaries in raster order, secondaries in random
directions, as scripts/coherence_probe.py makes them) through the C ABI in BVH
mode, REPS times each, and reports k_trace_fast / k_fast_resolve / k_fast_hard
durations per subset from a rocprofv3 kernel trace.

run:   rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 scripts/small_launch_probe.py DIR
parse: python3 scripts/small_launch_probe.py --parse DIR
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import coherence_probe as cp  # noqa: E402

REPS = 3


def run():
    from winmad_rt import native, scenes
    import tempfile
    W, H = 1920, 1080
    tmp = tempfile.mkdtemp()
    sc = native.Scene(scenes.write(os.path.join(tmp, "t.scene"), scenes.torus_scene(W, H)))
    ctx = native.Context(sc, 0)
    ctx.set_trace_mode(native.TRACE_BVH)
    pos = np.array([-603.8923, 1013.96, 1823.33], np.float32)
    fwd = np.array([0.11, -0.373, -0.921], np.float32)
    up = np.array([-0.25, 0.885, -0.389], np.float32)
    fwd /= np.linalg.norm(fwd)
    right = np.cross(fwd, up)
    right /= np.linalg.norm(right)
    up2 = np.cross(right, fwd)
    tx = np.tan(np.radians(34.6222) / 2)
    ys, xs = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    u = ((xs + 0.5) / W * 2 - 1) * tx
    v = ((ys + 0.5) / H * 2 - 1) * tx * H / W
    d = fwd[None] + u.reshape(-1, 1) * right[None] + v.reshape(-1, 1) * up2[None]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.broadcast_to(pos, d.shape)
    prim = native.rays_from_arrays(o, d)
    hits = ctx.trace_closest(prim)
    ok = hits["prim"] >= 0
    p, nrm = hits["p"][ok], hits["n"][ok]
    rng = np.random.default_rng(1)
    sd = rng.normal(size=p.shape).astype(np.float32)
    sd /= np.linalg.norm(sd, axis=1, keepdims=True)
    flip = (sd * nrm).sum(1) * (d[ok] * nrm).sum(1) > 0
    sd[flip] *= -1
    sec = native.rays_from_arrays((p + 1e-2 * sd).astype(np.float32), sd)
    names = []
    for n in (1024, 8192, 54144, 216576, 1048576):
        for kind, rays in (("primary", prim), ("secondary", sec)):
            idx = rng.choice(len(rays), n, replace=False)
            idx.sort()
            sub = rays[idx]
            for _ in range(REPS):
                ctx.trace_closest(sub)
                names.append((f"{kind} {n}", n))
    return names


if __name__ == "__main__":
    if sys.argv[1] == "--parse":
        cp.parse(sys.argv[2], json.load(open(os.path.join(sys.argv[2], "order.json"))))
    else:
        names = run()
        os.makedirs(sys.argv[1], exist_ok=True)
        with open(os.path.join(sys.argv[1], "order.json"), "w") as f:
            json.dump(names, f)
