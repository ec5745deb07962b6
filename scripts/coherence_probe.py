"""How much does ray order (coherence) change the BVH search's cost?

Traces the same ray sets in several orders through the C ABI (BVH mode) and
reports k_trace_fast's kernel duration per order from a rocprofv3 kernel trace
(usage at the bottom: a profiled run, then a parse step).

Ray sets (torus.scene, BDPT camera): primaries in raster order, and secondary
rays leaving the primaries' hit points in uniformly random directions.  Orders:
raster (path index), shuffled, Morton code of the origin, direction octant then
Morton code, and orders an append-time binning could give (octant, sign of x,
octant within blocks of consecutive rays).
"""
import csv
import glob
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))
REPS = 3


def morton(p, lo, hi, bits=10):
    q = np.clip(((p - lo) / np.maximum(hi - lo, 1e-9) * (1 << bits)).astype(np.int64), 0, (1 << bits) - 1)
    key = np.zeros(len(p), np.int64)
    for b in range(bits):
        for a in range(3):
            key |= ((q[:, a] >> b) & 1) << (3 * b + a)
    return key


def local_order(key, block):
    """Stable sort by `key` within each block of `block` consecutive rays."""
    i = np.arange(len(key))
    return np.lexsort((i, key, i // block))


def run():
    from winmad_rt import native, scenes
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
    p = hits["p"][ok]
    nrm = hits["n"][ok]
    rng = np.random.default_rng(1)
    sd = rng.normal(size=p.shape).astype(np.float32)
    sd /= np.linalg.norm(sd, axis=1, keepdims=True)
    flip = (sd * nrm).sum(1) * (d[ok] * nrm).sum(1) > 0  # leave on the incoming side
    sd[flip] *= -1
    so = (p + 1e-2 * sd).astype(np.float32)
    sec = native.rays_from_arrays(so, sd)
    lo, hi = so.min(0), so.max(0)
    m = morton(so, lo, hi)
    octant = ((sd[:, 0] > 0) * 1 + (sd[:, 1] > 0) * 2 + (sd[:, 2] > 0) * 4).astype(np.int64)
    sets = [
        ("primary raster", prim),
        ("primary shuffled", prim[rng.permutation(len(prim))]),
        ("secondary raster", sec),
        ("secondary shuffled", sec[rng.permutation(len(sec))]),
        ("secondary morton", sec[np.argsort(m, kind="stable")]),
        ("secondary octant+morton", sec[np.argsort(octant << 40 | m, kind="stable")]),
        ("secondary dir-morton", sec[np.argsort(morton(sd, -1, 1, 6), kind="stable")]),
        # what an append-time binning could give without a sort pass: the
        # octant alone (8 segments), the sign of x (both ends of one queue),
        # and octant bins within blocks of 64 / 4,096 consecutive rays
        ("secondary octant", sec[np.argsort(octant, kind="stable")]),
        ("secondary x-sign", sec[np.argsort(octant & 1, kind="stable")]),
        ("secondary octant/64", sec[local_order(octant, 64)]),
        ("secondary octant/4096", sec[local_order(octant, 4096)]),
    ]
    names = []
    for name, r in sets:
        for _ in range(REPS):
            ctx.trace_closest(r)
            names.append((name, len(r)))
    return names


def parse(d, names):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    allrows = list(csv.DictReader(open(f)))
    out = {}
    for k in ("k_trace_fast", "k_fast_resolve", "k_fast_hard"):
        rows = sorted((r for r in allrows if k in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
        rows = rows[1:]  # the primary trace that made the secondary rays
        for (name, n), r in zip(names, rows):
            us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            out.setdefault(name, {}).setdefault(k, []).append(us)
    for (name, n) in dict.fromkeys(map(tuple, names)):
        v = {k: min(x) for k, x in out[name].items()}
        print(f"{name:26s} rays {n:8d} " + " ".join(f"{k} {us:7.1f} us" for k, us in v.items())
              + f"  search {n / v['k_trace_fast']:7.1f} Mrays/s")


if __name__ == "__main__":
    # run:   rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 scripts/coherence_probe.py DIR
    # parse: python3 scripts/coherence_probe.py --parse DIR
    if sys.argv[1] == "--parse":
        parse(sys.argv[2], json.load(open(os.path.join(sys.argv[2], "order.json"))))
    else:
        names = run()
        os.makedirs(sys.argv[1], exist_ok=True)
        with open(os.path.join(sys.argv[1], "order.json"), "w") as f:
            json.dump(names, f)
