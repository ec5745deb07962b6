#!/usr/bin/env python3
"""Validation of the verified-BVH traversal mode on full bench workloads:
every ray of the renders is traced twice -- the BVH mode's answer, then the
reference's KD walk (k_fast_verify, WR_BVH_VERIFY=1) -- and the (t, primitive)
pairs are compared bit for bit.  Writes one JSON line per configuration.

    python scripts/verify_bvh.py [--configs c2,vcm,c3,c4] [--iters 256,64,64,16] [--seed S] [--out FILE]
"""
import argparse
import json
import os
import sys
import tempfile
import time

os.environ["WR_BVH_VERIFY"] = "1"
os.environ["GPU_MAX_HW_QUEUES"] = str(max(16, int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)))
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))
import bench  # noqa: E402  (make_scene, CONFIGS)
from winmad_rt import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,vcm,c3,c4")
    ap.add_argument("--iters", default="256,64,64,16")
    ap.add_argument("--out", default=None)
    ap.add_argument("--seed", type=int, default=5489, help="another seed traces another ray set")
    a = ap.parse_args()
    W, H = 1920, 1080
    tmp = tempfile.mkdtemp(prefix="wr_verify_")
    lines = []
    for cfg, k in zip(a.configs.split(","), map(int, a.iters.split(","))):
        sc = native.Scene(bench.make_scene(cfg, W, H, tmp))
        ctx = native.Context(sc, 0)
        ctx.set_trace_mode(native.TRACE_BVH)
        t0 = time.perf_counter()
        integ = bench.CONFIGS[cfg]["integrator"]
        if integ == "pt":
            _, st = ctx.render_path(W, H, spp=512, max_depth=7, seed=a.seed, sample_begin=0, sample_count=k)
        elif integ == "vcm":
            _, st = ctx.render_vcm(W, H, iterations=k, seed=a.seed)
        else:
            _, st = ctx.render_bdpt(W, H, iterations=k, seed=a.seed)
        rays = st.closest_rays + st.shadow_rays
        d = {"config": cfg, "workload": f"{bench.CONFIGS[cfg]['desc']} {W}x{H}, {k} "
             f"{'samples' if integ == 'pt' else 'iterations'}, seed {a.seed}",
             "rays": int(rays), "verified_rays": int(st.verify_rays), "mismatches": int(st.verify_mismatches),
             "seconds": round(time.perf_counter() - t0, 1)}
        assert st.verify_rays == rays, (st.verify_rays, rays)
        print(json.dumps(d), flush=True)
        lines.append(d)
        ctx.close()
        sc.close()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(lines, f, indent=1)


if __name__ == "__main__":
    main()
