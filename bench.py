#!/usr/bin/env python3
"""Benchmark: torus.scene BDPT at 1920x1080 on N MI355X (BASELINE.json configs[1]).

One "step" = one BDPT iteration (BidirPathTracing::runIteration, 1 sample per
pixel) over the full 1920x1080 frame.  Weak scaling: every rank renders K
iterations of its own (iteration indices rank*K + s, counter RNG), into a film
in HBM; one RCCL reduce(sum) of the films to rank 0 per batch is inside the
timed region.  value = (closest + shadow traversals of all ranks) / max-rank
wall time, in Mrays/s.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (the driver's N > 1 form)

Extra JSON keys: spp_per_sec, roofline (dominant kernel = KD traversal, HIP
events on the context stream), cpu_baseline (the oracle's C port, MT-serial,
single thread, bounded sample of the same frame).
"""
import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# HBM bytes per k_trace launch from the PMC passes of the same bench command
# (scripts/profile_round.sh + scripts/summarize_profile.py; counters cannot be
# read from inside the timed run)
TRAFFIC_JSON = os.path.join(REPO, "profiles", "r1", "traffic.json")


def pmc_traffic():
    try:
        with open(TRAFFIC_JSON) as f:
            t = json.load(f)
        return t.get("hbm_bytes_per_launch"), os.path.relpath(TRAFFIC_JSON, REPO)
    except (OSError, ValueError):
        return None, None


def algorithmic_bytes(rays, inner, leaves, refs):
    """B_ray = 32 (ray) + 16 (hit) + 8 x (inner + leaf visits)
    + 4 x (primitive refs read) + 40 x (triangles tested)."""
    return 48.0 * rays + 8.0 * (inner + leaves) + 4.0 * refs + 40.0 * refs


def cpu_baseline(scene_path, W, H, budget_paths, chunks=16):
    """Oracle (oracle/cpuref.c, C port of the reference path), MT-serial RNG,
    one thread, on `budget_paths` path indices of one iteration taken as
    `chunks` evenly spaced contiguous runs (so sky rows and floor rows are
    sampled in proportion)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle
    s = _oracle.Scene(scene_path)
    P = W * H
    per = budget_paths // chunks
    rays = 0
    dt = 0.0
    for c in range(chunks):
        b = c * P // chunks
        t0 = time.perf_counter()
        _, st = s.bdpt(W, H, 1, 5489 + c, mode=0, path_range=(b, b + per))
        dt += time.perf_counter() - t0
        rays += st.closest_rays + st.shadow_rays
    n = per * chunks
    return {"value": round(rays / dt / 1e6, 4), "unit": "Mrays/s", "cores": 1, "kind": "port",
            "sample": f"oracle/cpuref.c MT-serial BDPT, torus {W}x{H}, {n} camera+light path pairs of one "
                      f"iteration in {chunks} evenly spaced runs ({rays} rays, {dt:.1f} s CPU); "
                      f"spp/s={n / dt:.0f}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--cpu-paths", type=int, default=1000000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-count", action="store_true", help="skip the work-counting replay")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from winmad_rt import native, scenes
    from winmad_rt import dist as wdist

    W, H, K = args.width, args.height, args.steps
    tmp = tempfile.mkdtemp(prefix=f"wr_bench_{rank}_")
    scene_path = scenes.write(os.path.join(tmp, "torus.scene"), scenes.torus_scene(W, H))
    sc = native.Scene(scene_path)
    ctx = native.Context(sc, local)
    film = torch.zeros((H, W, 3), dtype=torch.float32, device=f"cuda:{local}")

    # warmup (iteration indices outside the timed ones)
    if args.warmup > 0:
        ctx.render_bdpt(W, H, iterations=args.warmup, seed=5489, iter_begin=1 << 20,
                        film_ptr=film.data_ptr())
    film.zero_()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    it0 = wdist.bdpt_iteration_begin(rank, K)
    _, st = ctx.render_bdpt(W, H, iterations=K, seed=5489, iter_begin=it0, film_ptr=film.data_ptr(),
                            time_kernels=1)
    wdist.reduce_film(film, dist)  # one film reduction per batch (RCCL)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    rays = st.closest_rays + st.shadow_rays
    trace_ms = st.kernel_ms[native.K_TRACE]
    trace_launches = st.kernel_launches[native.K_TRACE]
    elapsed, total_rays = wdist.job_totals(elapsed, rays, dist, film.device)

    roofline = None
    if not args.no_count and rank == 0:
        # replay the same iterations with per-traversal counters (identical ray set:
        # the counter RNG makes the work a pure function of (seed, iteration, path))
        _, cst = ctx.render_bdpt(W, H, iterations=K, seed=5489, iter_begin=it0, count_work=1,
                                 film=None)
        assert cst.closest_rays == st.closest_rays and cst.shadow_rays == st.shadow_rays
        total_bytes = algorithmic_bytes(rays, cst.inner_visits, cst.leaf_visits, cst.prim_refs)
        per_launch = total_bytes / max(1, trace_launches)
        avg_launch_s = trace_ms / 1e3 / max(1, trace_launches)
        achieved = per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
        traffic, traffic_src = pmc_traffic()
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": round(traffic) if traffic else None, "traffic_source": traffic_src,
                    "kernel": "k_trace (KD closest-hit traversal)",
                    "bytes_per_launch": round(per_launch), "avg_launch_ms": round(avg_launch_s * 1e3, 4),
                    "launches": int(trace_launches),
                    "tests_per_ray": round(cst.prim_refs / rays, 2),
                    "nodes_per_ray": round((cst.inner_visits + cst.leaf_visits) / rays, 2),
                    "trace_share_of_gpu_time": round(trace_ms / max(1e-9, sum(st.kernel_ms)), 3)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(scene_path, W, H, args.cpu_paths)

    if rank == 0:
        value = total_rays / elapsed / 1e6
        out = {
            "metric": "Mrays/sec + spp/sec at 1920x1080, torus.scene BDPT, 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world, "steps": K,
            "warmup": args.warmup, "ms_per_step": round(elapsed / K * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: torus.scene (reference assets), counter RNG, faithful ray set",
            "config": {"workload": f"torus.scene BDPT {W}x{H}, {K} iterations (spp) per GPU, controlLength 3, "
                                   f"maxPathLength 10", "width": W, "height": H,
                       "iterations_per_gpu": K, "parallelism": f"sample-batch x{world}"},
            "spp_per_sec": round(W * H * K * world / elapsed, 1),
            "rays_per_iteration": round(total_rays / (K * world)),
            "roofline": roofline, "cpu_baseline": cpu,
        }
        if cpu:
            out["speedup_vs_cpu_port"] = round(value / cpu["value"], 1)
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
