#!/usr/bin/env python3
"""Benchmark: torus.scene BDPT at 1920x1080 on N MI355X (BASELINE.json configs[1]).

One "step" = one BDPT iteration (BidirPathTracing::runIteration, 1 sample per
pixel) over the full 1920x1080 frame.  Weak scaling: every rank renders K
iterations of its own (iteration indices rank*K + s, counter RNG), into a film
in HBM; one RCCL reduce(sum) of the films to rank 0 per batch is inside the
timed region.  value = (closest + shadow traversals of all ranks) / max-rank
wall time, in Mrays/s.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4]
    torchrun --nproc-per-node N bench.py --gpus N ...   (the driver's N > 1 form)

--config picks the SURVEY.md 8(d) configuration: c2 (default; the BASELINE.json
metric), c3 (cbox + dragon PT, one step = one sample index of a 512-spp
stratified render), c4 (the 1M-triangle synthetic torus, BDPT), vcm (torus.scene
with VertexCM, SURVEY 8(f) item 4: one step = one VCM iteration, merge radius
0.003 x sceneRadius shrinking with the global iteration index).

Extra JSON keys: spp_per_sec, roofline (dominant kernel = KD traversal, HIP
events on the context stream), cpu_baseline (the reference itself, built from
its sources by oracle/Makefile, one thread, the same scene at reduced
resolution), cpu_port (the oracle's C port, MT-serial, one thread, a bounded
sample of the full frame).
"""
import argparse
import json
import os
import sys
import tempfile
import time

# At least 16 hardware queues for this process (HIP's default, and the GPU
# box's environment, is 4) so that the library runs 16 concurrent render
# pipelines; must be set before HIP initialises.  DESIGN.md section 4.
os.environ["GPU_MAX_HW_QUEUES"] = str(max(16, int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)))

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md: L2, 8 XCDs x 4 MiB, ~34.5 TB/s aggregate
# HBM bytes per traversal launch from the PMC passes of the same bench command
# and configuration (scripts/profile_round.sh + scripts/summarize_profile.py:
# rocprofv3 counters cannot be read from inside the timed run, which is not
# run under the profiler).  One file per configuration
# (profiles/<round>/traffic_<config>.json; C2's older rounds: traffic.json);
# the newest round's file wins and its name is in the line (traffic_source).
PROFILES = os.path.join(REPO, "profiles")
ROUNDS = ("r6", "r5", "r4", "r3", "r2", "r1")


def pmc_traffic(config):
    names = [f"traffic_{config}.json"] + (["traffic.json"] if config == "c2" else [])
    for r in ROUNDS:
        for n in names:
            p = os.path.join(PROFILES, r, n)
            try:
                with open(p) as f:
                    t = json.load(f)
            except (OSError, ValueError):
                continue
            return t, os.path.relpath(p, REPO)
    return None, None


def algorithmic_bytes(rays, inner, leaves, refs, tests):
    """B_ray = 32 (ray) + 16 (hit) + 8 x (inner + leaf visits)
    + 4 x (primitive refs read) + 40 x (triangles tested).  Tests = the ones
    the kernel runs (repeats of a (ray, primitive) pair are skipped)."""
    return 48.0 * rays + 8.0 * (inner + leaves) + 4.0 * refs + 40.0 * tests


def cpu_baseline(kind, scene_path, W, H, budget, chunks=16):
    """Oracle (oracle/cpuref.c, C port of the reference path), MT-serial RNG,
    one thread, on a bounded sample of the same frame: `budget` path indices
    (BDPT) or pixels at 1 spp (PT), taken as `chunks` evenly spaced contiguous
    runs so sky rows and geometry rows are sampled in proportion."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle
    s = _oracle.Scene(scene_path)
    P = W * H
    per = budget // chunks
    rays = 0
    dt = 0.0
    for c in range(chunks):
        b = c * P // chunks
        t0 = time.perf_counter()
        if kind == "bdpt":
            _, st = s.bdpt(W, H, 1, 5489 + c, mode=0, path_range=(b, b + per))
        elif kind == "vcm":
            _, st = s.vcm(W, H, 1, 5489 + c, mode=0, path_range=(b, b + per))
        else:
            _, st = s.pt(W, H, 1, 7, 5489 + c, mode=0, pix_range=(b, b + per))
        dt += time.perf_counter() - t0
        rays += st.closest_rays + st.shadow_rays
    n = per * chunks
    what = "pixels at 1 spp" if kind == "pt" else "camera+light path pairs of one iteration"
    return {"value": round(rays / dt / 1e6, 4), "unit": "Mrays/s", "cores": 1, "kind": "port",
            "sample": f"oracle/cpuref.c MT-serial {kind.upper()}, {os.path.basename(scene_path)} {W}x{H}, "
                      f"{n} {what} in {chunks} evenly spaced runs ({rays} rays, {dt:.1f} s CPU); "
                      f"spp/s={n / dt:.0f}"}


REFDRV = os.path.join(REPO, "oracle", "_ref", "refdrv")


def _cpu_share():
    """CPUs this process may run on (its affinity mask), else os.cpu_count();
    env WR_CPU_BASELINE_CORES overrides (a positive integer; anything else is
    ignored)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    v = os.environ.get("WR_CPU_BASELINE_CORES", "").strip()
    if v.isdigit() and int(v) > 0:
        n = int(v)
    return max(1, n)


def cpu_reference(cfg_name, kind, W, H, tmp, shrink):
    """The reference ITSELF on the host: oracle/_ref/refdrv is the reference's own
    translation units compiled by oracle/Makefile (test infrastructure).  It
    renders whole frames only, so the bounded sample is the same scene at
    (W/shrink) x (H/shrink), one iteration / one sample per pixel, one thread;
    time = its render() wall time (refdrv prints it, scene load and KD build
    excluded).  The reference counts no rays: the count of that exact run comes
    from the oracle's MT-serial replica, whose film must equal the reference's
    bit for bit (checked, reported as film_bit_exact)."""
    import subprocess
    import numpy as np
    from winmad_rt import scenes
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle
    if not os.path.exists(REFDRV):
        return None
    w, h = max(8, W // shrink), max(8, H // shrink)
    d = os.path.join(tmp, "ref")
    os.makedirs(d, exist_ok=True)
    scene = make_scene(cfg_name, w, h, d, obj=os.path.join(tmp, "torus_1m.obj"))
    para = scenes.write(os.path.join(d, "ref.para"), scenes.params_text(w, h, 7, 1))
    out = os.path.join(d, "ref.f32")
    args = {"bdpt": ["bdpt", scene, para, 1, 5489, out], "vcm": ["vcm", scene, para, 1, 5489, out],
            "pt": ["pt", scene, para, 5489, out]}[kind]
    env = dict(os.environ, REFDRV_CWD=d)
    r = subprocess.run([REFDRV, *map(str, args)], capture_output=True, text=True, timeout=600, env=env)
    if r.returncode != 0:
        return None
    sec = float(next(l for l in r.stdout.splitlines() if l.startswith("render_seconds")).split()[1])
    # all cores of this box's CPU share: the same sample in `ncores` concurrent
    # single-threaded reference processes (the reference has no threading).
    # The GPU box gives one job 16 CPUs while os.cpu_count() shows the whole
    # machine's: the CPUs this process may run on, capped at that share
    ncores = max(1, min(16, _cpu_share()))
    machine_cpus = os.cpu_count()
    procs = [subprocess.Popen([REFDRV, *map(str, args[:-1]), out + f".{k}"], stdout=subprocess.PIPE,
                              stderr=subprocess.DEVNULL, text=True, env=env) for k in range(ncores)]
    outs = [p.communicate(timeout=900) for p in procs]
    ok = all(p.returncode == 0 for p in procs)
    # slowest process's render() time (scene load and KD build excluded, as above)
    wall_all = max(float(next(l for l in o.splitlines() if l.startswith("render_seconds")).split()[1])
                   for o, _ in outs) if ok else 0.0
    s = _oracle.Scene(scene)
    if kind == "bdpt":
        film, st = s.bdpt(w, h, 1, 5489, mode=0)
    elif kind == "vcm":
        film, st = s.vcm(w, h, 1, 5489, mode=0)
    else:
        film, st = s.pt(w, h, 1, 7, 5489, mode=0)
    ref = np.fromfile(out, np.float32).reshape(h, w, 3)
    rays = st.closest_rays + st.shadow_rays
    res = {"value": round(rays / sec / 1e6, 4), "unit": "Mrays/s", "cores": 1, "kind": "reference",
           "sample": f"oracle/_ref/refdrv {kind} (the reference's own code, g++ -O3), {os.path.basename(scene)} "
                     f"{w}x{h}, 1 {'spp' if kind == 'pt' else 'iteration'}, {rays} rays in {sec:.2f} s; "
                     f"spp/s={w * h / sec:.0f}",
           "film_bit_exact": bool(np.array_equal(film.view(np.uint32), ref.view(np.uint32)))}
    if ok:
        res["all_cores"] = {"value": round(ncores * rays / wall_all / 1e6, 4), "unit": "Mrays/s", "cores": ncores,
                            "machine_cpus": machine_cpus,
                            "sample": f"{ncores} concurrent refdrv processes of the same sample, "
                                      f"slowest render() {wall_all:.2f} s; {ncores} = this job's CPU share "
                                      f"(the machine shows {machine_cpus} CPUs)"}
    return res


# SURVEY.md 8(d) configurations a bench line can be quoted on
CONFIGS = {
    # steps: default iterations (spp) per GPU -- BASELINE.json configs[1] is 256
    # spp BDPT, configs[3] 64 spp; c3's 512-spp grid is shared by the ranks
    "c2": {"desc": "torus.scene BDPT", "integrator": "bdpt", "steps": 256},
    "c3": {"desc": "cbox + dragon PT, 512 spp stratification, MAX_TRACING_DEPTH 7", "integrator": "pt",
           "steps": 64},
    "c4": {"desc": "1M-triangle synthetic torus BDPT", "integrator": "bdpt", "steps": 64},
    "vcm": {"desc": "torus.scene VertexCM", "integrator": "vcm", "steps": 256},
    # not a BASELINE config: the Sphere::hit path (Cornell box, glass / mirror / glossy spheres)
    "sph": {"desc": "Cornell box + three spheres BDPT", "integrator": "bdpt", "steps": 64},
}
METRIC = "Mrays/sec + spp/sec at 1920x1080, torus.scene BDPT, 1/2/4/8 MI355X"


def make_scene(cfg, W, H, tmp, obj=None):
    from winmad_rt import scenes
    if cfg in ("c2", "vcm"):
        return scenes.write(os.path.join(tmp, "torus.scene"), scenes.torus_scene(W, H))
    if cfg == "c3":
        return scenes.write(os.path.join(tmp, "cbox.scene"), scenes.cbox_scene(W, H))
    if cfg == "sph":
        return scenes.write(os.path.join(tmp, "spheres.scene"), scenes.spheres_scene(W, H))
    obj = obj or os.path.join(tmp, "torus_1m.obj")
    if not os.path.exists(obj):
        scenes.synth_torus_obj(obj)
    return scenes.write(os.path.join(tmp, "torus_1m.scene"), scenes.torus_scene(W, H, torus_obj=obj))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="iterations (spp) per GPU; default per config: c2/vcm 256, c3/c4 64")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2",
                    help="c2 (default, the BASELINE metric), c3 PT, c4 1M triangles, vcm VertexCM, sph spheres")
    ap.add_argument("--spp", type=int, default=512, help="c3: stratification grid of the PT render")
    ap.add_argument("--cpu-paths", type=int, default=1000000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-count", action="store_true", help="skip the work-counting replay")
    ap.add_argument("--trace", choices=["auto", "reference", "bvh"], default="auto",
                    help="traversal: the reference's KD walk, or the verified BVH search (same (t, primitive) "
                         "answers, DESIGN.md section 4b); auto = the faster one: bvh for every config")
    ap.add_argument("--no-compare", action="store_true",
                    help="skip the single-GPU comparison run in the other traversal mode")
    ap.add_argument("--no-cut", action="store_true",
                    help="c3/vcm: shadow rays run to the end of the walk (no occlusion cutoff)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="N > 1: torch.distributed backend (nccl = RCCL over xGMI; gloo = the film reduction "
                         "through host memory, for ranks sharing one GPU in tests)")
    ap.add_argument("--iter-begin", type=int, default=0,
                    help="global index of rank 0's first iteration (sample): one rank's shard of a bigger job, "
                         "e.g. --config c4 --steps 512 --iter-begin 512 = rank 1 of SURVEY 8(d) C5")
    ap.add_argument("--dump-film", default=None, help="rank 0 writes the reduced film here (.npy, float32 H x W x 3)")
    ap.add_argument("--rccl-self-check", action="store_true",
                    help="N = 1 with --backend nccl: run the library's RCCL communicator and film reduce anyway "
                         "(the N > 1 code path on one GPU; a test of it)")
    args = ap.parse_args()
    if args.no_cut:
        os.environ["WR_TRACE_NO_CUT"] = "1"  # read by wr_create

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank; ranks beyond the visible GPUs share them round-robin
    # (tests run 2 ranks on a one-GPU box with --backend gloo)
    local = local % max(1, torch.cuda.device_count())
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    from winmad_rt import native
    from winmad_rt import dist as wdist

    cfg = CONFIGS[args.config]
    trace = args.trace
    if trace == "auto":
        trace = "bvh"
    W, H = args.width, args.height
    K = args.steps if args.steps is not None else cfg["steps"]
    pt = cfg["integrator"] == "pt"
    tmp = tempfile.mkdtemp(prefix=f"wr_bench_{rank}_")
    scene_path = make_scene(args.config, W, H, tmp)
    sc = native.Scene(scene_path)
    ctx = native.Context(sc, local)
    # (the library's default is the BVH search: the reference's walk is selected explicitly)
    ctx.set_trace_mode(native.TRACE_BVH if trace == "bvh" else native.TRACE_REFERENCE)
    film = torch.zeros((H, W, 3), dtype=torch.float32, device=f"cuda:{local}")
    # N > 1 over RCCL: the library's own communicator (wr_comm_init; its unique
    # id travels over torch.distributed) reduces the films, and its size is read
    # back from RCCL (wr_comm_info) into the line -- the job checks it spans N ranks
    comm = None
    if args.backend == "nccl" and (world > 1 or args.rccl_self_check):
        uid = [native.comm_unique_id() if rank == 0 else None]
        if dist:
            dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(uid[0], world, rank)
        comm = ctx.comm_info()
        if comm != (world, rank):
            raise SystemExit(f"RCCL communicator reports {comm}, expected ({world}, {rank})")

    # one step = one iteration (BDPT) / one sample index of the spp grid (PT);
    # every rank renders K of its own (weak scaling)
    def render(begin, count, **kw):
        if pt:
            return ctx.render_path(W, H, spp=args.spp, max_depth=7, seed=5489, sample_begin=begin,
                                   sample_count=count, **kw)
        if cfg["integrator"] == "vcm":
            return ctx.render_vcm(W, H, iterations=count, seed=5489, iter_begin=begin, **kw)
        return ctx.render_bdpt(W, H, iterations=count, seed=5489, iter_begin=begin, **kw)

    if pt and (args.iter_begin + world * K > args.spp or args.warmup > args.spp):
        raise SystemExit(f"c3: --iter-begin + --steps x ranks ({args.iter_begin + world * K}) must not exceed "
                         f"--spp ({args.spp})")
    if args.warmup > 0:  # warm-up samples / iterations outside the timed ones
        # run as the counting build of the traversal (k_trace<true, ...>): the
        # same caches and allocations warm up, and a rocprofv3 summary of this
        # command then lists exactly the timed launches under k_trace<false, ...>
        render((args.spp - args.warmup) if pt else (1 << 20), args.warmup, film_ptr=film.data_ptr(),
               count_work=1)
    film.zero_()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    it0 = args.iter_begin + wdist.bdpt_iteration_begin(rank, K)
    _, st = render(it0, K, film_ptr=film.data_ptr(), time_kernels=1)
    torch.cuda.synchronize()
    tr0 = time.perf_counter()
    if comm:  # one film reduction per batch: RCCL through the library (wr_film_reduce)
        ctx.film_reduce(film.data_ptr(), film.numel(), 0)
    else:  # gloo (ranks sharing a GPU in tests): through host memory
        wdist.reduce_film(film, dist)
    torch.cuda.synchronize()
    reduce_s = time.perf_counter() - tr0
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    if args.dump_film and rank == 0:
        import numpy as np
        np.save(args.dump_film, film.cpu().numpy())
    rays = st.closest_rays + st.shadow_rays
    trace_ms = st.kernel_ms[native.K_TRACE]
    trace_launches = st.kernel_launches[native.K_TRACE]
    elapsed, total_rays = wdist.job_totals(elapsed, rays, dist, film.device)
    # the reduce as each rank saw it: the last rank to arrive waits for nobody,
    # so the minimum is the collective itself, the maximum adds arrival skew
    red_min, red_max = wdist.min_max(reduce_s, dist, film.device)

    roofline = None
    if not args.no_count and rank == 0:
        # replay the same iterations with per-traversal counters (identical ray set:
        # the counter RNG makes the work a pure function of (seed, iteration, path))
        _, cst = render(it0, K, count_work=1, film=None)
        assert cst.closest_rays == st.closest_rays and cst.shadow_rays == st.shadow_rays
        total_bytes = algorithmic_bytes(rays, cst.inner_visits, cst.leaf_visits, cst.prim_refs, cst.prim_tests)
        bvh = None
        if trace == "bvh":
            # the KD counters cover only the fallback rays (their own B_ray terms
            # minus the ray load / hit store, which every ray pays once here):
            # + 64 B per BVH node record (128 B per 4-wide node), 48 B per
            # triangle record, 8 B per KD path entry replayed
            node_bytes = 128.0 if cst.bvh_width == 4 else 64.0
            total_bytes += node_bytes * cst.bvh_nodes + 48.0 * cst.bvh_tests + 8.0 * cst.kd_replay_steps \
                - 48.0 * cst.fallback_rays
            bvh = {"width": int(cst.bvh_width), "nodes_per_ray": round(cst.bvh_nodes / rays, 2),
                   "tests_per_ray": round(cst.bvh_tests / rays, 2),
                   "replay_steps_per_ray": round(cst.kd_replay_steps / rays, 2),
                   "fallback_frac": round(cst.fallback_rays / rays, 5),
                   "kd_tests_per_fallback_ray": round(cst.prim_tests / max(1, cst.fallback_rays), 1)}
        per_launch = total_bytes / max(1, trace_launches)
        # the same bytes over the driver-comparable clock: the timed steps' wall
        # time (every kernel of the step, not only the traversal's intervals)
        achieved_step = total_bytes / elapsed / 1e9
        # launches of the concurrent pipelines overlap: the rate is the bytes over
        # the union of the traversal launch intervals (HIP events on each stream);
        # the per-launch event average is reported beside it
        avg_launch_s = trace_ms / 1e3 / max(1, trace_launches)
        wall_s = st.trace_wall_ms / 1e3
        achieved = total_bytes / wall_s / 1e9 if wall_s > 0 else 0.0
        tr_rec, traffic_src = pmc_traffic(args.config)
        traffic = tr_rec.get("hbm_bytes_per_launch") if tr_rec else None
        # The scene is cache-resident (torus: 1.8 MB, L2; 1M triangles: 78 MB,
        # Infinity Cache), so the algorithmic bytes are served by L2, not HBM:
        # PMC HBM traffic per launch is ~1 % of them.  The bytes are priced
        # against the L2 aggregate, the tightest bandwidth ceiling they can
        # meet; the measured HBM rate is reported beside it (`hbm`).  What
        # actually limits the kernel (PMC) is the latency
        # of dependent L2 round trips plus VALU issue, not any bandwidth.
        hbm = None
        lib_sha = native.library_sha16()
        if traffic and wall_s > 0:
            hbm_gbs = traffic * trace_launches / wall_s / 1e9
            hbm = {"achieved": round(hbm_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": round(hbm_gbs / HBM_PEAK_GBS, 4), "source": "PMC FETCH_SIZE x2 + WRITE_SIZE per launch "
                   "x launches / trace_wall_ms", "l2_hit_rate": tr_rec.get("l2_hit_rate"),
                   "pmc_build": tr_rec.get("head"), "pmc_lib_sha": tr_rec.get("lib_sha"),
                   "pmc_lib_is_this_run": tr_rec.get("lib_sha") == lib_sha}
        state_hbm = None
        if tr_rec and tr_rec.get("state_bytes_per_launch") and traffic:
            # the path-state kernels (gen, vertex, resolve) beside the traversal:
            # the whole step's HBM bytes over the whole timed wall
            sb = tr_rec["state_bytes_per_launch"] * trace_launches
            tb = traffic * trace_launches
            state_hbm = {"bytes_per_trace_step": round(tr_rec["state_bytes_per_launch"]),
                         "achieved": round(sb / elapsed / 1e9, 1), "unit": "GB/s",
                         "whole_step_achieved": round((sb + tb) / elapsed / 1e9, 1), "peak": HBM_PEAK_GBS,
                         "whole_step_frac": round((sb + tb) / elapsed / 1e9 / HBM_PEAK_GBS, 4),
                         "source": "PMC FETCH_SIZE x2 + WRITE_SIZE of every non-traversal kernel, per traversal step "
                                   "x launches / elapsed (traversal: roofline.traffic)",
                         "top": sorted(((k, round(v["bytes_per_step"])) for k, v in tr_rec["state_kernels"].items()),
                                       key=lambda kv: -kv[1])[:4]}
        roofline = {"bound": "l2", "achieved": round(achieved, 1), "peak": L2_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / L2_PEAK_GBS, 4),
                    "limiter": "latency of dependent L2 round trips + VALU issue (PMC, DESIGN.md section 4)",
                    "algorithmic_bytes": "SURVEY.md 8(d) B_ray, counted by a replay of the timed iterations",
                    "traffic": round(traffic) if traffic else None, "traffic_source": traffic_src, "hbm": hbm,
                    "state_hbm": state_hbm,
                    "kernel": "k_trace (KD closest-hit traversal)",
                    "bytes_per_launch": round(per_launch), "avg_launch_ms": round(avg_launch_s * 1e3, 4),
                    "trace_wall_ms": round(st.trace_wall_ms, 3),
                    "wall_ms_per_launch": round(st.trace_wall_ms / max(1, trace_launches), 4),
                    "launches": int(trace_launches),
                    "refs_per_ray": round(cst.prim_refs / rays, 2),
                    "tests_per_ray": round(cst.prim_tests / rays, 2),
                    "nodes_per_ray": round((cst.inner_visits + cst.leaf_visits) / rays, 2),
                    "trace_share_of_wall": round(st.trace_wall_ms / 1e3 / max(1e-9, elapsed), 3),
                    "algorithmic_bytes_per_step": round(total_bytes / K),
                    "achieved_step": round(achieved_step, 1),
                    "frac_step": round(achieved_step / L2_PEAK_GBS, 4),
                    "frac_step_note": "algorithmic_bytes_per_step / ms_per_step / peak: the driver-timed form; "
                                      "frac uses the union of the traversal launches' intervals (trace_wall_ms), "
                                      "reproduced from a rocprofv3 kernel trace by scripts/trace_union.py"}
        if traffic:
            # measured HBM bytes per traversal step against the minimum ray I/O
            # (48 B per ray: origin, direction, hit t and primitive)
            roofline["traffic_over_ray_io"] = round(traffic / (48.0 * rays / max(1, trace_launches)), 3)
        if bvh:
            roofline["kernel"] = "k_trace_fast (verified BVH closest hit) + k_trace over its fallback rays"
            roofline["algorithmic_bytes"] = ("BVH: 48 B per ray + 64 B per node (128 per 4-wide node) + 48 B per triangle test + 8 B per "
                                             "KD path entry replayed; fallback rays: SURVEY.md 8(d) B_ray")
            roofline["bvh"] = bvh

    other = None
    if rank == 0 and world == 1 and not args.no_compare:
        # the same K steps in the other traversal mode (same rays, same answers),
        # timed the same way, for the line's `other_trace`
        o_mode = "reference" if trace == "bvh" else "bvh"
        try:
            ctx.set_trace_mode(native.TRACE_BVH if o_mode == "bvh" else native.TRACE_REFERENCE)
            render((args.spp - 1) if pt else (1 << 20) + 64, 1, film_ptr=film.data_ptr())
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            _, ost = render(it0, K, film_ptr=film.data_ptr())
            torch.cuda.synchronize()
            odt = time.perf_counter() - t1
            orays = ost.closest_rays + ost.shadow_rays
            other = {"trace": o_mode, "value": round(orays / odt / 1e6, 2), "ms_per_step": round(odt / K * 1e3, 3),
                     "same_ray_count": bool(orays == rays)}
        except native.WrError as e:  # e.g. a scene without a verified BVH
            other = {"trace": o_mode, "error": str(e)}

    cpu = port = None
    if rank == 0 and world == 1 and not args.no_cpu:
        # the reference on the full frame for C2 (the config's
        # resolution, fewer iterations: 1 iteration is ~35-40 s of one core);
        # the 1M-triangle C4 at a quarter of it per axis
        cpu = cpu_reference(args.config, cfg["integrator"], W, H, tmp, {"c4": 4, "c2": 1}.get(args.config, 2))
        budget = {"c2": args.cpu_paths, "c3": args.cpu_paths // 4, "c4": args.cpu_paths // 20,
                  "vcm": args.cpu_paths // 2, "sph": args.cpu_paths // 4}[args.config]
        port = cpu_baseline(cfg["integrator"], scene_path, W, H, budget)
        if cpu is None:  # no reference build on this machine: the port is the baseline
            cpu, port = port, None

    if rank == 0:
        value = total_rays / elapsed / 1e6
        unit_name = "samples (spp)" if pt else "iterations (spp)"
        metric = METRIC if args.config == "c2" else \
            f"Mrays/sec + spp/sec at {W}x{H}, {cfg['desc']} ({args.config.upper()}), MI355X"
        out = {
            "metric": metric,
            "value": round(value, 2), "unit": "Mrays/s", "n_gpus": world, "steps": K,
            "warmup": args.warmup, "ms_per_step": round(elapsed / K * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: reference scene assets, counter RNG, faithful ray set",
            "config": {"workload": f"{cfg['desc']} {W}x{H}, {K} {unit_name} per GPU"
                                   + ("" if pt else ", maxPathLength 10" if cfg["integrator"] == "vcm"
                                      else ", controlLength 3, maxPathLength 10"),
                       "scene_config": args.config.upper(), "width": W, "height": H,
                       "steps_per_gpu": K, "iter_begin": it0, "parallelism": f"sample-batch x{world}",
                       "backend": args.backend if world > 1 else None, "trace": trace,
                       "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"]), "pipelines": int(st.pipelines)},
            "spp_per_sec": round(W * H * K * world / elapsed, 1),
            "rays_per_step": round(total_rays / (K * world)),
            "roofline": roofline, "cpu_baseline": cpu,
            "lib_sha": native.library_sha16(),
        }
        if world > 1 or comm:
            out["rccl_ranks"] = comm[0] if comm else None  # from ncclCommCount (wr_comm_info)
            out["reduce_ms"] = round(red_min * 1e3, 3)
            out["reduce_ms_max"] = round(red_max * 1e3, 3)
            out["reduce"] = ("wr_film_reduce (RCCL reduce-sum of the H x W x 3 fp32 film to rank 0, "
                             f"{H * W * 12 / 1e6:.1f} MB), inside the timed region; reduce_ms = fastest rank "
                             "(the collective), reduce_ms_max = slowest (plus arrival skew)") if comm else \
                ("gloo reduce through host memory (ranks sharing a GPU)")
        if trace == "bvh":
            out["trace_note"] = ("verified BVH traversal: every ray gets the reference KD walk's (t, primitive) "
                                 "answer, bit for bit (argument in DESIGN.md 4b; rays running inside the plane of a "
                                 "triangle the search tests take the KD walk; 0 mismatches on the plane-grazing probe, "
                                 "tests/test_gpu_bvh.py, and on the bench workloads, profiles/r5/bvh_verify.json, 4.13e9 rays incl. spheres); the "
                                 "same rays are traced and counted")
        if other:
            out["other_trace"] = other
        if cfg["integrator"] in ("pt", "vcm"):
            # dead-work elision is flagged; --no-cut measures without it.
            # Only the KD walk has the cutoff: the BVH mode traces every shadow ray
            # to its closest hit
            cut = not args.no_cut and trace == "reference"
            out["config"]["occlusion_cutoff"] = cut
            if cut:
                out["dead_work_elision"] = ("occlusion cutoff: a shadow ray ends once a hit below occl_cut "
                                            "settles 'occluded' (exact, DESIGN.md section 4); every ray is "
                                            "still traced and counted; bench.py --no-cut runs without it")
        if cfg["integrator"] == "vcm":
            out["merges_per_step"] = round(st.vm_merged / K)
            out["merge_queries_per_step"] = round(st.vm_queries / K)
        if cpu:
            out["speedup_vs_cpu_baseline"] = round(value / cpu["value"], 1)
            if "all_cores" in cpu:
                out["speedup_vs_cpu_all_cores"] = round(value / cpu["all_cores"]["value"], 1)
        if port:
            out["cpu_port"] = port
            out["speedup_vs_cpu_port"] = round(value / port["value"], 1)
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
