"""The N > 1 path of bench.py on the HIP renderer (SURVEY 8(e), C5's layout).

Two ranks launched by torch.distributed.run exactly as the driver launches
bench.py, here sharing the one GPU of the box (each rank its own wr_context,
--backend gloo: the film reduction goes through host memory; on an 8-GPU node
the same code reduces over RCCL).  Each rank renders its own iteration range
(bidirPathTracing.cpp:25-26 sharded, lightPathNum global, :55); the reduced
film must equal one process rendering all iterations, and the ray counts must
add up.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import _scenes
from test_gpu import ctx
from winmad_rt import native

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("config,W,H,K,it0", [("c2", 192, 112, 3, 0), ("c4", 96, 56, 2, 512)])
def test_two_ranks_on_the_hip_renderer_reduce_to_the_one_process_film(config, W, H, K, it0, tmp_path):
    out = tmp_path / "film.npy"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", WR_PIPES="4", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--backend", "gloo", "--config", config, "--width", str(W), "--height", str(H),
           "--steps", str(K), "--warmup", "1", "--iter-begin", str(it0), "--no-cpu", "--no-compare", "--no-count",
           "--dump-film", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["backend"] == "gloo"
    reduced = np.load(out)
    # the same iterations [it0, it0 + 2K) in one process
    if config == "c2":
        path = _scenes.torus(W, H)
    else:
        from test_gpu_bvh import big_torus
        path = big_torus(W, H)
    c = ctx(path)
    c.set_trace_mode(native.TRACE_BVH)
    try:
        film, st = c.render_bdpt(W, H, iterations=2 * K, seed=5489, iter_begin=it0)
    finally:
        c.set_trace_mode(native.TRACE_REFERENCE)
    assert line["rays_per_step"] * 2 * K == pytest.approx(st.closest_rays + st.shadow_rays, abs=2 * K)
    assert reduced.shape == film.shape and reduced.max() > 0
    assert np.allclose(reduced, film, rtol=1e-4, atol=1e-6)
