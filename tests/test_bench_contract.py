"""bench.py's output contract on the GPU box (`-m gpu`): one JSON line with the
driver's keys, a roofline object whose frac is achieved / peak in (0, 1], and the
whole-job value consistent with rays_per_step / ms_per_step.  Short runs
(2 timed steps, no CPU leg) of every configuration, each in a child process.
On a host without a GPU (CPU suite) it must fail loudly: no CPU fallback.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
        "roofline")
ROOF = ("bound", "achieved", "peak", "unit", "frac", "traffic")


def run_bench(*args):
    out = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--no-cpu", *args],
                         cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "vcm"])
def test_bench_line(cfg):
    d = run_bench("--config", cfg)
    for k in KEYS:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["unit"] == "Mrays/s" and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["width"] == 1920 and d["config"]["height"] == 1080
    # whole-job rays / time (one GPU): value == rays_per_step / ms_per_step
    assert abs(d["value"] - d["rays_per_step"] / d["ms_per_step"] / 1e3) <= 1e-2 * d["value"]
    r = d["roofline"]
    for k in ROOF:
        assert k in r, k
    # the algorithmic bytes of the cache-resident scene are priced against L2
    assert r["bound"] == "l2" and r["peak"] > 0 and r["achieved"] > 0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) <= 1e-3 * max(r["frac"], 1e-9) + 1e-4
    assert 0 < r["frac"] <= 1, r["frac"]  # a fraction of a peak the kernel can actually meet
    # the driver-timed form: the step's algorithmic bytes over ms_per_step
    assert abs(r["achieved_step"] - r["algorithmic_bytes_per_step"] / d["ms_per_step"] / 1e6) \
        <= 1e-2 * r["achieved_step"]
    assert 0 < r["frac_step"] <= r["frac"] * 1.001
    if r.get("hbm"):
        assert 0 < r["hbm"]["frac"] <= 1 and r["hbm"]["peak"] == 8000.0


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU may be visible here")
@pytest.mark.parametrize("cfg", ["c2"])
def test_bench_fails_loudly_without_gpu(cfg):
    """No CPU fallback: without a HIP device bench.py exits non-zero naming it."""
    out = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "0", "--no-cpu",
                          "--config", cfg], cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert out.returncode != 0
    assert "no HIP device" in out.stderr
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.gpu
def test_bench_reference_trace_is_the_kd_walk():
    """`--trace reference` times the reference's KD walk (the library's default
    is the BVH search, so bench.py must select the walk explicitly)."""
    d = run_bench("--config", "c2", "--trace", "reference", "--no-compare")
    assert d["config"]["trace"] == "reference"
    assert d["roofline"]["kernel"].startswith("k_trace (KD"), d["roofline"]["kernel"]
    assert "bvh" not in d["roofline"]


@pytest.mark.gpu
def test_bench_rccl_self_check_reads_the_communicator():
    """The N > 1 reduce path on one GPU: the library's RCCL communicator
    (wr_comm_init) over one rank, its size read back from RCCL (wr_comm_info)
    into the line, and the film reduce (wr_film_reduce) timed."""
    d = run_bench("--config", "c2", "--rccl-self-check", "--no-compare", "--no-count")
    assert d["rccl_ranks"] == 1
    assert d["reduce_ms"] > 0 and d["reduce_ms_max"] >= d["reduce_ms"]
    assert d["reduce"].startswith("wr_film_reduce")
