"""bench.py's CPU-baseline legs run on the host alone (CPU suite): the
reference itself (oracle/_ref/refdrv, one process and the all-cores form) and
the oracle port, on a small sample of the C2 scene.  The `-m gpu` bench tests
run with --no-cpu, so without this a fault in these legs first shows in the
driver's default run."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_cpu_reference_leg(tmp_path, monkeypatch):
    if not os.path.exists(bench.REFDRV):
        pytest.skip("oracle/_ref/refdrv not built")
    monkeypatch.setenv("WR_CPU_BASELINE_CORES", "2")
    r = bench.cpu_reference("c2", "bdpt", 1920, 1080, str(tmp_path), 40)
    assert r is not None and r["value"] > 0 and r["kind"] == "reference"
    assert r["film_bit_exact"] is True
    assert r["all_cores"]["cores"] == 2 and r["all_cores"]["value"] > 0
    assert r["all_cores"]["machine_cpus"] == os.cpu_count()


def test_cpu_port_leg(tmp_path):
    scene = bench.make_scene("c2", 96, 54, str(tmp_path))
    r = bench.cpu_baseline("bdpt", scene, 96, 54, 512, chunks=4)
    assert r["value"] > 0 and r["kind"] == "port" and r["cores"] == 1
