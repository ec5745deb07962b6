"""The cell filter of the tie resolution and membership replays
(cell_may_be_reached, csrc/wr_fast.h) must never drop a KD leaf the
reference's walk reaches (KDtreeAccel.cpp:309-388) -- CPU only.

tests/native/cell_filter_check.cpp walks rays over the tree wr_scene.cpp
builds, exactly as kd_walk does, and gives every reached leaf to a host copy of
the filter.  Rays: plane-grazing and random ones generated there, and
tests/golden/grazing_cbox_phantom.f32 -- rays of tests/test_gpu_bvh.py's
Cornell-box grazing corpus (scripts/dump_grazing.py) whose origin lies just
outside the root box with the ray pointing away: the walk still runs, ends in
leaves whose cells the ray's line never meets, and hits a wall there at
t > 0 (the case that made the filter drop reached leaves before it learned to
keep every leaf of a ray whose root interval is not positive)."""
import os
import subprocess
import tempfile

import pytest

import _scenes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "winmad-s-raytracer-v1.0_amd", "csrc")
_bin = []


def checker():
    if not _bin:
        out = os.path.join(tempfile.mkdtemp(prefix="wr_cfc_"), "cell_filter_check")
        subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-I", CSRC, "-I", os.path.join(REPO, "include"),
                        os.path.join(REPO, "tests", "native", "cell_filter_check.cpp"),
                        os.path.join(CSRC, "wr_scene.cpp"), "-o", out, "-lpthread"], check=True)
        _bin.append(out)
    return _bin[0]


def run(*args):
    r = subprocess.run([checker(), *args], capture_output=True, text=True, timeout=600)
    return r.returncode, r.stdout


def test_phantom_leaves_of_the_grazing_corpus_are_kept():
    rc, out = run(_scenes.cbox(256, 192), "--rays", os.path.join(REPO, "tests", "golden", "grazing_cbox_phantom.f32"))
    assert rc == 0, out[-3000:]
    last = out.strip().splitlines()[-1]
    assert " dropped 0 " in last, last
    assert int(last.split("all-negative leaves ")[1]) > 100, last  # the case is exercised


@pytest.mark.parametrize("name,maker", [("cbox", lambda: _scenes.cbox(256, 192)),
                                        ("torus", lambda: _scenes.torus(256, 256))])
def test_no_reached_leaf_dropped(name, maker):
    rc, out = run(maker(), "400000", "17")
    assert rc == 0, out[-3000:]
