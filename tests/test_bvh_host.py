"""CPU checks of the verified-BVH data built on the host (wr_bvh.cpp): every
triangle / sphere in exactly one BVH leaf with its Triangle::hit record (a
sphere: centre and radius, its box inside the leaf's), boxes nested and
holding their triangles, and the KD membership data (each primitive's leaves,
its position in them, the root paths) equal to the reference tree's
(tests/native/bvh_check.cpp, compiled here from the product's own sources)."""
import os
import subprocess
import tempfile

import pytest

import _scenes
from winmad_rt import scenes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "winmad-s-raytracer-v1.0_amd", "csrc")
_bin = {}


def checker(wide=None, quant=False):
    """The checker built from the product's sources; wide=4 / 8 builds the 4- / 8-wide
    search tree (WR_BVH_WIDE=4) as well and checks it against the binary one;
    quant: the 4-wide tree of byte-quantised nodes (WR_BVH4_QUANT=1)."""
    key = f"{wide or 'default'}{'q' if quant else ''}"
    if key not in _bin:
        out = os.path.join(tempfile.mkdtemp(prefix="wr_bvhchk_"), "bvh_check")
        flags = ([f"-DWR_BVH_WIDE={wide}"] if wide else []) + (["-DWR_BVH4_QUANT=1"] if quant else [])
        subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", *flags, "-I", CSRC, "-I",
                        os.path.join(REPO, "include"), os.path.join(REPO, "tests", "native", "bvh_check.cpp"),
                        os.path.join(CSRC, "wr_scene.cpp"), os.path.join(CSRC, "wr_bvh.cpp"), "-o", out, "-lpthread"],
                       check=True)
        _bin[key] = out
    return _bin[key]


def small_torus():
    p = os.path.join(_scenes._DIR, "torus_small.obj")
    if not os.path.exists(p):
        scenes.synth_torus_obj(p, U=200, V=100)
    return _scenes.path("torus_small.scene", scenes.torus_scene(64, 64, "bdpt", torus_obj=p))


@pytest.mark.parametrize("maker", [lambda: _scenes.torus(64, 64), lambda: _scenes.cbox(64, 48), small_torus,
                                   lambda: _scenes.spheres(64, 64)],
                         ids=["torus", "cbox_dragon", "synthetic_torus_40k", "spheres"])
def test_bvh_structure(maker):
    r = subprocess.run([checker(), maker()], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr


@pytest.mark.parametrize("knobs", [{"WR_BVH_SWEEP": "100000"}, {"WR_BVH_BINS": "64", "WR_BVH_CT": "1"},
                                   {"WR_BVH_SWEEP": "64", "WR_BVH_CT": "0.25"}], ids=["sweep", "bins64_ct1", "sweep64_ct025"])
def test_bvh_build_knobs_keep_the_structure(knobs):
    """The SAH build knobs (measurement only) change the tree, never its contract."""
    env = dict(os.environ, **knobs)
    r = subprocess.run([checker(), _scenes.torus(64, 64)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr


def test_bvh_parallel_build_equals_serial():
    """The threaded build (subtrees, top splits, boxes) lays out exactly the
    serial build's data (WR_BVH_SERIAL=1), on a scene big enough to thread."""
    scene = small_torus()
    outs = []
    for serial in ("0", "1"):
        r = subprocess.run([checker(), scene], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, WR_BVH_SERIAL=serial))
        assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
        outs.append(r.stdout.split(" hash ")[1].strip())
    assert outs[0] == outs[1]


def test_bvh_wide_tree_structure():
    r = subprocess.run([checker(4), _scenes.torus(64, 64)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr


@pytest.mark.parametrize("maker", [lambda: _scenes.torus(64, 64), small_torus, lambda: _scenes.spheres(64, 64)],
                         ids=["torus", "synthetic_torus_40k", "spheres"])
def test_bvh_4wide_quantised_tree_structure(maker):
    """The 64-byte 4-wide node (WR_BVH4_QUANT=1, round 6: measured and left off
    by default): the binary tree's leaves, each once, every decoded leaf box
    containing the binary one and every decoded inner box its subtree's."""
    r = subprocess.run([checker(4, quant=True), maker()], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr


@pytest.mark.parametrize("maker", [lambda: _scenes.torus(64, 64), lambda: _scenes.cbox(64, 48), small_torus,
                                   lambda: _scenes.spheres(64, 64)],
                         ids=["torus", "cbox_dragon", "synthetic_torus_40k", "spheres"])
def test_bvh_8wide_quantised_tree_structure(maker):
    """The 8-wide search tree (WR_BVH_WIDE=8): the binary tree's leaves, each
    once, every byte-quantised child box decoded with the device's formula
    containing the binary box, children inside their parents."""
    r = subprocess.run([checker(8), maker()], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
