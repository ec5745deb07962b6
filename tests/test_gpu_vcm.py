"""GPU parity for VertexCM (wr_render_vcm) against the oracle's restatement of
vertexcm.cpp:47-285 (itself pinned bit for bit to the reference, test_oracle.py).

The GPU and the oracle draw the same counter-RNG numbers and compute the same
floats (glibc-exact libm on the device, tests/test_libm.py), and the hash grid
finds the same SET of light vertices in the merge radius as the reference's KD
tree (tests/test_oracle.py test_vcm_kdtree_search_is_the_brute_force_set); only
the order in which merges and splats are summed differs.  Gates: every pixel
as for BDPT (tests/_parity.py), ray counts and merge counts (queries, vertices
found in radius, merges) equal.
"""
import numpy as np
import pytest

import _oracle
import _scenes
from _parity import assert_vcm_parity
from test_gpu import ctx
from winmad_rt import native

pytestmark = pytest.mark.gpu


def _check(film, st, ref, rst):
    assert_vcm_parity(film, ref)
    for k in ("closest_rays", "shadow_rays", "vm_queries", "vm_found", "vm_merged"):
        assert getattr(st, k) == getattr(rst, k), (k, getattr(st, k), getattr(rst, k))


@pytest.mark.parametrize("name,maker,W,H,it,seed,rf", [
    ("torus64", lambda: _scenes.torus(64, 64), 64, 64, 1, 5489, 0.003),   # the reference's own radius
    ("torus64", lambda: _scenes.torus(64, 64), 64, 64, 3, 3, 0.05),       # many merges, radius schedule
    ("spheres64", lambda: _scenes.spheres(64, 64), 64, 64, 2, 11, 0.1),   # glass / mirror: delta vertices
    ("cboxb64x48", lambda: _scenes.cbox(64, 48, "bdpt"), 64, 48, 3, 3, 0.05),
    ("torus96x64", lambda: _scenes.torus(96, 64), 96, 64, 2, 7, 0.02),    # non-square film[x][y]
    ("tent64", lambda: _scenes.tent(64, 64), 64, 64, 2, 3, 0.05),          # emitter-first light vertices
])
def test_vcm_matches_oracle_counter_rng(name, maker, W, H, it, seed, rf):
    path = maker()
    film, st = ctx(path).render_vcm(W, H, iterations=it, seed=seed, radius_factor=rf)
    ref, rst = _oracle.Scene(path).vcm(W, H, it, seed, mode=1, radius_factor=rf)
    assert rst.vm_merged > 0
    _check(film, st, ref, rst)


@pytest.mark.parametrize("lo,hi", [(3, 5), (0, 2), (2, 3)])
def test_vcm_path_length_window(lo, hi):
    """min / max path length (RangeQuery::process :61-63, connection loop
    :236-244, light pass :129): narrow windows match the oracle too."""
    path = _scenes.torus(64, 64)
    film, st = ctx(path).render_vcm(64, 64, iterations=2, seed=5, min_path_length=lo, max_path_length=hi,
                                    radius_factor=0.05)
    ref, rst = _oracle.Scene(path).vcm(64, 64, 2, 5, mode=1, min_len=lo, max_len=hi, radius_factor=0.05)
    _check(film, st, ref, rst)


def test_vcm_1080p_matches_oracle_counter_rng():
    """torus.scene at 1920x1080 with the reference's own merge radius, one
    iteration, against the oracle (counter RNG)."""
    W, H = 1920, 1080
    path = _scenes.torus(W, H)
    film, st = ctx(path).render_vcm(W, H, iterations=1, seed=5489)
    ref, rst = _oracle.Scene(path).vcm(W, H, 1, 5489, mode=1)
    assert rst.vm_merged > 1000000
    _check(film, st, ref, rst)


def test_vcm_iteration_sharding_is_additive_at_1080p():
    """Full C2 frame: iterations [0, 2) == [0, 1) + [1, 2) (each iteration has
    its own radius, keyed by the global index), identical ray and merge counts."""
    W, H = 1920, 1080
    c = ctx(_scenes.torus(W, H))
    both, s2 = c.render_vcm(W, H, iterations=2, seed=5489)
    a, sa = c.render_vcm(W, H, iterations=1, seed=5489, iter_begin=0)
    b, sb = c.render_vcm(W, H, iterations=1, seed=5489, iter_begin=1)
    assert np.all(np.isfinite(both)) and both.min() >= 0 and both.max() > 0
    assert sa.closest_rays + sb.closest_rays == s2.closest_rays
    assert sa.shadow_rays + sb.shadow_rays == s2.shadow_rays
    assert sa.vm_found + sb.vm_found == s2.vm_found
    assert np.allclose(a + b, both, rtol=1e-4, atol=1e-6)


def test_vcm_tiny_films_and_errors():
    path = _scenes.torus(7, 5)
    film, st = ctx(path).render_vcm(7, 5, iterations=3, seed=17, radius_factor=0.05)
    ref, rst = _oracle.Scene(path).vcm(7, 5, 3, 17, mode=1, radius_factor=0.05)
    assert st.closest_rays == rst.closest_rays
    assert_vcm_parity(film, ref)
    c = ctx(_scenes.torus(16, 16))
    film, st = c.render_vcm(16, 16, iterations=0)
    assert st.closest_rays == 0 and not film.any()
    for kw in ({"max_path_length": 11}, {"max_path_length": 0}, {"iterations": -1}, {"radius_factor": 0.0},
               {"min_path_length": -1}):
        with pytest.raises(native.WrError) as e:
            c.render_vcm(16, 16, **kw)
        assert e.value.code == native.WR_E_ARG
