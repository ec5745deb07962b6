"""BVH mode vs the reference's KD walk on rays that run along the plane of the
surface they leave (the open case of the margins argument)."""
import numpy as np
import pytest

from test_gpu_bvh import SCENES, _same_hits, _unit, big_torus, pair
from winmad_rt import native

pytestmark = pytest.mark.gpu


def _plane_grazing_rays(ref, n, seed):
    """From hit points on every surface: directions in the surface's plane
    tilted out of it by log-uniform angles in [1e-8, 3e-3] rad either way,
    from the hit point itself and from points lifted off the plane by
    log-uniform 1e-7..1e-3 of the scene's size.  On flat walls and floors
    every coplanar neighbour's plane is grazed too."""
    rng = np.random.default_rng(seed)
    ps, ns = [], []
    for _ in range(16):  # until n / 2 hits (closed scenes like the Cornell box hit rarely from outside)
        for size in (2000.0, 400.0, 60.0, 3.0):  # scenes of every scale: hits from each
            o = (rng.uniform(-1, 1, (n // 4, 3)) * size).astype(np.float32)
            h = ref.trace_closest(native.rays_from_arrays(o, _unit(rng.normal(size=(n // 4, 3)))))
            hit = h["prim"] >= 0
            ps.append(h["p"][hit].astype(np.float64))
            ns.append(h["n"][hit].astype(np.float64))
        if sum(x.shape[0] for x in ps) >= n // 2:
            break
    p, nn = np.concatenate(ps)[:n], np.concatenate(ns)[:n]
    m = p.shape[0]
    scale = float(np.abs(p).max())
    u = np.cross(nn, rng.normal(size=(m, 3)))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    ang = 10.0 ** rng.uniform(-8, np.log10(3e-3), m) * np.where(rng.random(m) < 0.5, 1.0, -1.0)
    dd = _unit(u * np.cos(ang)[:, None] + nn * np.sin(ang)[:, None])
    lift = np.where(rng.random(m) < 0.5, 0.0, 10.0 ** rng.uniform(-7, -3, m) * scale)
    lift *= np.where(rng.random(m) < 0.5, 1.0, -1.0)
    oo = (p + nn * lift[:, None]).astype(np.float32)
    ok = np.isfinite(dd).all(axis=1)
    return native.rays_from_arrays(oo[ok], dd[ok])


@pytest.mark.parametrize("name,maker", SCENES + [("torus1m", lambda: big_torus(64, 64))])
def test_bvh_matches_reference_mode_on_plane_grazing_rays(name, maker):
    ref, fast = pair(maker())
    n = 600_000 if name != "torus1m" else 200_000
    rays = _plane_grazing_rays(ref, n, 99)
    assert rays.shape[0] >= 0.4 * n
    a = ref.trace_closest(rays)
    b = fast.trace_closest(rays)
    ok = _same_hits(a, b)
    print(name, rays.shape[0], "rays,", int((~ok).sum()), "mismatches")
    assert ok.all(), (name, int((~ok).sum()), rays.shape[0], np.nonzero(~ok)[0][:8])
