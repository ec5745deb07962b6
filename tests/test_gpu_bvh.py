"""GPU parity of the verified-BVH traversal mode (WR_TRACE_BVH).

The BVH mode must return exactly what the reference's KD walk returns: the same
winning primitive and the same float t for every ray (bit-exact), the same
occlusion answers, and therefore renders with the same ray set.  Checked
against the reference mode of the same library (itself bit-exact against the
reference's own golden corpus, tests/test_gpu.py) on
  * the golden corpus (reference outputs, tests/golden/rays_*.txt);
  * large ray corpora built like the renderer's rays: camera rays, random rays,
    extension rays leaving surface hits (origin + EPS along d, the BDPT / PT
    extension rule) in every direction including grazing ones, and shadow rays
    from hit points (no offset, BDPT's connections) to points on other surfaces;
  * full BDPT / VCM / PT renders: identical ray counts, films equal up to the
    order of float atomics.
"""
import os

import numpy as np
import pytest

import _scenes
from test_gpu import _check_golden_corpus, normalize_f32
from winmad_rt import native, scenes

pytestmark = pytest.mark.gpu
EPS = np.float32(1e-3)

_cache = {}


def pair(path):
    """(reference-mode context, BVH-mode context) on one scene."""
    if path not in _cache:
        s = native.Scene(path)
        a = native.Context(s, 0, trace=native.TRACE_REFERENCE)
        b = native.Context(s, 0, trace=native.TRACE_BVH)
        _cache[path] = (s, a, b)
    return _cache[path][1], _cache[path][2]


def big_torus(W, H):
    p = os.path.join(_scenes._DIR, "torus1m.obj")
    if not os.path.exists(p):
        scenes.synth_torus_obj(p)
    return _scenes.path(f"torus1m_{W}x{H}.scene", scenes.torus_scene(W, H, "bdpt", torus_obj=p))


SCENES = [("torus", lambda: _scenes.torus(256, 256)), ("cbox", lambda: _scenes.cbox(256, 192)),
          ("spheres", lambda: _scenes.spheres(256, 256))]


@pytest.mark.parametrize("name,maker", [("torus64", lambda: _scenes.torus(64, 64)),
                                        ("cbox64x48", lambda: _scenes.cbox(64, 48)),
                                        ("spheres64", lambda: _scenes.spheres(64, 64))])
def test_bvh_golden_corpus_bit_exact(name, maker):
    _check_golden_corpus(pair(maker())[1], name)


def test_bvh_is_the_default_for_sphere_scenes():
    """Spheres are in the verified BVH (round 5): a scene with spheres gets the
    BVH search by default -- the binary tree (PT), and the 4-wide one for a
    BDPT render short enough to take the latency path (one group) -- with the
    same film and rays as the KD walk's."""
    c = native.Context(native.Scene(_scenes.spheres(64, 64)), 0)
    fb, sb = c.render_bdpt(64, 64, iterations=2, seed=3)
    fp, sp = c.render_path(64, 64, spp=4, seed=3)
    assert sb.bvh_width == 4 and sp.bvh_width == 2, (sb.bvh_width, sp.bvh_width)
    c.set_trace_mode(native.TRACE_REFERENCE)
    fb0, sb0 = c.render_bdpt(64, 64, iterations=2, seed=3)
    fp0, sp0 = c.render_path(64, 64, spp=4, seed=3)
    assert sb0.bvh_width == 0
    assert (sb.closest_rays, sb.shadow_rays, sp.closest_rays) == (sb0.closest_rays, sb0.shadow_rays, sp0.closest_rays)
    assert _film_close(fb, fb0) and _film_close(fp, fp0)


def _unit(v):
    with np.errstate(invalid="ignore", divide="ignore"):
        return normalize_f32(v.astype(np.float32))


def _valid(o, d):
    """Rays with finite origins and unit directions only (a zero-length
    direction normalises to NaN; neither mode is asked about such rays)."""
    ok = np.isfinite(o).all(axis=1) & np.isfinite(d).all(axis=1)
    ok &= np.abs(np.sqrt((d.astype(np.float64) ** 2).sum(axis=1)) - 1.0) < 1e-3
    return ok


def _corpus(ref, n, seed):
    """Rays shaped like the renderer's: camera / random rays, then extension
    and shadow rays spawned from their hits."""
    rng = np.random.default_rng(seed)
    # first generation: random origins inside a big box around the scene, random dirs
    info_o = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    hits0 = None
    for scale in (2000.0, 400.0, 60.0, 3.0):
        o = (info_o * scale).astype(np.float32)
        d = _unit(rng.normal(size=(n, 3)))
        h = ref.trace_closest(native.rays_from_arrays(o, d))
        if hits0 is None or (h["prim"] >= 0).mean() > (hits0[2]["prim"] >= 0).mean():
            hits0 = (o, d, h)
    o0, d0, h0 = hits0
    hit = h0["prim"] >= 0
    p = h0["p"][hit].astype(np.float32)
    nn = h0["n"][hit].astype(np.float32)
    m = p.shape[0]
    # extension rays: cosine-ish around +-n, a quarter of them grazing
    side = np.where(rng.random(m) < 0.5, 1.0, -1.0).astype(np.float32)[:, None]
    dd = _unit(nn * side + rng.normal(size=(m, 3)).astype(np.float32))
    g = rng.random(m) < 0.25
    t = np.cross(nn[g], rng.normal(size=(g.sum(), 3)).astype(np.float32))
    dd[g] = _unit(t + nn[g] * side[g] * rng.uniform(-1e-3, 1e-3, (g.sum(), 1)).astype(np.float32))
    ext_o = (p + dd * EPS).astype(np.float32)
    # shadow rays: hit point -> another hit point, no offset (BDPT connections)
    q = p[rng.permutation(m)]
    sd = _unit(q - p)
    ok0, oke, ok = _valid(o0, d0), _valid(ext_o, dd), _valid(p, sd)
    rays = [native.rays_from_arrays(o0[ok0], d0[ok0]), native.rays_from_arrays(ext_o[oke], dd[oke]),
            native.rays_from_arrays(p[ok], sd[ok])]
    return np.concatenate(rays), (p[ok], sd[ok], q[ok])


def _same_hits(a, b):
    same_prim = a["prim"] == b["prim"]
    same_t = (a["t"].view(np.int32) == b["t"].view(np.int32)) | (a["prim"] < 0)
    return same_prim & same_t


@pytest.mark.parametrize("name,maker", SCENES + [("torus1m", lambda: big_torus(64, 64))])
def test_bvh_matches_reference_mode_on_ray_corpus(name, maker):
    ref, fast = pair(maker())
    n = 400_000 if name != "torus1m" else 150_000
    rays, (p, sd, q) = _corpus(ref, n, 1234)
    a = ref.trace_closest(rays)
    b = fast.trace_closest(rays)
    ok = _same_hits(a, b)
    assert ok.all(), (name, int((~ok).sum()), rays.shape[0], np.nonzero(~ok)[0][:8])
    for fld in ("p", "n", "inside", "mat_id"):
        assert np.array_equal(a[fld], b[fld]), fld
    r8 = native.rays_from_arrays(p, sd)
    assert np.array_equal(ref.occluded(r8, q), fast.occluded(r8, q))


def _film_close(fa, fb):
    fa = fa.astype(np.float64)
    fb = fb.astype(np.float64)
    rms = np.sqrt((fa ** 2).mean())
    return np.sqrt(((fa - fb) ** 2).mean()) <= 1e-5 * max(rms, 1e-30)


def test_bvh_bdpt_render_same_rays_and_film():
    ref, fast = pair(_scenes.torus(256, 256))
    fa, sa = ref.render_bdpt(256, 256, iterations=4, seed=5489, count_work=True)
    fb, sb = fast.render_bdpt(256, 256, iterations=4, seed=5489, count_work=True)
    assert sa.closest_rays == sb.closest_rays and sa.shadow_rays == sb.shadow_rays
    assert _film_close(fa, fb)
    rays = sb.closest_rays + sb.shadow_rays
    assert sb.bvh_nodes > 0 and sb.bvh_tests > 0
    assert sb.fallback_rays < 0.1 * rays, (sb.fallback_rays, rays)
    # the BVH search does far less work than the reference's walk
    assert sb.bvh_tests + sb.prim_tests < 0.5 * sa.prim_tests


def test_bvh_vcm_and_pt_renders_same_rays_and_film():
    ref, fast = pair(_scenes.torus(128, 128))
    fa, sa = ref.render_vcm(128, 128, iterations=2, seed=7)
    fb, sb = fast.render_vcm(128, 128, iterations=2, seed=7)
    assert sa.closest_rays == sb.closest_rays and sa.shadow_rays == sb.shadow_rays
    assert sa.vm_merged == sb.vm_merged
    assert _film_close(fa, fb)
    ref, fast = pair(_scenes.cbox(128, 96))
    fa, sa = ref.render_path(128, 96, spp=4, max_depth=7, seed=11)
    fb, sb = fast.render_path(128, 96, spp=4, max_depth=7, seed=11)
    assert sa.closest_rays == sb.closest_rays and sa.shadow_rays == sb.shadow_rays
    assert _film_close(fa, fb)


def test_bvh_bdpt_render_1m_triangles():
    ref, fast = pair(big_torus(192, 108))
    fa, sa = ref.render_bdpt(192, 108, iterations=2, seed=3)
    fb, sb = fast.render_bdpt(192, 108, iterations=2, seed=3, count_work=True)
    assert sa.closest_rays == sb.closest_rays and sa.shadow_rays == sb.shadow_rays
    assert _film_close(fa, fb)


@pytest.mark.parametrize("kind", ["bdpt", "vcm", "pt"])
def test_resolve_list_same_rays_and_film(kind, monkeypatch):
    """The search settles the rays its first membership test proves and lists
    the rest for k_fast_resolve (WR_RESOLVE_LIST, the default): the same rays
    and film as the resolve over every ray."""
    out = []
    for rl in ("1", "0"):
        monkeypatch.setenv("WR_RESOLVE_LIST", rl)
        c = native.Context(native.Scene(_scenes.torus(192, 144) if kind != "pt" else _scenes.cbox(192, 144)), 0)
        if kind == "bdpt":
            out.append(c.render_bdpt(192, 144, iterations=4, seed=13))
        elif kind == "vcm":
            out.append(c.render_vcm(192, 144, iterations=2, seed=13))
        else:
            out.append(c.render_path(192, 144, spp=4, max_depth=7, seed=13))
        c.close()
    (fa, sa), (fb, sb) = out
    assert sa.closest_rays == sb.closest_rays and sa.shadow_rays == sb.shadow_rays
    assert _film_close(fa, fb)


@pytest.mark.parametrize("kind", ["bdpt", "vcm", "bdpt1m"])
def test_pair_record_same_rays_and_film(kind, monkeypatch):
    """Near-ties settled from the search's pair record (WR_PAIR_RECORD: 2 = the
    pair list, one near-tie per lane, the default; 1 = the record in the tie
    list only) give the rays and the film of the tie resolution's own BVH
    collection (0).  (Every answer of the default against the KD walk:
    test_bvh_verify_every_ray_against_the_kd_walk.)"""
    W, H = (128, 72) if kind == "bdpt1m" else (192, 144)
    out = []
    for mode in ("2", "1", "0"):
        monkeypatch.setenv("WR_PAIR_RECORD", mode)
        c = native.Context(native.Scene(big_torus(W, H) if kind == "bdpt1m" else _scenes.torus(W, H)), 0)
        if kind == "vcm":
            out.append(c.render_vcm(W, H, iterations=2, seed=13))
        else:
            out.append(c.render_bdpt(W, H, iterations=4, seed=13))
        c.close()
    f0, s0 = out[0]
    for f, s in out[1:]:
        assert s.closest_rays == s0.closest_rays and s.shadow_rays == s0.shadow_rays
        assert _film_close(f0, f)


@pytest.mark.parametrize("diag", [16, 32, 48, 64, 128])
def test_capacity_diagnostics_keep_primitive_indices_valid(diag, monkeypatch):
    """WR_BVH_DIAG's capacity probes skip the resolve or the hard launch (wrong
    answers, measurement only): the rays those kernels would settle keep the
    search's winner with its marks cleared, so a render completes (a marked
    primitive index used to reach the vertex kernels)."""
    monkeypatch.setenv("WR_BVH_DIAG", str(diag))
    c = native.Context(native.Scene(_scenes.torus(128, 96)), 0)
    film, st = c.render_bdpt(128, 96, iterations=2, seed=3)
    c.close()
    assert np.isfinite(film).all() and st.closest_rays > 0


@pytest.mark.parametrize("name,maker,kind", [("torus", lambda: _scenes.torus(256, 256), "bdpt"),
                                             ("torus_vcm", lambda: _scenes.torus(256, 256), "vcm"),
                                             ("cbox", lambda: _scenes.cbox(256, 192), "pt"),
                                             ("torus1m", lambda: big_torus(128, 72), "bdpt"),
                                             ("spheres", lambda: _scenes.spheres(256, 256), "bdpt"),
                                             ("spheres_pt", lambda: _scenes.spheres(256, 192, "pt"), "pt"),
                                             ("spheres_vcm", lambda: _scenes.spheres(256, 256), "vcm")])
def test_bvh_verify_every_ray_against_the_kd_walk(name, maker, kind, monkeypatch):
    """WR_BVH_VERIFY: every ray of a render is traced again by the reference's
    KD walk inside the library and the (t, primitive) pairs are compared bit for
    bit: no mismatch, and every ray checked."""
    monkeypatch.setenv("WR_BVH_VERIFY", "1")
    s = native.Scene(maker())
    c = native.Context(s, 0)
    c.set_trace_mode(native.TRACE_BVH)
    if kind == "pt":
        _, st = c.render_path(256, 192, spp=4, max_depth=7, seed=3)
    elif kind == "vcm":
        _, st = c.render_vcm(256, 256, iterations=2, seed=3)
    elif name == "torus1m":
        _, st = c.render_bdpt(128, 72, iterations=2, seed=3)
    else:
        _, st = c.render_bdpt(256, 256, iterations=4, seed=3)
    assert st.verify_rays == st.closest_rays + st.shadow_rays > 0
    assert st.verify_mismatches == 0, (st.verify_mismatches, st.verify_rays)
    # the tree each render searched: the 1M scene has only the 4-wide tree; the
    # torus render's 4 pieces make two groups on its one pipeline (not the
    # latency path), so it searches the binary tree, as VCM and PT do
    assert st.bvh_width == {"torus": 2, "torus_vcm": 2, "cbox": 2, "torus1m": 4, "spheres": 2, "spheres_pt": 2,
                            "spheres_vcm": 2}[name], (name, st.bvh_width)


@pytest.mark.parametrize("lat", ["latency", "full"])
def test_bvh_tree_of_each_schedule_verified(lat, monkeypatch):
    """Pins the two trees a binary-tree scene's BDPT renders search, each with
    every ray verified against the KD walk (WR_BVH_VERIFY):
      * latency: a short render (two iterations = two pieces = one group on
        one pipeline) searches the 4-wide tree (wide_now) -- the path of the
        round-4 fault, where the searched scene was copied before its KD stack
        depth was set;
      * full: pieces that fill 16 pipelines with several groups each, and
        WR_BVH_WIDE_LAT=0, search the binary tree -- the headline's tree."""
    monkeypatch.setenv("WR_BVH_VERIFY", "1")
    W = H = 256
    if lat == "full":
        monkeypatch.setenv("WR_BVH_WIDE_LAT", "0")
        monkeypatch.setenv("WR_PIECE_MIN", "4096")
        monkeypatch.setenv("WR_PIECE_CAP", "4096")
    s = native.Scene(_scenes.torus(W, H))
    c = native.Context(s, 0, trace=native.TRACE_BVH)
    if lat == "full":
        c.set_pipelines(16)
    _, st = c.render_bdpt(W, H, iterations=4 if lat == "full" else 2, seed=31)
    c.close()
    assert st.verify_rays == st.closest_rays + st.shadow_rays > 0
    assert st.verify_mismatches == 0, (st.verify_mismatches, st.verify_rays)
    if lat == "full":
        assert st.pipelines == 16 and st.bvh_width == 2, (st.pipelines, st.bvh_width)
    else:
        assert st.pipelines == 1 and st.bvh_width == 4, (st.pipelines, st.bvh_width)


@pytest.mark.parametrize("name,maker,n", [("torus", lambda: _scenes.torus(256, 256), 200_000),
                                          ("cbox", lambda: _scenes.cbox(256, 192), 200_000),
                                          ("torus1m", lambda: big_torus(64, 64), 60_000)])
def test_wave_kd_walk_matches_reference_mode(name, maker, n, monkeypatch):
    """WR_BVH_DIAG=256 sends every ray to k_fast_hard's KD walk: the API calls
    walk them one ray per wave (kd_walk_wave: the wave expands the crossed
    nodes together and replays the reference's first-found rule over the hits
    in walk order).  Same (t, primitive) as the reference mode, bit for bit."""
    ref, _ = pair(maker())
    monkeypatch.setenv("WR_BVH_DIAG", "256")
    s = native.Scene(maker())
    walk = native.Context(s, 0, trace=native.TRACE_BVH)
    rays, (p, sd, q) = _corpus(ref, n, 77)
    a = ref.trace_closest(rays)
    b = walk.trace_closest(rays)
    ok = _same_hits(a, b)
    assert ok.all(), (name, int((~ok).sum()), rays.shape[0], np.nonzero(~ok)[0][:8])
    r8 = native.rays_from_arrays(p, sd)
    assert np.array_equal(ref.occluded(r8, q), walk.occluded(r8, q))


@pytest.mark.parametrize("name,maker", [("torus", lambda: _scenes.torus(128, 128)),
                                        ("torus1m", lambda: big_torus(96, 54))])
def test_wave_kd_walk_in_pipelines_verified(name, maker, monkeypatch):
    """Every ray of a BDPT render to the KD walk (WR_BVH_DIAG=256): the
    pipelines' k_fast_hard takes them one per lane and each lane hands its walk
    to its wave; WR_BVH_VERIFY checks every answer against the serial walk."""
    monkeypatch.setenv("WR_BVH_DIAG", "256")
    monkeypatch.setenv("WR_BVH_VERIFY", "1")
    s = native.Scene(maker())
    c = native.Context(s, 0, trace=native.TRACE_BVH)
    W, H = (128, 128) if name == "torus" else (96, 54)
    _, st = c.render_bdpt(W, H, iterations=1, seed=9, count_work=True)
    assert st.verify_rays == st.closest_rays + st.shadow_rays > 0
    assert st.verify_mismatches == 0, (st.verify_mismatches, st.verify_rays)
    assert st.fallback_rays >= 0.5 * st.closest_rays, (st.fallback_rays, st.closest_rays)  # walked


@pytest.mark.parametrize("name,maker,W,H,its", [("torus", lambda: _scenes.torus(256, 256), 256, 256, 3),
                                                ("cbox", lambda: _scenes.cbox(96, 72, "bdpt"), 96, 72, 3),
                                                ("torus1m", lambda: big_torus(192, 108), 192, 108, 1)])
def test_deferred_hard_rays_render_the_same_film(name, maker, W, H, its, monkeypatch):
    """BDPT hard rays off the critical path (WR_DEFER=1): the
    deferred rays get the same answers (WR_BVH_VERIFY checks them against the KD
    walk), their paths are shaded a step later with their own state and random
    numbers, so the render has the same rays and the same film as the
    synchronous one (up to the order of float atomics) and as the oracle."""
    import _oracle
    from _parity import assert_film_parity, assert_ray_counts
    path = maker()
    s = native.Scene(path)
    films = {}
    monkeypatch.setenv("WR_PIECE_MIN", "4096")  # every pipeline gets a share of these small renders
    for defer in ("1", "0"):
        monkeypatch.setenv("WR_DEFER", defer)
        c = native.Context(s, 0)
        c.set_trace_mode(native.TRACE_BVH)
        c.set_pipelines(4)
        films[defer] = c.render_bdpt(W, H, iterations=its, seed=5489)
        c.close()
    (fa, sa), (fb, sb) = films["1"], films["0"]
    assert sa.pipelines == 4
    assert sa.deferred_rays > 0 and sb.deferred_rays == 0, (sa.deferred_rays, sb.deferred_rays)
    assert sa.closest_rays == sb.closest_rays and sa.shadow_rays == sb.shadow_rays
    assert _film_close(fa, fb)
    ref, rst = _oracle.Scene(path).bdpt(W, H, its, 5489, mode=1)
    assert_film_parity(fa, ref, case=f"bdpt_{name}{W}x{H}_i{its}_s5489_defer")
    assert_ray_counts(sa, rst)
    # and every deferred answer is the KD walk's, bit for bit
    monkeypatch.setenv("WR_DEFER", "1")
    monkeypatch.setenv("WR_BVH_VERIFY", "1")
    c = native.Context(s, 0)
    c.set_trace_mode(native.TRACE_BVH)
    c.set_pipelines(4)
    _, st = c.render_bdpt(W, H, iterations=its, seed=5489)
    c.close()
    assert st.deferred_rays > 0
    assert st.verify_rays == st.closest_rays + st.shadow_rays
    assert st.verify_mismatches == 0, (st.verify_mismatches, st.verify_rays)


def _plane_grazing_rays(ref, n, seed):
    """Rays that run along the plane of the surface they leave (DESIGN.md 4b,
    the near-grazing case of the margins argument): from hit points on every
    surface, directions in the surface's plane tilted out of it by log-uniform
    angles in [1e-8, 3e-3] rad either way, from the hit point itself and from
    points lifted off the plane by log-uniform 1e-7..1e-3 of the scene's size.
    On flat walls and floors every coplanar neighbour's plane is grazed too.

    Hit points come from random rays whose origins fill the box spanned by a
    first sample of hits, so a closed scene (the Cornell box, seen from inside)
    yields its quota as well as an open one."""
    rng = np.random.default_rng(seed)
    o = (rng.uniform(-1, 1, (4 * n, 3)) * np.repeat([2000.0, 400.0, 60.0, 3.0], n)[:, None]).astype(np.float32)
    h = ref.trace_closest(native.rays_from_arrays(o, _unit(rng.normal(size=(4 * n, 3)))))
    first = h["p"][h["prim"] >= 0].astype(np.float64)
    assert first.shape[0] > 100, "no hits from the first sample"
    lo, hi = first.min(axis=0), first.max(axis=0)
    pad = 0.05 * (hi - lo)
    ps, ns = [], []
    got = 0
    for _ in range(32):
        o = rng.uniform(lo - pad, hi + pad, (n, 3)).astype(np.float32)
        h = ref.trace_closest(native.rays_from_arrays(o, _unit(rng.normal(size=(n, 3)))))
        hit = h["prim"] >= 0
        ps.append(h["p"][hit].astype(np.float64))
        ns.append(h["n"][hit].astype(np.float64))
        got += int(hit.sum())
        if got >= n:
            break
    p, nn = np.concatenate(ps)[:n], np.concatenate(ns)[:n]
    m = p.shape[0]
    scale = float(np.abs(p).max())
    u = np.cross(nn, rng.normal(size=(m, 3)))
    with np.errstate(invalid="ignore", divide="ignore"):
        u /= np.linalg.norm(u, axis=1, keepdims=True)
    ang = 10.0 ** rng.uniform(-8, np.log10(3e-3), m) * np.where(rng.random(m) < 0.5, 1.0, -1.0)
    dd = _unit(u * np.cos(ang)[:, None] + nn * np.sin(ang)[:, None])
    lift = np.where(rng.random(m) < 0.5, 0.0, 10.0 ** rng.uniform(-7, -3, m) * scale)
    lift *= np.where(rng.random(m) < 0.5, 1.0, -1.0)
    oo = (p + nn * lift[:, None]).astype(np.float32)
    ok = _valid(oo, dd)
    return native.rays_from_arrays(oo[ok], dd[ok])


@pytest.mark.parametrize("name,maker", SCENES + [("torus1m", lambda: big_torus(64, 64))])
def test_bvh_matches_reference_mode_on_plane_grazing_rays(name, maker):
    """The targeted probe of DESIGN.md 4b's near-grazing case: BVH mode vs the
    reference's KD walk, (t, primitive) bit for bit, on rays grazing the plane
    of the surface they leave (and of its coplanar neighbours)."""
    ref, fast = pair(maker())
    n = 600_000 if name != "torus1m" else 200_000
    rays = _plane_grazing_rays(ref, n, 99)
    assert rays.shape[0] >= 0.9 * n, (name, rays.shape[0], n)
    a = ref.trace_closest(rays)
    b = fast.trace_closest(rays)
    ok = _same_hits(a, b)
    print(name, rays.shape[0], "rays,", int((a["prim"] >= 0).sum()), "hits,", int((~ok).sum()), "mismatches")
    assert ok.all(), (name, int((~ok).sum()), rays.shape[0], np.nonzero(~ok)[0][:8])


def _sphere_rim_rays(rng, n, centres, radii, lo, hi):
    """Rays passing a sphere at its rim: closest approach r (1 + s), s from
    -1e-2 to 1e-2 on a log scale down to 1e-8 (both signs), from origins
    anywhere in the scene box -- where Sphere::hit's t_hc is at its rounding
    noise (wr_bvh.cpp, sphere_grow)."""
    k = rng.integers(0, len(radii), n)
    c, r = centres[k], radii[k]
    o = rng.uniform(lo, hi, (n, 3))
    to_c = c - o
    dist = np.linalg.norm(to_c, axis=1)
    u = to_c / dist[:, None]
    w = np.cross(u, rng.normal(size=(n, 3)))
    w /= np.linalg.norm(w, axis=1, keepdims=True)
    s = 10.0 ** rng.uniform(-8, -2, n) * np.where(rng.random(n) < 0.5, 1.0, -1.0)
    b = np.clip(r * (1 + s) / np.maximum(dist, 1e-9), -1.0, 1.0)  # sin of the angle off the centre
    d = u * np.sqrt(1 - b * b)[:, None] + w * b[:, None]
    ok = dist > r * 1.05
    return native.rays_from_arrays(o[ok].astype(np.float32), _unit(d[ok]))


def test_bvh_matches_reference_mode_on_sphere_rim_rays():
    """Spheres in the verified BVH: rays grazing a sphere's rim, where the
    reference's t_hc is decided by rounding, from origins inside the scene (the
    search's sphere boxes cover them) and far outside it (taken to the KD walk):
    the BVH mode's (t, primitive) equals the reference KD walk's bit for bit,
    and so do the occlusion answers."""
    ref, fast = pair(_scenes.spheres(256, 256))
    rng = np.random.default_rng(17)
    centres = np.array([[-0.5, 0.3, -0.82], [0.55, 0.6, -0.86], [0.05, -0.45, -1.0]])
    radii = np.array([0.45, 0.42, 0.28])
    near = _sphere_rim_rays(rng, 400_000, centres, radii, np.array([-1.0, -1.0, -1.3]), np.array([1.0, 1.0, 1.0]))
    far = _sphere_rim_rays(rng, 100_000, centres, radii, np.array([-60.0, -60.0, -60.0]), np.array([60.0, 60.0, 60.0]))
    for name, rays in (("near", near), ("far", far)):
        a = ref.trace_closest(rays)
        b = fast.trace_closest(rays)
        ok = _same_hits(a, b)
        pd = a["p"].astype(np.float64)
        on = np.abs(np.linalg.norm(pd[:, None, :] - centres[None], axis=2) - radii[None]).min(axis=1) < 1e-3
        sph = (a["prim"] >= 0) & on
        print(name, rays.shape[0], "rays,", int(sph.sum()), "sphere hits,", int((~ok).sum()), "mismatches")
        assert ok.all(), (name, int((~ok).sum()), rays.shape[0], np.nonzero(~ok)[0][:8])
        # (half of the rim rays pass outside; most far ones meet the box's walls first)
        assert sph.sum() > (0.1 if name == "near" else 0.01) * rays.shape[0], (name, int(sph.sum()))
    o = near[:200_000, 0:3]
    q = o + near[:200_000, 3:6] * 2.0
    assert np.array_equal(ref.occluded(near[:200_000], q), fast.occluded(near[:200_000], q))


def test_bvh_sphere_films_match_the_oracle():
    """Spheres scene in the BVH mode (the library default) against the oracle:
    BDPT and PT films under the same gates as the KD walk's, same ray counts."""
    import _oracle
    from _parity import assert_film_parity, assert_ray_counts
    path = _scenes.spheres(64, 64)
    c = native.Context(native.Scene(path), 0, trace=native.TRACE_BVH)
    film, st = c.render_bdpt(64, 64, iterations=4, seed=5489)
    ref, rst = _oracle.Scene(path).bdpt(64, 64, 4, 5489, mode=1)
    assert_film_parity(film, ref, case="bdpt_spheres64x64_i4_s5489")
    assert_ray_counts(st, rst)
    assert st.bvh_width == 2
    film, st = c.render_path(64, 64, spp=16, max_depth=7, seed=5489)
    ref, rst = _oracle.Scene(path).pt(64, 64, 16, 7, 5489, mode=1)
    assert_film_parity(film * np.float32(1.0 / 16), ref, case="pt_spheres64x64_spp16_s5489")
    assert_ray_counts(st, rst)
