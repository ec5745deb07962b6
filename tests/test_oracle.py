"""Pin oracle/cpuref.c to the reference's own outputs (tests/golden/, made by
tests/golden/make_golden.py from oracle/_ref/refdrv).  CPU only.

Everything here is bit-exact: same float evaluation order, same libm.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import _oracle
import _scenes

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
META = json.load(open(os.path.join(GOLD, "golden.json")))


def hx(t):
    return np.float32(float.fromhex(t))


@pytest.mark.parametrize("seed", [5489, 12345])
def test_mt19937_matches_reference(seed):
    ref = np.loadtxt(os.path.join(GOLD, f"mt_{seed}.txt"), dtype=np.uint64).astype(np.uint32)
    out = np.zeros(len(ref), np.uint32)
    import ctypes as C
    _oracle.lib().cr_mt_outputs(seed, len(ref), out.ctypes.data_as(C.POINTER(C.c_uint32)))
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("name,maker", [("torus64", lambda: _scenes.torus(64, 64)),
                                        ("torus256", lambda: _scenes.torus(256, 256)),
                                        ("cbox64x48", lambda: _scenes.cbox(64, 48)),
                                        ("spheres64", lambda: _scenes.spheres(64, 64))])
def test_scene_and_kdtree_dump_bit_exact(name, maker, tmp_path):
    """Loader (scene.cpp:259-467 + tinyobj), camera matrices (camera.cpp:3-29) and
    the whole KD tree incl. leaf order (KDtreeAccel.cpp:12-307) hash-equal."""
    s = _oracle.Scene(maker())
    txt = s.dump(str(tmp_path / "d.txt"))
    m = META[name]
    lines = txt.splitlines()
    assert s.nobjs == m["nobjs"]
    assert sum(1 for l in lines if l.startswith("L ")) == m["leaves"]
    assert sum(1 for l in lines if l.startswith("I ")) == m["inner"]
    assert hashlib.sha256(txt.encode()).hexdigest() == m["scene_sha256"]


def parse_rays(path):
    out = []
    for line in open(path):
        tok = line.split()
        occ = int(tok[-1])
        if tok[0] == "-1":
            out.append((-1, None, None, None, occ))
        else:
            vals = np.array([hx(t) for t in tok[1:8]], np.float32)
            out.append((int(tok[0]), vals, int(tok[8]), int(tok[9]), occ))
    return out


@pytest.mark.parametrize("name,maker", [("torus64", lambda: _scenes.torus(64, 64)),
                                        ("cbox64x48", lambda: _scenes.cbox(64, 48)),
                                        ("spheres64", lambda: _scenes.spheres(64, 64))])
def test_trace_corpus_bit_exact(name, maker):
    """Scene::intersect + Scene::occluded on the golden ray corpus."""
    s = _oracle.Scene(maker())
    rays = np.fromfile(os.path.join(GOLD, f"rays_{name}.f32"), np.float32).reshape(-1, 9)
    ref = parse_rays(os.path.join(GOLD, f"rays_{name}.txt"))
    oi, of, oc, st = s.trace(rays)
    assert st.closest_rays == len(rays) and st.shadow_rays == len(rays)
    for k, (prim, vals, inside, mat, occ) in enumerate(ref):
        assert oi[k, 0] == prim, k
        assert oc[k] == occ, k
        if prim >= 0:
            assert np.array_equal(of[k], vals), k
            assert oi[k, 1] == inside and oi[k, 2] == mat, k


def kat_lines(name, tag):
    return [l.split()[1:] for l in open(os.path.join(GOLD, f"kat_{name}.txt")) if l.startswith(tag + " ")]


def test_kat_samplers():
    L = _oracle.lib()
    F = _oracle.fptr
    cosh = kat_lines("torus64", "cosh")
    pcosh = kat_lines("torus64", "pcosh")
    assert len(cosh) == len(pcosh) > 0
    for a, b in zip(cosh, pcosh):
        u = np.array([hx(t) for t in a[0:3]], np.float32)
        power = hx(b[3])
        o = np.zeros(9, np.float32)
        L.cr_kat_sampler(F(u), power, F(o))
        assert np.array_equal(o[0:4], [hx(t) for t in a[3:7]])
        assert np.array_equal(o[4:9], [hx(t) for t in b[4:9]])
    for a in kat_lines("torus64", "tri"):
        v = np.array([hx(t) for t in a], np.float32)
        o = np.zeros(3, np.float32)
        L.cr_kat_triangle(F(v[0:3]), F(np.ascontiguousarray(v[3:12])), F(o))
        assert np.array_equal(o, v[12:15])
    for a in kat_lines("torus64", "frame"):
        v = np.array([hx(t) for t in a], np.float32)
        o = np.zeros(9, np.float32)
        L.cr_kat_frame(F(np.ascontiguousarray(v[0:3])), F(o))
        assert np.array_equal(o, v[3:12])
    for a in kat_lines("torus64", "fresnel"):
        assert L.cr_kat_fresnel(hx(a[0]), hx(a[1])) == hx(a[2])
    for a in kat_lines("torus64", "strat"):
        k, tot = int(a[0]), int(a[1])
        v = np.array([hx(t) for t in a[2:]], np.float32)
        o = np.zeros(3, np.float32)
        L.cr_kat_strat(F(np.ascontiguousarray(v[0:3])), k, tot, F(o))
        assert np.array_equal(o, v[3:6])


@pytest.mark.parametrize("name,maker", [("torus64", lambda: _scenes.torus(64, 64)),
                                        ("cbox64x48", lambda: _scenes.cbox(64, 48)),
                                        ("spheres64", lambda: _scenes.spheres(64, 64))])
def test_kat_bsdf_lights_camera(name, maker):
    """BSDF init/f/pdf/sample (bsdf.h:66-89, bsdf.cpp), AreaLight (light.cpp:4-100)
    and Camera (camera.cpp:31-42) known answers per material / light."""
    s = _oracle.Scene(maker())
    L, F = s.L, _oracle.fptr
    nb = 0
    for a in kat_lines(name, "bsdf"):
        m = int(a[0])
        v = np.array([hx(t) for t in a[1:13]], np.float32)
        o = np.zeros(26, np.float32)
        valid = L.cr_kat_bsdf(s.h, m, F(v[0:3].copy()), F(v[3:6].copy()), F(v[6:9].copy()),
                              F(v[9:12].copy()), F(o))
        assert valid == int(a[14])
        if not valid:
            continue
        nb += 1
        rest = a[15:]
        exp = [float(rest[0])] + [hx(t) for t in rest[1:8]]  # isDelta, cosWi, cont, fres, 4 probs
        assert np.array_equal(o[0:8], np.array(exp, np.float32)), (m, a)
        fi = rest.index("f")
        assert np.array_equal(o[8:14], [hx(t) for t in rest[fi + 1:fi + 7]]), (m, a)
        pi = rest.index("pdf")
        assert np.array_equal(o[14:16], [hx(t) for t in rest[pi + 1:pi + 3]]), (m, a)
        si = rest.index("smp")
        assert int(o[16]) == int(rest[si + 1])
        assert np.array_equal(o[17:25], [hx(t) for t in rest[si + 2:si + 10]]), (m, a)
    assert nb > 100
    for tag_i, tag_e, tag_r in zip(kat_lines(name, "illu"), kat_lines(name, "emit"), kat_lines(name, "rad")):
        li = int(tag_i[0])
        vi = np.array([hx(t) for t in tag_i[1:]], np.float32)
        ve = np.array([hx(t) for t in tag_e[1:]], np.float32)
        vr = np.array([hx(t) for t in tag_r[1:]], np.float32)
        o = np.zeros(27, np.float32)
        L.cr_kat_light(s.h, li, F(vi[0:3].copy()), F(vi[3:6].copy()), F(ve[0:3].copy()),
                       F(ve[3:6].copy()), F(vr[0:3].copy()), F(o))
        assert np.array_equal(o[0:10], vi[6:16])
        assert np.array_equal(o[10:22], ve[6:18])
        assert np.array_equal(o[22:27], vr[6:11])
    for a in kat_lines(name, "cam"):
        v = np.array([hx(t) for t in a[:-1]], np.float32)
        o = np.zeros(10, np.float32)
        L.cr_kat_camera(s.h, v[0], v[1], F(v[8:11].copy()), F(o))
        assert np.array_equal(o[0:6], v[2:8])
        assert np.array_equal(o[6:9], v[11:14])
        assert int(o[9]) == int(a[-1])


@pytest.mark.parametrize("it,seed", [(1, 5489), (4, 5489), (2, 7)])
def test_bdpt_film_mt_serial_bit_exact(it, seed):
    """Whole BDPT render (bidirPathTracing.cpp:53-665) replayed on the MT stream."""
    s = _oracle.Scene(_scenes.torus(64, 64))
    film, st = s.bdpt(64, 64, it, seed, mode=0)
    ref = np.fromfile(os.path.join(GOLD, f"bdpt_torus64_i{it}_s{seed}.f32"), np.float32).reshape(64, 64, 3)
    assert np.array_equal(film, ref)
    assert st.closest_rays > 0 and st.shadow_rays > 0


@pytest.mark.slow
def test_bdpt_256_mt_serial_bit_exact():
    s = _oracle.Scene(_scenes.torus(256, 256))
    film, st = s.bdpt(256, 256, 4, 5489, mode=0)
    m = META["bdpt_torus256_i4_s5489"]
    assert hashlib.sha256(film.tobytes()).hexdigest() == m["sha256"]
    # torus BDPT at 256^2: ~190 triangle tests per traversal
    assert 150 < st.tri_tests / (st.closest_rays + st.shadow_rays) < 230


def test_pt_film_mt_serial_bit_exact():
    """PathIntegrator (pathIntegrator.cpp:29-148) via SurfaceIntegrator::render."""
    s = _oracle.Scene(_scenes.cbox(64, 48))
    film, _ = s.pt(64, 48, 16, 7, 5489, mode=0)
    ref = np.fromfile(os.path.join(GOLD, "pt_cbox64x48_spp16_s5489.f32"), np.float32).reshape(48, 64, 3)
    assert np.array_equal(film, ref)


def test_spheres_bdpt_and_pt_films_mt_serial_bit_exact():
    """Sphere::hit (sphere.cpp:17-78) and the glass / mirror BSDF branches, whole
    renders against the reference's own films."""
    s = _oracle.Scene(_scenes.spheres(64, 64))
    film, _ = s.bdpt(64, 64, 2, 5489, mode=0)
    ref = np.fromfile(os.path.join(GOLD, "bdpt_spheres64_i2_s5489.f32"), np.float32).reshape(64, 64, 3)
    assert np.array_equal(film, ref)
    film, _ = s.pt(64, 64, 4, 7, 5489, mode=0)
    ref = np.fromfile(os.path.join(GOLD, "pt_spheres64_spp4_s5489.f32"), np.float32).reshape(64, 64, 3)
    assert np.array_equal(film, ref)


VCM_SCENES = {"torus64": (lambda: _scenes.torus(64, 64), 64, 64),
              "spheres64": (lambda: _scenes.spheres(64, 64), 64, 64),
              "cboxb64x48": (lambda: _scenes.cbox(64, 48, "bdpt"), 64, 48),
              "tent64": (lambda: _scenes.tent(64, 64), 64, 64)}


@pytest.mark.parametrize("name,it,seed,rf", [("torus64", 1, 5489, None), ("torus64", 3, 3, 0.05),
                                             ("spheres64", 2, 11, 0.1), ("cboxb64x48", 3, 3, 0.05),
                                             ("tent64", 2, 3, 0.05), ("tent64", 4, 5, 0.05)])
def test_vcm_film_mt_serial_bit_exact(name, it, seed, rf):
    """VertexCM::runIteration (vertexcm.cpp:47-285): light pass with light
    tracing, the point KD tree (KDtree.h:88-175), camera pass with NEE, vertex
    connection and merging -- replayed on the MT stream, bit for bit, including
    the radius schedule over iterations (:53-56) and the emitter light vertices
    that inherit the previous BSDF's probabilities."""
    maker, W, H = VCM_SCENES[name]
    s = _oracle.Scene(maker())
    film, st = s.vcm(W, H, it, seed, mode=0, radius_factor=0.003 if rf is None else rf)
    fx = f"vcm_{name}_i{it}_s{seed}" + ("" if rf is None else f"_r{rf}") + ".f32"
    ref = np.fromfile(os.path.join(GOLD, fx), np.float32).reshape(H, W, 3)
    assert np.array_equal(film.view(np.uint32), ref.view(np.uint32))
    assert st.vm_queries > 0 and st.vm_merged > 0 and st.vm_found >= st.vm_merged
    if name == "tent64":  # the cross-path stale-BSDF case is exercised (~500 per iteration)
        assert st.vm_emitter_first > 100 * it


def test_vcm_kdtree_search_is_the_brute_force_set():
    """KdTree::searchInRadius prunes with |pos[axis] - split| < radius, which is
    exact in float: the found set equals every point with |q - p| < radius.  So
    the GPU may replace the tree by a hash grid; only the summation order of the
    merge contributions differs.  Point clouds with tied coordinates (the
    comparator's address tie-break, KDtree.h:74-86) and duplicate points."""
    import ctypes as C
    rng = np.random.default_rng(3)
    for n, grid in ((1, None), (2, None), (7, None), (500, None), (3000, 16), (3000, 4)):
        p = rng.random((n, 3)).astype(np.float32)
        if grid:
            p = (np.floor(p * grid) / grid).astype(np.float32)
        q = np.concatenate([p[: min(n, 200)] + rng.normal(0, 0.02, (min(n, 200), 3)).astype(np.float32),
                            rng.random((200, 3)).astype(np.float32)])
        out = np.zeros((len(q), 4), np.int64)
        for r in (0.01, 0.07, 0.25):
            _oracle.lib().cr_kat_vkd(_oracle.fptr(np.ascontiguousarray(p)), n,
                                     _oracle.fptr(np.ascontiguousarray(q)), len(q), r,
                                     out.ctypes.data_as(C.POINTER(C.c_int64)))
            assert np.array_equal(out[:, :2], out[:, 2:]), (n, grid, r)
        assert out[:, 0].sum() > 0


def test_counter_mode_is_statistically_the_reference():
    """Counter-RNG oracle vs the reference's 256^2 x4 statistics: same estimator,
    independent random numbers => agreement to within Monte-Carlo noise."""
    s = _oracle.Scene(_scenes.torus(256, 256))
    film, _ = s.bdpt(256, 256, 4, 5489, mode=1)
    m = META["bdpt_torus256_i4_s5489"]
    ref_mean = np.array(m["mean"])
    mean = film.mean(axis=(0, 1))
    assert np.all(np.abs(mean - ref_mean) < 0.15 * ref_mean + 1e-5), (mean, ref_mean)
    rms = float(np.sqrt((film.astype(np.float64) ** 2).mean()))
    assert abs(rms - m["rms"]) < 0.3 * m["rms"]


def test_counter_rng_streams():
    L = _oracle.lib()
    k1 = L.cr_stream_key(5489, 0, 0, 0)
    k2 = L.cr_stream_key(5489, 0, 1, 0)
    k3 = L.cr_stream_key(5489, 1, 0, 0)
    assert len({k1, k2, k3}) == 3
    u = np.array([L.cr_stream_u32(k1, i) & 0xffffff for i in range(20000)], np.float64) / 2 ** 24
    assert abs(u.mean() - 0.5) < 0.01 and abs(u.var() - 1 / 12) < 0.005
