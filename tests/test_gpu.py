"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference's golden fixtures.  Runs on the MI355X box (`-m gpu`).

Tolerances
  * traversal (wr_trace_closest / wr_occluded): bit-exact vs the reference's own
    outputs (tests/golden/rays_*.txt) -- same float ops, no FMA contraction;
  * films: the GPU and the oracle draw the same counter-RNG numbers; they differ
    only where OCML and glibc cosf/sinf/powf round differently.  The gates
    (tests/_parity.py, set from scripts/parity_stats.py's measurements): a few
    pixels of "split" paths may differ freely, every other pixel agrees to
    1e-5 (relative RMSE and summed bias), per-channel RMSE < 1e-3 (north_star),
    ray counts equal up to the split paths' rays;
  * full-size runs: size-independent properties (finite, non-negative,
    iteration additivity == sharding invariance, determinism of the ray set).
"""
import os

import numpy as np
import pytest

import _oracle
import _scenes
from _parity import assert_film_parity, assert_ray_counts
from test_oracle import parse_rays
from winmad_rt import native

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

_cache = {}


def ctx(path):
    if path not in _cache:
        s = native.Scene(path)
        _cache[path] = (s, native.Context(s, 0))
    return _cache[path][1]


def normalize_f32(d):
    d = d.astype(np.float32)
    l = np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2])
    return (d / l[:, None]).astype(np.float32)


@pytest.mark.parametrize("name,maker", [("torus64", lambda: _scenes.torus(64, 64)),
                                        ("cbox64x48", lambda: _scenes.cbox(64, 48)),
                                        ("spheres64", lambda: _scenes.spheres(64, 64))])
def test_trace_closest_bit_exact_vs_reference(name, maker):
    """The reference's own outputs: the library default (verified BVH on
    triangle scenes) and the KD walk, forced."""
    _check_golden_corpus(ctx(maker()), name)
    _check_golden_corpus(native.Context(native.Scene(maker()), 0, trace=native.TRACE_REFERENCE), name)


@pytest.mark.parametrize("name,maker", [("torus64", lambda: _scenes.torus(64, 64)),
                                        ("cbox64x48", lambda: _scenes.cbox(64, 48)),
                                        ("spheres64", lambda: _scenes.spheres(64, 64))])
def test_trace_dense_variant_bit_exact_vs_reference(name, maker, monkeypatch):
    """TRACE_DENSE (PT's launches: owner rays by ds_bpermute, 20 waves/CU),
    forced on the API: the reference's corpus, closest hits and occlusion."""
    monkeypatch.setenv("WR_TRACE_DENSE", "1")
    _check_golden_corpus(native.Context(native.Scene(maker()), 0, trace=native.TRACE_REFERENCE), name)


def _check_golden_corpus(c, name):
    rays = np.fromfile(os.path.join(GOLD, f"rays_{name}.f32"), np.float32).reshape(-1, 9)
    ref = parse_rays(os.path.join(GOLD, f"rays_{name}.txt"))
    r8 = native.rays_from_arrays(rays[:, 0:3], normalize_f32(rays[:, 3:6]))  # Ray ctor normalises
    hits = c.trace_closest(r8)
    bad = 0
    for k, (prim, vals, inside, mat, occ) in enumerate(ref):
        if hits["prim"][k] != prim:
            bad += 1
            continue
        if prim >= 0:
            got = np.concatenate([[hits["t"][k]], hits["p"][k], hits["n"][k]]).astype(np.float32)
            assert np.array_equal(got, vals), (k, got, vals)
            assert hits["inside"][k] == inside and hits["mat_id"][k] == mat
    assert bad == 0
    occ = c.occluded(native.rays_from_arrays(rays[:, 0:3], rays[:, 3:6]), rays[:, 6:9])
    assert np.array_equal(occ, np.array([r[4] for r in ref], np.uint8))


def test_trace_edge_cases():
    c = ctx(_scenes.torus(64, 64))
    o = np.array([[0, 5000, 0], [0, 5000, 0], [1e6, 1e6, 1e6]], np.float32)
    d = np.array([[0, -1, 0], [0, 1, 0], [1, 0, 0]], np.float32)
    h = c.trace_closest(native.rays_from_arrays(o, d))
    assert h["prim"][1] == -1 and h["prim"][2] == -1  # away from the scene
    assert c.trace_closest(np.zeros((0, 8), np.float32)).shape == (0,)
    # tmax clips
    h2 = c.trace_closest(native.rays_from_arrays(o[:1], d[:1], tmax=1.0))
    assert h2["prim"][0] == -1


def film_err(a, b):
    rmse = float(np.sqrt(((a.astype(np.float64) - b) ** 2).mean()))
    rms = float(np.sqrt((b.astype(np.float64) ** 2).mean()))
    ch = np.sqrt(((a.astype(np.float64) - b) ** 2).mean(axis=(0, 1)))
    return rmse, rms, ch


@pytest.mark.parametrize("W,H,it", [(64, 64, 4), (96, 64, 2)])
def test_bdpt_matches_oracle_counter_rng(W, H, it):
    """Same counter-RNG streams => the GPU film is the oracle's film up to libm
    rounding; non-square films exercise the film[x][y] orientation."""
    path = _scenes.torus(W, H)
    film, st = ctx(path).render_bdpt(W, H, iterations=it, seed=5489)
    ref, rst = _oracle.Scene(path).bdpt(W, H, it, 5489, mode=1)
    assert_film_parity(film, ref, case=f"bdpt_torus{W}x{H}_i{it}_s5489")
    assert_ray_counts(st, rst)


def test_bdpt_all_lengths_and_control_length_filter():
    path = _scenes.torus(64, 64)
    f_all, _ = ctx(path).render_bdpt(64, 64, iterations=2, seed=11, control_length=0)
    r_all, _ = _oracle.Scene(path).bdpt(64, 64, 2, 11, mode=1, control_length=0)
    assert_film_parity(f_all, r_all, case="bdpt_torus64x64_i2_s11_ctl0")
    f3, _ = ctx(path).render_bdpt(64, 64, iterations=2, seed=11)
    assert f_all.mean() > f3.mean()  # the length-3 filter drops energy


def test_bdpt_statistically_matches_reference_mt_run():
    """Independent RNG (counter vs the reference's MT stream): 256^2 x 4
    iterations agree with the reference's film statistics to within noise."""
    import json
    m = json.load(open(os.path.join(GOLD, "golden.json")))["bdpt_torus256_i4_s5489"]
    film, _ = ctx(_scenes.torus(256, 256)).render_bdpt(256, 256, iterations=4, seed=5489)
    mean = film.mean(axis=(0, 1))
    assert np.all(np.abs(mean - np.array(m["mean"])) < 0.15 * np.array(m["mean"]) + 1e-5)
    blocks = film.reshape(8, 32, 8, 32, 3).mean(axis=(1, 3))
    ref_blocks = np.array(m["block32_mean"])
    assert np.abs(blocks - ref_blocks).mean() < 0.25 * ref_blocks.mean() + 1e-5


def test_pt_matches_oracle_counter_rng():
    path = _scenes.cbox(64, 48)
    film, st = ctx(path).render_path(64, 48, spp=16, max_depth=7, seed=5489)
    ref, rst = _oracle.Scene(path).pt(64, 48, 16, 7, 5489, mode=1)
    film = film * np.float32(1.0 / 16)  # the oracle (like the reference) scales by 1/spp
    assert_film_parity(film, ref, case="pt_cbox64x48_spp16_s5489")
    assert_ray_counts(st, rst)


def test_pt_sample_sharding_is_additive():
    path = _scenes.cbox(64, 48)
    c = ctx(path)
    full, _ = c.render_path(64, 48, spp=16, seed=3)
    a, _ = c.render_path(64, 48, spp=16, seed=3, sample_begin=0, sample_count=7)
    b, _ = c.render_path(64, 48, spp=16, seed=3, sample_begin=7, sample_count=9)
    assert np.allclose(a + b, full, rtol=1e-5, atol=1e-6)


def test_pt_sample_range_matches_oracle():
    """One rank's share (samples [3, 8) of a 9-sample grid, stratified over the
    whole grid) equals the oracle's cr_render_pt_samples of the same range."""
    path = _scenes.cbox(64, 48)
    film, st = ctx(path).render_path(64, 48, spp=9, max_depth=7, seed=8, sample_begin=3, sample_count=5)
    ref, rst = _oracle.Scene(path).pt_samples(64, 48, 9, 3, 5, 7, 8)
    assert_film_parity(film, ref, case="pt_cbox64x48_spp9_k3n5_s8")
    assert_ray_counts(st, rst)


def test_bdpt_1080p_properties_and_sharding():
    """Full C2 frame size: finite, non-negative, iteration-sharded renders sum
    to the unsharded one (multi-GPU invariance), identical ray sets."""
    W, H = 1920, 1080
    c = ctx(_scenes.torus(W, H))
    both, s2 = c.render_bdpt(W, H, iterations=2, seed=5489)
    a, sa = c.render_bdpt(W, H, iterations=1, seed=5489, iter_begin=0)
    b, sb = c.render_bdpt(W, H, iterations=1, seed=5489, iter_begin=1)
    assert np.all(np.isfinite(both)) and both.min() >= 0 and both.max() > 0
    assert sa.closest_rays + sb.closest_rays == s2.closest_rays
    assert sa.shadow_rays + sb.shadow_rays == s2.shadow_rays
    assert np.allclose(a + b, both, rtol=1e-4, atol=1e-6)
    # rays per pixel per iteration near the reference's 4.16
    rpp = (sa.closest_rays + sa.shadow_rays) / (W * H)
    assert 3.5 < rpp < 4.8, rpp


def test_4k_frames_properties_and_sharding():
    """3840x2160 frames (4x BASELINE.json's) for BDPT, VCM and PT: the work
    buffers scale with the frame (2 pipelines here, up to ~105 GB), renders
    stay finite and non-negative, iteration / sample shards add up, and BDPT's
    ray density per pixel is the 1080p frame's."""
    W, H = 3840, 2160
    s = native.Scene(_scenes.torus(W, H))
    c = native.Context(s, 0)
    try:
        c.set_pipelines(2)
        both, s2 = c.render_bdpt(W, H, iterations=2, seed=77)
        a, sa = c.render_bdpt(W, H, iterations=1, seed=77, iter_begin=0)
        b, sb = c.render_bdpt(W, H, iterations=1, seed=77, iter_begin=1)
        assert np.all(np.isfinite(both)) and both.min() >= 0 and both.max() > 0
        assert sa.closest_rays + sb.closest_rays == s2.closest_rays
        assert sa.shadow_rays + sb.shadow_rays == s2.shadow_rays
        assert np.allclose(a + b, both, rtol=1e-4, atol=1e-6)
        rpp = (sa.closest_rays + sa.shadow_rays) / (W * H)
        assert 3.5 < rpp < 4.8, rpp
        # VCM and PT on the same frame: shards add up as well
        vb, _ = c.render_vcm(W, H, iterations=2, seed=77)
        va, _ = c.render_vcm(W, H, iterations=1, seed=77, iter_begin=0)
        vc, _ = c.render_vcm(W, H, iterations=1, seed=77, iter_begin=1)
        assert np.all(np.isfinite(vb)) and vb.min() >= 0 and vb.max() > 0
        assert np.allclose(va + vc, vb, rtol=1e-4, atol=1e-6)
    finally:
        c.close()
    cb = native.Context(native.Scene(_scenes.cbox(W, H)), 0)
    try:
        cb.set_pipelines(2)
        full, _ = cb.render_path(W, H, spp=4, seed=7)
        p0, _ = cb.render_path(W, H, spp=4, seed=7, sample_begin=0, sample_count=1)
        p1, _ = cb.render_path(W, H, spp=4, seed=7, sample_begin=1, sample_count=3)
        assert np.all(np.isfinite(full)) and full.min() >= 0 and full.max() > 0
        assert np.allclose(p0 + p1, full, rtol=1e-4, atol=1e-6)
    finally:
        cb.close()


def test_bdpt_1080p_matches_oracle_counter_rng():
    """BASELINE.json's own frame (torus.scene 1920x1080, C2), one iteration:
    the GPU film against the oracle's counter-RNG film -- the same gates as the
    small films (the oracle needs ~5-15 s of one CPU core here)."""
    W, H = 1920, 1080
    path = _scenes.torus(W, H)
    film, st = ctx(path).render_bdpt(W, H, iterations=1, seed=5489)
    ref, rst = _oracle.Scene(path).bdpt(W, H, 1, 5489, mode=1)
    assert_film_parity(film, ref, case="bdpt_torus1920x1080_i1_s5489")
    assert_ray_counts(st, rst)
    # the gates catch the GPU film damaged the ways tests/test_parity_gates.py
    # damages oracle films: one 8-row tile band not written (verdict r4: at
    # 1080p that moves the per-channel RMSE by only ~3e-4), one row's splats a
    # pixel off
    sums = np.abs(ref).reshape(H // 8, 8, -1).sum(axis=(1, 2))
    lit = np.nonzero(sums > 0)[0]
    for band in (int(np.argmax(sums)), int(lit[len(lit) // 2])):
        bad = film.copy()
        bad[8 * band:8 * band + 8] = 0
        with pytest.raises(AssertionError):
            assert_film_parity(bad, ref, case="bdpt_torus1920x1080_i1_s5489")
    row = int(np.argmax(np.abs(ref).sum(axis=(1, 2))))
    bad = film.copy()
    bad[row] = np.roll(film[row], 1, axis=0)
    with pytest.raises(AssertionError):
        assert_film_parity(bad, ref, case="bdpt_torus1920x1080_i1_s5489")
    # and one pixel off by 1e-3 of its value (a single path's share gone)
    y, x = np.argwhere(ref.any(axis=-1))[len(np.argwhere(ref.any(axis=-1))) // 2]
    bad = film.copy()
    bad[y, x] *= 1.001
    with pytest.raises(AssertionError):
        assert_film_parity(bad, ref, case="bdpt_torus1920x1080_i1_s5489")


# Seeds none of the other cases use, each run once (verdict r5, next 1): the
# films must equal the oracle's on every pixel for any random numbers, not
# only for the seeds the gates were first measured on.
SWEEP_SEEDS = (1, 7, 41, 97, 1234)


@pytest.mark.parametrize("seed", SWEEP_SEEDS)
@pytest.mark.parametrize("name,maker,W,H,it,ctl", [
    ("cbox", lambda: _scenes.cbox(64, 48, "bdpt"), 64, 48, 3, 0),  # every path length, NEE + connections
    ("torus", lambda: _scenes.torus(256, 256), 256, 256, 1, 3),
])
def test_bdpt_seed_sweep_matches_oracle(name, maker, W, H, it, ctl, seed):
    path = maker()
    film, st = ctx(path).render_bdpt(W, H, iterations=it, seed=seed, control_length=ctl)
    ref, rst = _oracle.Scene(path).bdpt(W, H, it, seed, mode=1, control_length=ctl)
    assert_film_parity(film, ref, case=f"bdpt_{name}{W}x{H}_i{it}_s{seed}_ctl{ctl}")
    assert_ray_counts(st, rst)


def test_bdpt_1080p_seed_sweep_matches_oracle():
    """The C2 frame (torus.scene 1920x1080, one iteration) at each sweep
    seed: every pixel equals the oracle's.  The oracle films are rendered on
    5 host threads (ctypes releases the GIL; the scene is read-only)."""
    from concurrent.futures import ThreadPoolExecutor
    W, H = 1920, 1080
    path = _scenes.torus(W, H)
    osc = _oracle.Scene(path)
    osc.bdpt(2, 2, 1, 1, mode=1)  # (the oracle's one-time constants, before the threads)
    with ThreadPoolExecutor(len(SWEEP_SEEDS)) as ex:
        refs = list(ex.map(lambda sd: osc.bdpt(W, H, 1, sd, mode=1), SWEEP_SEEDS))
    for seed, (ref, rst) in zip(SWEEP_SEEDS, refs):
        film, st = ctx(path).render_bdpt(W, H, iterations=1, seed=seed)
        assert_film_parity(film, ref, case=f"bdpt_torus1920x1080_i1_s{seed}")
        assert_ray_counts(st, rst)


def test_path_radiance_per_ray_matches_oracle():
    """wr_path_radiance == PathIntegrator::raytracing per caller ray (same
    counter-RNG stream): camera rays through random raster points and random
    rays inside the box.  Every ray's radiance agrees to 1e-5 relative (the
    same path, summed in the same order: glibc-exact libm on the device), and
    the traversal counts are equal."""
    path = _scenes.cbox(64, 48)
    rng = np.random.default_rng(9)
    n = 20000
    cam = np.array([-0.0439815, -4.12529, 0.222539], np.float32)
    tgt = np.stack([rng.uniform(-1.2, 1.2, n), np.full(n, 1.3), rng.uniform(-1.2, 1.2, n)], 1).astype(np.float32)
    d = normalize_f32(tgt - cam)
    o = np.repeat(cam[None], n, 0)
    o[n // 2:] = rng.uniform(-1.0, 1.0, (n - n // 2, 3)).astype(np.float32)
    d[n // 2:] = normalize_f32(rng.normal(size=(n - n // 2, 3)))
    rays = native.rays_from_arrays(o, d)
    rad, st = ctx(path).path_radiance(rays, max_depth=7, seed=77, sample=3)
    ref, rst = _oracle.Scene(path).pt_radiance(np.concatenate([o, d], 1), 7, 77, sample=3)
    assert np.all(np.isfinite(rad)) and rad.min() >= 0 and ref.sum() > 0
    close = np.all(np.abs(rad - ref) <= 1e-5 * np.abs(ref) + 1e-30, axis=1)
    assert close.all(), (np.count_nonzero(~close), np.argwhere(~close)[:5].ravel())
    assert st.closest_rays == rst.closest_rays and st.shadow_rays == rst.shadow_rays
    with pytest.raises(native.WrError):
        ctx(path).path_radiance(rays[:4], max_depth=-1)


def test_film_on_device_pointer():
    torch = pytest.importorskip("torch")
    path = _scenes.torus(64, 64)
    c = ctx(path)
    dev = torch.zeros((64, 64, 3), dtype=torch.float32, device="cuda:0")
    c.render_bdpt(64, 64, iterations=1, seed=9, film_ptr=dev.data_ptr())
    torch.cuda.synchronize()
    host, _ = c.render_bdpt(64, 64, iterations=1, seed=9)
    assert np.allclose(dev.cpu().numpy(), host, rtol=1e-5, atol=1e-7)


def test_device_film_is_ordered_after_pending_default_stream_work():
    """A device film zeroed by torch on the default stream right before the
    call (no synchronize) is zeroed before the render adds into it: the
    library's non-blocking streams wait for the legacy null stream."""
    torch = pytest.importorskip("torch")
    path = _scenes.torus(64, 64)
    c = ctx(path)
    host, _ = c.render_bdpt(64, 64, iterations=1, seed=9)
    a = torch.randn((4096, 4096), device="cuda:0")
    dev = torch.full((64, 64, 3), 1e6, dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    for _ in range(8):  # several ms of default-stream work ahead of the zeroing
        a = a @ a
        a = a / a.abs().max()
    dev.zero_()
    c.render_bdpt(64, 64, iterations=1, seed=9, film_ptr=dev.data_ptr())
    torch.cuda.synchronize()
    assert np.allclose(dev.cpu().numpy(), host, rtol=1e-5, atol=1e-7)


def test_pt_sample_range_is_validated():
    c = ctx(_scenes.cbox(16, 12))
    for kw in ({"sample_begin": -1, "sample_count": 1}, {"sample_begin": 0, "sample_count": -2},
               {"sample_begin": 3, "sample_count": 2}, {"sample_begin": 5, "sample_count": 0}):
        with pytest.raises(native.WrError) as e:
            c.render_path(16, 12, spp=4, **kw)
        assert e.value.code == native.WR_E_ARG, kw
    film, _ = c.render_path(16, 12, spp=4, sample_begin=4, sample_count=0)  # empty rest range
    assert not film.any()
    with pytest.raises(ValueError):  # host film of the wrong shape / dtype: refused before the call
        c.render_path(16, 12, spp=4, film=np.zeros((12, 16, 3), np.float64))


def _check_trace_vs_oracle(c, oracle_scene, rays9):
    """GPU closest hit (wr_trace_closest) == the oracle's Scene::intersect, bit for bit."""
    oi, of, _, _ = oracle_scene.trace(rays9)
    hits = c.trace_closest(native.rays_from_arrays(rays9[:, 0:3], normalize_f32(rays9[:, 3:6])))
    assert np.array_equal(hits["prim"], oi[:, 0])
    m = oi[:, 0] >= 0
    got = np.concatenate([hits["t"][:, None], hits["p"], hits["n"]], axis=1).astype(np.float32)
    assert np.array_equal(got[m], of[m])
    assert np.array_equal(hits["inside"][m], oi[m, 1]) and np.array_equal(hits["mat_id"][m], oi[m, 2])
    return int(m.sum())


def test_trace_wide_stack_variant_bit_exact(monkeypatch):
    """The 32-bit-stack traversal (trees > 65536 nodes) forced on the golden corpus."""
    monkeypatch.setenv("WR_TRACE_WIDE", "1")
    path = _scenes.torus(64, 64)
    s = native.Scene(path)
    c = native.Context(s, 0, trace=native.TRACE_REFERENCE)
    rays = np.fromfile(os.path.join(GOLD, f"rays_torus64.f32"), np.float32).reshape(-1, 9)
    assert _check_trace_vs_oracle(c, _oracle.Scene(path), rays) > 500


def test_trace_1m_triangle_scene_matches_oracle(tmp_path, monkeypatch):
    """C4 scene (1,005,486 prims, 292,937 nodes: the wide-stack variant, depth 18)."""
    from winmad_rt import scenes
    obj = str(tmp_path / "torus_1m.obj")
    scenes.synth_torus_obj(obj)
    path = scenes.write(str(tmp_path / "torus_1m.scene"), scenes.torus_scene(64, 64, torus_obj=obj))
    s = native.Scene(path)
    assert s.info()["kd_inner"] + s.info()["kd_leaves"] > 65536
    c = native.Context(s, 0, trace=native.TRACE_REFERENCE)
    rng = np.random.default_rng(42)
    n = 4096
    o = rng.uniform([-250, -150, -120], [280, 350, 90], size=(n, 3))
    d = rng.normal(size=(n, 3))
    rays = np.zeros((n, 9), np.float32)
    rays[:, 0:3], rays[:, 3:6] = o, d
    orc = _oracle.Scene(path)
    assert _check_trace_vs_oracle(c, orc, rays) > n // 4
    assert _check_trace_vs_oracle(native.Context(s, 0), orc, rays) > n // 4  # library default (BVH)
    monkeypatch.setenv("WR_TRACE_DENSE", "1")  # wide stack + TRACE_DENSE
    assert _check_trace_vs_oracle(native.Context(s, 0, trace=native.TRACE_REFERENCE), orc, rays) > n // 4


def test_trace_large_batch_matches_oracle_and_small_batches():
    """4M rays in one wr_trace_closest call (grid-stride refill, queue
    reservations across many waves): a random sample of 4,096 equals the
    oracle bit for bit and the same rays traced as a small batch."""
    path = _scenes.torus(64, 64)
    c = ctx(path)
    rng = np.random.default_rng(5)
    n = 1 << 22
    o = rng.uniform([-250, -150, -120], [280, 350, 90], size=(n, 3)).astype(np.float32)
    draw = rng.normal(size=(n, 3)).astype(np.float32)
    d = normalize_f32(draw)  # as the Ray constructor the oracle runs
    big = c.trace_closest(native.rays_from_arrays(o, d))
    idx = np.sort(rng.choice(n, 4096, replace=False))
    rays = np.zeros((idx.size, 9), np.float32)
    rays[:, 0:3], rays[:, 3:6] = o[idx], draw[idx]
    oi, of, _, _ = _oracle.Scene(path).trace(rays)
    assert np.array_equal(big["prim"][idx], oi[:, 0])
    m = oi[:, 0] >= 0
    assert m.sum() > 500
    got = np.concatenate([big["t"][idx][:, None], big["p"][idx], big["n"][idx]], axis=1).astype(np.float32)
    assert np.array_equal(got[m], of[m])
    small = c.trace_closest(native.rays_from_arrays(o[idx], d[idx]))
    for k in ("prim", "t", "p", "n", "inside", "mat_id"):
        assert np.array_equal(small[k], big[k][idx]), k


@pytest.mark.parametrize("pipes", [1, 3, 8])
def test_pipeline_count_does_not_change_the_render(pipes, monkeypatch):
    """Iterations / samples dealt to 1..16 concurrent streams: same rays, same film
    up to the order of float atomics.  (WR_PIECE_MIN: shares of this small
    render go to every pipeline.)"""
    monkeypatch.setenv("WR_PIECE_MIN", "1024")
    path = _scenes.torus(96, 64)
    s = native.Scene(path)
    c = native.Context(s, 0)
    c.set_pipelines(2)
    ref, rs = c.render_bdpt(96, 64, iterations=5, seed=21)
    c.set_pipelines(pipes)
    got, gs = c.render_bdpt(96, 64, iterations=5, seed=21)
    assert rs.pipelines == 2 and gs.pipelines == pipes, (rs.pipelines, gs.pipelines)
    assert gs.closest_rays == rs.closest_rays and gs.shadow_rays == rs.shadow_rays
    assert np.allclose(got, ref, rtol=1e-4, atol=1e-6)
    cb = native.Context(native.Scene(_scenes.cbox(64, 48)), 0)
    cb.set_pipelines(1)
    pref, _ = cb.render_path(64, 48, spp=9, seed=4)
    cb.set_pipelines(pipes)
    pgot, _ = cb.render_path(64, 48, spp=9, seed=4)
    assert np.allclose(pgot, pref, rtol=1e-4, atol=1e-6)
    with pytest.raises(native.WrError):
        c.set_pipelines(0)


@pytest.mark.parametrize("W,H", [(256, 256), (100, 60)])
def test_bdpt_pieces_render_like_whole_iterations(W, H, monkeypatch):
    """Iterations cut into path-range pieces over 8 pipelines (plan_pieces:
    light path i and camera path i stay together, lightPathNum stays W*H):
    the same rays as whole iterations on one pipeline, the same film up to the
    order of float atomics, and the oracle's film.  100x60 is not a multiple of
    the 8x8 camera tiles (64-path units instead of 8-row bands)."""
    path = _scenes.torus(W, H)
    s = native.Scene(path)
    monkeypatch.setenv("WR_PIECE_MIN", "1024")
    monkeypatch.setenv("WR_PIECE_CAP", "4096")
    cut = native.Context(s, 0)
    cut.set_pipelines(8)
    got, gs = cut.render_bdpt(W, H, iterations=3, seed=21)
    one, os_ = cut.render_bdpt(W, H, iterations=1, seed=21, iter_begin=2)  # one iteration over 8 pipelines
    cut.close()
    monkeypatch.setenv("WR_PIECE_MIN", str(1 << 30))
    monkeypatch.setenv("WR_PIECE_CAP", str(1 << 21))
    whole = native.Context(s, 0)
    whole.set_pipelines(1)
    ref, rs = whole.render_bdpt(W, H, iterations=3, seed=21)
    ref1, rs1 = whole.render_bdpt(W, H, iterations=1, seed=21, iter_begin=2)
    whole.close()
    assert gs.closest_rays == rs.closest_rays and gs.shadow_rays == rs.shadow_rays
    assert os_.closest_rays == rs1.closest_rays and os_.shadow_rays == rs1.shadow_rays
    assert np.allclose(got, ref, rtol=1e-4, atol=1e-6)
    assert np.allclose(one, ref1, rtol=1e-4, atol=1e-6)
    orc, ost = _oracle.Scene(path).bdpt(W, H, 3, 21, mode=1)
    assert_film_parity(got, orc, case=f"bdpt_torus{W}x{H}_i3_s21")
    assert_ray_counts(gs, ost)


@pytest.mark.parametrize("name,maker,W,H", [("torus", lambda: _scenes.torus(96, 64), 96, 64),
                                             ("cbox", lambda: _scenes.cbox(64, 48, "bdpt"), 64, 48),
                                             ("spheres", lambda: _scenes.spheres(64, 64), 64, 64)])
@pytest.mark.parametrize("ctl", [3, 0])
def test_bdpt_overlapped_passes_equal_the_sequential_schedule(name, maker, W, H, ctl, monkeypatch):
    """The overlapped schedule (light and camera passes bounce by bounce in
    one launch; each (light vertex, camera vertex) pair connected by the
    vertex made second, wr_bdpt.h) against the reference's order (the whole
    light pass, then the camera pass; WR_BDPT_OVERLAP=0): the same rays, the
    same film up to the order of float atomics, and the oracle's film --
    controlLength 3 and every path length (connections of all lengths, the
    Cornell box and spheres where they carry 12-15 % of the image)."""
    path = maker()
    s = native.Scene(path)
    films = {}
    for ov in ("1", "0"):
        monkeypatch.setenv("WR_BDPT_OVERLAP", ov)
        c = native.Context(s, 0)
        films[ov] = c.render_bdpt(W, H, iterations=3, seed=77, control_length=ctl)
        c.close()
    (fa, sa), (fb, sb) = films["1"], films["0"]
    assert sa.closest_rays == sb.closest_rays and sa.shadow_rays == sb.shadow_rays
    assert np.allclose(fa, fb, rtol=1e-4, atol=1e-6)
    orc, ost = _oracle.Scene(path).bdpt(W, H, 3, 77, mode=1, control_length=ctl)
    # with every path length counted, a split path moves more pixels (the
    # gates of test_cbox_bdpt_film_matches_oracle); the rest keep the 2e-6 gate
    assert_film_parity(fa, orc, case=f"bdpt_{name}{W}x{H}_i3_s77_ctl{ctl}")
    assert_ray_counts(sa, ost)


@pytest.mark.parametrize("W,H,cap,pipes", [(100, 60, 3000, 1), (100, 60, 1000, 2), (99, 61, 2049, 1)])
def test_bdpt_pieces_never_exceed_the_buffer_capacity(W, H, cap, pipes, monkeypatch):
    """A film whose sides are not multiples of 8 (64-path units) with a
    WR_PIECE_CAP that is not a multiple of 64: the iteration's last piece ends
    at the iteration's end, not on a unit, and must still fit the buffer set
    (cut_pieces counts whole units per piece).  Same rays and film as whole
    iterations on one pipeline, and the oracle's film."""
    path = _scenes.torus(W, H)
    s = native.Scene(path)
    monkeypatch.setenv("WR_PIECE_MIN", "64")
    monkeypatch.setenv("WR_PIECE_CAP", str(cap))
    cut = native.Context(s, 0)
    cut.set_pipelines(pipes)
    got, gs = cut.render_bdpt(W, H, iterations=2, seed=33)
    cut.close()
    monkeypatch.setenv("WR_PIECE_MIN", str(1 << 30))
    monkeypatch.setenv("WR_PIECE_CAP", str(1 << 21))
    whole = native.Context(s, 0)
    whole.set_pipelines(1)
    ref, rs = whole.render_bdpt(W, H, iterations=2, seed=33)
    whole.close()
    assert gs.closest_rays == rs.closest_rays and gs.shadow_rays == rs.shadow_rays
    assert np.allclose(got, ref, rtol=1e-4, atol=1e-6)
    orc, ost = _oracle.Scene(path).bdpt(W, H, 2, 33, mode=1)
    assert_film_parity(got, orc, case=f"bdpt_torus{W}x{H}_i2_s33")
    assert_ray_counts(gs, ost)


@pytest.mark.parametrize("mode,W,H", [("-bpt", 64, 64), ("-vcm", 64, 64), ("-p", 64, 48)])
def test_cli_renders_like_the_reference_main(mode, W, H, tmp_path):
    """wr_tot (the C++ mirror of main.cpp's -bpt / -p branches) end to end on the GPU."""
    import subprocess
    scene = _scenes.torus(W, H) if mode in ("-bpt", "-vcm") else _scenes.cbox(W, H)
    para = tmp_path / "p.para"  # parameters.para: depth, spp, light / hemisphere samples, W, H, phong, lights
    para.write_text(f"#\n7\n#\n4\n8\n4\n{W}\n{H}\n5\n400\n")
    out = tmp_path / "o.ppm"
    r = subprocess.run([os.path.join(native.PKG_DIR, "wr_tot"), scene, str(out), mode, "--params", str(para),
                        "--iterations", "2"], capture_output=True, text=True, cwd=tmp_path, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Mrays/s" in r.stdout
    data = out.read_bytes()
    header = f"P6\n{W} {H}\n255\n".encode()
    assert data.startswith(header) and len(data) == len(header) + W * H * 3
    assert max(data[len(header):]) > 0
    assert (tmp_path / "time.txt").exists()


def test_spheres_bdpt_and_pt_match_oracle_counter_rng():
    """The SPH traversal variant, Sphere::hit and the glass / mirror BSDF branches."""
    path = _scenes.spheres(64, 64)
    film, st = ctx(path).render_bdpt(64, 64, iterations=4, seed=5489)
    ref, rst = _oracle.Scene(path).bdpt(64, 64, 4, 5489, mode=1)
    assert_film_parity(film, ref, case="bdpt_spheres64x64_i4_s5489")
    assert_ray_counts(st, rst)
    film, st = ctx(path).render_path(64, 64, spp=16, max_depth=7, seed=5489)
    ref, rst = _oracle.Scene(path).pt(64, 64, 16, 7, 5489, mode=1)
    assert_film_parity(film * np.float32(1.0 / 16), ref, case="pt_spheres64x64_spp16_s5489")
    assert_ray_counts(st, rst)


def test_render_argument_and_scene_errors(tmp_path):
    """Failures are WR_E_* codes with a message, never a crash (the reference
    would index an empty light list or overrun its buffers)."""
    from winmad_rt import scenes
    text = scenes.torus_scene(16, 16)
    nolight = "\n".join(l for l in text.splitlines() if "area_light" not in l and "torus_light" not in l
                        and "intensity" not in l)
    s = native.Scene(scenes.write(str(tmp_path / "nolight.scene"), nolight))
    c = native.Context(s, 0)
    with pytest.raises(native.WrError) as e:
        c.render_bdpt(16, 16, iterations=1)
    assert e.value.code == native.WR_E_SCENE
    with pytest.raises(native.WrError) as e:
        c.render_path(16, 16, spp=1)
    assert e.value.code == native.WR_E_SCENE
    c2 = ctx(_scenes.torus(16, 16))
    for kw in ({"max_path_length": 11}, {"iterations": -1}):
        with pytest.raises(native.WrError) as e:
            c2.render_bdpt(16, 16, **kw)
        assert e.value.code == native.WR_E_ARG
    with pytest.raises(native.WrError):
        c2.render_bdpt(0, 16)
    with pytest.raises(native.WrError):
        c2.render_path(16, 16, spp=4, max_depth=62)


@pytest.mark.parametrize("W,H", [(1, 1), (7, 5), (3, 130)])
def test_bdpt_tiny_and_ragged_films_match_oracle(W, H):
    """Films smaller than a wave / not a multiple of the 8x8 camera tiles."""
    path = _scenes.torus(W, H)
    film, st = ctx(path).render_bdpt(W, H, iterations=3, seed=17)
    ref, rst = _oracle.Scene(path).bdpt(W, H, 3, 17, mode=1)
    assert_ray_counts(st, rst)
    assert_film_parity(film, ref, case=f"bdpt_torus{W}x{H}_i3_s17")


def test_zero_iterations_and_depth_zero():
    c = ctx(_scenes.torus(16, 16))
    film, st = c.render_bdpt(16, 16, iterations=0)
    assert st.closest_rays == 0 and not film.any()
    path = _scenes.cbox(16, 12)
    film, st = ctx(path).render_path(16, 12, spp=4, max_depth=0, seed=2)
    ref, rst = _oracle.Scene(path).pt(16, 12, 4, 0, 2, mode=1)
    assert st.closest_rays == rst.closest_rays
    assert_film_parity(film * np.float32(1.0 / 4), ref, case="pt_cbox16x12_spp4_d0_s2")


@pytest.mark.parametrize("spp", [8, 12])
def test_pt_non_square_spp_stratification_matches_oracle(spp):
    """len = floor(sqrt(spp)) strata; samples past len^2 overshoot the pixel
    exactly as SurfaceIntegrator::render does (surfaceIntegrator.cpp:26-32,
    sampleRectangleStratified sampler.cpp:28-42) -- the C3 config's 512 spp."""
    path = _scenes.cbox(40, 30)
    film, st = ctx(path).render_path(40, 30, spp=spp, max_depth=7, seed=31)
    ref, rst = _oracle.Scene(path).pt(40, 30, spp, 7, 31, mode=1)
    assert_film_parity(film * np.float32(1.0 / spp), ref, case=f"pt_cbox40x30_spp{spp}_s31")
    assert_ray_counts(st, rst)


def test_cbox_bdpt_film_matches_oracle():
    """BDPT on the Cornell box (unit-scale geometry: vertex connections carry
    12 % of this film, where on torus.scene they add nothing -- DESIGN.md 8)."""
    path = _scenes.cbox(64, 48, "bdpt")
    for ctl in (3, 0):
        film, st = ctx(path).render_bdpt(64, 48, iterations=3, seed=5489, control_length=ctl)
        ref, rst = _oracle.Scene(path).bdpt(64, 48, 3, 5489, mode=1, control_length=ctl)
        # every path length counts with control_length 0, so a split path (tests/_parity.py)
        # moves more pixels: 113 of 3,072 measured; the other pixels keep the 2e-6 gate
        assert_film_parity(film, ref, case=f"bdpt_cbox64x48_i3_s5489_ctl{ctl}")
        assert_ray_counts(st, rst)


def test_bdpt_1m_scene_film_matches_oracle():
    """C4's scene (the 1M-triangle torus: deep KD tree, wide-stack traversal),
    BDPT at 384x216 (a fifth of the C4 frame per axis), one iteration, against
    the oracle's film: the same gates as every BDPT film."""
    from test_gpu_bvh import big_torus
    W, H = 384, 216
    path = big_torus(W, H)
    film, st = ctx(path).render_bdpt(W, H, iterations=1, seed=5489)
    ref, rst = _oracle.Scene(path).bdpt(W, H, 1, 5489, mode=1)
    assert_film_parity(film, ref, case="bdpt_torus1m384x216_i1_s5489")
    assert_ray_counts(st, rst)


def test_pt_c3_film_480x270_matches_oracle():
    """C3 (Cornell box + dragon, PT, MAX_TRACING_DEPTH 7) at 480x270 with 4
    stratified samples against the oracle's film."""
    W, H = 480, 270
    path = _scenes.cbox(W, H)
    film, st = ctx(path).render_path(W, H, spp=4, max_depth=7, seed=5489)
    ref, rst = _oracle.Scene(path).pt(W, H, 4, 7, 5489, mode=1)
    assert_film_parity(film * np.float32(1.0 / 4), ref, case="pt_cbox480x270_spp4_s5489")
    assert_ray_counts(st, rst)
