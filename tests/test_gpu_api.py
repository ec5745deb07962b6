"""API versions 5-6 on the GPU: several devices behind one context
(wr_create_multi), the one-process-per-GPU communicator (wr_comm_*), a scene
handed over as flat arrays (wr_scene_from_desc), and checkpoint / resume in
the reference-compatible CLI.  The box has one GPU, so the multi-device
context lists device 0 twice (its films are then summed by copies; distinct
devices use one RCCL reduce) and the communicator has one rank."""
import os
import subprocess

import numpy as np
import pytest

import _scenes
from test_gpu import ctx
from test_host_api import _xml_desc
from winmad_rt import native

pytestmark = pytest.mark.gpu


def _same(a, sa, b, sb):
    assert sa.closest_rays == sb.closest_rays and sa.shadow_rays == sb.shadow_rays
    assert np.allclose(a, b, rtol=1e-4, atol=1e-6)


@pytest.fixture(scope="module")
def multi():
    s = native.Scene(_scenes.torus(256, 256))
    m = native.Context(s, devices=[0, 0])
    yield s, m
    m.close()


def test_multi_device_bdpt_equals_one_device(multi):
    s, m = multi
    assert m.devices() == [0, 0]
    one = ctx(_scenes.torus(256, 256))
    for it, begin in ((3, 0), (1, 7)):  # 1 iteration: shared out by path ranges
        a, sa = m.render_bdpt(256, 256, iterations=it, seed=13, iter_begin=begin)
        b, sb = one.render_bdpt(256, 256, iterations=it, seed=13, iter_begin=begin)
        _same(a, sa, b, sb)


def test_multi_device_vcm_pt_and_traversal_equal_one_device(multi):
    s, m = multi
    one = ctx(_scenes.torus(256, 256))
    a, sa = m.render_vcm(256, 256, iterations=3, seed=5, radius_factor=0.02)
    b, sb = one.render_vcm(256, 256, iterations=3, seed=5, radius_factor=0.02)
    _same(a, sa, b, sb)
    assert sa.vm_merged == sb.vm_merged
    a, sa = m.render_path(256, 256, spp=5, seed=2)
    b, sb = one.render_path(256, 256, spp=5, seed=2)
    _same(a, sa, b, sb)
    rng = np.random.default_rng(1)
    n = 5000
    o = rng.uniform([-250, -150, -120], [280, 350, 90], size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r8 = native.rays_from_arrays(o, d)
    ha, hb = m.trace_closest(r8), one.trace_closest(r8)
    for k in ("prim", "t", "p", "n"):
        assert np.array_equal(ha[k], hb[k]), k


def test_multi_device_film_on_device_and_bvh_mode(multi):
    torch = pytest.importorskip("torch")
    s, m = multi
    m.set_trace_mode(native.TRACE_BVH)
    try:
        dev = torch.full((256, 256, 3), 0.5, dtype=torch.float32, device="cuda:0")
        _, st = m.render_bdpt(256, 256, iterations=2, seed=3, film_ptr=dev.data_ptr())
        torch.cuda.synchronize()
        host, hs = ctx(_scenes.torus(256, 256)).render_bdpt(256, 256, iterations=2, seed=3)
        assert st.closest_rays == hs.closest_rays
        assert np.allclose(dev.cpu().numpy() - 0.5, host, rtol=1e-4, atol=1e-5)  # accumulated into the film
    finally:
        m.set_trace_mode(native.TRACE_REFERENCE)


def test_multi_device_errors():
    s = native.Scene(_scenes.torus(16, 16))
    for bad in ([], [-1], [0, 999]):
        with pytest.raises((native.WrError, ValueError)):
            native.Context(s, devices=bad)


def test_comm_single_rank_reduce():
    """wr_comm_unique_id -> wr_comm_init -> wr_film_reduce over RCCL with one
    rank: the film comes back unchanged (a sum over one rank)."""
    torch = pytest.importorskip("torch")
    c = ctx(_scenes.torus(64, 64))
    uid = native.comm_unique_id()
    assert len(uid) == 128
    c.comm_init(uid, 1, 0)
    f = torch.rand((64, 64, 3), dtype=torch.float32, device="cuda:0")
    ref = f.clone()
    c.film_reduce(f.data_ptr(), f.numel(), 0)
    torch.cuda.synchronize()
    assert torch.equal(f, ref)
    with pytest.raises(native.WrError):
        c.film_reduce(f.data_ptr(), f.numel(), 1)  # no rank 1


def test_scene_from_desc_renders_like_the_file(tmp_path):
    path = _scenes.torus(128, 128)
    loaded = native.Scene(path)
    built = native.Scene.from_desc(**_xml_desc(path, loaded.dump(str(tmp_path / "d.txt"))))
    a, sa = native.Context(built, 0).render_bdpt(128, 128, iterations=2, seed=4)
    b, sb = ctx(path).render_bdpt(128, 128, iterations=2, seed=4)
    _same(a, sa, b, sb)


def _tot(args, cwd):
    r = subprocess.run([os.path.join(native.PKG_DIR, "wr_tot"), *map(str, args)], capture_output=True, text=True,
                       cwd=cwd, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


def _pfm(path):
    data = open(path, "rb").read()
    head = data.split(b"\n", 3)
    w, h = map(int, head[1].split())
    return np.frombuffer(head[3], np.float32).reshape(h, w, 3)


@pytest.mark.parametrize("mode", ["-bpt", "-p"])
def test_cli_checkpoint_resume_and_devices(mode, tmp_path):
    """wr_tot: an interrupted render (--stop-after) resumes from its checkpoint
    and ends with the film of an uninterrupted one; --devices 0,0 shares it out."""
    W, H = 96, 64
    scene = _scenes.torus(W, H) if mode == "-bpt" else _scenes.cbox(W, H)
    para = tmp_path / "p.para"
    para.write_text(f"#\n7\n#\n6\n8\n4\n{W}\n{H}\n5\n400\n")  # PT: 6 spp
    base = [scene, None, mode, "--params", para, "--iterations", 6, "--seed", 9]
    out = _tot([base[0], tmp_path / "full.pfm", *base[2:]], tmp_path)
    assert "trace bvh" in out
    ck = tmp_path / "ck.bin"
    stop = _tot([base[0], tmp_path / "part.pfm", *base[2:], "--checkpoint", ck, "--checkpoint-every", 2,
                 "--stop-after", 4], tmp_path)
    assert "stopped" in stop and ck.exists() and not (tmp_path / "part.pfm").exists()
    _, info = native.checkpoint_load(str(ck))
    assert info["done"] == 4 and info["total"] == 6
    assert info["fingerprint"] != 0
    # a checkpoint of another scene (same film size, kind, total, seed) is refused
    other = _scenes.cbox(W, H) if mode == "-bpt" else _scenes.torus(W, H, "pt")
    r = subprocess.run([os.path.join(native.PKG_DIR, "wr_tot"), *map(str, [other, tmp_path / "x.pfm", *base[2:],
                        "--checkpoint", ck])], capture_output=True, text=True, cwd=tmp_path, timeout=300)
    assert r.returncode != 0 and "another scene" in r.stderr, (r.returncode, r.stderr)
    # a film of the same render shape without a fingerprint (pre-v7, or saved with 0) is refused too
    film0, info0 = native.checkpoint_load(str(ck))
    nofp = tmp_path / "nofp.bin"
    native.checkpoint_save(str(nofp), film0, info0["kind"], info0["done"], info0["total"], info0["seed"],
                           fingerprint=0)
    r = subprocess.run([os.path.join(native.PKG_DIR, "wr_tot"), *map(str, [base[0], tmp_path / "y.pfm", *base[2:],
                        "--checkpoint", nofp])], capture_output=True, text=True, cwd=tmp_path, timeout=300)
    assert r.returncode != 0 and "no scene fingerprint" in r.stderr, (r.returncode, r.stderr)
    _tot([base[0], tmp_path / "resumed.pfm", *base[2:], "--checkpoint", ck, "--checkpoint-every", 2], tmp_path)
    assert np.allclose(_pfm(tmp_path / "resumed.pfm"), _pfm(tmp_path / "full.pfm"), rtol=1e-4, atol=1e-6)
    two = _tot([base[0], tmp_path / "two.pfm", *base[2:], "--devices", "0,0", "--trace", "reference"], tmp_path)
    assert "2 GPU(s)" in two and "trace reference" in two
    assert np.allclose(_pfm(tmp_path / "two.pfm"), _pfm(tmp_path / "full.pfm"), rtol=1e-4, atol=1e-6)


def test_reserve_then_render_equals_render(multi):
    """wr_reserve (API v6) allocates the work buffers ahead of the first render;
    the render after it is the same render (rays, film) and reports how many
    pipelines ran.  Bad arguments are refused."""
    s, m = multi
    a = native.Context(s, 0)
    a.set_trace_mode(native.TRACE_BVH)
    a.reserve(native.INTEGRATOR_BDPT, 256, 256)
    fa, sa = a.render_bdpt(256, 256, iterations=2, seed=9)
    b = native.Context(s, 0)
    b.set_trace_mode(native.TRACE_BVH)
    fb, sb = b.render_bdpt(256, 256, iterations=2, seed=9)
    _same(fa, sa, fb, sb)
    assert sa.pipelines >= 1 and sa.pipelines == sb.pipelines
    for kind, (W, H) in ((native.INTEGRATOR_VCM, (64, 64)), (native.INTEGRATOR_PATH, (64, 48))):
        a.reserve(kind, W, H)
    m.reserve(native.INTEGRATOR_BDPT, 128, 128)  # every device of a multi-device context
    for bad in ((3, 64, 64), (-1, 64, 64), (native.INTEGRATOR_BDPT, 0, 64)):
        with pytest.raises(native.WrError):
            a.reserve(*bad)
    a.close()
    b.close()


def test_reference_main_with_the_mirror_runs_at_the_bench_rate(tmp_path):
    """INTEGRATION.md section 1 built as a program (csrc/example_main.cpp: the
    reference's main() with the three integrator branches swapped for the
    winmad:: mirror, nothing else) at the headline configuration, 1920x1080
    torus.scene BDPT, 256 iterations, in a fresh process with the box's own
    environment: its wr_request_hw_queues(16) and the library's default
    traversal must give it bench.py's rate (verdict r3: within 10 %; asserted
    at 20 % against run-to-run noise, both rates printed)."""
    import json
    import re
    import sys
    W, H, it = 1920, 1080, 256
    (tmp_path / "src").mkdir()
    (tmp_path / "src" / "parameters.para").write_text(f"7\n1\n8\n4\n{W}\n{H}\n5\n400\n")
    scene = _scenes.torus(W, H)
    env = {k: v for k, v in os.environ.items() if k not in ("WR_HW_QUEUES",)}
    r = subprocess.run([os.path.join(native.PKG_DIR, "example_main"), scene, str(tmp_path / "o.ppm"), "-bpt", str(it)],
                       capture_output=True, text=True, cwd=tmp_path, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    m = re.search(r"= ([0-9.]+) Mrays/s, ([0-9]+) pipelines", r.stdout)
    assert m, r.stdout
    main_rate, pipes = float(m.group(1)), int(m.group(2))
    assert (tmp_path / "o.ppm").exists() and (tmp_path / "time.txt").exists()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    b = subprocess.run([sys.executable, "bench.py", "--steps", str(it), "--warmup", "3", "--no-cpu", "--no-count",
                        "--no-compare"], cwd=root, capture_output=True, text=True, timeout=300, env=env)
    assert b.returncode == 0, b.stderr[-2000:]
    bench_rate = json.loads([ln for ln in b.stdout.splitlines() if ln.startswith("{")][-1])["value"]
    bench_pipes = json.loads([ln for ln in b.stdout.splitlines() if ln.startswith("{")][-1])["config"]["pipelines"]
    print(f"example_main {main_rate:.1f} Mrays/s ({pipes} pipelines) vs bench.py {bench_rate:.1f} "
          f"({bench_pipes} pipelines): {main_rate / bench_rate:.3f}")
    # wr_request_hw_queues gave the program bench.py's queues: the same
    # pipeline count (16 on an idle GPU; fewer when this test process still
    # holds device memory, as both size their pipelines by the free memory)
    assert pipes == bench_pipes, (pipes, bench_pipes)
    assert main_rate >= 0.8 * bench_rate, (main_rate, bench_rate)
