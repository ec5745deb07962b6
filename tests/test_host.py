"""Host side of the product (CPU, no GPU needed): the C-ABI library loads and
exports every symbol of include/winmad_rt.h; its .scene/.obj loader, camera and
KD builder (csrc/wr_scene.cpp) reproduce the reference's dump bit for bit;
error behaviour; the film writer."""
import hashlib
import json
import os
import re

import numpy as np
import pytest

import _scenes
from winmad_rt import native

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(REPO, "tests", "golden")
META = json.load(open(os.path.join(GOLD, "golden.json")))


def test_library_exports_every_declared_symbol():
    L = native.lib()
    hdr = open(os.path.join(REPO, "include", "winmad_rt.h")).read()
    declared = set(re.findall(r"\b(wr_[a-z_]+)\s*\(", hdr))
    assert declared == set(native.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name
    assert L.wr_api_version() == 8


@pytest.mark.parametrize("name,maker", [("torus64", lambda: _scenes.torus(64, 64)),
                                        ("torus256", lambda: _scenes.torus(256, 256)),
                                        ("cbox64x48", lambda: _scenes.cbox(64, 48)),
                                        ("spheres64", lambda: _scenes.spheres(64, 64))])
def test_product_loader_and_kdtree_match_reference(name, maker, tmp_path):
    """wr_scene_load == Scene::init of the reference (scene.cpp:259-489,
    KDtreeAccel.cpp:12-307): identical triangles, lights, camera matrices and tree."""
    s = native.Scene(maker())
    txt = s.dump(str(tmp_path / "p.txt"))
    assert hashlib.sha256(txt.encode()).hexdigest() == META[name]["scene_sha256"]
    info = s.info()
    m = META[name]
    assert info["nprims"] == m["nobjs"]
    assert info["kd_inner"] == m["inner"] and info["kd_leaves"] == m["leaves"]
    assert info["kd_refs"] == m["refs"] and info["kd_depth_max"] == m["depmax"]
    assert 1 <= info["kd_max_stack"] <= m["depmax"]


def test_host_buffers_are_validated_before_the_library_sees_them():
    """Host films are accumulated in place and rays / targets are read by
    hipMemcpy: a wrong shape, dtype or layout raises instead of reaching C."""
    f = np.zeros((4, 5, 3), np.float32)
    assert native._host_film(f, 4, 5) is f
    assert native._host_film(None, 4, 5).shape == (4, 5, 3)
    for bad in (np.zeros((4, 5, 3), np.float64), np.zeros((5, 4, 3), np.float32), np.zeros((4, 4, 3), np.float32),
                np.zeros((4, 10, 3), np.float32)[:, ::2], np.zeros(60, np.float32), [[0.0] * 3] * 20):
        with pytest.raises(ValueError):
            native._host_film(bad, 4, 5)
    ro = np.zeros((4, 5, 3), np.float32)
    ro.setflags(write=False)
    with pytest.raises(ValueError):
        native._host_film(ro, 4, 5)
    assert native._rays8(np.zeros((3, 8), np.float64)).dtype == np.float32
    for bad in (np.zeros((3, 7)), np.zeros(8), np.zeros((2, 3, 8))):
        with pytest.raises(ValueError):
            native._rays8(bad)
    with pytest.raises(ValueError):
        native.write_image(np.zeros((4, 5), np.float32), "x.ppm")


def test_missing_obj_is_skipped_like_the_reference():
    # torus.scene names torus_mirror.obj, absent in the reference's ObjFiles too
    info = native.Scene(_scenes.torus(64, 64)).info()
    assert info["missing_files"] == 1
    assert info["nlights"] == 2 and info["ntriangles"] == 13486


def test_missing_scene_is_an_io_error(tmp_path):
    with pytest.raises(native.WrError) as e:
        native.Scene(str(tmp_path / "nope.scene"))
    assert e.value.code == native.WR_E_IO


def test_obj_index_out_of_range_is_an_io_error(tmp_path):
    obj = tmp_path / "bad.obj"
    obj.write_text("v 0 0 0\nv 1 0 0\nf 1 2 7\n")
    sc = tmp_path / "bad.scene"
    sc.write_text(f'<scene><object><file_path path="{obj}"/><matid matid="1"/></object></scene>')
    with pytest.raises(native.WrError) as e:
        native.Scene(str(sc))
    assert e.value.code == native.WR_E_IO


def test_obj_polygon_fan_negative_indices_and_water(tmp_path):
    """tinyobj semantics: quads fan into (0,1,2),(0,2,3); negative indices are
    relative; a shape named "water" gets its winding flipped when n.y < EPS."""
    obj = tmp_path / "q.obj"
    obj.write_text("v 0 0 0\nv 1 0 0\nv 1 0 1\nv 0 0 1\nf -4 -3 -2 -1\no water\nf 1 2 3\n")
    sc = tmp_path / "q.scene"
    sc.write_text(f'<scene><object><file_path path="{obj}"/><matid matid="2"/></object></scene>')
    txt = native.Scene(str(sc)).dump(str(tmp_path / "d.txt"))
    tris = [l.split() for l in txt.splitlines() if l.startswith("tri ")]
    assert len(tris) == 3
    v = lambda t: [float.fromhex(x) for x in t[2:11]]
    assert v(tris[0]) == [0, 0, 0, 1, 0, 0, 1, 0, 1]
    assert v(tris[1]) == [0, 0, 0, 1, 0, 1, 0, 0, 1]
    # water: n = (p1-p0)x(p2-p0) = (0,-1,0) -> n.y < EPS -> p0 <-> p2
    assert v(tris[2]) == [1, 0, 1, 1, 0, 0, 0, 0, 0]


def test_create_without_gpu_fails_loudly():
    if native.device_count() > 0:
        pytest.skip("GPU present")
    s = native.Scene(_scenes.torus(64, 64))
    with pytest.raises(native.WrError) as e:
        native.Context(s)
    assert e.value.code == native.WR_E_NODEVICE


IMAGE_CASES = [("sq37", 37, 37, 3, 1), ("r23x41", 23, 41, 1, 0), ("bdpt_torus64_i4_s5489", 64, 64, 4, 1)]


def _png_rgb(raw, h, w):
    """Decode the writer's PNG (stored-deflate IDAT, filter 0 rows)."""
    import zlib
    assert raw[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat = 8, b""
    while pos < len(raw):
        n = int.from_bytes(raw[pos:pos + 4], "big")
        if raw[pos + 4:pos + 8] == b"IDAT":
            idat += raw[pos + 8:pos + 8 + n]
        pos += 12 + n
    rows = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 3 * w + 1)
    assert (rows[:, 0] == 0).all()
    return rows[:, 1:].reshape(h, w, 3)


@pytest.mark.parametrize("name,h,w,iters,tr", IMAGE_CASES)
def test_film_writer_bytes_equal_the_reference(name, h, w, iters, tr, tmp_path):
    """8-bit output, bit-exact against the reference's own ImageFilm::scale ->
    clamp -> gamma(2.2) -> Color3::R/G/B (film.cpp:11-30, 45-60; color.h:47-75)
    run by oracle/_ref/refdrv `image` on the same float film (after the BDPT
    transpose, bidirPathTracing.cpp:31-41, for the square cases): every byte of
    .ppm, .bmp and .png, NaN / inf / negative inputs and the exact float
    boundaries of the 8-bit levels included (tests/golden/make_golden.py)."""
    src = os.path.join(GOLD, f"image_in_{name}.f32" if not name.startswith("bdpt_") else name + ".f32")
    film = np.fromfile(src, np.float32).reshape(h, w, 3)
    want = np.fromfile(os.path.join(GOLD, f"image_{name}.rgb"), np.uint8).reshape(h, w, 3)
    scale = float(np.float32(1) / np.float32(iters))  # 1.f / iterations (bidirPathTracing.cpp:45)
    p = tmp_path / "f.ppm"
    native.write_ppm(film, str(p), scale=scale, gamma=2.2, transpose=bool(tr))
    raw = p.read_bytes()
    hdr = f"P6\n{w} {h}\n255\n".encode()
    assert raw.startswith(hdr)
    got = np.frombuffer(raw[len(hdr):], np.uint8).reshape(h, w, 3)
    assert np.array_equal(got, want), int((got != want).sum())
    for ext in (".ppm", ".bmp", ".png"):
        q = tmp_path / f"g{ext}"
        native.write_image(film, str(q), scale=scale, gamma=2.2, transpose=bool(tr))
        raw = q.read_bytes()
        if ext == ".ppm":
            img = np.frombuffer(raw[len(hdr):], np.uint8).reshape(h, w, 3)
        elif ext == ".bmp":  # bottom-up BGR rows padded to 4 bytes
            row = (3 * w + 3) & ~3
            img = np.frombuffer(raw[54:], np.uint8).reshape(h, row)[::-1, :3 * w].reshape(h, w, 3)[..., ::-1]
        else:
            img = _png_rgb(raw, h, w)
        assert np.array_equal(img, want), (ext, int((img != want).sum()))


def test_cli_mirrors_reference_main(tmp_path):
    import subprocess
    exe = os.path.join(native.PKG_DIR, "wr_tot")
    r = subprocess.run([exe, _scenes.torus(64, 64), str(tmp_path / "o.ppm"), "-xyz",
                        "--params", str(tmp_path / "none")], capture_output=True, text=True)
    assert r.returncode != 0  # missing parameter file
    para = tmp_path / "p.para"
    para.write_text("#a\n7\n#b\n1\n8\n4\n64\n64\n5\n400\n")
    r = subprocess.run([exe, _scenes.torus(64, 64), str(tmp_path / "o.ppm"), "-xyz", "--params", str(para)],
                       capture_output=True, text=True)
    assert "error!" in r.stdout  # unknown mode (main.cpp:88-91)


def _expected_8bit(film, scale, gamma):
    """ImageFilm::outputImage's pipeline in float32 (film.cpp:39-64, color.h:47-75)."""
    v = film.astype(np.float32) * np.float32(scale)
    v = np.minimum(np.float32(1), np.where(v < 0, np.float32(0), v))  # clampVal; NaN -> 1 below
    v = np.where(np.isnan(v), np.float32(1), v)
    v = np.power(v, np.float32(1) / np.float32(gamma))
    return (v.astype(np.float64) * 255.0).astype(np.uint8)


def test_image_writer_formats(tmp_path):
    """wr_film_write_image: the reference's 8-bit pipeline into PPM / BMP / PNG
    (decoded here independently) and linear PFM."""
    import struct
    import zlib
    rng = np.random.default_rng(3)
    H, W = 5, 7  # odd width: BMP row padding, PNG scanlines
    film = (rng.random((H, W, 3)) * 1.4 - 0.1).astype(np.float32)
    film[0, 0, 0] = np.nan
    exp = _expected_8bit(film, 0.9, 2.2)
    native.write_image(film, tmp_path / "a.ppm", scale=0.9)
    data = (tmp_path / "a.ppm").read_bytes()
    head = f"P6\n{W} {H}\n255\n".encode()
    assert data.startswith(head)
    got = np.frombuffer(data[len(head):], np.uint8).reshape(H, W, 3)
    # libm powf vs numpy float32 power may differ in the last bit before truncation
    assert np.abs(got.astype(int) - exp).max() <= 1 and (got == exp).mean() > 0.97
    assert got[0, 0, 0] == 255
    native.write_image(film, tmp_path / "a.bmp", scale=0.9)
    b = (tmp_path / "a.bmp").read_bytes()
    assert b[:2] == b"BM" and struct.unpack("<iiHH", b[18:30]) == (W, H, 1, 24)
    row = (3 * W + 3) & ~3
    bgr = np.array([np.frombuffer(b[54 + r * row: 54 + r * row + 3 * W], np.uint8).reshape(W, 3)
                    for r in range(H)])[::-1][..., ::-1]
    assert np.array_equal(bgr, got)
    native.write_image(film, tmp_path / "a.png", scale=0.9)
    p = (tmp_path / "a.png").read_bytes()
    assert p[:8] == b"\x89PNG\r\n\x1a\n"
    chunks, off = {}, 8
    while off < len(p):
        n, typ = struct.unpack(">I4s", p[off:off + 8])
        body = p[off + 8: off + 8 + n]
        assert struct.unpack(">I", p[off + 8 + n: off + 12 + n])[0] == zlib.crc32(typ + body)
        chunks.setdefault(typ, b"")
        chunks[typ] += body
        off += 12 + n
    assert struct.unpack(">IIBBBBB", chunks[b"IHDR"]) == (W, H, 8, 2, 0, 0, 0)
    raw = np.frombuffer(zlib.decompress(chunks[b"IDAT"]), np.uint8).reshape(H, 3 * W + 1)
    assert not raw[:, 0].any() and np.array_equal(raw[:, 1:].reshape(H, W, 3), got)
    native.write_image(film, tmp_path / "a.pfm", scale=0.5)
    f = (tmp_path / "a.pfm").read_bytes()
    head = f"PF\n{W} {H}\n-1.0\n".encode()
    assert f.startswith(head)
    lin = np.frombuffer(f[len(head):], "<f4").reshape(H, W, 3)[::-1]
    assert np.array_equal(lin, film * np.float32(0.5), equal_nan=True)
    native.write_image(film[:5, :5], tmp_path / "t.png", transpose=True)  # square transpose
    with pytest.raises(native.WrError):
        native.write_image(film, tmp_path / "a.jpg")
    with pytest.raises(native.WrError):
        native.write_image(film, tmp_path / "t.ppm", transpose=True)  # non-square


def test_occlusion_cutoff_margin_holds_in_float32():
    """occl_cut (wr_traverse.h): a shadow ray may stop once its best hit t is
    below cut = proj - 2 (EPS + 1e-6 M); then the hit point o + d t must differ
    from the target by more than EPS in some component (Scene::occluded's
    position test, vector.cpp:43-47), whatever t in [0, cut) the traversal
    ends with.  Checked in float32 (same operations, no FMA) at the extreme
    t just below cut, for targets on and off the ray and scene scales from
    1e-2 to 1e4."""
    rng = np.random.default_rng(12)
    f = np.float32
    EPS = f(1e-3)
    bad = 0
    for scale in (1e-2, 1.0, 30.0, 1e3, 1e4):
        n = 20000
        o = (rng.uniform(-1, 1, (n, 3)) * scale).astype(f)
        tgt = (rng.uniform(-1, 1, (n, 3)) * scale).astype(f)
        off = rng.random(n) < 0.5  # half: target off the ray direction a little
        v = (tgt - o).astype(f)
        l = np.sqrt((v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1] + v[:, 2] * v[:, 2]).astype(f)).astype(f)
        d = (v / l[:, None]).astype(f)
        jitter = (rng.normal(size=(n, 3)) * 0.01 * scale).astype(f)
        tgt = np.where(off[:, None], (tgt + jitter).astype(f), tgt)
        w = (tgt - o).astype(f)
        proj = ((w[:, 0] * d[:, 0] + w[:, 1] * d[:, 1]).astype(f) + (w[:, 2] * d[:, 2]).astype(f)).astype(f)
        m = np.max(np.abs(np.concatenate([o, tgt, proj[:, None]], 1)), axis=1).astype(f)
        cut = (proj - f(2) * (EPS + f(1e-6) * m)).astype(f)
        ok = cut > 0
        t = np.nextafter(cut, f(-np.inf)).astype(f)
        p = (o + (d * t[:, None]).astype(f)).astype(f)
        diff = (p - tgt).astype(f)
        equal = np.all((diff >= -EPS) & (diff <= EPS), axis=1)
        bad += int(np.sum(equal & ok))
    assert bad == 0
