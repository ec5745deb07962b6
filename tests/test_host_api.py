"""Host-side entry points added in API version 5 (CPU, no GPU needed):
wr_scene_from_desc (the reference's in-memory Scene as flat arrays, scene.h:35-42)
and the film checkpoint."""
import os
import re

import numpy as np
import pytest

import _scenes
from winmad_rt import native


def _xml_desc(scene_path, dump_text):
    """Flat arrays of a scene: primitives (exact floats) from the product's own
    dump, lights = the emitter primitives in order with the XML intensity,
    materials and camera from the .scene XML (converted like the loader's
    (float)atof)."""
    xml = open(scene_path).read()
    f = np.float32
    prim_type, prim_data, prim_mat = [], [], []
    for line in dump_text.splitlines():
        w = line.split()
        if w[0] == "tri":
            prim_type.append(0)
            prim_mat.append(int(w[1]))
            prim_data.append([float.fromhex(x) for x in w[2:11]])
        elif w[0] == "sph":
            prim_type.append(1)
            prim_mat.append(int(w[1]))
            prim_data.append([float.fromhex(x) for x in w[2:6]] + [0.0] * 5)
    le = [f(float(v)) for v in re.search(r'<intensity r="([^"]+)" g="([^"]+)" b="([^"]+)"', xml).groups()] \
        if "<intensity" in xml else None
    light_tri = [d for d, m in zip(prim_data, prim_mat) if m < 0]
    mats = []
    for m in re.finditer(r"<material>(.*?)</material>", xml, re.S):
        body = m.group(1)
        rgb = [[f(float(x)) for x in t] for t in re.findall(r'r="([^"]+)" g="([^"]+)" b="([^"]+)"', body)]
        e = f(float(re.search(r'phongExp="([^"]+)"', body).group(1)))
        n = f(float(re.search(r'refracIndex="([^"]+)"', body).group(1)))
        mats.append(rgb[0] + rgb[1] + rgb[2] + [e, n])
    cam = re.search(r"<camera>(.*?)</camera>", xml, re.S).group(1)
    vec = [[f(float(x)) for x in t] for t in re.findall(r'x="([^"]+)" y="([^"]+)" z="([^"]+)"', cam)]
    res = re.search(r'height="([^"]+)" width="([^"]+)"', cam).groups()
    fov = re.search(r'horizontalFOV="([^"]+)"', cam).group(1)
    return dict(prim_type=prim_type, prim_data=prim_data, prim_mat=prim_mat, light_tri=light_tri,
                light_le=[le] * len(light_tri), materials=mats, cam_pos=vec[0], cam_fwd=vec[1], cam_up=vec[2],
                cam_xres=f(float(res[0])), cam_yres=f(float(res[1])), cam_hfov=f(float(fov)))


@pytest.mark.parametrize("maker", [lambda: _scenes.torus(64, 64), lambda: _scenes.cbox(64, 48),
                                   lambda: _scenes.spheres(64, 64)])
def test_scene_from_desc_equals_the_loaded_scene(maker, tmp_path):
    """The same Scene handed over as arrays builds the identical scene: same
    primitives, lights, camera matrices and KD tree (dump text equal)."""
    path = maker()
    loaded = native.Scene(path)
    text = loaded.dump(str(tmp_path / "a.txt"))
    built = native.Scene.from_desc(**_xml_desc(path, text))
    assert built.dump(str(tmp_path / "b.txt")) == text
    a, b = built.info(), loaded.info()
    a.pop("missing_files"), b.pop("missing_files")  # files are the loader's business
    assert a == b


def test_scene_from_desc_rejects_malformed_arrays():
    tri = np.array([[0, 0, 0, 1, 0, 0, 0, 1, 0]], np.float32)
    base = dict(prim_type=[0], prim_data=tri, prim_mat=[0], light_tri=np.zeros((0, 9)), light_le=np.zeros((0, 3)),
                materials=np.zeros((1, 11)), cam_pos=[0, 0, 5], cam_fwd=[0, 0, -1], cam_up=[0, 1, 0], cam_xres=8,
                cam_yres=8, cam_hfov=45)
    native.Scene.from_desc(**base)
    for bad in (dict(prim_mat=[-1]),        # an emitter without its light
                dict(prim_type=[7]),        # unknown primitive type
                dict(prim_type=[1], prim_data=np.zeros((1, 9)))):  # sphere of radius 0
        with pytest.raises(native.WrError) as e:
            native.Scene.from_desc(**dict(base, **bad))
        assert e.value.code == native.WR_E_ARG
    with pytest.raises(ValueError):
        native.Scene.from_desc(**dict(base, prim_mat=[0, 0]))


def test_checkpoint_round_trip_and_corruption(tmp_path):
    rng = np.random.default_rng(3)
    film = rng.random((6, 10, 3), dtype=np.float32)
    p = str(tmp_path / "ck.bin")
    native.checkpoint_save(p, film, native.CKPT_BDPT, 3, 8, 5489, fingerprint=0x0123456789ABCDEF)
    got, info = native.checkpoint_load(p)
    assert np.array_equal(got, film)
    assert info == {"width": 10, "height": 6, "kind": native.CKPT_BDPT, "done": 3, "total": 8, "seed": 5489,
                    "fingerprint": 0x0123456789ABCDEF}
    assert not os.path.exists(p + ".tmp")
    raw = bytearray(open(p, "rb").read())
    raw[-5] ^= 0x40  # one flipped bit in the film
    open(p, "wb").write(bytes(raw))
    with pytest.raises(native.WrError) as e:
        native.checkpoint_load(p)
    assert e.value.code == native.WR_E_IO
    open(p, "wb").write(bytes(raw[:40]))  # truncated
    with pytest.raises(native.WrError):
        native.checkpoint_load(p)
    with pytest.raises(native.WrError):
        native.checkpoint_load(str(tmp_path / "missing.bin"))
    with pytest.raises(native.WrError) as e:  # done > total
        native.checkpoint_save(p, film, native.CKPT_BDPT, 9, 8, 1)
    assert e.value.code == native.WR_E_ARG


def test_scene_fingerprint_tells_scenes_apart(tmp_path):
    """wr_scene_fingerprint (what a checkpoint is bound to): equal for the same
    scene loaded twice, different for another scene, another camera or
    another material."""
    a = native.Scene(_scenes.torus(64, 64)).fingerprint()
    assert a == native.Scene(_scenes.torus(64, 64)).fingerprint() != 0
    assert a != native.Scene(_scenes.cbox(64, 64)).fingerprint()
    assert a != native.Scene(_scenes.torus(64, 48)).fingerprint()  # camera resolution
