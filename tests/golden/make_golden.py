#!/usr/bin/env python3
"""Regenerate tests/golden/ from the reference itself.

Test infrastructure: runs oracle/_ref/refdrv -- the reference's own translation
units compiled from /root/reference by `make -C oracle ref` -- and stores its
outputs as fixtures.  Only data is written here (inputs and expected outputs);
no reference source text.  Needs /root/reference (this container only); the GPU
box uses the committed fixtures.

    python tests/golden/make_golden.py          (everything)
    python tests/golden/make_golden.py image    (the 8-bit image fixtures only)
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))
from winmad_rt import scenes  # noqa: E402

REFDRV = os.path.join(REPO, "oracle", "_ref", "refdrv")

# (scene, iterations, seed, radius factor or None = the reference's 0.003)
VCM_CASES = [("torus64", 1, 5489, None), ("torus64", 3, 3, 0.05), ("spheres64", 2, 11, 0.1),
             ("cboxb64x48", 3, 3, 0.05), ("tent64", 2, 3, 0.05), ("tent64", 4, 5, 0.05)]


def vcm_fixture(name, it, seed, rf):
    return f"vcm_{name}_i{it}_s{seed}" + ("" if rf is None else f"_r{rf}") + ".f32"


def refdrv(*args, cwd):
    env = dict(os.environ, REFDRV_CWD=cwd)
    return subprocess.run([REFDRV, *map(str, args)], check=True, capture_output=True,
                          text=True, env=env).stdout


def sha(text):
    return hashlib.sha256(text.encode()).hexdigest()


def ray_corpus(scene_dump, n, seed):
    """Half camera-like rays from the camera position through random raster
    points of the scene's own camera, half random rays inside the root box;
    occlusion targets are random points (half of them on the first hit of a
    pilot ray are not needed: occlusion is checked both ways by mixing near and
    far targets)."""
    rng = np.random.default_rng(seed)
    lines = scene_dump.splitlines()
    cam = [float.fromhex(t) for t in next(l for l in lines if l.startswith("camera")).split()[1:]]
    kd = [float.fromhex(t) for t in next(l for l in lines if l.startswith("kd ")).split()[2:]]
    lo, hi = np.array(kd[:3]), np.array(kd[3:6])
    pos = np.array(cam[:3])
    out = np.zeros((n, 9), np.float32)
    h = n // 2
    tgt = lo + (hi - lo) * rng.random((h, 3))
    out[:h, 0:3] = pos
    out[:h, 3:6] = tgt - pos
    out[:h, 6:9] = lo + (hi - lo) * rng.random((h, 3))
    o = lo + (hi - lo) * rng.random((n - h, 3))
    d = rng.normal(size=(n - h, 3))
    out[h:, 0:3] = o
    out[h:, 3:6] = d
    out[h:, 6:9] = o + d * rng.random((n - h, 1)) * np.linalg.norm(hi - lo)
    return out


# 8-bit output (film.cpp:39-64 + color.h:47-75): (name, height, width, ITERS, transpose)
IMAGE_CASES = [("sq37", 37, 37, 3, 1), ("r23x41", 23, 41, 1, 0), ("bdpt_torus64_i4_s5489", 64, 64, 4, 1)]


def image_film(name, h, w):
    """Input films of the image fixtures: random radiance over six decades,
    the exact float boundaries of the 8-bit levels (x with pow(x, 1/2.2) * 255
    at or next to an integer, and one ulp either side), zero, negatives,
    values above the clamp, NaN and infinities.  The BDPT case is the
    reference's own torus film."""
    if name.startswith("bdpt_"):
        return np.fromfile(os.path.join(HERE, name + ".f32"), np.float32).reshape(h, w, 3)
    rng = np.random.default_rng(2024 + h * w)
    f = (10.0 ** rng.uniform(-4, 2, (h, w, 3))).astype(np.float32)
    flat = f.reshape(-1)
    k = np.arange(256, dtype=np.float64)
    edge = ((k / 255.0) ** 2.2).astype(np.float32)
    specials = np.concatenate([edge, np.nextafter(edge, np.float32(0)), np.nextafter(edge, np.float32(2)),
                               np.array([0, -0.0, -1, -1e-30, 1, 1.0000001, 3, 1e30, np.nan, np.inf, -np.inf],
                                        np.float32)])
    idx = rng.choice(flat.size, specials.size, replace=False)
    flat[idx] = specials * np.float32(1 if name != "sq37" else 3)  # ITERS = 3 scales them back
    return f


def image_fixtures(tmp):
    for name, h, w, iters, tr in IMAGE_CASES:
        film = image_film(name, h, w)
        src = os.path.join(HERE, f"image_in_{name}.f32")
        if not name.startswith("bdpt_"):
            film.astype(np.float32).tofile(src)
        else:
            src = os.path.join(HERE, name + ".f32")
        refdrv("image", h, w, iters, tr, src, os.path.join(HERE, f"image_{name}.rgb"), cwd=tmp)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "image":  # the image fixtures alone
        image_fixtures(tempfile.mkdtemp(prefix="wr_golden_"))
        return
    if not os.path.exists(REFDRV):
        sys.exit("build the reference driver first: make -C oracle ref")
    tmp = tempfile.mkdtemp(prefix="wr_golden_")
    meta = {}
    # MT19937 streams (rng.cpp)
    for seed in (5489, 12345):
        txt = refdrv("mt", seed, 2000, cwd=tmp)
        with open(os.path.join(HERE, f"mt_{seed}.txt"), "w") as f:
            f.write(txt)
    cases = {
        "torus64": (scenes.torus_scene(64, 64), scenes.params_text(64, 64)),
        "torus256": (scenes.torus_scene(256, 256), scenes.params_text(256, 256)),
        "cbox64x48": (scenes.cbox_scene(64, 48), scenes.params_text(64, 48, 7, 16)),
        "spheres64": (scenes.spheres_scene(64, 64), scenes.params_text(64, 64, 7, 4)),
    }
    for name, (sc, pa) in cases.items():
        sp = scenes.write(os.path.join(tmp, name + ".scene"), sc)
        pp = scenes.write(os.path.join(tmp, name + ".para"), pa)
        dump = refdrv("scene", sp, pp, cwd=tmp)
        lines = dump.splitlines()
        meta[name] = {
            "scene_sha256": sha(dump),
            "nobjs": int(lines[0].split()[1]),
            "inner": sum(1 for l in lines if l.startswith("I ")),
            "leaves": sum(1 for l in lines if l.startswith("L ")),
            "refs": sum(int(l.split()[1]) for l in lines if l.startswith("L ")),
            "depmax": int(next(l for l in lines if l.startswith("kd ")).split()[1]),
        }
        if name == "torus256":
            continue
        corpus = ray_corpus(dump, 2048 if name == "torus64" else 1024, 99)
        if name == "spheres64":  # aim half of the random rays at the spheres
            c = np.array([[-0.5, 0.3, -0.82], [0.55, 0.6, -0.86], [0.05, -0.45, -1.0]], np.float32)
            k = np.arange(512, 1024, 2)
            corpus[k, 3:6] = c[k % 3] - corpus[k, 0:3]
        cp = os.path.join(HERE, f"rays_{name}.f32")
        corpus.tofile(cp)
        # second pass: every other hitting ray gets its own hit point as the
        # occlusion target, so both outcomes of the position-equality test
        # (scene.cpp:65) are covered
        for k, line in enumerate(refdrv("rays", sp, pp, cp, cwd=tmp).splitlines()):
            tok = line.split()
            if tok[0] != "-1" and k % 2 == 0:
                corpus[k, 6:9] = [float.fromhex(t) for t in tok[2:5]]
        corpus.tofile(cp)
        with open(os.path.join(HERE, f"rays_{name}.txt"), "w") as f:
            f.write(refdrv("rays", sp, pp, cp, cwd=tmp))
        with open(os.path.join(HERE, f"kat_{name}.txt"), "w") as f:
            f.write(refdrv("kat", sp, pp, 128, 777, cwd=tmp))
    # films (pre-transpose, accumulated), MT-serial
    for name, it, seed in (("torus64", 1, 5489), ("torus64", 4, 5489), ("torus64", 2, 7)):
        sp, pp = os.path.join(tmp, name + ".scene"), os.path.join(tmp, name + ".para")
        out = os.path.join(HERE, f"bdpt_{name}_i{it}_s{seed}.f32")
        refdrv("bdpt", sp, pp, it, seed, out, cwd=tmp)
    sp, pp = os.path.join(tmp, "torus256.scene"), os.path.join(tmp, "torus256.para")
    tmpf = os.path.join(tmp, "b256.f32")
    refdrv("bdpt", sp, pp, 4, 5489, tmpf, cwd=tmp)
    film = np.fromfile(tmpf, np.float32).reshape(256, 256, 3)
    meta["bdpt_torus256_i4_s5489"] = {
        "mean": film.mean(axis=(0, 1)).tolist(),
        "rms": float(np.sqrt((film.astype(np.float64) ** 2).mean())),
        "block32_mean": film.reshape(8, 32, 8, 32, 3).mean(axis=(1, 3)).tolist(),
        "sha256": hashlib.sha256(film.tobytes()).hexdigest(),
    }
    sp, pp = os.path.join(tmp, "cbox64x48.scene"), os.path.join(tmp, "cbox64x48.para")
    refdrv("pt", sp, pp, 5489, os.path.join(HERE, "pt_cbox64x48_spp16_s5489.f32"), cwd=tmp)
    # spheres: Sphere::hit and the specular (glass / mirror) BSDF branches
    sp, pp = os.path.join(tmp, "spheres64.scene"), os.path.join(tmp, "spheres64.para")
    refdrv("bdpt", sp, pp, 2, 5489, os.path.join(HERE, "bdpt_spheres64_i2_s5489.f32"), cwd=tmp)
    refdrv("pt", sp, pp, 5489, os.path.join(HERE, "pt_spheres64_spp4_s5489.f32"), cwd=tmp)
    # VCM (vertexcm.cpp + KDtree.h): the reference radius on torus, larger radii
    # (baseRadius set through refdrv's RADIUS_FACTOR) so 64^2 films merge a lot;
    # cbox in the BDPT orientation (raster x = film row) has emitter light vertices
    sp = scenes.write(os.path.join(tmp, "cboxb64x48.scene"), scenes.cbox_scene(64, 48, "bdpt"))
    pp = scenes.write(os.path.join(tmp, "cboxb64x48.para"), scenes.params_text(64, 48))
    # tent luminaire: light paths whose first vertex is another emitter (their
    # BSDF probabilities come from the previous light path's last BSDF)
    sp = scenes.write(os.path.join(tmp, "tent64.scene"), scenes.tent_scene(64, 64))
    pp = scenes.write(os.path.join(tmp, "tent64.para"), scenes.params_text(64, 64))
    for name, it, seed, rf in VCM_CASES:
        sp, pp = os.path.join(tmp, name + ".scene"), os.path.join(tmp, name + ".para")
        extra = [] if rf is None else [rf]
        refdrv("vcm", sp, pp, it, seed, os.path.join(HERE, vcm_fixture(name, it, seed, rf)), *extra, cwd=tmp)
    image_fixtures(tmp)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps({k: v for k, v in meta.items() if "block32_mean" not in v}, indent=1))


if __name__ == "__main__":
    main()
