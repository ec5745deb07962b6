"""The device's cosf / sinf / powf (winmad-s-raytracer-v1.0_amd/csrc/wr_libm.h)
return glibc's float bit for bit (verdict r5, next 1): the reference takes
every sampled direction and Phong lobe through libm (sampler.cpp:97-136,
bsdf.cpp:99), and one ulp of a direction can send a path elsewhere.

CPU test: tests/native/libm_check.c runs the header's functions (the code the
GPU kernels inline, compiled for the host) beside this machine's glibc --
every cos / sin input the samplers can produce (2*PI*k/2^24, all k), a stride
of all floats in [-256, 256], powf of a stride of the float cosines in (0, 1]
and of every sampler value for the scenes' Phong exponents, and random pairs.
scripts/libm_check_full.sh runs the same checks on every input
(profiles/r6/libm_check.json: 0 differences in 5.5e9 comparisons).
"""
import json
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("libm") / "libm_check")
    subprocess.run(["gcc", "-O2", "-std=c99", "-ffp-contract=off", "-Wall", "-o", exe,
                    os.path.join(HERE, "native", "libm_check.c"), "-lm"], check=True)
    return exe


def run(exe, *args):
    out = subprocess.run([exe, *map(str, args)], check=True, capture_output=True, text=True, timeout=300).stdout
    return [json.loads(l) for l in out.splitlines() if l.strip()]


def test_cos_sin_of_every_sampler_input(checker):
    rows = run(checker, "sampler")
    assert {r["check"] for r in rows} == {"cos_sampler", "sin_sampler"}
    for r in rows:
        assert r["n"] == 1 << 24 and r["diff"] == 0, r


def test_cos_sin_over_the_float_range(checker):
    # every quadrant, the small-|x| paths (|x| < 2^-12, < PI/4), the fast
    # reduction (< 120) and the large one (>= 120)
    for lo, hi, step in ((0.0, 256.0, 97), (0.0, 1e-3, 1009), (256.0, 3.4e38, 3001)):
        for r in run(checker, "range", lo, hi, step):
            assert r["n"] > 100000 and r["diff"] == 0, (lo, hi, r)


@pytest.mark.parametrize("exponent", [0, 1, 20, 90, 400])
def test_powf_for_the_scene_phong_exponents(checker, exponent):
    # powf(cos, phongExp) (bsdf.cpp:99, sampler.cpp:135) and
    # powf(u, 1 / (phongExp + 1)) (sampler.cpp:119)
    for r in run(checker, "powexp", exponent, 61):
        assert r["n"] > 1000000 and r["diff"] == 0, r


def test_powf_random_pairs(checker):
    for r in run(checker, "powrand", 3000000, 7):
        assert r["diff"] == 0, r
