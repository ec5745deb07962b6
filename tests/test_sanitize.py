"""Sanitizer builds of the host code (ASan on the host side; VERDICT
r3 item 9), CPU only.

tests/native/host_sanitize.cpp drives the product's host translation units --
the in-place .scene/.obj loader and the threaded KD build (wr_scene.cpp; the
reference's scene.cpp:259-489, tiny_obj_loader.cpp:461-661 semantics and
KDtreeAccel.cpp:12-307), the threaded verified-BVH build (wr_bvh.cpp), the image
writers (wr_image.cpp) and the checkpoint (wr_checkpoint.cpp) -- over the
reference scenes, a synthetic torus large enough for both builders to spawn
helper threads, and malformed inputs.  Two builds: AddressSanitizer +
UndefinedBehaviorSanitizer (every report fatal) and ThreadSanitizer.  The logs
of the runs are written to profiles/r4/sanitize_{asan,tsan}.log when
WR_SANITIZE_LOG=1 (scripts/sanitize_host.sh)."""
import os
import subprocess
import tempfile

import pytest

import _scenes
from winmad_rt import scenes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "winmad-s-raytracer-v1.0_amd", "csrc")
SRCS = ["wr_scene.cpp", "wr_bvh.cpp", "wr_image.cpp", "wr_checkpoint.cpp"]
FLAGS = {
    "asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-O1", "-g"],
    "tsan": ["-fsanitize=thread", "-fno-omit-frame-pointer", "-O1", "-g"],
}
ENV = {
    "asan": {"ASAN_OPTIONS": "halt_on_error=1:detect_leaks=1:exitcode=86:verify_asan_link_order=0",
             "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"},
    "tsan": {"TSAN_OPTIONS": "halt_on_error=1:exitcode=87:second_deadlock_stack=1"},
}
_bin = {}


def build(kind):
    if kind not in _bin:
        out = os.path.join(tempfile.mkdtemp(prefix=f"wr_{kind}_"), "host_sanitize")
        subprocess.run(["g++", "-std=c++17", "-ffp-contract=off", *FLAGS[kind], "-I", CSRC, "-I",
                        os.path.join(REPO, "include"), os.path.join(REPO, "tests", "native", "host_sanitize.cpp"),
                        *[os.path.join(CSRC, s) for s in SRCS], "-o", out, "-lpthread"], check=True)
        _bin[kind] = out
    return _bin[kind]


def threaded_torus():
    """90,000 triangles: above both builders' thresholds for helper threads
    (KD subtrees >= 4,096 refs a side, BVH subtrees >= 8,192 and the BVH's
    one-axis-per-thread top splits >= 65,536)."""
    p = os.path.join(_scenes._DIR, "torus_90k.obj")
    if not os.path.exists(p):
        scenes.synth_torus_obj(p, U=300, V=150)
    return _scenes.path("torus_90k.scene", scenes.torus_scene(64, 64, "bdpt", torus_obj=p))


def malformed(d):
    """Inputs the loader must survive: the bad .scene files must be refused,
    the odd .obj files loaded or refused without touching memory it does not
    own (tinyobj semantics: tiny_obj_loader.cpp:461-661)."""
    objs = {
        "range.obj": "v 0 0 0\nv 1 0 0\nf 1 2 7\n",
        "neg.obj": "v 0 0 0\nv 1 0 0\nv 0 1 0\nf -1 -2 -9\n",
        "zero.obj": "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n",
        "short.obj": "v 0 0\nv 1\nf 1 2 3\nf 1\n",
        "junk.obj": "v 1e99999 nan inf\nv -0 -0 -0\nv 1 2 3\nf 1 2 3 4 5 6 7 8 9 10\nvn 1\nvt\nf 3/2/1 2//1 1/1\n",
        "empty.obj": "",
        "binary.obj": "\x00\xff\x7f v f \x01\x02\n" * 64,
        "long.obj": "v " + "1" * 5000 + " 0 0\nv 0 1 0\nv 0 0 1\nf 1 2 3\n",
        "noeol.obj": "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3",
    }
    out = []
    for name, text in objs.items():
        p = os.path.join(d, name)
        with open(p, "w", encoding="latin-1") as f:
            f.write(text)
        sc = os.path.join(d, name + ".scene")
        with open(sc, "w") as f:
            f.write(f'<scene>{scenes._mat()}<object><file_path path="{p}"/><matid matid="0"/></object></scene>')
        out.append(sc)
    bad_scenes = {"truncated.scene": "<scene><object><file_path path=\"x.obj\"/", "notxml.scene": "\x00\x01garbage",
                  "empty.scene": ""}
    for name, text in bad_scenes.items():
        p = os.path.join(d, name)
        with open(p, "w", encoding="latin-1") as f:
            f.write(text)
        out.append("!" + p)
    out.append("!" + os.path.join(d, "does_not_exist.scene"))
    return out


def run(kind, args, timeout=600):
    env = dict(os.environ, **ENV[kind])
    r = subprocess.run([build(kind), *args], capture_output=True, text=True, timeout=timeout, env=env)
    log = os.environ.get("WR_SANITIZE_LOG")
    if log:
        os.makedirs(os.path.join(REPO, "profiles", "r4"), exist_ok=True)
        with open(os.path.join(REPO, "profiles", "r4", f"sanitize_{kind}.log"), "a") as f:
            f.write(f"$ host_sanitize[{kind}] {' '.join(os.path.basename(a) for a in args)}\n"
                    f"{r.stdout}{r.stderr}exit {r.returncode}\n\n")
    return r


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_code_is_clean_under_sanitizers(kind, tmp_path):
    scenes_ = [_scenes.torus(64, 64), _scenes.cbox(64, 48), _scenes.spheres(64, 64), threaded_torus()]
    if kind == "asan":
        scenes_ += malformed(str(tmp_path))
    r = run(kind, [str(tmp_path), *scenes_])
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "DONE" in r.stdout, out[-4000:]
    for bad in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "LeakSanitizer"):
        assert bad not in out, out[-4000:]
