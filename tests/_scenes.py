"""Scene files for tests: written into a temp dir with absolute asset paths."""
import os
import tempfile

from winmad_rt import scenes

_DIR = tempfile.mkdtemp(prefix="wr_tests_")


def path(name, text):
    p = os.path.join(_DIR, name)
    if not os.path.exists(p):
        scenes.write(p, text)
    return p


def torus(W, H, mode="bdpt"):
    return path(f"torus_{W}x{H}_{mode}.scene", scenes.torus_scene(W, H, mode))


def cbox(W, H, mode="pt"):
    return path(f"cbox_{W}x{H}_{mode}.scene", scenes.cbox_scene(W, H, mode))


def spheres(W, H, mode="bdpt"):
    return path(f"spheres_{W}x{H}_{mode}.scene", scenes.spheres_scene(W, H, mode))


def tent(W, H, mode="bdpt"):
    return path(f"tent_{W}x{H}_{mode}.scene", scenes.tent_scene(W, H, mode))
