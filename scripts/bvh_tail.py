"""Latency tail of the BVH mode's resolve / hard kernels (WR_TRACE_LOG=1 output
on stderr): one pipeline, a counting render of a few iterations.
Usage: WR_TRACE_LOG=1 WR_PIPES=1 python3 scripts/bvh_tail.py [c2|c4|vcm] [iterations]"""
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "winmad-s-raytracer-v1.0_amd"))
import torch  # noqa: E402
from winmad_rt import native, scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
W, H = 1920, 1080
tmp = tempfile.mkdtemp()
obj = None
if cfg == "c4":
    obj = os.path.join(tmp, "torus_1m.obj")
    scenes.synth_torus_obj(obj)
sc = native.Scene(scenes.write(os.path.join(tmp, "t.scene"), scenes.torus_scene(W, H, torus_obj=obj)))
ctx = native.Context(sc, 0)
ctx.set_trace_mode(native.TRACE_BVH)
film = torch.zeros((H, W, 3), device="cuda")
render = ctx.render_vcm if cfg == "vcm" else ctx.render_bdpt
_, st = render(W, H, iterations=K, seed=5489, film_ptr=film.data_ptr(), count_work=1)
print("rays", st.closest_rays + st.shadow_rays, "fallback", st.fallback_rays, file=sys.stderr)
