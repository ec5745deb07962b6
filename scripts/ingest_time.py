"""Time to first frame's inputs: scene load (wr_scene_load: .obj parse + KD
build) and context creation (wr_create: verified-BVH build + upload to HBM) for
the C2 torus and the C4 1M-triangle scene.  Prints one JSON line per scene.
Usage (GPU box): python3 scripts/ingest_time.py"""
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))
from winmad_rt import native, scenes  # noqa: E402

native.lib()  # the HIP runtime's own load is not part of either step
tmp = tempfile.mkdtemp()
obj = os.path.join(tmp, "torus_1m.obj")
scenes.synth_torus_obj(obj)
for name, kw in (("c2 torus", {}), ("c4 1M-triangle torus", {"torus_obj": obj})):
    path = scenes.write(os.path.join(tmp, name.split()[0] + ".scene"), scenes.torus_scene(1920, 1080, **kw))
    t0 = time.perf_counter()
    sc = native.Scene(path)
    t1 = time.perf_counter()
    ctx = native.Context(sc, 0)
    ctx.set_trace_mode(native.TRACE_BVH)
    t2 = time.perf_counter()
    print(json.dumps({"scene": name, "scene_load_s": round(t1 - t0, 3), "context_create_s": round(t2 - t1, 3),
                      "cpus": os.cpu_count()}))
    ctx.close()
    sc.close()
