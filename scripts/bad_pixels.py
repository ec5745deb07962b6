#!/usr/bin/env python3
"""Where GPU and oracle films disagree (relative > 1e-4): pixel, values, sign;
with and without the occlusion cutoff (WR_TRACE_NO_CUT) and in both traversal
modes, for the cases whose bias is one-sided."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402

import _oracle  # noqa: E402
import _scenes  # noqa: E402
from winmad_rt import native  # noqa: E402


def report(name, film, ref, extra):
    a, b = film.astype(np.float64), ref.astype(np.float64)
    d = a - b
    rel = np.abs(d) / np.maximum(np.abs(b), 1e-3 * np.abs(b).mean() + 1e-30)
    bad = np.argwhere((rel > 1e-4).any(-1))
    rows = [[int(i), int(j), [float(x) for x in a[i, j]], [float(x) for x in b[i, j]]] for i, j in bad[:40]]
    print(json.dumps({"case": name, **extra, "bias": float(d.sum() / b.sum()), "nbad": int(len(bad)), "bad": rows}),
          flush=True)


cases = [("cbox_bdpt", _scenes.cbox(64, 48, "bdpt"), "bdpt", dict(iterations=3, seed=5489)),
         ("torus_vcm_l3", _scenes.torus(64, 64), "vcm", dict(iterations=3, seed=3, radius_factor=1e-9,
                                                              min_path_length=3, max_path_length=3)),
         ("torus_bdpt256", _scenes.torus(256, 256), "bdpt", dict(iterations=2, seed=5))]
for name, path, kind, kw in cases:
    s = native.Scene(path)
    o = _oracle.Scene(path)
    W = int(path.split("_")[-2].split("x")[0]) if False else None
    info = s.info()
    H_, W_ = (48, 64) if "cbox" in name else ((64, 64) if "64" in path else (256, 256))
    if kind == "bdpt":
        ref, _ = o.bdpt(W_, H_, kw["iterations"], kw["seed"], mode=1)
    else:
        ref, _ = o.vcm(W_, H_, kw["iterations"], kw["seed"], mode=1, radius_factor=kw["radius_factor"],
                       min_len=kw["min_path_length"], max_len=kw["max_path_length"])
    for nocut in ("0", "1"):
        os.environ["WR_TRACE_NO_CUT"] = nocut
        for mode in (native.TRACE_REFERENCE, native.TRACE_BVH):
            c = native.Context(s, 0)
            c.set_trace_mode(mode)
            film, _ = (c.render_bdpt if kind == "bdpt" else c.render_vcm)(W_, H_, **kw)
            report(name, film, ref, {"no_cut": nocut, "trace": mode})
            c.close()
