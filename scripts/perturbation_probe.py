#!/usr/bin/env python3
"""How much of a BDPT film the connectVertices strategy carries: the same
render with the product library and with the WR_TEST_CONN_W=1.001 variant
(scripts/build_variant.sh perturb_conn -DWR_TEST_CONN_W=1.001f), compared.
Each render runs in its own process (one library per process).

    python scripts/perturbation_probe.py [--out gpurun_out/perturbation_probe.jsonl]
"""
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANT = os.path.join(REPO, "winmad-s-raytracer-v1.0_amd", "variants", "perturb_conn.so")
CASES = [("torus256_ctl3", 256, 256, 4, 3), ("torus256_ctl0", 256, 256, 4, 0), ("torus1080p_ctl3", 1920, 1080, 1, 3)]


def child(out, W, H, it, ctl):
    sys.path.insert(0, os.path.join(REPO, "winmad-s-raytracer-v1.0_amd"))
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import numpy as np
    import _scenes
    from winmad_rt import native
    c = native.Context(native.Scene(_scenes.torus(W, H)), 0)
    film, _ = c.render_bdpt(W, H, iterations=it, seed=5489, control_length=ctl)
    np.save(out, film)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2], *map(int, sys.argv[3:7]))
        return
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    import numpy as np
    tmp = tempfile.mkdtemp()
    for name, W, H, it, ctl in CASES:
        films = []
        for lib in (None, VARIANT):
            f = os.path.join(tmp, f"{name}_{'v' if lib else 'p'}.npy")
            env = dict(os.environ)
            if lib:
                env["WR_LIB"] = lib
            subprocess.run([sys.executable, __file__, "--child", f, str(W), str(H), str(it), str(ctl)], check=True,
                           env=env, timeout=300)
            films.append(np.load(f).astype(np.float64))
        p, v = films
        d = v - p
        r = {"case": name, "bias": float(d.sum() / np.abs(p).sum()),
             "rel_rmse": float(np.sqrt((d ** 2).mean()) / np.sqrt((p ** 2).mean())),
             "pix_changed_gt_1e-6": float((np.abs(d) > 1e-6 * np.maximum(np.abs(p), 1e-12)).any(-1).mean()),
             "max_rel": float((np.abs(d) / np.maximum(np.abs(p), 1e-3 * np.abs(p).mean())).max())}
        line = json.dumps(r)
        print(line, flush=True)
        if out:
            with open(out, "a") as fo:
                fo.write(line + "\n")


if __name__ == "__main__":
    main()
