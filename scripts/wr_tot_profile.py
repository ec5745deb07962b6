"""Throughput of the drop-in CLI (wr_tot, the twin of the reference's main.cpp:29-97)
at the headline configuration: torus.scene BDPT 1920x1080, beside bench.py.

    python3 scripts/wr_tot_profile.py [iterations ...] > profiles/r3/wr_tot_c2.jsonl

wr_tot raises GPU_MAX_HW_QUEUES itself and picks the verified-BVH traversal, so it
runs with the box's own environment (GPU_MAX_HW_QUEUES=4 there).  Its stats
seconds are the render call's wall time (context creation and image output
excluded, like bench.py's timed region but including the one-time pipeline
buffer allocation of a first render).
"""
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "winmad-s-raytracer-v1.0_amd")
sys.path.insert(0, PKG)
from winmad_rt import scenes  # noqa: E402


def main():
    its = [int(a) for a in sys.argv[1:]] or [20, 256]
    d = tempfile.mkdtemp(prefix="wr_tot_")
    W, H = 1920, 1080
    scene = scenes.write(os.path.join(d, "torus.scene"), scenes.torus_scene(W, H))
    para = os.path.join(d, "p.para")
    with open(para, "w") as f:  # parameters.para: depth, spp, light / hemisphere samples, W, H, phong, lights
        f.write(f"#\n7\n#\n4\n8\n4\n{W}\n{H}\n5\n400\n")
    exe = os.path.join(PKG, "wr_tot")
    for n in its:
        r = subprocess.run([exe, scene, os.path.join(d, "o.ppm"), "-bpt", "--params", para, "--iterations", str(n)],
                           capture_output=True, text=True, cwd=d, timeout=600)
        if r.returncode != 0:
            print(r.stdout, r.stderr, file=sys.stderr)
            sys.exit(r.returncode)
        m = re.search(r"rays (\d+) .* in ([0-9.]+) s: ([0-9.]+) Mrays/s \[trace (\w+)", r.stdout)
        with open(os.path.join(d, "time.txt")) as f:
            total = f.read().strip()
        print(json.dumps({"cmd": f"wr_tot torus.scene out.ppm -bpt --iterations {n} (1920x1080)",
                          "env_GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"),
                          "rays": int(m.group(1)), "render_s": float(m.group(2)),
                          "mrays_per_s": float(m.group(3)), "trace": m.group(4),
                          "time_txt": total, "stdout": r.stdout.strip()}), flush=True)


if __name__ == "__main__":
    main()
