"""Per-launch traversal latency vs ray count through the C ABI (diagnostic):
WR_TRACE_LOG=1 prints each launch's rays and microseconds on stderr."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "winmad-s-raytracer-v1.0_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import _scenes  # noqa: E402
from winmad_rt import native  # noqa: E402

s = native.Scene(_scenes.torus(256, 256))
rng = np.random.default_rng(1)
for mode in (native.TRACE_REFERENCE, native.TRACE_BVH):
    c = native.Context(s, 0)
    c.set_trace_mode(mode)
    for n in (64, 4096, 65536, 1 << 20):
        o = np.zeros((n, 3), np.float32) + np.array([0, 300, 0], np.float32)
        d = rng.normal(size=(n, 3)).astype(np.float32)
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        r8 = native.rays_from_arrays(o, d.astype(np.float32))
        c.trace_closest(r8)
        t0 = time.perf_counter()
        c.trace_closest(r8)
        print(f"mode {mode} n {n}: {1e3 * (time.perf_counter() - t0):.2f} ms wall", file=sys.stderr, flush=True)
