import sys, os, tempfile
sys.path.insert(0, "winmad-s-raytracer-v1.0_amd")
import torch
from winmad_rt import native, scenes
W, H = 1920, 1080
tmp = tempfile.mkdtemp()
p = scenes.write(os.path.join(tmp, "t.scene"), scenes.torus_scene(W, H))
c = native.Context(native.Scene(p), 0)
film = torch.zeros((H, W, 3), device="cuda")
for pipes in (1, 4):
    c.set_pipelines(pipes)
    c.render_bdpt(W, H, iterations=2, seed=1, iter_begin=999, film_ptr=film.data_ptr())
    _, st = c.render_bdpt(W, H, iterations=12, seed=1, film_ptr=film.data_ptr(), time_kernels=1)
    names = ["trace", "shade", "resolve", "gen", "other"]
    print(pipes, "wall %.1f ms" % (st.seconds * 1e3), "trace_wall %.1f" % st.trace_wall_ms,
          {n: round(st.kernel_ms[i], 1) for i, n in enumerate(names)},
          {n: st.kernel_launches[i] for i, n in enumerate(names)})
