"""Scene-file writers for the configurations in BASELINE.json.

The reference reads `.scene` XML (`src/scene/scene.cpp:259-467`) whose object
paths are opened relative to the process CWD.  The shipped `torus.scene`
(`torus.scene:56-76`) carries Windows-absolute paths, so every run here writes a
local copy with the same camera, materials and objects but paths that point at
`assets/` (the .obj data files copied verbatim from the reference's
`ObjFiles/`).  Resolution follows the reference's convention: the XML
`height` attribute becomes `camera.xResolution` (`scene.cpp:292-295`).

Writers:
  torus_scene(W, H)     -- torus.scene (C1/C2), mirror object kept (file absent
                           in the reference => 0 triangles, as there)
  cbox_scene(W, H)      -- Cornell box + test_out_dragon.obj (C3)
  synth_torus_obj(path) -- the 1M-triangle torus of C4/C5
"""
import math
import os

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ASSETS = os.path.join(REPO, "assets")

_MAT = """\t<material>
\t\t<diffuse r="{d[0]}" g="{d[1]}" b="{d[2]}"/>
\t\t<glossy r="{g[0]}" g="{g[1]}" b="{g[2]}"/>
\t\t<specular r="{s[0]}" g="{s[1]}" b="{s[2]}"/>
\t\t<phongExp phongExp="{e}"/>
\t\t<refracIndex refracIndex="{n}"/>
\t</material>
"""


def _camera(pos, fwd, up, xres, yres, fov):
    return ("\t<camera>\n"
            f"\t\t<position x=\"{pos[0]}\" y=\"{pos[1]}\" z=\"{pos[2]}\"/>\n"
            f"\t\t<forward x=\"{fwd[0]}\" y=\"{fwd[1]}\" z=\"{fwd[2]}\"/>\n"
            f"\t\t<up x=\"{up[0]}\" y=\"{up[1]}\" z=\"{up[2]}\"/>\n"
            f"\t\t<resolution height=\"{xres}\" width=\"{yres}\"/>\n"
            f"\t\t<horizontalFOV horizontalFOV=\"{fov}\"/>\n"
            "\t</camera>\n")


def _mat(d=(0, 0, 0), g=(0, 0, 0), s=(0, 0, 0), e=0, n=-1):
    return _MAT.format(d=d, g=g, s=s, e=e, n=n)


def _obj(path, matid):
    return (f"\t<object>\n\t\t<file_path path=\"{path}\"/>\n"
            f"\t\t<matid matid=\"{matid}\"/>\n\t</object>\n")


def _area(path, le):
    return (f"\t<area_light>\n\t\t<file_path path=\"{path}\"/>\n"
            f"\t\t<intensity r=\"{le}\" g=\"{le}\" b=\"{le}\"/>\n\t</area_light>\n")


def torus_scene(width, height, mode="bdpt", torus_obj=None, assets=ASSETS):
    """torus.scene with local paths.  For BDPT the raster x axis runs over film
    rows (`bidirPathTracing.cpp:422-423`), so xResolution = HEIGHT; for PT the
    raster x axis runs over columns (`surfaceIntegrator.cpp:26-34`), so
    xResolution = WIDTH."""
    xres, yres = (height, width) if mode == "bdpt" else (width, height)
    a = lambda f: os.path.join(assets, f)
    out = "<scene>\n"
    out += _camera(("-603.8923", "1013.96", "1823.33"), ("0.11", "-0.373", "-0.921"),
                   ("-0.25", "0.885", "-0.389"), xres, yres, "34.6222")
    out += _mat()
    out += _mat(d=("0.933", "0.929", "0.424"))
    out += _mat(s=(1, 1, 1), n="1.5")
    out += _mat(d=("0.733", "0.733", "0.733"))
    out += _mat(s=(1, 1, 1))
    out += _obj(torus_obj or a("torus_torus.obj"), 1)
    out += _obj(a("torus_glass.obj"), 2)
    out += _obj(a("torus_floor.obj"), 3)
    out += _obj(a("torus_mirror.obj"), 4)  # absent in the reference too
    out += _area(a("torus_light.obj"), 70)
    out += "</scene>\n"
    return out


def cbox_scene(width, height, mode="pt", assets=ASSETS):
    """Cornell box + dragon: camera of the built-in scene
    (`scene.cpp:152-155`), luminaire intensity of `scene.cpp:288-292`."""
    xres, yres = (width, height) if mode == "pt" else (height, width)
    a = lambda f: os.path.join(assets, f)
    out = "<scene>\n"
    out += _camera(("-0.0439815", "-4.12529", "0.222539"),
                   ("0.00688625", "0.998505", "-0.0542161"),
                   ("3.73896e-4", "0.0542148", "0.998529"), xres, yres, "45")
    out += _mat()
    out += _mat(d=("0.803922", "0.803922", "0.803922"), e=1)
    out += _mat(d=("0.156863", "0.803922", "0.172549"), e=1)
    out += _mat(d=("0.803922", "0.152941", "0.152941"), e=1)
    out += _mat(d=("0.1", "0.1", "0.1"), g=("0.7", "0.7", "0.7"), e=90)
    for f in ("cbox_floor.obj", "cbox_back.obj", "cbox_ceiling.obj"):
        out += _obj(a(f), 1)
    out += _obj(a("cbox_greenwall.obj"), 2)
    out += _obj(a("cbox_redwall.obj"), 3)
    out += _obj(a("test_out_dragon.obj"), 4)
    out += _area(a("cbox_luminaire.obj"), "25.03329895614464")
    out += "</scene>\n"
    return out


def _sphere(c, r, matid):
    """<sphere> element (scene.cpp:375-396): origin, radius, material id."""
    return (f"\t<sphere>\n\t\t<origin x=\"{c[0]}\" y=\"{c[1]}\" z=\"{c[2]}\"/>\n"
            f"\t\t<radius radius=\"{r}\"/>\n\t\t<matid matid=\"{matid}\"/>\n\t</sphere>\n")


def spheres_scene(width, height, mode="bdpt", assets=ASSETS):
    """Cornell-box walls and luminaire with three spheres -- glass (IOR 1.5),
    mirror and diffuse -- for the Sphere::hit path and the specular BSDF
    branches (the reference's configs use triangles only)."""
    xres, yres = (width, height) if mode == "pt" else (height, width)
    a = lambda f: os.path.join(assets, f)
    out = "<scene>\n"
    out += _camera(("-0.0439815", "-4.12529", "0.222539"),
                   ("0.00688625", "0.998505", "-0.0542161"),
                   ("3.73896e-4", "0.0542148", "0.998529"), xres, yres, "45")
    out += _mat()
    out += _mat(d=("0.803922", "0.803922", "0.803922"), e=1)
    out += _mat(d=("0.156863", "0.803922", "0.172549"), e=1)
    out += _mat(d=("0.803922", "0.152941", "0.152941"), e=1)
    out += _mat(s=("1", "1", "1"), n="1.5")                   # 4 glass
    out += _mat(s=("0.95", "0.95", "0.95"))                    # 5 mirror
    out += _mat(d=("0.2", "0.3", "0.7"), g=("0.3", "0.3", "0.3"), e=20)  # 6 glossy blue
    for f in ("cbox_floor.obj", "cbox_back.obj", "cbox_ceiling.obj"):
        out += _obj(a(f), 1)
    out += _obj(a("cbox_greenwall.obj"), 2)
    out += _obj(a("cbox_redwall.obj"), 3)
    out += _sphere(("-0.5", "0.3", "-0.82"), "0.45", 4)
    out += _sphere(("0.55", "0.6", "-0.86"), "0.42", 5)
    out += _sphere(("0.05", "-0.45", "-1.0"), "0.28", 6)
    out += _area(a("cbox_luminaire.obj"), "25.03329895614464")
    out += "</scene>\n"
    return out


def tent_scene(width, height, mode="bdpt", assets=ASSETS):
    """Cornell-box walls under a tent-shaped luminaire (assets/tent_luminaire.obj,
    four emitting faces turned inward): light subpaths can start on one slope
    and hit another emitter first -- the VCM light vertex that inherits the
    previous light path's BSDF probabilities (vertexcm.cpp:90-113, bsdf.h:78-83)."""
    xres, yres = (width, height) if mode == "pt" else (height, width)
    a = lambda f: os.path.join(assets, f)
    out = "<scene>\n"
    out += _camera(("-0.0439815", "-4.12529", "0.222539"),
                   ("0.00688625", "0.998505", "-0.0542161"),
                   ("3.73896e-4", "0.0542148", "0.998529"), xres, yres, "45")
    out += _mat()
    out += _mat(d=("0.803922", "0.803922", "0.803922"), e=1)
    out += _mat(d=("0.156863", "0.803922", "0.172549"), e=1)
    out += _mat(d=("0.803922", "0.152941", "0.152941"), e=1)
    out += _mat(s=("1", "1", "1"), n="1.5")
    for f in ("cbox_floor.obj", "cbox_back.obj", "cbox_ceiling.obj"):
        out += _obj(a(f), 1)
    out += _obj(a("cbox_greenwall.obj"), 2)
    out += _obj(a("cbox_redwall.obj"), 3)
    out += _sphere(("0.1", "0.2", "-0.8"), "0.35", 4)
    out += _area(a("tent_luminaire.obj"), "12")
    out += "</scene>\n"
    return out


def synth_torus_obj(path, U=1000, V=500, R=150.0, r=45.0, center=(17.0, 102.0, -15.0)):
    """The C4/C5 synthetic torus: U x V quad grid in the xy-plane, each quad
    (a b c d) written as `f a b c` / `f a c d` => 2*U*V = 1,000,000 triangles."""
    cx, cy, cz = center
    with open(path, "w") as f:
        f.write(f"# synthetic torus U={U} V={V} R={R} r={r}\n")
        for i in range(U):
            u = 2.0 * math.pi * i / U
            cu, su = math.cos(u), math.sin(u)
            for j in range(V):
                v = 2.0 * math.pi * j / V
                rr = R + r * math.cos(v)
                f.write(f"v {cx + rr * cu:.6f} {cy + rr * su:.6f} {cz + r * math.sin(v):.6f}\n")
        for i in range(U):
            i1 = (i + 1) % U
            for j in range(V):
                j1 = (j + 1) % V
                a = i * V + j + 1
                b = i1 * V + j + 1
                c = i1 * V + j1 + 1
                d = i * V + j1 + 1
                f.write(f"f {a} {b} {c}\nf {a} {c} {d}\n")


def write(path, text):
    with open(path, "w") as f:
        f.write(text)
    return path


def params_text(width, height, max_depth=7, spp=1):
    """`src/parameters.para` format: 8 positional ints with # comments
    (`parameters.cpp:22-34`)."""
    return (f"#MAX_TRACING_DEPTH\n{max_depth}\n\n#SAMPLES_PER_PIXEL\n{spp}\n\n"
            f"#SAMPLES_OF_LIGHT(path_tracing)\n8\n\n#SAMPLES_OF_HEMISPHERE(path_tracing)\n4\n\n"
            f"#WIDTH\n{width}\n\n#HEIGHT\n{height}\n\n#PHONG_POWER_INDEX\n5\n\n#POINT_LIGHT_NUM\n400\n")
