"""ctypes binding to oracle/liboracle.so (the C restatement of the reference).

Test infrastructure only: used by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker -- never by the product path.
"""
import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(REPO, "oracle")
_lib = None


class Stats(C.Structure):
    _fields_ = [("closest_rays", C.c_int64), ("shadow_rays", C.c_int64),
                ("inner_visits", C.c_int64), ("leaf_visits", C.c_int64),
                ("prim_refs", C.c_int64), ("tri_tests", C.c_int64),
                ("sph_tests", C.c_int64), ("seconds", C.c_double),
                ("vm_queries", C.c_int64), ("vm_found", C.c_int64), ("vm_merged", C.c_int64),
                ("vm_emitter_first", C.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def lib():
    global _lib
    if _lib is None:
        so = os.environ.get("WR_ORACLE_SO") or os.path.join(ORACLE, "liboracle.so")  # debugging variants
        if not os.path.exists(so):
            subprocess.run(["make", "-C", ORACLE, "oracle"], check=True, capture_output=True)
        L = C.CDLL(so)
        P, F, I, I64, U32 = C.c_void_p, C.POINTER(C.c_float), C.c_int, C.c_int64, C.c_uint32
        L.cr_scene_load.restype = P
        L.cr_scene_load.argtypes = [C.c_char_p]
        L.cr_scene_free.argtypes = [P]
        L.cr_last_error.restype = C.c_char_p
        L.cr_scene_nobjs.argtypes = [P]
        L.cr_scene_nlights.argtypes = [P]
        L.cr_scene_dump.argtypes = [P, C.c_char_p]
        L.cr_trace.argtypes = [P, F, I64, C.POINTER(C.c_int32), F, C.POINTER(C.c_uint8), C.POINTER(Stats)]
        L.cr_render_bdpt.argtypes = [P, I, I, I, I, U32, I, I, I64, I64, F, C.POINTER(Stats)]
        L.cr_render_vcm.argtypes = [P, I, I, I, I, U32, I, I, I, C.c_float, C.c_float, I64, I64, F,
                                    C.POINTER(Stats)]
        L.cr_render_pt.argtypes = [P, I, I, I, I, U32, I, I64, I64, F, C.POINTER(Stats)]
        L.cr_render_pt_samples.argtypes = [P, I, I, I, I, I, I, U32, I, I64, I64, F, C.POINTER(Stats)]
        L.cr_pt_radiance.argtypes = [P, F, I64, I, U32, U32, F, C.POINTER(Stats)]
        L.cr_stream_key.restype = C.c_uint64
        L.cr_stream_key.argtypes = [U32, U32, U32, U32]
        L.cr_stream_u32.restype = C.c_uint32
        L.cr_stream_u32.argtypes = [C.c_uint64, U32]
        L.cr_mt_outputs.argtypes = [U32, I, C.POINTER(C.c_uint32)]
        L.cr_kat_sampler.argtypes = [F, C.c_float, F]
        L.cr_kat_triangle.argtypes = [F, F, F]
        L.cr_kat_frame.argtypes = [F, F]
        L.cr_kat_fresnel.restype = C.c_float
        L.cr_kat_fresnel.argtypes = [C.c_float, C.c_float]
        L.cr_kat_strat.argtypes = [F, I, I, F]
        L.cr_kat_bsdf.argtypes = [P, I, F, F, F, F, F]
        L.cr_kat_light.argtypes = [P, I, F, F, F, F, F, F]
        L.cr_kat_vkd.argtypes = [F, I, F, I, C.c_float, C.POINTER(C.c_int64)]
        L.cr_kat_camera.argtypes = [P, C.c_float, C.c_float, F, F]
        _lib = L
    return _lib


def fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def f32(*vals):
    return np.array(vals, np.float32)


class Scene:
    def __init__(self, path):
        self.L = lib()
        self.h = self.L.cr_scene_load(path.encode())
        if not self.h:
            raise RuntimeError(self.L.cr_last_error().decode())

    def __del__(self):
        if getattr(self, "h", None):
            self.L.cr_scene_free(self.h)
            self.h = None

    @property
    def nobjs(self):
        return self.L.cr_scene_nobjs(self.h)

    def dump(self, path):
        assert self.L.cr_scene_dump(self.h, path.encode()) == 0
        with open(path) as f:
            return f.read()

    def trace(self, rays9):
        rays9 = np.ascontiguousarray(rays9, np.float32)
        n = rays9.shape[0]
        oi = np.zeros((n, 3), np.int32)
        of = np.zeros((n, 7), np.float32)
        oc = np.zeros(n, np.uint8)
        st = Stats()
        self.L.cr_trace(self.h, fptr(rays9), n, oi.ctypes.data_as(C.POINTER(C.c_int32)), fptr(of),
                        oc.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(st))
        return oi, of, oc, st

    def bdpt(self, W, H, iterations, seed, mode=0, control_length=3, iter_begin=0,
             path_range=None):
        film = np.zeros((H, W, 3), np.float32)
        st = Stats()
        pb, pe = path_range or (0, W * H)
        rc = self.L.cr_render_bdpt(self.h, W, H, iter_begin, iterations, seed, mode, control_length,
                                   pb, pe, fptr(film), C.byref(st))
        if rc:
            raise RuntimeError(self.L.cr_last_error().decode())
        return film, st

    def vcm(self, W, H, iterations, seed, mode=0, iter_begin=0, min_len=0, max_len=10,
            radius_factor=0.003, alpha=0.75, path_range=None):
        film = np.zeros((H, W, 3), np.float32)
        st = Stats()
        pb, pe = path_range or (0, W * H)
        rc = self.L.cr_render_vcm(self.h, W, H, iter_begin, iterations, seed, mode, min_len, max_len,
                                  radius_factor, alpha, pb, pe, fptr(film), C.byref(st))
        if rc:
            raise RuntimeError(self.L.cr_last_error().decode())
        return film, st

    def pt_radiance(self, rays6, max_depth, seed, sample=0):
        rays6 = np.ascontiguousarray(rays6, np.float32)
        out = np.zeros((rays6.shape[0], 3), np.float32)
        st = Stats()
        rc = self.L.cr_pt_radiance(self.h, fptr(rays6), rays6.shape[0], max_depth, seed, sample, fptr(out),
                                   C.byref(st))
        if rc:
            raise RuntimeError(self.L.cr_last_error().decode())
        return out, st

    def pt(self, W, H, spp, max_depth, seed, mode=0, pix_range=None):
        film = np.zeros((H, W, 3), np.float32)
        st = Stats()
        pb, pe = pix_range or (0, W * H)
        rc = self.L.cr_render_pt(self.h, W, H, spp, max_depth, seed, mode, pb, pe, fptr(film), C.byref(st))
        if rc:
            raise RuntimeError(self.L.cr_last_error().decode())
        return film, st

    def pt_samples(self, W, H, spp, k_begin, k_count, max_depth, seed, mode=1, pix_range=None):
        """Samples [k_begin, k_begin + k_count) of the spp grid, summed (no 1/spp)."""
        film = np.zeros((H, W, 3), np.float32)
        st = Stats()
        pb, pe = pix_range or (0, W * H)
        rc = self.L.cr_render_pt_samples(self.h, W, H, spp, k_begin, k_count, max_depth, seed, mode, pb, pe,
                                         fptr(film), C.byref(st))
        if rc:
            raise RuntimeError(self.L.cr_last_error().decode())
        return film, st
