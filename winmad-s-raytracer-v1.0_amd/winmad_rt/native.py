"""ctypes binding to libwinmad_rt.so (include/winmad_rt.h).

The library is built in-tree (`make -C winmad-s-raytracer-v1.0_amd`, or
`__graft_entry__.build()`).  There is no fallback: if the HIP library cannot be
loaded every call raises.
"""
import ctypes as C
import os
import sys

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# WR_LIB selects another build of the same library (kernel variants under test)
LIB_PATH = os.environ.get("WR_LIB") or os.path.join(PKG_DIR, "libwinmad_rt.so")

WR_OK, WR_E_ARG, WR_E_IO, WR_E_HIP, WR_E_SCENE, WR_E_NODEVICE = 0, -1, -2, -3, -4, -5
K_TRACE, K_SHADE, K_RESOLVE, K_GEN, K_OTHER = 0, 1, 2, 3, 4
TRACE_REFERENCE, TRACE_BVH = 0, 1
INTEGRATOR_BDPT, INTEGRATOR_VCM, INTEGRATOR_PATH = 0, 1, 2

# every entry point declared in include/winmad_rt.h
EXPORTS = ["wr_scene_load", "wr_scene_from_desc", "wr_scene_info_get", "wr_scene_fingerprint", "wr_scene_dump", "wr_scene_free",
           "wr_device_count", "wr_create", "wr_create_multi", "wr_context_devices", "wr_destroy", "wr_comm_unique_id",
           "wr_comm_init", "wr_comm_info", "wr_film_reduce", "wr_set_pipelines", "wr_set_trace_mode", "wr_trace_closest", "wr_occluded",
           "wr_render_bdpt", "wr_render_path", "wr_render_vcm", "wr_path_radiance", "wr_film_write_ppm",
           "wr_film_write_image", "wr_checkpoint_save", "wr_checkpoint_load", "wr_last_error", "wr_api_version",
           "wr_reserve", "wr_request_hw_queues"]
CKPT_BDPT, CKPT_VCM, CKPT_PT = 1, 2, 3


class WrRay(C.Structure):
    _fields_ = [("o", C.c_float * 3), ("d", C.c_float * 3), ("tmin", C.c_float), ("tmax", C.c_float)]


class WrHit(C.Structure):
    _fields_ = [("t", C.c_float), ("p", C.c_float * 3), ("n", C.c_float * 3), ("prim", C.c_int32),
                ("inside", C.c_int32), ("mat_id", C.c_int32)]


class WrSceneInfo(C.Structure):
    _fields_ = [("nprims", C.c_int32), ("ntriangles", C.c_int32), ("nspheres", C.c_int32),
                ("nlights", C.c_int32), ("nmaterials", C.c_int32), ("kd_depth_max", C.c_int32),
                ("kd_inner", C.c_int32), ("kd_leaves", C.c_int32), ("kd_refs", C.c_int64),
                ("kd_max_stack", C.c_int32), ("missing_files", C.c_int32), ("camera_xres", C.c_float),
                ("camera_yres", C.c_float), ("device_bytes", C.c_int64)]


class WrSceneDesc(C.Structure):
    _fields_ = [("n_prims", C.c_int32), ("prim_type", C.POINTER(C.c_int32)), ("prim_data", C.POINTER(C.c_float)),
                ("prim_mat", C.POINTER(C.c_int32)), ("n_lights", C.c_int32), ("light_tri", C.POINTER(C.c_float)),
                ("light_le", C.POINTER(C.c_float)), ("n_materials", C.c_int32), ("materials", C.POINTER(C.c_float)),
                ("cam_pos", C.c_float * 3), ("cam_fwd", C.c_float * 3), ("cam_up", C.c_float * 3),
                ("cam_xres", C.c_float), ("cam_yres", C.c_float), ("cam_hfov", C.c_float)]


class WrCheckpointInfo(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("kind", C.c_int32), ("done", C.c_int32),
                ("total", C.c_int32), ("seed", C.c_uint32), ("fingerprint", C.c_uint32 * 2)]


class WrBdptParams(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("iterations", C.c_int32),
                ("iter_begin", C.c_int32), ("control_length", C.c_int32), ("max_path_length", C.c_int32),
                ("seed", C.c_uint32), ("faithful", C.c_int32), ("time_kernels", C.c_int32),
                ("count_work", C.c_int32)]


class WrPathParams(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_int32), ("max_depth", C.c_int32),
                ("sample_begin", C.c_int32), ("sample_count", C.c_int32), ("seed", C.c_uint32),
                ("time_kernels", C.c_int32), ("count_work", C.c_int32)]


class WrVcmParams(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("iterations", C.c_int32),
                ("iter_begin", C.c_int32), ("min_path_length", C.c_int32), ("max_path_length", C.c_int32),
                ("radius_factor", C.c_float), ("radius_alpha", C.c_float), ("seed", C.c_uint32),
                ("time_kernels", C.c_int32), ("count_work", C.c_int32)]


class WrStats(C.Structure):
    _fields_ = [("closest_rays", C.c_int64), ("shadow_rays", C.c_int64), ("inner_visits", C.c_int64),
                ("leaf_visits", C.c_int64), ("prim_refs", C.c_int64), ("seconds", C.c_double),
                ("kernel_ms", C.c_double * 8), ("kernel_launches", C.c_int64 * 8), ("trace_wall_ms", C.c_double),
                ("vm_queries", C.c_int64), ("vm_found", C.c_int64), ("vm_merged", C.c_int64),
                ("prim_tests", C.c_int64), ("bvh_nodes", C.c_int64), ("bvh_tests", C.c_int64),
                ("kd_replay_steps", C.c_int64), ("fallback_rays", C.c_int64), ("verify_rays", C.c_int64),
                ("verify_mismatches", C.c_int64), ("pipelines", C.c_int64),
                ("deferred_rays", C.c_int64), ("bvh_width", C.c_int64), ("work_bytes", C.c_int64),
                ("work_paths", C.c_int64), ("redone", C.c_int64)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in ("kernel_ms", "kernel_launches")}
        d["kernel_ms"] = list(self.kernel_ms)
        d["kernel_launches"] = list(self.kernel_launches)
        return d


class WrError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"winmad_rt error {code}: {msg}")
        self.code = code


_lib = None


def _share_torch_runtime():
    """PyTorch-ROCm ships its own libamdhip64 with the same SONAME
    (libamdhip64.so.7) as /opt/rocm's.  If torch is loaded first, the dynamic
    linker binds libwinmad_rt.so to that copy and the process has ONE HIP
    runtime (device pointers of torch tensors are then valid for wr_* calls).
    Loaded the other way round there would be two runtimes and torch's fails to
    initialise, so torch -- when installed -- is imported before our library."""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def _hip_is_up():
    torch = sys.modules.get("torch")
    try:
        return torch is not None and torch.cuda.is_initialized()
    except Exception:
        return False


def _request_hw_queues(L):
    """One hardware queue per render pipeline (concurrent
    pipelines): HIP reads GPU_MAX_HW_QUEUES once, when it initialises, and the
    library sizes its pipelines by it.  If HIP is not up yet, ask for 16
    (env WR_HW_QUEUES=n asks for n; a larger GPU_MAX_HW_QUEUES is kept) through
    wr_request_hw_queues -- the library never changes the environment by
    itself.  If torch already initialised HIP, the variable stays as HIP read
    it, so the library starts no more pipelines than there are queues."""
    if _hip_is_up():
        return
    want = 16
    try:
        want = max(1, min(32, int(os.environ.get("WR_HW_QUEUES", "16"))))
    except ValueError:
        pass
    L.wr_request_hw_queues(want)


def lib():
    """Load the in-tree HIP library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        _share_torch_runtime()
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: build it with `make -C {PKG_DIR}` "
                               "(or __graft_entry__.build()); there is no CPU fallback")
        L = C.CDLL(LIB_PATH)
        L.wr_request_hw_queues.argtypes = [C.c_int]
        _request_hw_queues(L)
        P, I, I64 = C.c_void_p, C.c_int, C.c_int64
        L.wr_scene_load.argtypes = [C.c_char_p, C.POINTER(P)]
        L.wr_scene_from_desc.argtypes = [C.POINTER(WrSceneDesc), C.POINTER(P)]
        L.wr_create_multi.argtypes = [P, C.POINTER(C.c_int), I, C.POINTER(P)]
        L.wr_context_devices.argtypes = [P, C.POINTER(C.c_int), I]
        L.wr_comm_unique_id.argtypes = [C.POINTER(C.c_uint8)]
        L.wr_comm_init.argtypes = [P, C.POINTER(C.c_uint8), I, I]
        L.wr_film_reduce.argtypes = [P, P, I64, I]
        L.wr_comm_info.argtypes = [P, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.wr_checkpoint_save.argtypes = [C.c_char_p, C.POINTER(WrCheckpointInfo), C.POINTER(C.c_float)]
        L.wr_checkpoint_load.argtypes = [C.c_char_p, C.POINTER(WrCheckpointInfo), C.POINTER(C.c_float), I64]
        L.wr_scene_info_get.argtypes = [P, C.POINTER(WrSceneInfo)]
        L.wr_scene_dump.argtypes = [P, C.c_char_p]
        L.wr_scene_fingerprint.argtypes = [P, C.POINTER(C.c_uint64)]
        L.wr_scene_free.argtypes = [P]
        L.wr_scene_free.restype = None
        L.wr_create.argtypes = [P, I, C.POINTER(P)]
        L.wr_destroy.argtypes = [P]
        L.wr_destroy.restype = None
        L.wr_set_pipelines.argtypes = [P, I]
        L.wr_set_trace_mode.argtypes = [P, I]
        L.wr_reserve.argtypes = [P, I, I, I]
        L.wr_trace_closest.argtypes = [P, C.POINTER(WrRay), I64, C.POINTER(WrHit)]
        L.wr_occluded.argtypes = [P, C.POINTER(WrRay), C.POINTER(C.c_float), I64, C.POINTER(C.c_uint8)]
        L.wr_render_bdpt.argtypes = [P, C.POINTER(WrBdptParams), P, I, C.POINTER(WrStats)]
        L.wr_render_path.argtypes = [P, C.POINTER(WrPathParams), P, I, C.POINTER(WrStats)]
        L.wr_render_vcm.argtypes = [P, C.POINTER(WrVcmParams), P, I, C.POINTER(WrStats)]
        L.wr_path_radiance.argtypes = [P, C.POINTER(WrRay), I64, I, C.c_uint32, I, C.POINTER(C.c_float),
                                       C.POINTER(WrStats)]
        L.wr_film_write_ppm.argtypes = [C.POINTER(C.c_float), I, I, C.c_float, C.c_float, I, C.c_char_p]
        L.wr_film_write_image.argtypes = [C.POINTER(C.c_float), I, I, C.c_float, C.c_float, I, C.c_char_p]
        L.wr_last_error.restype = C.c_char_p
        _lib = L
    return _lib


def library_sha16():
    """sha256 prefix (16 hex digits) of the library file this process loads:
    ties a measurement (profiles/*/traffic_*.json, lib_sha) to a build."""
    import hashlib
    try:
        with open(LIB_PATH, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def check(rc):
    if rc != WR_OK:
        raise WrError(rc, lib().wr_last_error().decode())
    return rc


def device_count():
    return lib().wr_device_count()


class Scene:
    """Scene::init (scene.cpp:469-489): .scene + .obj + KD tree, host side."""

    def __init__(self, path=None, _handle=None):
        if _handle is not None:
            self.h = _handle
            return
        h = C.c_void_p()
        check(lib().wr_scene_load(os.fsencode(path), C.byref(h)))
        self.h = h

    @classmethod
    def from_desc(cls, prim_type, prim_data, prim_mat, light_tri, light_le, materials, cam_pos, cam_fwd, cam_up,
                  cam_xres, cam_yres, cam_hfov):
        """wr_scene_from_desc: the reference's in-memory Scene as flat arrays
        (include/winmad_rt.h wr_scene_desc): prim_type (n,) int32 0/1,
        prim_data (n, 9) float32, prim_mat (n,) int32, light_tri (m, 9),
        light_le (m, 3), materials (k, 11), camera vectors and raster / FOV."""
        pt = np.ascontiguousarray(prim_type, np.int32).reshape(-1)
        pd = np.ascontiguousarray(prim_data, np.float32).reshape(-1, 9)
        pm = np.ascontiguousarray(prim_mat, np.int32).reshape(-1)
        lt = np.ascontiguousarray(light_tri, np.float32).reshape(-1, 9)
        le = np.ascontiguousarray(light_le, np.float32).reshape(-1, 3)
        mt = np.ascontiguousarray(materials, np.float32).reshape(-1, 11)
        if not (pt.size == pd.shape[0] == pm.size) or lt.shape[0] != le.shape[0]:
            raise ValueError("inconsistent primitive / light array lengths")
        d = WrSceneDesc()
        d.n_prims = pt.size
        d.prim_type = pt.ctypes.data_as(C.POINTER(C.c_int32))
        d.prim_data = pd.ctypes.data_as(C.POINTER(C.c_float))
        d.prim_mat = pm.ctypes.data_as(C.POINTER(C.c_int32))
        d.n_lights = lt.shape[0]
        d.light_tri = lt.ctypes.data_as(C.POINTER(C.c_float))
        d.light_le = le.ctypes.data_as(C.POINTER(C.c_float))
        d.n_materials = mt.shape[0]
        d.materials = mt.ctypes.data_as(C.POINTER(C.c_float))
        for k in range(3):
            d.cam_pos[k], d.cam_fwd[k], d.cam_up[k] = float(cam_pos[k]), float(cam_fwd[k]), float(cam_up[k])
        d.cam_xres, d.cam_yres, d.cam_hfov = float(cam_xres), float(cam_yres), float(cam_hfov)
        h = C.c_void_p()
        check(lib().wr_scene_from_desc(C.byref(d), C.byref(h)))
        return cls(_handle=h)

    def close(self):
        if getattr(self, "h", None):
            lib().wr_scene_free(self.h)
            self.h = None

    __del__ = close

    def info(self):
        i = WrSceneInfo()
        check(lib().wr_scene_info_get(self.h, C.byref(i)))
        return {k: getattr(i, k) for k, _ in i._fields_}

    def fingerprint(self):
        """wr_scene_fingerprint: 64-bit hash of the primitives, lights, materials, camera."""
        v = C.c_uint64()
        check(lib().wr_scene_fingerprint(self.h, C.byref(v)))
        return v.value

    def dump(self, path):
        check(lib().wr_scene_dump(self.h, os.fsencode(path)))
        with open(path) as f:
            return f.read()


def _rays8(rays8):
    """(n, 8) float32 C-contiguous rays (o, d, tmin, tmax); anything else raises."""
    rays8 = np.ascontiguousarray(rays8, np.float32)
    if rays8.ndim != 2 or rays8.shape[1] != 8:
        raise ValueError(f"rays8 must have shape (n, 8), got {rays8.shape}")
    return rays8


def _host_film(film, height, width):
    """The caller's accumulating host film: the library adds height*width*3
    floats into it in place, so it must be exactly a C-contiguous float32
    (height, width, 3) array -- no silent conversion (a copy would drop the
    result, a smaller buffer would be overrun)."""
    if film is None:
        return np.zeros((height, width, 3), np.float32)
    if not isinstance(film, np.ndarray) or film.dtype != np.float32 or film.shape != (height, width, 3) \
            or not film.flags["C_CONTIGUOUS"] or not film.flags["WRITEABLE"]:
        raise ValueError(f"film must be a writeable C-contiguous float32 array of shape ({height}, {width}, 3), "
                         f"got {type(film).__name__} "
                         f"{getattr(film, 'dtype', None)} {getattr(film, 'shape', None)}")
    return film


def rays_from_arrays(o, d, tmin=0.0, tmax=1e7):
    n = o.shape[0]
    arr = np.zeros((n, 8), np.float32)
    arr[:, 0:3] = o
    arr[:, 3:6] = d
    arr[:, 6] = tmin
    arr[:, 7] = tmax
    return arr


class Context:
    """Scene resident in HBM on one device (or on several: `devices`, a list of
    HIP device ids, wr_create_multi) + its HIP streams."""

    def __init__(self, scene, device=0, devices=None, trace=None):
        """trace: None keeps the library default (the verified BVH for triangle
        scenes, the KD walk with spheres), else TRACE_REFERENCE / TRACE_BVH."""
        h = C.c_void_p()
        if devices is not None:
            ids = (C.c_int * len(devices))(*devices)
            check(lib().wr_create_multi(scene.h, ids, len(devices), C.byref(h)))
        else:
            check(lib().wr_create(scene.h, device, C.byref(h)))
        self.h = h
        self.scene = scene
        if trace is not None:
            self.set_trace_mode(trace)

    def devices(self):
        buf = (C.c_int * 64)()
        n = lib().wr_context_devices(self.h, buf, 64)
        if n < 0:
            check(n)
        return list(buf[:n])

    def comm_init(self, unique_id, nranks, rank):
        """wr_comm_init: this rank's RCCL communicator (one process per GPU)."""
        idb = (C.c_uint8 * 128)(*bytes(unique_id))
        check(lib().wr_comm_init(self.h, idb, nranks, rank))

    def comm_info(self):
        """wr_comm_info: (ranks, this rank) as the RCCL communicator reports them."""
        n, r = C.c_int(0), C.c_int(0)
        check(lib().wr_comm_info(self.h, C.byref(n), C.byref(r)))
        return n.value, r.value

    def film_reduce(self, film_ptr, nfloat, root=0):
        """wr_film_reduce: sum the ranks' device films into rank `root`'s, in place."""
        check(lib().wr_film_reduce(self.h, C.c_void_p(film_ptr), nfloat, root))

    def set_pipelines(self, n):
        """Concurrent render pipelines (streams) for render_bdpt / render_path."""
        check(lib().wr_set_pipelines(self.h, n))

    def reserve(self, integrator, width, height):
        """wr_reserve: allocate the work buffers of renders of this kind
        (INTEGRATOR_BDPT / _VCM / _PATH) and film size now."""
        check(lib().wr_reserve(self.h, integrator, width, height))

    def set_trace_mode(self, mode):
        """TRACE_REFERENCE (the reference's KD walk) or TRACE_BVH (verified BVH
        search + KD fallback, same answers): include/winmad_rt.h."""
        check(lib().wr_set_trace_mode(self.h, mode))

    def close(self):
        if getattr(self, "h", None):
            lib().wr_destroy(self.h)
            self.h = None

    __del__ = close

    def trace_closest(self, rays8):
        """rays8: (n, 8) float32 = o, d, tmin, tmax (d used as given)."""
        rays8 = _rays8(rays8)
        n = rays8.shape[0]
        hits = np.zeros(n, dtype=np.dtype([("t", "f4"), ("p", "f4", 3), ("n", "f4", 3), ("prim", "i4"),
                                           ("inside", "i4"), ("mat_id", "i4")]))
        check(lib().wr_trace_closest(self.h, rays8.ctypes.data_as(C.POINTER(WrRay)), n,
                                     hits.ctypes.data_as(C.POINTER(WrHit))))
        return hits

    def occluded(self, rays8, targets):
        rays8 = _rays8(rays8)
        targets = np.ascontiguousarray(targets, np.float32)
        n = rays8.shape[0]
        if targets.shape != (n, 3):
            raise ValueError(f"targets must have shape ({n}, 3), got {targets.shape}")
        out = np.zeros(n, np.uint8)
        check(lib().wr_occluded(self.h, rays8.ctypes.data_as(C.POINTER(WrRay)),
                                targets.ctypes.data_as(C.POINTER(C.c_float)), n,
                                out.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out

    def render_bdpt(self, width, height, iterations=1, seed=5489, iter_begin=0, control_length=3,
                    max_path_length=10, faithful=1, time_kernels=0, count_work=0, film=None, film_ptr=None):
        """BidirPathTracing::render.  Host film (numpy, accumulated) or a device
        pointer (film_ptr, e.g. a torch tensor's data_ptr())."""
        p = WrBdptParams(width, height, iterations, iter_begin, control_length, max_path_length, seed,
                         faithful, time_kernels, count_work)
        st = WrStats()
        if film_ptr is not None:
            check(lib().wr_render_bdpt(self.h, C.byref(p), C.c_void_p(film_ptr), 1, C.byref(st)))
            return None, st
        film = _host_film(film, height, width)
        check(lib().wr_render_bdpt(self.h, C.byref(p), film.ctypes.data_as(C.c_void_p), 0, C.byref(st)))
        return film, st

    def render_vcm(self, width, height, iterations=1, seed=5489, iter_begin=0, min_path_length=0,
                   max_path_length=10, radius_factor=0.003, radius_alpha=0.75, time_kernels=0, count_work=0,
                   film=None, film_ptr=None):
        """VertexCM::render (vertex connection and merging).  Film as render_bdpt."""
        p = WrVcmParams(width, height, iterations, iter_begin, min_path_length, max_path_length, radius_factor,
                        radius_alpha, seed, time_kernels, count_work)
        st = WrStats()
        if film_ptr is not None:
            check(lib().wr_render_vcm(self.h, C.byref(p), C.c_void_p(film_ptr), 1, C.byref(st)))
            return None, st
        film = _host_film(film, height, width)
        check(lib().wr_render_vcm(self.h, C.byref(p), film.ctypes.data_as(C.c_void_p), 0, C.byref(st)))
        return film, st

    def path_radiance(self, rays8, max_depth=7, seed=5489, sample=0):
        """PathIntegrator::raytracing for each ray of rays8 ((n, 8) float32:
        o, d, tmin, tmax; d used as given).  Returns (n, 3) radiance, stats."""
        rays8 = _rays8(rays8)
        n = rays8.shape[0]
        out = np.zeros((n, 3), np.float32)
        st = WrStats()
        check(lib().wr_path_radiance(self.h, rays8.ctypes.data_as(C.POINTER(WrRay)), n, max_depth, seed, sample,
                                     out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st)))
        return out, st

    def render_path(self, width, height, spp, max_depth=7, seed=5489, sample_begin=0, sample_count=0,
                    time_kernels=0, count_work=0, film=None, film_ptr=None):
        """SurfaceIntegrator::render + PathIntegrator (film = SUM over samples)."""
        p = WrPathParams(width, height, spp, max_depth, sample_begin, sample_count, seed, time_kernels,
                         count_work)
        st = WrStats()
        if film_ptr is not None:
            check(lib().wr_render_path(self.h, C.byref(p), C.c_void_p(film_ptr), 1, C.byref(st)))
            return None, st
        film = _host_film(film, height, width)
        check(lib().wr_render_path(self.h, C.byref(p), film.ctypes.data_as(C.c_void_p), 0, C.byref(st)))
        return film, st


def comm_unique_id():
    """wr_comm_unique_id: 128 bytes rank 0 hands to every rank's comm_init."""
    buf = (C.c_uint8 * 128)()
    check(lib().wr_comm_unique_id(buf))
    return bytes(buf)


def checkpoint_save(path, film, kind, done, total, seed, fingerprint=0):
    """wr_checkpoint_save: the accumulated film + how many iterations it sums
    (+ the 64-bit scene / settings fingerprint the resume must match)."""
    film = np.ascontiguousarray(film, np.float32)
    if film.ndim != 3 or film.shape[2] != 3:
        raise ValueError(f"film must have shape (height, width, 3), got {film.shape}")
    info = WrCheckpointInfo(film.shape[1], film.shape[0], kind, done, total, seed,
                            (C.c_uint32 * 2)(fingerprint & 0xFFFFFFFF, (fingerprint >> 32) & 0xFFFFFFFF))
    check(lib().wr_checkpoint_save(os.fsencode(path), C.byref(info), film.ctypes.data_as(C.POINTER(C.c_float))))


def checkpoint_load(path):
    """wr_checkpoint_load -> (film, dict(width, height, kind, done, total, seed, fingerprint))."""
    info = WrCheckpointInfo()
    check(lib().wr_checkpoint_load(os.fsencode(path), C.byref(info), None, 0))
    film = np.zeros((info.height, info.width, 3), np.float32)
    check(lib().wr_checkpoint_load(os.fsencode(path), C.byref(info), film.ctypes.data_as(C.POINTER(C.c_float)),
                                   film.size))
    d = {k: getattr(info, k) for k in ("width", "height", "kind", "done", "total", "seed")}
    d["fingerprint"] = int(info.fingerprint[0]) | (int(info.fingerprint[1]) << 32)
    return film, d


def write_ppm(film, path, scale=1.0, gamma=2.2, transpose=False):
    """ImageFilm::outputImage pipeline (film.cpp:39-64) to a binary PPM."""
    film = np.ascontiguousarray(film, np.float32)
    if film.ndim != 3 or film.shape[2] != 3:
        raise ValueError(f"film must have shape (height, width, 3), got {film.shape}")
    h, w = film.shape[:2]
    check(lib().wr_film_write_ppm(film.ctypes.data_as(C.POINTER(C.c_float)), h, w, scale, gamma,
                                  1 if transpose else 0, os.fsencode(path)))


def write_image(film, path, scale=1.0, gamma=2.2, transpose=False):
    """ImageFilm::outputImage into .ppm / .bmp / .png, or linear .pfm."""
    film = np.ascontiguousarray(film, np.float32)
    if film.ndim != 3 or film.shape[2] != 3:
        raise ValueError(f"film must have shape (height, width, 3), got {film.shape}")
    h, w = film.shape[:2]
    check(lib().wr_film_write_image(film.ctypes.data_as(C.POINTER(C.c_float)), h, w, scale, gamma,
                                    1 if transpose else 0, os.fsencode(path)))
