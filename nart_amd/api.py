"""ctypes bindings of the nart_amd C ABI (include/nart_scene.h, include/nart_hip.h).

Mirrors the reference's host surface for the render path:
    Scene(path)                        <- Scene::Scene (src/core/scene.cpp:3-26)
    parse_args(argv) / load_sessions   <- ParseRenderParamArguments / LoadSessions (render.cpp:236-414)
    HipRenderer(scene).render(params)  <- RenderSession::Render (render.cpp:114-206), on the GPU
    write_exr(path, params, image)     <- RenderSession::WriteImageToEXR (render.cpp:208-234)
The render path has no CPU fallback: without the HIP library (or a GPU) it raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(_HERE, "lib")

NART_OK = 0
ERRORS = {-1: "NART_E_INVALID", -2: "NART_E_IO", -3: "NART_E_HIP", -4: "NART_E_OOM", -5: "NART_E_RCCL",
          -6: "NART_E_UNSUPPORTED"}
NART_E_UNSUPPORTED = -6

PIXEL_FLOATS = 5  # struct Pixel { vec4 contribution; float filterWeightSum; } (render.h:18-21)


class NativeLibraryMissing(RuntimeError):
    pass


class NartError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__("%s (%d)%s" % (ERRORS.get(code, "error"), code, (": " + msg) if msg else ""))
        self.code = code


class RenderParams(ctypes.Structure):
    """struct RenderParams (include/nart/core/scene.h:25-36)."""
    _fields_ = [("integrator", ctypes.c_int32), ("image_width", ctypes.c_uint32), ("image_height", ctypes.c_uint32),
                ("bucket_size", ctypes.c_uint32), ("spp", ctypes.c_uint32), ("bounces", ctypes.c_uint32),
                ("filter_width", ctypes.c_float), ("roughening_factor", ctypes.c_float)]

    def __repr__(self):
        return "RenderParams(%s)" % ", ".join("%s=%r" % (f, getattr(self, f)) for f, _ in self._fields_)

    def copy(self):
        p = RenderParams()
        ctypes.pointer(p)[0] = self
        return p


class SessionGeometry(ctypes.Structure):
    _fields_ = [("filter_bounds", ctypes.c_uint32), ("tile_size", ctypes.c_uint32), ("total_width", ctypes.c_uint32),
                ("total_height", ctypes.c_uint32), ("n_buckets_x", ctypes.c_uint32), ("n_buckets_y", ctypes.c_uint32)]


class BvhInfo(ctypes.Structure):
    """nart_bvh_info (include/nart_hip.h)."""
    _fields_ = [("num_nodes", ctypes.c_uint32), ("stack_depth", ctypes.c_uint32), ("num_leaf_tris", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


# nart_render_stats.schedule bits (include/nart_hip.h NART_SCHED_*)
SCHED = {"probe_queue": 0x1, "priority": 0x2, "spec_pairs": 0x4, "wave_groups": 0x8, "vol_queue": 0x10,
         "vol_sparse": 0x20, "splat_skew": 0x40, "primary": 0x80, "splat_rows": 0x100,
         "half_waves": 0x200, "specialized": 0x400,
         "lean": 0x800}

# scene feature bits (include/nart_hip.h NART_FT_*; nart_hip_scene_features)
FEATURES = {"lambert": 0x1, "specular": 0x2, "glass": 0x4, "glossy": 0x8, "plastic": 0x10, "disk": 0x20,
            "ring": 0x40, "environment": 0x80, "texture": 0x100, "normal_map": 0x200}
FT_ALL = 0x3FF


class RenderStats(ctypes.Structure):
    _fields_ = [("render_ms", ctypes.c_double), ("kernel_ms", ctypes.c_double), ("splat_ms", ctypes.c_double),
                ("kernel_launches", ctypes.c_uint32), ("schedule", ctypes.c_uint32), ("samples", ctypes.c_uint64),
                ("traced_samples", ctypes.c_uint64), ("rays_extend", ctypes.c_uint64), ("rays_shadow", ctypes.c_uint64),
                ("node_visits", ctypes.c_uint64), ("tri_tests", ctypes.c_uint64), ("bounces", ctypes.c_uint64),
                ("latin_ms", ctypes.c_double), ("octree_checks", ctypes.c_uint64),
                ("octree_replays", ctypes.c_uint64), ("primary_ms", ctypes.c_double)]

    def schedule_names(self):
        return sorted(k for k, v in SCHED.items() if self.schedule & v)

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


_P = ctypes.c_void_p


class _Texture(ctypes.Structure):
    """nart_texture (include/nart_scene.h)."""
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("rgba", _P)]


class _BlobHead(ctypes.Structure):
    """Leading fields of nart_scene_blob (include/nart_scene.h)."""
    _fields_ = [("num_triangles", ctypes.c_uint32), ("num_meshes", ctypes.c_uint32),
                ("num_materials", ctypes.c_uint32), ("num_lights", ctypes.c_uint32),
                ("num_textures", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("triangles", _P),
                ("meshes", _P), ("materials", _P), ("lights", _P), ("textures", ctypes.POINTER(_Texture)),
                ("cam_fov", ctypes.c_float), ("cam_m", ctypes.c_float * 16)]


_SCENE_SIGS = {
    "nart_scene_load": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(_P)]),
    "nart_scene_blob_of": (_P, [_P]),
    "nart_scene_free": (None, [_P]),
    "nart_scene_last_error": (ctypes.c_char_p, []),
    "nart_render_params_init": (None, [ctypes.POINTER(RenderParams)]),
    "nart_parse_args": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(RenderParams)]),
    "nart_load_sessions": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(RenderParams), ctypes.POINTER(RenderParams),
                                          ctypes.c_int]),
    "nart_session_geometry_of": (None, [ctypes.POINTER(RenderParams), ctypes.POINTER(SessionGeometry)]),
    "nart_filter_table": (None, [ctypes.POINTER(ctypes.c_float)]),
    "nart_combine_tiles": (None, [ctypes.POINTER(RenderParams), _P, _P]),
    "nart_write_exr": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(RenderParams), _P, ctypes.c_int]),
    "nart_float_to_half": (ctypes.c_uint16, [ctypes.c_float]),
    "nart_half_to_float": (ctypes.c_float, [ctypes.c_uint16]),
    "nart_read_exr_rgba": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint32),
                                          ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(_P)]),
    "nart_free": (None, [_P]),
}
_HIP_SIGS = {
    "nart_hip_create": (ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(_P)]),
    "nart_hip_destroy": (None, [_P]),
    "nart_hip_last_error": (ctypes.c_char_p, [_P]),
    "nart_hip_render": (ctypes.c_int, [_P, ctypes.POINTER(RenderParams), _P, ctypes.POINTER(RenderStats)]),
    "nart_hip_render_device": (ctypes.c_int, [_P, ctypes.POINTER(RenderParams), ctypes.POINTER(_P),
                                              ctypes.POINTER(RenderStats)]),
    "nart_hip_render_buckets_async": (ctypes.c_int, [_P, ctypes.POINTER(RenderParams), ctypes.POINTER(ctypes.c_uint32),
                                                     ctypes.c_uint32, _P, _P, ctypes.POINTER(RenderStats)]),
    "nart_hip_combine_async": (ctypes.c_int, [_P, ctypes.POINTER(RenderParams), _P, _P, _P]),
    "nart_hip_render_samples": (ctypes.c_int, [_P, ctypes.POINTER(RenderParams), ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.c_uint32, ctypes.c_uint32, _P]),
    "nart_hip_set_counters": (ctypes.c_int, [_P, ctypes.c_int]),
    "nart_hip_eval_sincos": (ctypes.c_int, [_P, _P, ctypes.c_uint32, _P, _P]),
    "nart_hip_set_variant": (ctypes.c_int, [_P, ctypes.c_int]),
    "nart_hip_set_splat_mode": (ctypes.c_int, [_P, ctypes.c_int]),
    "nart_hip_set_specialize": (ctypes.c_int, [_P, ctypes.c_int]),
    "nart_hip_scene_features": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    "nart_hip_scene_features_of": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint32)]),
    "nart_hip_splat_thresholds": (ctypes.c_int, [ctypes.c_float, _P]),
    "nart_hip_env_search": (ctypes.c_int, [_P, ctypes.c_uint32, _P, ctypes.c_uint32, _P, _P]),
    "nart_hip_splat_lut": (ctypes.c_int, [ctypes.c_float, _P, ctypes.POINTER(ctypes.c_uint32),
                                          ctypes.POINTER(ctypes.c_uint32)]),
    "nart_hip_bvh_info": (ctypes.c_int, [_P, ctypes.POINTER(BvhInfo)]),
    "nart_hip_create_multi": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(_P)]),
    "nart_hip_context_devices": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "nart_hip_debug_fault": (ctypes.c_int, [_P, ctypes.c_int]),
    "nart_hip_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "nart_hip_context_bvh": (ctypes.c_int, [_P, ctypes.POINTER(BvhInfo), ctypes.POINTER(ctypes.c_double)]),
    "nart_hip_shard_buckets": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                              ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
}
SCENE_SYMBOLS = tuple(_SCENE_SIGS)
HIP_SYMBOLS = tuple(_HIP_SIGS)

_libs = {}


def _load(name, sigs):
    if name in _libs:
        return _libs[name]
    path = os.path.join(LIB_DIR, name)
    if not os.path.exists(path):
        raise NativeLibraryMissing("%s not built (run nart_amd/build.py or __graft_entry__.build())" % path)
    lib = ctypes.CDLL(path)
    for fn, (res, args) in sigs.items():
        f = getattr(lib, fn)
        f.restype = res
        f.argtypes = args
    _libs[name] = lib
    return lib


def scene_lib():
    return _load("libnart_scene.so", _SCENE_SIGS)


def _missing_entry(fn, path):
    """Stand-in for an entry point an alternative build (NART_HIP_LIB) lacks: calling it raises
    a NartError naming the symbol and the build instead of an AttributeError or a call through an
    untyped pointer."""
    def call(*args):
        raise NartError(NART_E_UNSUPPORTED, "%s is not exported by the build %s" % (fn, path))
    return call


def hip_lib():
    # NART_HIP_LIB: an alternative build of the same ABI (A/B experiments, tools/ab.sh)
    alt = os.environ.get("NART_HIP_LIB")
    if alt:
        if "libnart_hip.so" not in _libs:
            scene_lib()  # its directory is on the alternative build's rpath too
            lib = ctypes.CDLL(os.path.abspath(alt))
            for fn, (res, args) in _HIP_SIGS.items():
                f = getattr(lib, fn, None)  # an older build may lack newer entry points
                if f is None:
                    setattr(lib, fn, _missing_entry(fn, alt))
                    continue
                f.restype = res
                f.argtypes = args
            _libs["libnart_hip.so"] = lib
        return _libs["libnart_hip.so"]
    return _load("libnart_hip.so", _HIP_SIGS)


def default_params():
    p = RenderParams()
    scene_lib().nart_render_params_init(ctypes.byref(p))
    return p


def parse_args(argv):
    """ParseRenderParamArguments: argv = [prog, scene, out, flags...]."""
    p = default_params()
    arr = (ctypes.c_char_p * len(argv))(*[a.encode() for a in argv])
    rc = scene_lib().nart_parse_args(len(argv), arr, ctypes.byref(p))
    if rc != NART_OK:
        raise NartError(rc, scene_lib().nart_scene_last_error().decode())
    return p


def load_sessions(path, cli=None):
    """LoadSessions: renderSessions[] resolved against CLI overrides."""
    lib = scene_lib()
    cli = cli if cli is not None else default_params()
    n = lib.nart_load_sessions(path.encode(), ctypes.byref(cli), None, 0)
    if n < 0:
        raise NartError(n, lib.nart_scene_last_error().decode())
    out = (RenderParams * max(n, 1))()
    lib.nart_load_sessions(path.encode(), ctypes.byref(cli), out, n)
    return [out[i].copy() for i in range(n)]


def session_geometry(p):
    g = SessionGeometry()
    scene_lib().nart_session_geometry_of(ctypes.byref(p), ctypes.byref(g))
    return g


def filter_table():
    t = (ctypes.c_float * 64)()
    scene_lib().nart_filter_table(t)
    return np.ctypeslib.as_array(t).copy()


def combine_tiles(p, tiles):
    g = session_geometry(p)
    tiles = np.ascontiguousarray(tiles, dtype=np.float32)
    img = np.zeros((g.total_height, g.total_width, PIXEL_FLOATS), np.float32)
    scene_lib().nart_combine_tiles(ctypes.byref(p), tiles.ctypes.data, img.ctypes.data)
    return img


def write_exr(path, p, image, compression=3):
    image = np.ascontiguousarray(image, dtype=np.float32)
    rc = scene_lib().nart_write_exr(path.encode(), ctypes.byref(p), image.ctypes.data, compression)
    if rc != NART_OK:
        raise NartError(rc, scene_lib().nart_scene_last_error().decode())


def read_exr(path):
    """RGBA halves as float32 array (H, W, 4)."""
    lib = scene_lib()
    w, h, ptr = ctypes.c_uint32(), ctypes.c_uint32(), _P()
    rc = lib.nart_read_exr_rgba(path.encode(), ctypes.byref(w), ctypes.byref(h), ctypes.byref(ptr))
    if rc != NART_OK:
        raise NartError(rc, lib.nart_scene_last_error().decode())
    n = w.value * h.value * 4
    halves = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint16)), shape=(n,)).copy()
    lib.nart_free(ptr)
    return halves.view(np.float16).astype(np.float32).reshape(h.value, w.value, 4)


def bvh_info(scene):
    """Host only: the BVH a render context would build for `scene` (nart_hip_bvh_info)."""
    info = BvhInfo()
    rc = hip_lib().nart_hip_bvh_info(_P(scene.blob), ctypes.byref(info))
    if rc != NART_OK:
        raise NartError(rc, "nart_hip_bvh_info")
    return {"num_nodes": info.num_nodes, "stack_depth": info.stack_depth, "num_leaf_tris": info.num_leaf_tris}


class Scene:
    """Scene::Scene(path): JSON + .geo + EXR ingestion into the flat nart_scene_blob."""

    def __init__(self, path):
        self.path = path
        self._lib = scene_lib()
        self._h = _P()
        rc = self._lib.nart_scene_load(path.encode(), ctypes.byref(self._h))
        if rc != NART_OK:
            raise NartError(rc, self._lib.nart_scene_last_error().decode())
        self.blob = self._lib.nart_scene_blob_of(self._h)

    def counts(self):
        c = ctypes.cast(self.blob, ctypes.POINTER(ctypes.c_uint32))
        return {"triangles": c[0], "meshes": c[1], "materials": c[2], "lights": c[3], "textures": c[4]}

    def _view(self):
        return ctypes.cast(self.blob, ctypes.POINTER(_BlobHead)).contents

    def triangles(self):
        """(n, 24) float32 copy of the blob's triangles (nart_triangle: v0 v1 v2 n0 n1 n2 uv0 uv1 uv2)."""
        h = self._view()
        if not h.num_triangles:
            return np.zeros((0, 24), np.float32)
        return np.ctypeslib.as_array(ctypes.cast(h.triangles, ctypes.POINTER(ctypes.c_float)),
                                     shape=(h.num_triangles * 24,)).copy().reshape(-1, 24)

    def camera(self):
        """(fov, m): the camera's fov and glm::mat4 storage (16 float32; pinholecamera.cpp:3-40)."""
        h = self._view()
        return float(h.cam_fov), np.array(list(h.cam_m), np.float32)

    def textures(self):
        """Loaded textures as (H, W, 4) uint16 half bit patterns (top row first), in load order."""
        h = self._view()
        out = []
        for i in range(h.num_textures):
            t = h.textures[i]
            out.append(np.ctypeslib.as_array(ctypes.cast(t.rgba, ctypes.POINTER(ctypes.c_uint16)),
                                             shape=(t.height * t.width * 4,)).copy().reshape(t.height, t.width, 4))
        return out

    def close(self):
        if self._h:
            self._lib.nart_scene_free(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def scene_features(scene):
    """Host only: the NART_FT_* feature mask a context would derive for the scene (it selects the
    scene-specialised path-kernel build; nart_hip_scene_features_of)."""
    m = ctypes.c_uint32()
    rc = hip_lib().nart_hip_scene_features_of(scene.blob, ctypes.byref(m))
    if rc != NART_OK:
        raise NartError(rc, "nart_hip_scene_features_of")
    return m.value


def shard_buckets(n_buckets_x, n_buckets, n_devices, device_index):
    """Host only: the bucket ids a multi-device context renders on device_index (diagonal lattice,
    nart_hip_shard_buckets; the same partition as nart_amd.dist.bucket_owners)."""
    lib = hip_lib()
    cnt = ctypes.c_uint32()
    rc = lib.nart_hip_shard_buckets(n_buckets_x, n_buckets, n_devices, device_index, None, ctypes.byref(cnt))
    if rc != NART_OK:
        raise NartError(rc, "nart_hip_shard_buckets")
    ids = np.zeros(max(1, cnt.value), np.uint32)
    lib.nart_hip_shard_buckets(n_buckets_x, n_buckets, n_devices, device_index,
                               ids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(cnt))
    return ids[:cnt.value]


class HipRenderer:
    """nart_ctx: the scene resident on one GPU (device) or on several (devices=[...], one
    process, library-owned RCCL gather: nart_hip_create_multi); Render()-equivalent entry points."""

    def __init__(self, scene, device=0, variant=None, splat_mode=None, devices=None):
        self._lib = hip_lib()
        self.scene = scene
        self.device = device if devices is None else devices[0]
        self._ctx = _P()
        if devices is None:
            rc = self._lib.nart_hip_create(scene.blob, device, ctypes.byref(self._ctx))
        else:
            arr = (ctypes.c_int * len(devices))(*devices)
            rc = self._lib.nart_hip_create_multi(scene.blob, arr, len(devices), ctypes.byref(self._ctx))
        if rc != NART_OK:
            raise NartError(rc, "nart_hip_create failed on device(s) %s" % (devices if devices is not None else device))
        if variant is not None:
            self.set_variant(variant)
        if splat_mode is not None:
            self.set_splat_mode(splat_mode)

    def set_variant(self, variant):
        """0 = megakernel with a wave ray queue (default), 3 = megakernel with one lane per pixel;
        identical results (1, the wavefront variant, and 2, the traversal-quorum megakernel, were
        retired)."""
        self._check(self._lib.nart_hip_set_variant(self._ctx, int(variant)))

    def set_splat_mode(self, mode):
        """-1 = automatic (default: the skewed-time splat on launches of >= 1 wave per SIMD, else
        its W-lanes-per-column form), 5 = skewed time with W lanes per tile column, 4 = skewed-time
        splat, 3 = four tile pixels per lane, 1-0 = one pixel per lane (include/nart_hip.h);
        identical results."""
        self._check(self._lib.nart_hip_set_splat_mode(self._ctx, int(mode)))

    def set_specialize(self, mode):
        """Path-kernel builds: 0 (or False) the generic build, 1 the scene-specialised builds, 2 (or
        True, the default) those plus the lean three-waves-per-SIMD build of throughput-bound
        launches; identical results (nart_hip_set_specialize)."""
        self._check(self._lib.nart_hip_set_specialize(self._ctx, int(mode) if not isinstance(mode, bool)
                                                      else (2 if mode else 0)))

    def scene_features(self):
        """(the scene's feature mask, the mask of the path-kernel build the last render launched;
        FT_ALL = generic), NART_FT_* bits (nart_hip_scene_features)."""
        f, b = ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self._lib.nart_hip_scene_features(self._ctx, ctypes.byref(f), ctypes.byref(b)))
        return f.value, b.value

    def _check(self, rc):
        if rc != NART_OK:
            raise NartError(rc, self._lib.nart_hip_last_error(self._ctx).decode())

    def bvh(self):
        """The acceleration structure this context built (nart_hip_context_bvh)."""
        info, ms = BvhInfo(), ctypes.c_double()
        self._check(self._lib.nart_hip_context_bvh(self._ctx, ctypes.byref(info), ctypes.byref(ms)))
        return {"num_nodes": info.num_nodes, "stack_depth": info.stack_depth, "num_leaf_tris": info.num_leaf_tris,
                "on_device": bool(info.reserved), "build_ms": ms.value}

    def devices(self):
        """(number of devices, gather over RCCL) of this context."""
        n, r = ctypes.c_int(), ctypes.c_int()
        self._check(self._lib.nart_hip_context_devices(self._ctx, ctypes.byref(n), ctypes.byref(r)))
        return n.value, r.value == 1

    def gather_mode(self):
        """"rccl", "copy", or "copy-fallback" (RCCL requested implicitly but unavailable)."""
        n, r = ctypes.c_int(), ctypes.c_int()
        self._check(self._lib.nart_hip_context_devices(self._ctx, ctypes.byref(n), ctypes.byref(r)))
        return {1: "rccl", 0: "copy", 2: "copy-fallback"}[r.value]

    def debug_fault(self, fault):
        """Test hook (nart_hip_debug_fault): 1 = the next RCCL gather posts an invalid peer."""
        self._check(self._lib.nart_hip_debug_fault(self._ctx, int(fault)))

    def set_counters(self, on):
        self._check(self._lib.nart_hip_set_counters(self._ctx, 1 if on else 0))

    def render(self, p, stats=None):
        """Whole session -> (totalH, totalW, 5) float32 image of Pixels (host)."""
        g = session_geometry(p)
        img = np.empty((g.total_height, g.total_width, PIXEL_FLOATS), np.float32)
        st = stats if stats is not None else RenderStats()
        self._check(self._lib.nart_hip_render(self._ctx, ctypes.byref(p), img.ctypes.data, ctypes.byref(st)))
        return img

    def render_device(self, p, stats=None):
        """Whole session, image left on the (first) device: returns its device address (totalH x
        totalW x 5 float32, owned by the context until the next render).  Multi-device contexts
        gather over their RCCL send/receive group first (nart_hip_render_device)."""
        st = stats if stats is not None else RenderStats()
        ptr = _P()
        self._check(self._lib.nart_hip_render_device(self._ctx, ctypes.byref(p), ctypes.byref(ptr), ctypes.byref(st)))
        return ptr.value

    def render_buckets_async(self, p, bucket_ids, d_tiles_ptr, stream_ptr=0, stats=None):
        ids = np.ascontiguousarray(bucket_ids, dtype=np.uint32)
        st = stats if stats is not None else RenderStats()
        self._check(self._lib.nart_hip_render_buckets_async(
            self._ctx, ctypes.byref(p), ids.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), len(ids),
            _P(d_tiles_ptr), _P(stream_ptr), ctypes.byref(st)))
        return st

    def combine_async(self, p, d_tiles_ptr, d_image_ptr, stream_ptr=0):
        self._check(self._lib.nart_hip_combine_async(self._ctx, ctypes.byref(p), _P(d_tiles_ptr), _P(d_image_ptr),
                                                     _P(stream_ptr)))

    def render_samples(self, p, x0, y0, w, h):
        out = np.empty((h, w, p.spp, 4), np.float32)
        self._check(self._lib.nart_hip_render_samples(self._ctx, ctypes.byref(p), x0, y0, w, h, out.ctypes.data))
        return out

    def eval_sincos(self, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        s = np.empty_like(x)
        c = np.empty_like(x)
        self._check(self._lib.nart_hip_eval_sincos(self._ctx, x.ctypes.data, len(x), s.ctypes.data, c.ctypes.data))
        return s, c

    def close(self):
        if self._ctx:
            self._lib.nart_hip_destroy(self._ctx)
            self._ctx = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def finalize(p, image):
    """WriteImageToEXR's per-pixel result = contribution / filterWeightSum (render.cpp:213-222)."""
    g = session_geometry(p)
    fb = g.filter_bounds
    crop = image[fb:fb + p.image_height, fb:fb + p.image_width]
    with np.errstate(divide="ignore", invalid="ignore"):
        return crop[..., :4] / crop[..., 4:5]
