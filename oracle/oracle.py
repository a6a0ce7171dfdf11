"""ctypes wrapper of the CPU restatement (oracle/nart_oracle.c).  TEST INFRASTRUCTURE ONLY:
imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
product path.  PARITY UNPINNED (see nart_oracle.h)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libnart_oracle.so")

_lib = None


def default_threads():
    """One worker per host core, capped at 16 (the GPU box's CPU share per GPU)."""
    return max(1, min(16, os.cpu_count() or 1))


REF_LIB = os.path.join(HERE, "_ref", "libref_util.so")
REF_SRC = os.environ.get("NART_REFERENCE", "/root/reference")


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])
    build_ref()
    return LIB


def build_ref():
    """oracle/_ref/libref_util.so: the reference's own util.cpp (BinarySearch), compiled in place
    from the reference checkout when it is present (this container; the GPU box gets the built
    file with the tree).  Returns the path, or None without the reference."""
    if os.path.exists(os.path.join(REF_SRC, "src", "core", "util.cpp")):
        subprocess.check_call(["make", "-s", "-C", HERE, "ref", "REF=" + REF_SRC])
    return REF_LIB if os.path.exists(REF_LIB) else None


def ref_binary_search():
    """The reference's BinarySearch (util.cpp:4-20) as f(value, cdf, start, end), or None."""
    if not os.path.exists(REF_LIB):
        return None
    ref = ctypes.CDLL(REF_LIB)
    ref.ref_binary_search.restype = ctypes.c_uint32
    ref.ref_binary_search.argtypes = [ctypes.c_float, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_uint32]

    def f(value, cdf, start, end):
        cdf = np.ascontiguousarray(cdf, np.float32)
        return ref.ref_binary_search(float(value), cdf.ctypes.data, len(cdf), start, end)
    return f


def binary_search(value, cdf, start, end):
    """The oracle's restatement of BinarySearch (nart_oracle.c)."""
    cdf = np.ascontiguousarray(cdf, np.float32)
    return lib().oracle_binary_search(float(value), cdf.ctypes.data, start, end)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        _lib.oracle_create.argtypes = [P, ctypes.POINTER(P)]
        _lib.oracle_destroy.argtypes = [P]
        _lib.oracle_render.argtypes = [P, P, P, ctypes.c_int]
        _lib.oracle_render_buckets.argtypes = [P, P, P, ctypes.c_uint32, P, ctypes.c_int]
        _lib.oracle_render_samples.argtypes = [P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.c_uint32, P, P]
        _lib.oracle_bvh_stats.argtypes = [P, P, P, P, P]
        _lib.oracle_rng_stream.argtypes = [ctypes.c_uint32, ctypes.c_uint32, P]
        _lib.oracle_latin_square.argtypes = [ctypes.c_uint32, ctypes.c_uint32, P, P]
        _lib.oracle_fresnel.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_float]
        _lib.oracle_fresnel.restype = ctypes.c_float
        _lib.oracle_binary_search.argtypes = [ctypes.c_float, P, ctypes.c_uint32, ctypes.c_uint32]
        _lib.oracle_binary_search.restype = ctypes.c_uint32
        _lib.oracle_max_list.argtypes = [ctypes.c_int]
        _lib.oracle_max_list.restype = ctypes.c_uint32
        _lib.oracle_camera_ray.argtypes = [P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_float, ctypes.c_float, P, P]
        _lib.oracle_trace.argtypes = [P, P, P, ctypes.c_float, P]
    return _lib


class Oracle:
    def __init__(self, scene):
        self.scene = scene  # keeps the blob alive
        self._h = ctypes.c_void_p()
        rc = lib().oracle_create(ctypes.c_void_p(scene.blob), ctypes.byref(self._h))
        if rc:
            raise RuntimeError("oracle_create failed: %d" % rc)

    def render(self, p, threads=None):
        from nart_amd import session_geometry
        g = session_geometry(p)
        img = np.zeros((g.total_height, g.total_width, 5), np.float32)
        rc = lib().oracle_render(self._h, ctypes.byref(p), img.ctypes.data, threads or default_threads())
        if rc:
            raise RuntimeError("oracle_render failed: %d" % rc)
        return img

    def render_buckets(self, p, ids, threads=None):
        from nart_amd import session_geometry
        g = session_geometry(p)
        ids = np.ascontiguousarray(ids, np.uint32)
        tiles = np.zeros((len(ids), g.tile_size * g.tile_size, 5), np.float32)
        rc = lib().oracle_render_buckets(self._h, ctypes.byref(p), ids.ctypes.data, len(ids), tiles.ctypes.data,
                                         threads or default_threads())
        if rc:
            raise RuntimeError("oracle_render_buckets failed: %d" % rc)
        return tiles

    def render_samples(self, p, x0, y0, w, h, with_uv=False):
        out = np.zeros((h, w, p.spp, 4), np.float32)
        uv = np.zeros((h, w, p.spp, 2), np.float32) if with_uv else None
        rc = lib().oracle_render_samples(self._h, ctypes.byref(p), x0, y0, w, h, out.ctypes.data,
                                         uv.ctypes.data if with_uv else None)
        if rc:
            raise RuntimeError("oracle_render_samples failed: %d" % rc)
        return (out, uv) if with_uv else out

    def bvh_stats(self):
        nc, mx, rl = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        gr = (ctypes.c_uint32 * 4)()
        lib().oracle_bvh_stats(self._h, ctypes.byref(nc), ctypes.byref(mx), ctypes.byref(rl), gr)
        return {"chunks": nc.value, "max_chunk_tris": mx.value, "root_is_leaf": bool(rl.value),
                "grid": tuple(gr[:3]), "reachable_tris": gr[3]}

    def __del__(self):
        try:
            if self._h:
                lib().oracle_destroy(self._h)
        except Exception:
            pass


def rng_stream(seed, n):
    out = np.zeros(n, np.float32)
    lib().oracle_rng_stream(seed, n, out.ctypes.data)
    return out


def latin_square(seed, spp):
    out = np.zeros((spp, 2), np.float32)
    st = ctypes.c_uint32()
    lib().oracle_latin_square(seed, spp, out.ctypes.data, ctypes.byref(st))
    return out, st.value


def fresnel(eta_o, eta_i, c):
    return lib().oracle_fresnel(eta_o, eta_i, c)


def camera_ray(orc, W, H, x, y, u, v):
    """Debug aid: the oracle's camera ray for pixel (x, y), sample (u, v)."""
    o = (ctypes.c_float * 3)()
    d = (ctypes.c_float * 3)()
    lib().oracle_camera_ray(orc._h, W, H, x, y, ctypes.c_float(u), ctypes.c_float(v), o, d)
    return np.array(o[:], np.float32), np.array(d[:], np.float32)


def trace(orc, o, d, tmax=float("inf")):
    """Debug aid: (octree triangle, t, brute-force triangle, t) for one ray."""
    o = np.ascontiguousarray(o, np.float32)
    d = np.ascontiguousarray(d, np.float32)
    out = (ctypes.c_int32 * 4)()
    lib().oracle_trace(orc._h, o.ctypes.data, d.ctypes.data, ctypes.c_float(tmax), out)
    t0 = np.array([out[1]], np.int32).view(np.float32)[0]
    t1 = np.array([out[3]], np.int32).view(np.float32)[0]
    return out[0], float(t0), out[2], float(t1)


def max_list_length(reset=False):
    """Longest nested-dielectric list (pathintegrator.h:9-19) any oracle path reached."""
    return int(lib().oracle_max_list(1 if reset else 0))
