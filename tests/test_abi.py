"""C ABI surface: both libraries load on a CPU-only host and export every function that
include/*.h declares (no compute calls: those need a GPU)."""
import ctypes
import os
import re

import nart_amd
from nart_amd import build as nb

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    text = open(os.path.join(REPO, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nart_\w+)\s*\(", text)))


def test_scene_lib_exports_header(built):
    lib = ctypes.CDLL(nb.build_scene_lib())
    names = declared("nart_scene.h")
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_hip_lib_exports_header(built):
    lib = ctypes.CDLL(nb.build_hip_lib())
    names = declared("nart_hip.h")
    assert len(names) >= 10
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_python_bindings_cover_abi(built):
    assert set(declared("nart_scene.h")) == set(nart_amd.SCENE_SYMBOLS)
    assert set(declared("nart_hip.h")) == set(nart_amd.HIP_SYMBOLS)


def test_hip_create_without_gpu_fails_cleanly(built, glass_scene):
    import torch
    if torch.cuda.is_available():
        return
    try:
        nart_amd.HipRenderer(glass_scene)
    except nart_amd.NartError as e:
        assert e.code == -3  # NART_E_HIP, no abort
    else:
        raise AssertionError("render context created without a GPU")


def test_splat_thresholds_reproduce_filter_index(built):
    """The splat's filter index from d2 thresholds equals AddSample's
    uint8((sqrt(d2) / fw) * 64) clamped to 63 (render.cpp:43-49), float32 throughout."""
    import numpy as np
    lib = nart_amd.api.hip_lib()
    rng = np.random.default_rng(7)
    for fw in (2.0, 1.5, 0.5, 1.0, 3.0, 0.75):
        thr = np.zeros(65, np.float32)
        assert lib.nart_hip_splat_thresholds(ctypes.c_float(fw), thr.ctypes.data) == 0
        hmax = np.float32(fw + 0.5)
        d2max = np.float32(2) * hmax * hmax
        d2 = np.concatenate([rng.uniform(0, d2max, 400000).astype(np.float32), thr[1:64],
                             np.nextafter(thr[1:64], np.float32(0)), np.float32([0.0, d2max])])
        d2 = d2[np.isfinite(d2) & (d2 <= d2max)]
        dist = np.sqrt(d2)
        q = (dist / np.float32(fw)).astype(np.float32) * np.float32(64)
        want = np.minimum(63, q.astype(np.int32) & 0xFF)
        got = np.searchsorted(thr[1:64], d2, side="right")  # #{k in 1..63: d2 >= thr[k]}
        assert np.array_equal(got, want), fw
    thr = np.zeros(65, np.float32)
    assert lib.nart_hip_splat_thresholds(ctypes.c_float(0.1), thr.ctypes.data) != 0


def test_bvh_depth_cap(built, glass_scene, monkeypatch):
    """Host BVH build (nart_hip_bvh_info, no device): binned SAH, and from NART_BVH_MEDIAN_DEPTH
    on object-median splits, which bound the traversal stack (LDS) by that depth plus
    log2(triangles / leaf size) -- the guard against SAH peeling one bin per level off clustered
    geometry.  glassSphere: 2,560 triangles, all visible to the reference octree."""
    import math
    info = nart_amd.bvh_info(glass_scene)
    assert info["num_leaf_tris"] == 2560
    assert 2 <= info["stack_depth"] <= 72
    for md in (1, 2, 5):
        monkeypatch.setenv("NART_BVH_MEDIAN_DEPTH", str(md))
        capped = nart_amd.bvh_info(glass_scene)
        assert capped["num_leaf_tris"] == 2560
        assert capped["stack_depth"] <= md + math.ceil(math.log2(2560 / 4)) + 2, (md, capped)


def test_multi_device_shard_partition(built):
    """nart_hip_shard_buckets (host only): the multi-device context's buckets per device partition
    the frame (every bucket exactly once, ascending per device), and the C ABI deals exactly as the
    one-process-per-GPU path does (nart_amd.dist.bucket_owners)."""
    import numpy as np
    from nart_amd.dist import bucket_owners
    for nbx, nb_, n in [(120, 8160, 8), (5, 15, 2), (7, 7, 4), (3, 3, 8), (240, 32400, 8), (1, 1, 1), (13, 104, 6)]:
        parts = [nart_amd.shard_buckets(nbx, nb_, n, d) for d in range(n)]
        allb = np.concatenate(parts)
        assert np.array_equal(np.sort(allb), np.arange(nb_))
        owners = bucket_owners(nbx, nb_, n)
        for d, ids in enumerate(parts):
            assert np.array_equal(ids, np.nonzero(owners == d)[0]) and np.all(np.diff(ids.astype(np.int64)) > 0)


def test_shard_spreads_regions_evenly():
    """Every block of the bucket grid (e.g. the C3 glass region) splits over 8 devices within a
    bucket or two per device, unlike b % 8 (whole stripes: a 4-bucket-wide column on 4 devices)."""
    import numpy as np
    from nart_amd.dist import bucket_owners
    nbx, nby = 120, 68
    b = np.arange(nbx * nby)
    lat, mod = bucket_owners(nbx, nbx * nby, 8), bucket_owners(nbx, nbx * nby, 8, "mod")
    for x0, x1, y0, y1 in [(40, 80, 20, 60), (50, 70, 30, 50), (58, 62, 40, 50), (0, 120, 0, 68)]:
        region = (b % nbx >= x0) & (b % nbx < x1) & (b // nbx >= y0) & (b // nbx < y1)
        per = np.bincount(lat[region], minlength=8)
        assert per.max() - per.min() <= 2, per
    region = (b % nbx >= 58) & (b % nbx < 62)
    assert np.bincount(mod[region], minlength=8).min() == 0


def test_multi_device_create_without_gpu_fails_cleanly(built, glass_scene):
    import ctypes as C
    lib = nart_amd.hip_lib()
    ctx = C.c_void_p()
    devs = (C.c_int * 2)(0, 1)
    rc = lib.nart_hip_create_multi(C.c_void_p(glass_scene.blob), devs, 2, C.byref(ctx))
    assert rc != 0 and not ctx.value
    cnt = C.c_int(-1)
    lib.nart_hip_device_count(C.byref(cnt))
    assert cnt.value == 0


def test_splat_weight_cells_reproduce_filter_weight(built):
    """The splat's weight-by-d2-cell table (nart_hip_splat_lut, k_splat_col4): for every d2 a hit can
    have, table[AddSample's filter index] (render.cpp:43-50) equals the cell lookup
    w = d2 >= t ? w_hi : w_lo with cell = clamp((bits(d2) >> 16) - b0, 0, n - 1)."""
    import numpy as np
    lib = nart_amd.api.hip_lib()
    table = nart_amd.filter_table()
    rng = np.random.default_rng(11)
    for fw in (2.0, 1.5, 0.5, 1.0, 3.0, 0.75):
        cells = np.zeros((2048, 4), np.float32)
        n, b0 = ctypes.c_uint32(), ctypes.c_uint32()
        assert lib.nart_hip_splat_lut(ctypes.c_float(fw), cells.ctypes.data, ctypes.byref(n), ctypes.byref(b0)) == 0
        cells = cells[:n.value]
        thr = np.zeros(65, np.float32)
        lib.nart_hip_splat_thresholds(ctypes.c_float(fw), thr.ctypes.data)
        hmax = np.float32(fw + 0.5)
        d2max = np.float32(2) * hmax * hmax
        edges = ((np.arange(n.value, dtype=np.uint32) + b0.value) << 16).view(np.float32)
        d2 = np.concatenate([rng.uniform(0, d2max, 400000).astype(np.float32), thr[1:64],
                             np.nextafter(thr[1:64], np.float32(0)), edges, np.nextafter(edges, np.float32(0)),
                             np.float32([0.0, 1e-30, d2max])])
        d2 = d2[np.isfinite(d2) & (d2 <= d2max) & (d2 >= 0)]
        q = (np.sqrt(d2) / np.float32(fw)).astype(np.float32) * np.float32(64)
        want = table[np.minimum(63, q.astype(np.int32) & 0xFF)]
        c = np.clip((d2.view(np.uint32) >> 16).astype(np.int64) - b0.value, 0, n.value - 1)
        e = cells[c]
        got = np.where(d2 >= e[:, 0], e[:, 2], e[:, 1])
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), fw


def _env_search(v, values):
    import numpy as np
    lib = nart_amd.api.hip_lib()
    v = np.ascontiguousarray(v, np.float32)
    values = np.ascontiguousarray(values, np.float32)
    full = np.zeros(len(values), np.uint32)
    guided = np.zeros(len(values), np.uint32)
    rc = lib.nart_hip_env_search(v.ctypes.data, len(v), values.ctypes.data, len(values), full.ctypes.data,
                                 guided.ctypes.data)
    assert rc >= 0
    return rc == 1, full, guided


def test_env_guided_search_matches_binary_search(built):
    """The environment light's guided CDF search (path.h guided_search + render.hip env_guide,
    ADVICE r04) returns BinarySearch's index (util.cpp:4-20) for every value: regular CDFs,
    plateaus (zero-pdf texels), one-entry ranges (1xN / Nx1 maps), values on guide-cell edges, on
    CDF entries and outside [0, 1); a non-monotone or NaN range gets no guide table (full search)."""
    import numpy as np
    rng = np.random.default_rng(5)
    K = 64
    edges = np.arange(K + 1, dtype=np.float32) / np.float32(K)
    probes = np.concatenate([edges, np.nextafter(edges, np.float32(0)), np.nextafter(edges, np.float32(2)),
                             rng.uniform(0, 1, 4000).astype(np.float32),
                             np.float32([0.0, -0.0, 1.0, 0.9999999, 1.5, -0.25, 1e-30, np.nan])])
    cases = []
    for n in (1, 2, 3, 7, 64, 65, 513, 1024):
        pdf = rng.exponential(1.0, n).astype(np.float32)
        pdf[rng.uniform(size=n) < 0.3] = 0.0                     # plateaus
        c = np.concatenate([[0.0], np.cumsum(pdf[:-1] / pdf.sum(), dtype=np.float32)]).astype(np.float32)
        cases.append(("cdf%d" % n, c, True))
    cases.append(("one-entry", np.float32([0.0]), True))
    cases.append(("all-equal", np.full(9, 0.5, np.float32), True))
    cases.append(("non-monotone", np.float32([0.0, 0.5, 0.4, 0.9]), False))
    cases.append(("nan-row", np.float32([0.0, np.nan, 0.6, 0.9]), False))
    cases.append(("nan-first", np.float32([np.nan, 0.2, 0.6]), False))
    for name, v, want_guide in cases:
        vals = np.concatenate([probes, v, np.nextafter(v, np.float32(-1)), np.nextafter(v, np.float32(2))])
        built_guide, full, guided = _env_search(v, vals)
        assert built_guide == want_guide, name
        assert np.array_equal(full, guided), (name, np.nonzero(full != guided)[0][:8])
