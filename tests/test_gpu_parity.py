"""GPU parity: the HIP render path against the CPU restatement (oracle/), bit for bit.

Parity bar: per-sample Li_alpha and the whole float32 framebuffer before the
half conversion must be bit-identical to the oracle on the same scene and per-pixel seeds.
Where an exact closest-hit tie is broken differently ("ties"), the tests report
the count of differing samples and require it to be zero at these sizes.
"""
import numpy as np
import pytest

import nart_amd
import oracle

pytestmark = pytest.mark.gpu


def _params(scene, w, h, spp, **kw):
    p = nart_amd.load_sessions(scene.path)[0]
    p.image_width, p.image_height, p.spp = w, h, spp
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


def _report(a, b):
    ne = a.view(np.uint32) != b.view(np.uint32)
    return "%d of %d floats differ, max abs diff %g" % (int(ne.sum()), ne.size, float(np.nanmax(np.abs(a - b))))


# ray-queue megakernel (default) and the one-lane-per-pixel megakernel (the fallback for deep
# BVHs; the wavefront variant was retired in round 3, the traversal-quorum variant in round 5)
VARIANTS = [0, 3]
VARIANT_IDS = ["rayqueue", "megakernel"]


@pytest.fixture(scope="module", params=VARIANTS, ids=VARIANT_IDS)
def glass_gpu(request, gpu, glass_scene):
    return nart_amd.HipRenderer(glass_scene, variant=request.param)


@pytest.fixture(scope="module")
def glass_oracle(glass_scene):
    return oracle.Oracle(glass_scene)


def test_device_sincos_matches_host_glibc(glass_gpu):
    """Device sinf/cosf port vs this host's glibc sinf/cosf (the reference's glm::sin/cos)."""
    import ctypes
    libm = ctypes.CDLL("libm.so.6")
    for f in (libm.sinf, libm.cosf):
        f.restype = ctypes.c_float
        f.argtypes = [ctypes.c_float]
    bits = np.arange(0, np.float32(6.2831855).view(np.uint32) + 1, 4099, dtype=np.uint32)
    x = bits.view(np.float32)
    x = np.concatenate([x, -x[::5], np.float32([6.2831855, 1e-30, 0.7853981, 0.7853982])]).astype(np.float32)
    s, c = glass_gpu.eval_sincos(x)
    hs = np.array([libm.sinf(float(v)) for v in x], np.float32)
    hc = np.array([libm.cosf(float(v)) for v in x], np.float32)
    assert _bits_equal(s, hs), _report(s, hs)
    assert _bits_equal(c, hc), _report(c, hc)


@pytest.mark.parametrize("rect", [(60, 40, 12, 12), (120, 100, 16, 8), (0, 0, 8, 8), (250, 255, 10, 5)])
def test_per_sample_glass_sphere(glass_gpu, glass_oracle, glass_scene, rect):
    """Li_alpha of every sample of a pixel block (sphere, backdrop, image corner, extra rows)."""
    p = _params(glass_scene, 256, 256, 16)
    x0, y0, w, h = rect
    g = glass_gpu.render_samples(p, x0, y0, w, h)
    r = glass_oracle.render_samples(p, x0, y0, w, h)
    assert _bits_equal(g, r), _report(g, r)


def test_framebuffer_glass_sphere_64(glass_gpu, glass_oracle, glass_scene):
    p = _params(glass_scene, 64, 64, 4)
    g = glass_gpu.render(p)
    r = glass_oracle.render(p)
    assert _bits_equal(g, r), _report(g, r)


def test_framebuffer_glass_sphere_c1(glass_gpu, glass_oracle, glass_scene):
    """C1: glassSphere 256x256 @ 16 spp (BASELINE.json configs[0])."""
    p = _params(glass_scene, 256, 256, 16)
    g = glass_gpu.render(p)
    r = glass_oracle.render(p)
    assert _bits_equal(g, r), _report(g, r)
    res = nart_amd.finalize(p, g)
    assert np.isfinite(res).all()


@pytest.mark.parametrize("w,h,spp,prio", [(1024, 576, 2, "1"), (1024, 576, 2, "2"), (512, 400, 2, "1"), (512, 400, 6, "1")],
                         ids=["k32", "k32-prio", "k8", "k8-6spp"])
def test_queue_scheduler_frames(gpu, glass_scene, monkeypatch, w, h, spp, prio):
    """More traced pixels than resident lanes: the megakernel runs the cost probe, the costly
    pixels are spread over the persistent waves and finished lanes refill from the queue
    (render.hip launch_render); in the ray-queue kernel they are priority lanes whose rays are
    traced first (small shards; NART_RQ_PRIO=2 forces them on at >= 3 rounds, k32-prio: 32
    costly pixels per wave as speculative pairs filling whole waves).  Only the order of work
    changes; the frame must not."""
    monkeypatch.setenv("NART_RQ_PRIO", prio)
    p = _params(glass_scene, w, h, spp)
    g = nart_amd.HipRenderer(glass_scene, variant=0).render(p)
    r = oracle.Oracle(glass_scene).render(p)
    assert _bits_equal(g, r), _report(g, r)


@pytest.mark.parametrize("pairs,extra", [("2", ""), ("4", ""), ("0", ""), ("2", "NART_RQ_QUAD=1"), ("2", "NART_RQ_HALF=0"),
                                         ("2", "NART_RQ_SETPRIO=0")],
                         ids=["speculative-pairs", "speculative-quads", "single-lanes", "quad-top", "all-waves",
                              "no-setprio"])
def test_queue_speculative_pairs(gpu, glass_scene, monkeypatch, pairs, extra):
    """A shard of ~1.2 rounds of resident waves at 24 spp: the costliest pixels run as speculative
    lane pairs (one lane on the chain's frontier sample, the other on the next sample from a
    predicted RNG state; kept only when the prediction was exact).  Long enough chains for both
    kept and dropped speculation; the frame must equal the oracle's bit for bit.  The default puts
    the costly pixels on one wave per SIMD at raised issue priority; variants: four lanes for every
    costly pixel, four for each first-round wave's costliest pixel only (NART_RQ_QUAD), the costly
    pixels dealt over every wave (NART_RQ_HALF=0), no raised priority (NART_RQ_SETPRIO=0)."""
    monkeypatch.setenv("NART_RQ_PAIRS", pairs)
    if extra:
        monkeypatch.setenv(*extra.split("="))
    p = _params(glass_scene, 512, 300, 24)
    g = nart_amd.HipRenderer(glass_scene, variant=0).render(p)
    r = oracle.Oracle(glass_scene).render(p)
    assert _bits_equal(g, r), _report(g, r)


@pytest.fixture(scope="module")
def full_frame_1spp(glass_scene):
    """The C3 frame size at 1 spp: ~16 rounds of resident waves, so the ray-queue kernel runs its
    wave-group refill (render.hip launch_render, R >= 12)."""
    p = _params(glass_scene, 1920, 1080, 1)
    return p, oracle.Oracle(glass_scene).render(p)


@pytest.mark.parametrize("order", ["0", "1", "2"], ids=["slot-order", "costliest-first", "top-class-first"])
def test_group_refill_order(gpu, glass_scene, full_frame_1spp, monkeypatch, order):
    """Wave-group refill on a full frame with the groups taken in slot order, costliest first
    (cost probe + sort), or the costliest NART_RQ_TOPF % first: only the order of work
    changes, so the frame must equal the oracle's bit for bit."""
    monkeypatch.setenv("NART_RQ_ORDER", order)
    monkeypatch.setenv("NART_RQ_TOPF", "15")
    p, r = full_frame_1spp
    g = nart_amd.HipRenderer(glass_scene, variant=0).render(p)
    assert _bits_equal(g, r), _report(g, r)


@pytest.mark.parametrize("sub", ["1", "8", "64"], ids=["probe-1-per-group", "probe-8-per-group", "probe-every-pixel"])
def test_group_probe_sampling(gpu, glass_scene, full_frame_1spp, monkeypatch, sub):
    """The wave-group order's cost probe samples NART_PROBE_SUB pixels of each 64-slot group (8 by
    default on launches of >= 12 rounds): the estimate only orders the groups, so every setting
    renders the oracle's frame bit for bit, on the wave-group path."""
    monkeypatch.setenv("NART_PROBE_SUB", sub)
    p, r = full_frame_1spp
    st = nart_amd.RenderStats()
    g = nart_amd.HipRenderer(glass_scene, variant=0).render(p, st)
    assert "wave_groups" in st.schedule_names(), st.schedule_names()
    assert _bits_equal(g, r), _report(g, r)


def test_queue_scheduler_environment(gpu, env_scene):
    p = _params(env_scene, 480, 300, 2)
    g = nart_amd.HipRenderer(env_scene, variant=0).render(p)
    r = oracle.Oracle(env_scene).render(p)
    assert _bits_equal(g, r), _report(g, r)


def test_framebuffer_ragged_buckets(glass_gpu, glass_oracle, glass_scene):
    """Image not a multiple of the bucket size: extra traced rows/cols (render.cpp:164-168)."""
    p = _params(glass_scene, 50, 37, 3, bucket_size=16, filter_width=1.5, bounces=7)
    g = glass_gpu.render(p)
    r = glass_oracle.render(p)
    assert _bits_equal(g, r), _report(g, r)


@pytest.mark.parametrize("variant", VARIANTS, ids=VARIANT_IDS)
def test_cornell_box(gpu, cornell_scene, variant):
    p = _params(cornell_scene, 96, 64, 8)
    g = nart_amd.HipRenderer(cornell_scene, variant=variant).render(p)
    r = oracle.Oracle(cornell_scene).render(p)
    assert _bits_equal(g, r), _report(g, r)


@pytest.mark.parametrize("variant", VARIANTS, ids=VARIANT_IDS)
def test_materials_scene(gpu, materials_scene, variant):
    """All five material types, textured rho_d / roughness / normal maps (EXR via the ZIP reader),
    ring + disk lights, nested dielectrics with priorities (scenes.materials)."""
    p = _params(materials_scene, 160, 120, 8)
    g = nart_amd.HipRenderer(materials_scene, variant=variant).render(p)
    r = oracle.Oracle(materials_scene).render(p)
    assert _bits_equal(g, r), _report(g, r)


def test_materials_per_sample(gpu, materials_scene):
    p = _params(materials_scene, 320, 240, 16)
    g = nart_amd.HipRenderer(materials_scene).render_samples(p, 140, 120, 24, 16)
    r = oracle.Oracle(materials_scene).render_samples(p, 140, 120, 24, 16)
    assert _bits_equal(g, r), _report(g, r)


@pytest.mark.parametrize("variant", VARIANTS, ids=VARIANT_IDS)
@pytest.mark.parametrize("which", ["textured", "constant"])
def test_environment_light(gpu, env_scene, env_const_scene, variant, which):
    """Environment light (environmentlight.cpp:9-79): lat-long Li via the glibc acosf/atan2f
    ports, Piecewise2DDistribution importance sampling (textured Le) or the constant pattern;
    textured + normal-mapped plastic, rough glass, textured ground."""
    sc = env_scene if which == "textured" else env_const_scene
    p = _params(sc, 128, 72, 8)
    g = nart_amd.HipRenderer(sc, variant=variant).render(p)
    r = oracle.Oracle(sc).render(p)
    assert _bits_equal(g, r), _report(g, r)


def test_environment_per_sample(gpu, env_scene):
    p = _params(env_scene, 320, 180, 16)
    g = nart_amd.HipRenderer(env_scene).render_samples(p, 60, 60, 32, 24)
    r = oracle.Oracle(env_scene).render_samples(p, 60, 60, 32, 24)
    assert _bits_equal(g, r), _report(g, r)


@pytest.mark.parametrize("kind", ["c5", "emissive"])
def test_volume_integrator(gpu, volume_scenes, kind):
    """VolumeIntegrator::Li_alpha (volumeintegrator.cpp): delta tracking with the width-1
    majorant grid, trilinear density, absorption/emission, isotropic scattering (acosf, logf
    ports), escape to the textured environment light."""
    sc = volume_scenes[kind]
    p = _params(sc, 96, 64, 8)
    g = nart_amd.HipRenderer(sc).render(p)
    r = oracle.Oracle(sc).render(p)
    assert _bits_equal(g, r), _report(g, r)


@pytest.mark.parametrize("sparse,rounds", [("64", "2"), ("16", "8"), ("4", "8")],
                         ids=["groups", "sparse16", "sparse4"])
@pytest.mark.parametrize("kind", ["c5", "emissive"])
def test_volume_queue_scheduler(gpu, volume_scenes, monkeypatch, kind, sparse, rounds):
    """More pixels than resident lanes: the volume kernel runs its cost probe (4 samples per
    pixel) and launches the costliest pixel groups first; on small shards the costliest groups run
    as sparse waves (NART_VOL_SPARSE pixels per wave, the other lanes idle; render.hip
    dispatch_volume).  Only the order of work changes."""
    monkeypatch.setenv("NART_VOL_SPARSE", sparse)
    monkeypatch.setenv("NART_VOL_SPARSE_ROUNDS", rounds)
    monkeypatch.setenv("NART_VOL_SPARSE_F", "1.1")  # some groups of this small frame count as costly
    sc = volume_scenes[kind]
    p = _params(sc, 640, 360, 8)
    st = nart_amd.RenderStats()
    g = nart_amd.HipRenderer(sc).render(p, st)
    r = oracle.Oracle(sc).render(p)
    assert _bits_equal(g, r), _report(g, r)
    # the scheduler path under test really ran: the cost-probe queue always (more
    # pixels than resident lanes), the sparse waves when asked for; nart_render_stats.schedule
    names = st.schedule_names()
    assert "vol_queue" in names, names
    assert ("vol_sparse" in names) == (sparse != "64"), names


def test_volume_per_sample(gpu, volume_scenes):
    sc = volume_scenes["c5"]
    p = _params(sc, 320, 180, 32)
    g = nart_amd.HipRenderer(sc).render_samples(p, 140, 70, 16, 12)
    r = oracle.Oracle(sc).render_samples(p, 140, 70, 16, 12)
    assert _bits_equal(g, r), _report(g, r)


@pytest.mark.parametrize("variant", VARIANTS, ids=VARIANT_IDS)
@pytest.mark.parametrize("name", ["ring", "veach"])
def test_reference_scenes_all_sessions(gpu, ref_scenes, name, variant):
    """The reference's own ring.json (every session: roughening 0 / 0.2 / 0.3) and veach.json
    (MIS over four disk lights of different radii, plastic plates with eta 8192)."""
    sc = ref_scenes[name]
    r = nart_amd.HipRenderer(sc, variant=variant)
    o = oracle.Oracle(sc)
    for p in nart_amd.load_sessions(sc.path):
        p.image_width, p.image_height, p.spp = 128, 72, 4
        g = r.render(p)
        ref = o.render(p)
        assert _bits_equal(g, ref), _report(g, ref)


def test_zero_direction_component_ray(gpu, glass_scene):
    """C3 pixel (1352, 136), sample 187 casts a camera ray with d.z == 0 exactly (found by the
    bench's in-run parity check): the slab test must not turn 1/0 into NaN boxes."""
    p = _params(glass_scene, 1920, 1080, 256)
    o = oracle.Oracle(glass_scene)
    _, uv = o.render_samples(p, 1352, 136, 1, 1, with_uv=True)
    _, d = oracle.camera_ray(o, 1920, 1080, 1352, 136, float(uv[0, 0, 187, 0]), float(uv[0, 0, 187, 1]))
    assert d[2] == 0.0
    g = nart_amd.HipRenderer(glass_scene).render_samples(p, 1344, 128, 16, 16)
    r = o.render_samples(p, 1344, 128, 16, 16)
    assert _bits_equal(g, r), _report(g, r)


@pytest.mark.parametrize("bounces", [0, 1, 2, 12, 20])
def test_bounce_limits(glass_gpu, glass_oracle, glass_scene, bounces):
    """Bounce caps (pathintegrator.cpp:165): none, shallow, and the overflow-list builds (> 10)."""
    p = _params(glass_scene, 24, 20, 5, bucket_size=8, bounces=bounces)
    g = glass_gpu.render(p)
    r = glass_oracle.render(p)
    assert _bits_equal(g, r), _report(g, r)


@pytest.mark.parametrize("variant", VARIANTS, ids=VARIANT_IDS)
@pytest.mark.parametrize("bounces", [16, 32])
def test_deep_dielectric_nesting(gpu, tmp_path, variant, bounces):
    """Nested-dielectric lists longer than the 10 entries the path kernels keep in registers
    (pathintegrator.cpp:123-142): 14 concentric glass shells, so paths through the middle push
    11+ entries, which live in the per-lane overflow columns (kernels.h IList<EXT>)."""
    from nart_amd import scenes
    sc = nart_amd.Scene(scenes.nested_glass(str(tmp_path), spp=6, bounces=bounces))
    p = nart_amd.load_sessions(sc.path)[0]
    g = nart_amd.HipRenderer(sc, variant=variant).render(p)
    oracle.max_list_length(reset=True)
    r = oracle.Oracle(sc).render(p)
    assert oracle.max_list_length() > 10  # the overflow entries were really used
    assert _bits_equal(g, r), _report(g, r)


def test_bucket_api_matches_render(gpu, glass_gpu, glass_scene):
    """render_buckets_async in a shuffled order + device combine == render()."""
    import torch
    p = _params(glass_scene, 80, 48, 4)
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    order = np.random.default_rng(1).permutation(nb).astype(np.uint32)
    tiles = torch.zeros((nb, g.tile_size * g.tile_size, 5), dtype=torch.float32, device="cuda")
    glass_gpu.render_buckets_async(p, order, tiles.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    by_id = torch.empty_like(tiles)
    by_id[torch.from_numpy(order.astype(np.int64)).cuda()] = tiles
    img = torch.zeros((g.total_height, g.total_width, 5), dtype=torch.float32, device="cuda")
    glass_gpu.combine_async(p, by_id.data_ptr(), img.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = glass_gpu.render(p)
    assert _bits_equal(img.cpu().numpy(), ref)


# C2 buckets (1920x1080x64) where the reference octree's unpadded slab tests reject the box
# holding the true closest hit (or a shadow blocker): found by tools/full_parity.py c2 before
# device/octree.h reproduced Octree::Intersect's reachability.
C2_OCTREE_BUCKETS = [1356, 1403, 1476, 1700, 1820, 2676, 3203, 4020, 4121, 5083, 5196, 6922, 7286, 7820, 8106]


@pytest.mark.parametrize("variant", VARIANTS, ids=VARIANT_IDS)
def test_octree_boundary_rejections(gpu, cornell_scene, variant):
    import torch
    p = _params(cornell_scene, 1920, 1080, 64)
    g = nart_amd.session_geometry(p)
    ids = np.array(C2_OCTREE_BUCKETS, np.uint32)
    tiles = torch.zeros((len(ids), g.tile_size * g.tile_size, 5), dtype=torch.float32, device="cuda")
    gpu_r = nart_amd.HipRenderer(cornell_scene, variant=variant)
    st = nart_amd.RenderStats()
    gpu_r.set_counters(True)
    gpu_r.render_buckets_async(p, ids, tiles.data_ptr(), torch.cuda.current_stream().cuda_stream, st)
    torch.cuda.synchronize()
    ref = oracle.Oracle(cornell_scene).render_buckets(p, ids)
    got = tiles.cpu().numpy()
    assert _bits_equal(got, ref), _report(got, ref)
    assert st.octree_replays > 0  # the emulation, not luck, decided these buckets


def test_octree_missed_camera_hit_samples(gpu, cornell_scene):
    """C2 pixel (331, 235): the octree misses triangle 465 at t = 3.1 for sample 30's camera ray
    and the reference renders that sample as a miss (alpha 0)."""
    p = _params(cornell_scene, 1920, 1080, 64)
    gs = nart_amd.HipRenderer(cornell_scene).render_samples(p, 328, 232, 8, 8)
    rs = oracle.Oracle(cornell_scene).render_samples(p, 328, 232, 8, 8)
    assert rs[3, 3, 30, 3] == 0.0
    assert _bits_equal(gs, rs), _report(gs, rs)


@pytest.mark.parametrize("spp", [65, 100, 256, 320, 512, 1024, 1040])
def test_latin_square_high_spp(gpu, glass_scene, glass_oracle, spp):
    """LatinSquare beyond the 256-spp LDS kernel: index shuffles in LDS with both arrays (<= 512
    spp) or one array per pass (<= 1024), and the global-memory kernel above that.  Per-sample
    Li_alpha of an 8x8 block (64 slots: the LDS-index kernel's minimum) and a 7x5 block (global
    kernel), bounces 1 so the samples' camera rays carry the Latin-square positions."""
    r = nart_amd.HipRenderer(glass_scene)
    p = _params(glass_scene, 64, 64, spp, bounces=1)
    for x0, y0, w, h in ((20, 20, 8, 8), (3, 50, 7, 5)):
        g = r.render_samples(p, x0, y0, w, h)
        o = glass_oracle.render_samples(p, x0, y0, w, h)
        assert _bits_equal(g, o), _report(g, o)


def test_latin_square_high_spp_frame(gpu, glass_scene, glass_oracle):
    """Bucket layout at 512 spp (LDS-index LatinSquare, sample-major buckets, splat): framebuffer."""
    p = _params(glass_scene, 24, 20, 512, bounces=2)
    g = nart_amd.HipRenderer(glass_scene).render(p)
    o = glass_oracle.render(p)
    assert _bits_equal(g, o), _report(g, o)


@pytest.mark.parametrize("bucket,fw", [(12, 2.0), (16, 1.0), (8, 2.5), (10, 0.75), (16, 3.0), (4, 0.25)])
@pytest.mark.parametrize("splat_mode", [5, 4, 3, 1, 0], ids=["rows", "skew", "col4", "threshold", "direct"])
def test_splat_bucket_and_filter_sizes(gpu, glass_scene, glass_oracle, bucket, fw, splat_mode):
    """Splat arithmetic paths: power-of-two buckets use the compare-only pair test, other sizes
    the direct one; filter widths with threshold-derived indices (fw > ~0.28) and without (0.25);
    the four-pixels-per-lane and one-pixel-per-lane kernels."""
    p = _params(glass_scene, 40, 30, 4, bucket_size=bucket, filter_width=fw, bounces=3)
    g = nart_amd.HipRenderer(glass_scene, splat_mode=splat_mode).render(p)
    o = glass_oracle.render(p)
    assert _bits_equal(g, o), _report(g, o)


@pytest.mark.parametrize("mode,bands", [(4, 1), (4, 2), (5, 0)], ids=["skew1", "skew2", "rows"])
@pytest.mark.parametrize("which", ["glass", "materials", "env", "volume"])
def test_skew_splat_frames(gpu, glass_scene, materials_scene, env_scene, volume_scenes, which, mode, bands,
                           monkeypatch):
    """The skewed-time splats over the pixel-major sample layout (forced: k_splat_skew runs by
    default only on launches of >= 1 wave per SIMD, k_splat_rows below that), k_splat_skew with
    one and two tile-row bands per bucket, on frames of the path and volume integrators with filter
    widths 2 and 1.5 and ragged edge buckets, against the oracle's framebuffer."""
    if bands:
        monkeypatch.setenv("NART_SKEW_BANDS", str(bands))
    sc = {"glass": glass_scene, "materials": materials_scene, "env": env_scene,
          "volume": volume_scenes["c5"]}[which]
    p = _params(sc, 72, 40, 16)
    g = nart_amd.HipRenderer(sc, splat_mode=mode).render(p)
    r = oracle.Oracle(sc).render(p)
    assert _bits_equal(g, r), _report(g, r)


def _edge_wrap_buckets(p, n_each=2):
    """Full buckets of a wide frame whose last-column / last-row samples round onto the next
    bucket's origin (render.cpp:52-61: splatted through glm::mod into the start of their own
    tile).  Far from the origin a float32 coordinate's spacing is 2^-8, so the last stratum's
    u rounds up often.  Returns bucket ids: x-wrap only, y-wrap only, and the corner pixel both."""
    g = nart_amd.session_geometry(p)
    B, fb = p.bucket_size, g.filter_bounds

    def wraps(x, y, axis):
        uv, _ = oracle.latin_square(y * g.total_width + x, p.spp)
        c = (x if axis == 0 else y) + fb
        return bool((np.float32(c) + uv[:, axis] >= np.float32(c + 1)).any())

    xs, ys, corner = [], [], []
    for by in range(g.n_buckets_y - 2, 0, -1):
        for bx in range(g.n_buckets_x - 2, g.n_buckets_x - 40, -1):
            x0, y0 = bx * B, by * B
            cx, cy = wraps(x0 + B - 1, y0 + B - 1, 0), wraps(x0 + B - 1, y0 + B - 1, 1)
            if cx and cy and len(corner) < 1:
                corner.append(by * g.n_buckets_x + bx)
            elif len(xs) < n_each and any(wraps(x0 + B - 1, y0 + j, 0) for j in range(B - 1)):
                xs.append(by * g.n_buckets_x + bx)
            elif len(ys) < n_each and any(wraps(x0 + i, y0 + B - 1, 1) for i in range(B - 1)):
                ys.append(by * g.n_buckets_x + bx)
            if corner and len(xs) == n_each and len(ys) == n_each:
                return xs + ys + corner
    raise AssertionError("no edge-wrap buckets found: xs %s ys %s corner %s" % (xs, ys, corner))


@pytest.mark.parametrize("splat_mode,bands", [(4, 1), (4, 2), (5, 0), (3, 0)], ids=["skew1", "skew2", "rows", "col4"])
def test_splat_bucket_edge_wraps(gpu, glass_scene, glass_oracle, splat_mode, bands, monkeypatch):
    """Edge-wrapped samples (x, y and the corner source with both) at their raster position in
    the tile pixels' sums: the skewed-time splat's flagged extra passes and the gather kernels'
    extra column / row, against the oracle's scatter, bit for bit."""
    import torch
    if bands:
        monkeypatch.setenv("NART_SKEW_BANDS", str(bands))
    p = _params(glass_scene, 32000, 32000, 16, bounces=1)
    ids = np.array(_edge_wrap_buckets(p), np.uint32)
    g = nart_amd.session_geometry(p)
    tiles = torch.zeros((len(ids), g.tile_size * g.tile_size, 5), dtype=torch.float32, device="cuda")
    r = nart_amd.HipRenderer(glass_scene, splat_mode=splat_mode)
    r.render_buckets_async(p, ids, tiles.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = glass_oracle.render_buckets(p, ids)
    got = tiles.cpu().numpy()
    assert _bits_equal(got, ref), _report(got, ref)


@pytest.fixture(scope="module")
def c4_scene(built, tmp_path_factory):
    from nart_amd import scenes
    return nart_amd.Scene(scenes.c4_teapot(str(tmp_path_factory.mktemp("c4"))))


@pytest.mark.parametrize("variant", [0, 3], ids=["rayqueue", "megakernel"])
def test_c4_teapot_scene(gpu, c4_scene, variant):
    """C4 on SURVEY 8(d)'s assets: the reference's teapot.geo (15,704 triangles; loaded without UVs,
    as the reference does) as plastic with uv.exr rho_d and the noise.exr normal map, a lambert
    plane, a generated 1024x512 environment light (importance sampled)."""
    p = _params(c4_scene, 160, 90, 4)
    g = nart_amd.HipRenderer(c4_scene, variant=variant).render(p)
    r = oracle.Oracle(c4_scene).render(p)
    assert _bits_equal(g, r), _report(g, r)


def test_c4_teapot_per_sample(gpu, c4_scene):
    p = _params(c4_scene, 384, 216, 8)
    g = nart_amd.HipRenderer(c4_scene).render_samples(p, 176, 96, 24, 16)
    r = oracle.Oracle(c4_scene).render_samples(p, 176, 96, 24, 16)
    assert _bits_equal(g, r), _report(g, r)


@pytest.mark.parametrize("packet", ["1", "0"], ids=["packet", "per-lane"])
def test_primary_packet_traversal(gpu, glass_scene, cornell_scene, c4_scene, monkeypatch, packet):
    """Camera rays traced as wave packets (the default, path.h traverse_packet: the wave walks one
    node at a time with a lane mask, each lane testing its own ray) or one ray per lane
    (NART_PRIMARY_PACKET=0).  Same closest hit and octree answer either way: C1 frame, the C3 block with a d.z == 0 camera ray,
    the C2 buckets whose octree answer differs from the true closest hit, a sample the octree
    misses, and the C4 teapot."""
    import torch
    monkeypatch.setenv("NART_PRIMARY_PACKET", packet)
    o = oracle.Oracle(glass_scene)
    p = _params(glass_scene, 256, 256, 16)
    g = nart_amd.HipRenderer(glass_scene).render(p)
    r = o.render(p)
    assert _bits_equal(g, r), _report(g, r)
    p = _params(glass_scene, 1920, 1080, 256)
    g = nart_amd.HipRenderer(glass_scene).render_samples(p, 1344, 128, 16, 16)
    r = o.render_samples(p, 1344, 128, 16, 16)
    assert _bits_equal(g, r), _report(g, r)
    p = _params(cornell_scene, 1920, 1080, 64)
    gm = nart_amd.session_geometry(p)
    ids = np.array(C2_OCTREE_BUCKETS, np.uint32)
    tiles = torch.zeros((len(ids), gm.tile_size * gm.tile_size, 5), dtype=torch.float32, device="cuda")
    nart_amd.HipRenderer(cornell_scene).render_buckets_async(p, ids, tiles.data_ptr(),
                                                             torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = oracle.Oracle(cornell_scene).render_buckets(p, ids)
    got = tiles.cpu().numpy()
    assert _bits_equal(got, ref), _report(got, ref)
    gs = nart_amd.HipRenderer(cornell_scene).render_samples(p, 328, 232, 8, 8)
    rs = oracle.Oracle(cornell_scene).render_samples(p, 328, 232, 8, 8)
    assert _bits_equal(gs, rs), _report(gs, rs)
    p = _params(c4_scene, 160, 90, 4)
    g = nart_amd.HipRenderer(c4_scene).render(p)
    r = oracle.Oracle(c4_scene).render(p)
    assert _bits_equal(g, r), _report(g, r)
