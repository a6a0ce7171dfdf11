"""Scene-specialised path kernels (render.hip dispatch_megakernel, path.h FT_*): the context
derives a feature mask from the scene (material kinds, light kinds, textured patterns, normal
maps) and runs the k_render_rq / k_primary build compiled for the first mask that covers it, so
glassSphere's kernel holds no plastic lobes, ring lights, texture fetches or normal-map frames.
Each kind's operations are the generic build's, so both builds must render the same bits on every
scene of the suite -- at sizes that take each scheduling path (wave-group refill, the probe queue
with priority lanes and speculative pairs, per-sample renders) -- and the scenes the BASELINE
configs name must really run their specialised build."""
import numpy as np
import pytest

import nart_amd
from nart_amd import scenes

pytestmark = pytest.mark.gpu

FT = nart_amd.api.FEATURES
FM_DIFFUSE = FT["lambert"] | FT["disk"]
FM_GLASS = FT["lambert"] | FT["glass"] | FT["disk"]
FM_ENVTEX = FT["lambert"] | FT["plastic"] | FT["environment"] | FT["texture"] | FT["normal_map"]


def _params(scene, w, h, spp, **kw):
    p = nart_amd.load_sessions(scene.path)[0]
    p.image_width, p.image_height, p.spp = w, h, spp
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _same_bits(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint32), np.ascontiguousarray(b).view(np.uint32))


def _both(scene, p, samples=None):
    """(specialised image, generic image, scene mask, specialised build mask, schedule names)."""
    r = nart_amd.HipRenderer(scene)
    st = nart_amd.RenderStats()
    if samples:
        a = r.render_samples(p, *samples)
    else:
        a = r.render(p, st)
    feats, build = r.scene_features()
    r.set_specialize(False)
    b = r.render_samples(p, *samples) if samples else r.render(p)
    _, gen = r.scene_features()
    r.close()
    assert gen == nart_amd.api.FT_ALL
    return a, b, feats, build, st.schedule_names()


@pytest.fixture(scope="module")
def c4_scene(built, tmp_path_factory):
    return nart_amd.Scene(scenes.c4_teapot(str(tmp_path_factory.mktemp("c4s"))))


@pytest.fixture(scope="module")
def nested_scene(built, tmp_path_factory):
    return nart_amd.Scene(scenes.nested_glass(str(tmp_path_factory.mktemp("nest")), spp=4, bounces=10))


@pytest.mark.parametrize("w,h,spp", [(1280, 720, 2), (480, 300, 4), (96, 64, 8)],
                         ids=["wave-groups", "probe-queue", "small"])
def test_glass_sphere_specialised(gpu, glass_scene, w, h, spp):
    a, b, feats, build, sched = _both(glass_scene, _params(glass_scene, w, h, spp))
    assert feats == FM_GLASS and build == FM_GLASS, (hex(feats), hex(build))
    assert "specialized" in sched and "lean" not in sched, sched
    assert _same_bits(a, b)


def test_cornell_specialised(gpu, cornell_scene):
    a, b, feats, build, _ = _both(cornell_scene, _params(cornell_scene, 480, 300, 4))
    assert feats == FM_DIFFUSE and build == FM_DIFFUSE, (hex(feats), hex(build))
    assert _same_bits(a, b)


@pytest.mark.parametrize("lds_levels", [None, "3"], ids=["default", "3-levels"])
def test_glass_sphere_lean_build(gpu, glass_scene, monkeypatch, lds_levels):
    """The whole-frame glassSphere launch runs the lean build, whose traversal stack keeps its top
    levels in LDS and the deeper ones in per-thread global columns (path.h SHORT); with 3 LDS
    levels most pushes of the 14-level BVH go to the columns.  Same bits as the generic build."""
    if lds_levels:
        monkeypatch.setenv("NART_LEAN_STACK", lds_levels)
    # a whole 1080p frame: 16 rounds of resident waves (glass scenes go lean from 12, render.hip lean_fits)
    a, b, feats, build, sched = _both(glass_scene, _params(glass_scene, 1920, 1080, 1))
    assert build == FM_GLASS and "lean" in sched, (hex(build), sched)
    assert _same_bits(a, b)


def test_cornell_lean_build(gpu, cornell_scene):
    """A throughput-bound Cornell frame (>= 3 rounds of resident waves) runs the lean build: no
    priority lanes or speculative pairs, 768-lane blocks at three waves per SIMD (kernels.h WV)."""
    a, b, feats, build, sched = _both(cornell_scene, _params(cornell_scene, 1280, 720, 2))
    assert build == FM_DIFFUSE and "lean" in sched, (hex(build), sched)
    assert _same_bits(a, b)


def test_cornell_lean_probe_queue(gpu, cornell_scene):
    """Scenes without glass or an environment light run the lean build from 1.5 rounds of resident
    waves (render.hip lean_fits): a 2-round Cornell frame takes it through the probe-ordered pixel
    queue (no wave groups below 3 rounds).  Same bits as the generic build."""
    a, b, feats, build, sched = _both(cornell_scene, _params(cornell_scene, 640, 480, 2))
    assert build == FM_DIFFUSE and "lean" in sched and "wave_groups" not in sched, (hex(build), sched)
    assert _same_bits(a, b)


@pytest.mark.parametrize("w,h,spp,lean", [(384, 216, 4, False), (1280, 720, 2, True)], ids=["small", "lean"])
def test_c4_specialised(gpu, c4_scene, w, h, spp, lean):
    a, b, feats, build, sched = _both(c4_scene, _params(c4_scene, w, h, spp))
    assert feats == FM_ENVTEX and build == FM_ENVTEX, (hex(feats), hex(build))
    assert ("lean" in sched) == lean, sched
    assert _same_bits(a, b)


def test_per_sample_specialised(gpu, glass_scene, c4_scene):
    for sc, win in ((glass_scene, (600, 300, 24, 16)), (c4_scene, (176, 96, 24, 16))):
        p = _params(sc, 1280, 720, 16) if sc is glass_scene else _params(sc, 384, 216, 8)
        a, b, _, build, _ = _both(sc, p, samples=win)
        assert build != nart_amd.api.FT_ALL
        assert _same_bits(a, b)


@pytest.mark.parametrize("which", ["materials", "env", "env_const", "ring", "veach", "nested"])
def test_other_scenes_generic_equals_specialised(gpu, materials_scene, env_scene, env_const_scene, ref_scenes,
                                                 nested_scene, which):
    """Every other scene of the suite: the dispatch takes the first build whose mask covers the
    scene's (the generic one when none does) and both builds render the same bits."""
    sc = {"materials": materials_scene, "env": env_scene, "env_const": env_const_scene, "ring": ref_scenes["ring"],
          "veach": ref_scenes["veach"], "nested": nested_scene}[which]
    p = _params(sc, 160, 96, 4)
    a, b, feats, build, _ = _both(sc, p)
    covering = [m for m in (FM_DIFFUSE, FM_GLASS) if not (feats & FT["environment"]) and (feats & ~m) == 0] + \
               [m for m in (FM_ENVTEX,) if (feats & FT["environment"]) and (feats & ~m) == 0]
    assert build == (covering[0] if covering else nart_amd.api.FT_ALL), (hex(feats), hex(build))
    assert _same_bits(a, b)
