"""Device-side BVH build (NART_BVH_BUILD=device, device/lbvh.h): a linear BVH
built by HIP kernels (Morton codes, radix sort, Karras hierarchy, bottom-up refit, breadth-first
emit) in the host build's node format.  Only the closest hit has to match the reference and the
traversal is exact for any tree, so every image must still equal the oracle's bit for bit."""
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


@pytest.fixture
def device_bvh(monkeypatch):
    monkeypatch.setenv("NART_BVH_BUILD", "device")


@pytest.mark.parametrize("variant", [0, 3], ids=["rayqueue", "megakernel"])
def test_device_bvh_glass_sphere(gpu, glass_scene, device_bvh, variant):
    r = nart_amd.HipRenderer(glass_scene, variant=variant)
    b = r.bvh()
    assert b["on_device"] and b["num_leaf_tris"] > 0 and b["num_nodes"] > 0, b
    p = _params(glass_scene, 128, 96, 4)
    assert _bits_equal(r.render(p), oracle.Oracle(glass_scene).render(p))


def test_device_bvh_cornell_octree_buckets(gpu, cornell_scene, device_bvh):
    """The C2 buckets whose octree answers need the exact emulation (test_gpu_parity)."""
    import torch
    from test_gpu_parity import C2_OCTREE_BUCKETS
    p = _params(cornell_scene, 1920, 1080, 16)
    g = nart_amd.session_geometry(p)
    ids = np.array(C2_OCTREE_BUCKETS[:6], np.uint32)
    tiles = torch.zeros((len(ids), g.tile_size * g.tile_size, 5), dtype=torch.float32, device="cuda")
    r = nart_amd.HipRenderer(cornell_scene)
    assert r.bvh()["on_device"]
    r.render_buckets_async(p, ids, tiles.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert _bits_equal(tiles.cpu().numpy(), oracle.Oracle(cornell_scene).render_buckets(p, ids))


def test_device_bvh_materials_and_teapot(gpu, materials_scene, tmp_path, device_bvh):
    from nart_amd import scenes
    for sc, (w, h, spp) in ((materials_scene, (160, 120, 4)),
                            (nart_amd.Scene(scenes.c4_teapot(str(tmp_path))), (160, 90, 4))):
        r = nart_amd.HipRenderer(sc)
        b = r.bvh()
        assert b["on_device"], b
        p = _params(sc, w, h, spp)
        assert _bits_equal(r.render(p), oracle.Oracle(sc).render(p)), sc.path


def test_device_bvh_matches_host_image_and_reports(gpu, glass_scene, monkeypatch):
    p = _params(glass_scene, 96, 64, 8)
    host = nart_amd.HipRenderer(glass_scene)
    hb = host.bvh()
    assert not hb["on_device"]
    monkeypatch.setenv("NART_BVH_BUILD", "device")
    dev = nart_amd.HipRenderer(glass_scene)
    db = dev.bvh()
    assert db["on_device"] and db["num_leaf_tris"] == hb["num_leaf_tris"]
    assert _bits_equal(dev.render(p), host.render(p))
