"""GPU robustness of the render context: allocation failure and recovery, batches holding more
than 2^32 samples (64-bit sample offsets), and a depth-capped BVH (median splits) rendering the
same bits as the oracle."""
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


def test_failed_allocation_then_render(gpu, glass_scene):
    """A render whose per-sample buffers cannot be allocated (256 slots x 70 M spp x 24 B =
    430 GB > 288 GB of HBM) fails with NART_E_OOM and leaves the context usable: the next,
    smaller render allocates again and matches the oracle (no stale capacity over freed
    buffers, no sticky HIP error)."""
    r = nart_amd.HipRenderer(glass_scene)
    small = _params(glass_scene, 24, 16, 4, bounces=3)
    first = r.render(small)  # buffers exist before the failing call
    with pytest.raises(nart_amd.NartError) as e:
        r.render(_params(glass_scene, 16, 16, 70_000_000))
    assert e.value.code == -4, e.value  # NART_E_OOM
    again = r.render(small)
    assert _bits_equal(again, first)
    assert _bits_equal(again, oracle.Oracle(glass_scene).render(small))


def test_batch_beyond_2_32_samples(gpu, glass_scene, monkeypatch):
    """One batch of 1920x1080 (+ the 4 extra traced rows) x 2070 spp = 4.31e9 samples > 2^32
    (NART_BATCH_BYTES raised to 130 GB; 28 B per sample: LatinSquare sample, radiance, camera-ray
    hit): 64-bit sample offsets.  The frame equals the same frame
    rendered in 16-GiB batches (each < 2^32 samples), and the last buckets -- whose samples sit
    beyond 2^32 in the single batch -- equal the oracle's."""
    import torch
    p = _params(glass_scene, 1920, 1080, 2070, bounces=1)
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    tpx = g.tile_size * g.tile_size
    ids = np.arange(nb, dtype=np.uint32)
    r = nart_amd.HipRenderer(glass_scene)
    stream = torch.cuda.current_stream().cuda_stream

    def frame(batch_bytes):
        monkeypatch.setenv("NART_BATCH_BYTES", str(batch_bytes))
        tiles = torch.zeros((nb, tpx, 5), dtype=torch.float32, device="cuda")
        st = nart_amd.RenderStats()
        r.render_buckets_async(p, ids, tiles.data_ptr(), stream, st)
        torch.cuda.synchronize()
        return tiles.cpu().numpy(), st

    one, st1 = frame(130_000_000_000)
    assert st1.kernel_launches == 1 and st1.traced_samples > 2 ** 32, (st1.kernel_launches, st1.traced_samples)
    many, st2 = frame(16 << 30)
    assert st2.kernel_launches > 1
    assert _bits_equal(one, many)
    tail = ids[-2:]
    ref = oracle.Oracle(glass_scene).render_buckets(p, tail)
    assert _bits_equal(one[-2:], ref)


def test_depth_capped_bvh_parity(gpu, glass_scene, monkeypatch):
    """Median splits from depth 2 on (NART_BVH_MEDIAN_DEPTH): another tree, the same image."""
    monkeypatch.setenv("NART_BVH_MEDIAN_DEPTH", "2")
    r = nart_amd.HipRenderer(glass_scene)
    p = _params(glass_scene, 64, 48, 4)
    assert _bits_equal(r.render(p), oracle.Oracle(glass_scene).render(p))


def test_rayqueue_lds_fallback(gpu, glass_scene, monkeypatch):
    """A scene whose BVH stack does not fit the ray-queue kernel's 512-lane LDS layout (stack depth
    > 24: 4 KiB per level + 60 KiB of outboxes) must still render with variant 0 -- on the 256-lane
    kernel -- bit-identically (such scenes passed create and failed at launch).  The
    LDS budget is lowered (NART_RQ_LDS_LIMIT) so that glassSphere's 14-level stack trips it."""
    monkeypatch.setenv("NART_RQ_LDS_LIMIT", str(100 * 1024))
    assert nart_amd.api.bvh_info(glass_scene)["stack_depth"] * 4096 + 61440 > 100 * 1024
    p = _params(glass_scene, 96, 64, 4)
    g = nart_amd.HipRenderer(glass_scene, variant=0).render(p)
    assert _bits_equal(g, oracle.Oracle(glass_scene).render(p))


@pytest.mark.parametrize("variant", [0, 3], ids=["rayqueue", "megakernel"])
def test_forced_octree_replay_single_pool_entry(gpu, cornell_scene, monkeypatch, variant):
    """Every query answered by replaying the reference octree search (NART_OCTREE_EXACT=2) with a
    replay pool of ONE entry (NART_OC_POOL=1): every wave that replays contends for the same
    heaps.  Lanes of a wave share the entry their lowest lane acquired, so no lane waits on a
    wave-mate; the frame must complete and equal the oracle's bit for bit."""
    import torch
    monkeypatch.setenv("NART_OCTREE_EXACT", "2")
    monkeypatch.setenv("NART_OC_POOL", "1")
    r = nart_amd.HipRenderer(cornell_scene, variant=variant)
    p = _params(cornell_scene, 96, 64, 4)
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    ids = np.arange(nb, dtype=np.uint32)
    tiles = torch.zeros((nb, g.tile_size * g.tile_size, 5), dtype=torch.float32, device="cuda")
    st = nart_amd.RenderStats()
    r.set_counters(True)
    r.render_buckets_async(p, ids, tiles.data_ptr(), torch.cuda.current_stream().cuda_stream, st)
    torch.cuda.synchronize()
    ref = oracle.Oracle(cornell_scene).render_buckets(p, ids)
    assert _bits_equal(tiles.cpu().numpy(), ref)
    assert st.octree_replays >= st.rays_extend  # every extension query (and shadow query) replayed
