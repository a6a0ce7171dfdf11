"""Multi-device context of the C ABI (nart_hip_create_multi, host/multi_gpu.h) on the one-GPU box:
the bucket sharding, per-device render threads and streams, the gather to device 0 and the
raster-order combine must reproduce the single-device image bit for bit.  Repeated ordinals
rehearse N devices on one GPU with device copies; NART_GATHER=rccl runs the gather through the
library's own RCCL communicator (one device: a self send/receive over RCCL).  The driver's 8-GPU
node runs the same code with eight distinct devices."""
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


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]], ids=["2-rehearsal", "3-rehearsal"])
def test_multi_device_matches_single(gpu, glass_scene, devices):
    p = _params(glass_scene, 200, 120, 8)  # 13 x 8 buckets: uneven shares
    m = nart_amd.HipRenderer(glass_scene, devices=devices)
    assert m.devices() == (len(devices), False)
    single = nart_amd.HipRenderer(glass_scene).render(p)
    got = m.render(p)
    assert _bits_equal(got, single)
    # a context renders several sessions (ring.json's use) and other sizes
    p2 = _params(glass_scene, 50, 37, 3, filter_width=1.5, bounces=7)
    assert _bits_equal(m.render(p2), oracle.Oracle(glass_scene).render(p2))


def test_multi_device_rccl_gather(gpu, glass_scene, monkeypatch):
    """The gather through RCCL (ncclCommInitAll + grouped ncclSend/ncclRecv), exercised on the one
    device of this box as a self send/receive."""
    monkeypatch.setenv("NART_GATHER", "rccl")
    p = _params(glass_scene, 96, 64, 4)
    m = nart_amd.HipRenderer(glass_scene, devices=[0])
    assert m.devices() == (1, True)
    st = nart_amd.RenderStats()
    got = m.render(p, st)
    assert _bits_equal(got, oracle.Oracle(glass_scene).render(p))
    assert st.traced_samples > 0 and st.kernel_ms > 0


def test_multi_device_volume_and_counters(gpu, volume_scenes):
    sc = volume_scenes["c5"]
    p = _params(sc, 96, 64, 8)
    m = nart_amd.HipRenderer(sc, devices=[0, 0])
    m.set_counters(True)
    st = nart_amd.RenderStats()
    got = m.render(p, st)
    assert _bits_equal(got, oracle.Oracle(sc).render(p))
    assert st.rays_extend > 0


def test_multi_device_rejects_bucket_api(gpu, glass_scene):
    import torch
    m = nart_amd.HipRenderer(glass_scene, devices=[0, 0])
    p = _params(glass_scene, 32, 32, 1)
    t = torch.zeros((4, 400, 5), dtype=torch.float32, device="cuda")
    with pytest.raises(nart_amd.NartError) as e:
        m.render_buckets_async(p, np.arange(4, dtype=np.uint32), t.data_ptr())
    assert e.value.code == -6  # NART_E_UNSUPPORTED: one context per rank for the bucket API


@pytest.mark.parametrize("devices", [[0], [0, 1]])
def test_rccl_gather_failure_marks_context(gpu, glass_scene, monkeypatch, devices):
    """A gather that fails inside the RCCL group (test hook: the last device that owns buckets sends
    to a rank that does not exist, after the other devices' receives are posted) closes the group,
    returns NART_E_RCCL and leaves the context refusing further renders; a fresh context then
    renders bit-identically (render.cpp:152-203 contract).  Two distinct devices need a node with
    two GPUs (skipped on the one-GPU box)."""
    import torch
    if len(set(devices)) > torch.cuda.device_count():
        pytest.skip("needs %d GPUs" % len(set(devices)))
    monkeypatch.setenv("NART_GATHER", "rccl")
    p = _params(glass_scene, 64, 48, 4)
    m = nart_amd.HipRenderer(glass_scene, devices=devices)
    assert m.gather_mode() == "rccl"
    m.debug_fault(1)
    with pytest.raises(nart_amd.NartError) as e:
        m.render(p)
    assert e.value.code == -5  # NART_E_RCCL
    with pytest.raises(nart_amd.NartError) as e2:
        m.render(p)
    assert e2.value.code == -5 and "destroy" in str(e2.value)
    m.close()
    fresh = nart_amd.HipRenderer(glass_scene, devices=devices)
    assert _bits_equal(fresh.render(p), oracle.Oracle(glass_scene).render(p))


def test_multi_device_stats_accumulate(gpu, glass_scene):
    """A stats struct reused over renders keeps accumulating on a multi-device context, as on one
    device (device times of the slowest device per render, added up)."""
    p = _params(glass_scene, 64, 48, 2)
    m = nart_amd.HipRenderer(glass_scene, devices=[0, 0])
    st = nart_amd.RenderStats()
    m.render(p, st)
    k1, s1 = st.kernel_ms, st.traced_samples
    m.render(p, st)
    assert st.kernel_ms > k1 and st.traced_samples == 2 * s1
