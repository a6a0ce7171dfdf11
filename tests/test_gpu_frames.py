"""Whole-frame parity at the BASELINE.json sizes (C2 1080p/64, C3 1080p/256, C4 4K/512, C5
1080p/1024): every bucket of the full frame rendered on the HIP path and compared, bucket by
bucket, with the oracle's tiles through the committed digests in tests/golden/frame_<cfg>.npz
(tests/golden/make_frame_digests.py: the oracle run in the build container).  Also the combined
framebuffer (render.cpp:183-203, in bucket raster order) and its finalised RGBA
(render.cpp:220-226).  Tolerance 0: a digest match means the float32 tiles are bit-identical,
so the per-pixel RMSE against the oracle is 0 (north_star asks < 1e-4)."""
import hashlib
import json
import os

import numpy as np
import pytest

import nart_amd
from frame_configs import FRAMES, frame_params, tile_digests

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _digest(a):
    return np.frombuffer(hashlib.blake2b(np.ascontiguousarray(a).tobytes(), digest_size=8).digest(), np.uint64)[0]


@pytest.mark.parametrize("name", ["c2", "c3", "c4", "c5"])
def test_whole_frame_matches_oracle_digests(gpu, name, tmp_path):
    import torch
    path = os.path.join(GOLDEN, "frame_%s.npz" % name)
    assert os.path.exists(path), "golden digests missing: run tests/golden/make_frame_digests.py %s" % name
    gold = np.load(path)
    meta = json.loads(str(gold["meta"]))
    sc, p = frame_params(name, str(tmp_path / "scene"))
    assert [p.image_width, p.image_height, p.spp] == meta["image"] + [meta["spp"]]
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    tpx = g.tile_size * g.tile_size
    assert nb == meta["buckets"] and tpx == meta["tile_pixels"]
    r = nart_amd.HipRenderer(sc)
    tiles = torch.zeros((nb, tpx, 5), dtype=torch.float32, device="cuda")
    r.render_buckets_async(p, np.arange(nb, dtype=np.uint32), tiles.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    host = tiles.cpu().numpy()
    del tiles
    r.close()
    got = tile_digests(host)
    bad = np.nonzero(got != gold["tile_digests"])[0]
    assert len(bad) == 0, "%s: %d of %d buckets differ from the oracle (first: %s)" % (name, len(bad), nb,
                                                                                       bad[:10].tolist())
    img = nart_amd.combine_tiles(p, host)
    assert _digest(img) == gold["image_digest"][0]
    fin = nart_amd.finalize(p, img).astype(np.float32)
    assert _digest(fin) == gold["final_digest"][0]
