"""Locate GPU-vs-oracle differences on a bucket sample of a full-size frame (GPU box)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import nart_amd  # noqa: E402
import oracle  # noqa: E402
from nart_amd import scenes  # noqa: E402

W, H, SPP, STRIDE = 1920, 1080, int(sys.argv[1]) if len(sys.argv) > 1 else 256, 29
path = scenes.glass_sphere("/tmp/fd_scene")
sc = nart_amd.Scene(path)
p = nart_amd.load_sessions(path)[0]
p.image_width, p.image_height, p.spp = W, H, SPP
g = nart_amd.session_geometry(p)
nb = g.n_buckets_x * g.n_buckets_y
ids = np.arange(0, nb, STRIDE, dtype=np.uint32)
gpu = nart_amd.HipRenderer(sc)
tpx = g.tile_size * g.tile_size
t = torch.zeros((len(ids), tpx, 5), dtype=torch.float32, device="cuda")
gpu.render_buckets_async(p, ids, t.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
gt = t.cpu().numpy()
orc = oracle.Oracle(sc)
rt = orc.render_buckets(p, ids, oracle.default_threads())
bad = np.nonzero((gt.view(np.uint32) != rt.view(np.uint32)).any(axis=2))
print("differing tile pixels:", len(bad[0]), "in buckets", sorted(set(int(ids[b]) for b in bad[0]))[:20])
# per-sample comparison of the source pixels of the first differing buckets
done = 0
for b in sorted(set(bad[0].tolist()))[:4]:
    bid = int(ids[b])
    bx, by = bid % g.n_buckets_x, bid // g.n_buckets_x
    x0, y0 = bx * p.bucket_size, by * p.bucket_size
    w = min(p.bucket_size, g.total_width - x0)
    h = min(p.bucket_size, g.total_height - y0)
    gs = gpu.render_samples(p, x0, y0, w, h)
    rs = orc.render_samples(p, x0, y0, w, h)
    ne = np.nonzero((gs.view(np.uint32) != rs.view(np.uint32)).any(axis=3))
    print("bucket", bid, "(x0 %d y0 %d)" % (x0, y0), "differing samples:", len(ne[0]))
    for k in range(min(5, len(ne[0]))):
        yy, xx, ss = ne[0][k], ne[1][k], ne[2][k]
        print("   px (%d,%d) s %d gpu %s oracle %s" % (x0 + xx, y0 + yy, ss, gs[yy, xx, ss].tolist(), rs[yy, xx, ss].tolist()))
