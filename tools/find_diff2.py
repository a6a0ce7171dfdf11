"""Locate GPU-vs-oracle differences over a whole frame of a bench config (GPU box)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import nart_amd  # noqa: E402
import oracle  # noqa: E402

name = sys.argv[1]
cfg = bench.CONFIGS[name]
path = cfg["scene"]("/tmp/fd2_" + name)
sc = nart_amd.Scene(path)
p = nart_amd.load_sessions(path)[0]
p.image_width, p.image_height, p.spp = cfg["w"], cfg["h"], cfg["spp"]
g = nart_amd.session_geometry(p)
nb = g.n_buckets_x * g.n_buckets_y
ids = np.arange(nb, dtype=np.uint32)
gpu = nart_amd.HipRenderer(sc)
t = torch.zeros((nb, g.tile_size ** 2, 5), dtype=torch.float32, device="cuda")
gpu.render_buckets_async(p, ids, t.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
gt = t.cpu().numpy()
orc = oracle.Oracle(sc)
rt = orc.render_buckets(p, ids, oracle.default_threads())
badb = sorted(set(np.nonzero((gt.view(np.uint32) != rt.view(np.uint32)).any(axis=2))[0].tolist()))
print("differing buckets:", len(badb), badb[:30])
for bid in badb[:6]:
    bx, by = bid % g.n_buckets_x, bid // g.n_buckets_x
    x0, y0 = bx * p.bucket_size, by * p.bucket_size
    w = min(p.bucket_size, g.total_width - x0)
    h = min(p.bucket_size, g.total_height - y0)
    gs = gpu.render_samples(p, x0, y0, w, h)
    rs, uv = orc.render_samples(p, x0, y0, w, h, with_uv=True)
    ne = np.nonzero((gs.view(np.uint32) != rs.view(np.uint32)).any(axis=3))
    if not len(ne[0]):
        print("bucket", bid, "no per-sample difference")
        continue
    yy, xx, ss = ne[0][0], ne[1][0], ne[2][0]
    o, d = oracle.camera_ray(orc, p.image_width, p.image_height, x0 + xx, y0 + yy, float(uv[yy, xx, ss, 0]),
                             float(uv[yy, xx, ss, 1]))
    print("bucket", bid, "px", (x0 + xx, y0 + yy), "s", ss, "n", len(ne[0]), "gpu", gs[yy, xx, ss].tolist(),
          "oracle", rs[yy, xx, ss].tolist(), "cam d", d.tolist(), "trace", oracle.trace(orc, o, d))
