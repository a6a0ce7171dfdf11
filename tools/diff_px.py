"""Per-sample GPU-vs-oracle check of one 16x16 region of the C3 frame (GPU box)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
import numpy as np  # noqa: E402
import nart_amd  # noqa: E402
import oracle  # noqa: E402
from nart_amd import scenes  # noqa: E402

x0, y0, spp = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
path = scenes.glass_sphere("/tmp/dp_scene")
sc = nart_amd.Scene(path)
p = nart_amd.load_sessions(path)[0]
p.image_width, p.image_height, p.spp = 1920, 1080, spp
gs = nart_amd.HipRenderer(sc).render_samples(p, x0, y0, 16, 16)
rs = oracle.Oracle(sc).render_samples(p, x0, y0, 16, 16)
ne = np.nonzero((gs.view(np.uint32) != rs.view(np.uint32)).any(axis=3))
first = {}
for yy, xx, ss in zip(*ne):
    first.setdefault((x0 + xx, y0 + yy), ss)
print(os.environ.get("TAG", ""), "differing samples", len(ne[0]), "first per pixel", sorted(first.items())[:6])
