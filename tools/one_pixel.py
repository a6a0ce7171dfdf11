"""Render one pixel rectangle (all spp) once -- a target for rocprofv3 counter passes.
    python tools/one_pixel.py X Y W H SPP"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import nart_amd  # noqa: E402
from nart_amd import scenes  # noqa: E402

x, y, w, h, spp = (int(v) for v in sys.argv[1:6])
path = scenes.glass_sphere(os.path.join("/tmp", "nart_px_%d" % os.getpid()))
scene = nart_amd.Scene(path)
p = nart_amd.load_sessions(path)[0]
p.image_width, p.image_height, p.spp = 1920, 1080, spp
gpu = nart_amd.HipRenderer(scene, device=0)
gpu.render_samples(p, x, y, w, h)
print("done")
