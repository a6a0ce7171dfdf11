"""Latency of one wave of the path kernel vs the number of pixels it holds (development aid).

Renders small pixel rectangles alone on the GPU (nart_hip_render_samples: one wave when the
rectangle has <= 64 pixels) at full spp and prints the wall time of each, so the latency of a
costly pixel chain can be compared with a full wave of such pixels.
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import nart_amd  # noqa: E402
from nart_amd import scenes  # noqa: E402


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    path = scenes.glass_sphere(os.path.join("/tmp", "nart_lat_%d" % os.getpid()))
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height, p.spp = 1920, 1080, spp
    gpu = nart_amd.HipRenderer(scene, device=0)
    gpu.render_samples(p, 0, 0, 4, 4)  # warm up
    for (x, y, w, h) in [(928, 712, 1, 1), (928, 712, 4, 1), (928, 712, 16, 1), (928, 712, 16, 4), (928, 712, 16, 16),
                         (100, 100, 16, 4), (100, 900, 16, 4), (928, 712, 64, 64), (928, 712, 256, 128)]:
        best = 1e9
        for _ in range(2):
            t = time.perf_counter()
            gpu.render_samples(p, x, y, w, h)
            best = min(best, time.perf_counter() - t)
        print("rect (%d,%d) %dx%d  %.2f ms" % (x, y, w, h, best * 1e3), flush=True)


if __name__ == "__main__":
    main()
