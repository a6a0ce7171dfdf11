"""Latency of one wave of the path / volume kernel vs the number of pixels it holds (development aid).

Renders small pixel rectangles alone on the GPU (nart_hip_render_samples: one wave when the
rectangle has <= 64 pixels) at full spp and prints the wall time of each, so the latency of a
costly pixel chain can be compared with a full wave of such pixels.
    python tools/latency_probe.py [--config c3|c5] [--spp N] [--grid G]
--grid G also probes a G x G grid of 8x8-pixel rectangles over the frame (one wave each), which
maps where the frame's longest chains are.
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import nart_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--grid", type=int, default=0)
    a = ap.parse_args()
    import bench
    cfg = bench.CONFIGS[a.config]
    path = cfg["scene"](os.path.join("/tmp", "nart_lat_%d" % os.getpid()))
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height = cfg["w"], cfg["h"]
    p.spp = a.spp or cfg["spp"]
    gpu = nart_amd.HipRenderer(scene, device=0)
    gpu.render_samples(p, 0, 0, 4, 4)  # warm up

    def probe(x, y, w, h):
        best = 1e9
        for _ in range(2):
            t = time.perf_counter()
            gpu.render_samples(p, x, y, w, h)
            best = min(best, time.perf_counter() - t)
        print("rect (%d,%d) %dx%d  %.2f ms" % (x, y, w, h, best * 1e3), flush=True)
        return best

    if a.config == "c3":
        rects = [(928, 712, 1, 1), (928, 712, 4, 1), (928, 712, 16, 1), (928, 712, 16, 4), (928, 712, 16, 16),
                 (100, 100, 16, 4), (100, 900, 16, 4), (928, 712, 64, 64)]
    else:
        rects = [(960, 540, 1, 1), (960, 540, 8, 8), (0, 0, 1, 1), (0, 0, 8, 8), (1912, 1072, 8, 8), (960, 0, 8, 8),
                 (0, 540, 8, 8)]
    for r in rects:
        probe(*r)
    if a.grid:
        worst = []
        for gy in range(a.grid):
            for gx in range(a.grid):
                x = min(p.image_width - 8, (gx * p.image_width) // a.grid)
                y = min(p.image_height - 8, (gy * p.image_height) // a.grid)
                worst.append((probe(x, y, 8, 8), x, y))
        worst.sort(reverse=True)
        print("slowest 8x8 waves:", ["(%d,%d) %.1f ms" % (x, y, t * 1e3) for t, x, y in worst[:8]], flush=True)


if __name__ == "__main__":
    main()
