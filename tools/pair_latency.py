"""Chain latency of costly glassSphere pixels with and without speculative lane pairs
(development aid): nart_hip_render_samples of small rects, NART_SAMPLES_PAIRS=0/2/4 (lanes per
pixel), results compared bit for bit with the single-lane run."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

import nart_amd  # noqa: E402
from nart_amd import scenes  # noqa: E402


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    path = scenes.glass_sphere(os.path.join("/tmp", "nart_pl_%d" % os.getpid()))
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height, p.spp = 1920, 1080, spp
    gpu = nart_amd.HipRenderer(scene, device=0)
    gpu.render_samples(p, 0, 0, 4, 4)
    for (x, y, w, h) in [(928, 712, 1, 1), (928, 712, 4, 1), (928, 712, 16, 1), (928, 712, 16, 4), (100, 100, 16, 4)]:
        res = {}
        for pairs in ("0", "2", "4"):
            os.environ["NART_SAMPLES_PAIRS"] = pairs
            best = 1e9
            for _ in range(2):
                t = time.perf_counter()
                out = gpu.render_samples(p, x, y, w, h)
                best = min(best, time.perf_counter() - t)
            res[pairs] = (best, out)
        same = all(np.array_equal(np.asarray(res["0"][1]).view(np.uint32), np.asarray(res[q][1]).view(np.uint32))
                   for q in ("2", "4"))
        print("rect (%d,%d) %dx%d  single %.2f ms  pairs %.2f ms  quads %.2f ms  identical %s" % (
            x, y, w, h, res["0"][0] * 1e3, res["2"][0] * 1e3, res["4"][0] * 1e3, same), flush=True)


if __name__ == "__main__":
    main()
