"""Cycle split of one costly pixel chain alone vs a wave of them (development aid; needs a
-DNART_WAVEPROF build via NART_HIP_LIB).  Prints the WAVEPROF lines of k_render_rq (stderr)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import nart_amd  # noqa: E402
from nart_amd import scenes  # noqa: E402


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    path = scenes.glass_sphere(os.path.join("/tmp", "nart_chain_%d" % os.getpid()))
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height, p.spp = 1920, 1080, spp
    gpu = nart_amd.HipRenderer(scene, device=0)
    gpu.set_counters(True)
    gpu.render_samples(p, 0, 0, 4, 4)
    for (x, y, w, h) in [(928, 712, 1, 1), (928, 712, 4, 1), (928, 712, 16, 4)]:
        sys.stderr.write("---- rect (%d,%d) %dx%d\n" % (x, y, w, h))
        sys.stderr.flush()
        t = time.perf_counter()
        gpu.render_samples(p, x, y, w, h)
        sys.stderr.write("---- %.2f ms\n" % ((time.perf_counter() - t) * 1e3))
        sys.stderr.flush()


if __name__ == "__main__":
    main()
