"""The BASELINE.json full-frame configurations and the per-bucket tile
digest shared by tests/golden/make_frame_digests.py (oracle side, build container) and
tests/test_gpu_frames.py (HIP side, GPU box).  Scene construction is bench.py's, so the
digests describe exactly the frames the bench renders."""
import hashlib

import numpy as np

import nart_amd
from nart_amd import scenes

FRAMES = {
    "c2": dict(scene=scenes.cornell, w=1920, h=1080, spp=64, chunk=680,
               workload="C2 synthesized Lambert Cornell box, 1920x1080 64spp"),
    "c3": dict(scene=scenes.glass_sphere, w=1920, h=1080, spp=256, chunk=340,
               workload="C3 glassSphere.json 1920x1080 256spp"),
    "c4": dict(scene=scenes.c4_teapot, w=3840, h=2160, spp=512, chunk=540,
               workload="C4 teapot + uv.exr/noise.exr + normal map + env light, 3840x2160 512spp"),
    "c5": dict(scene=lambda d: scenes.volume(d, kind="c5"), w=1920, h=1080, spp=1024, chunk=1360,
               workload="C5 homogeneous medium, volume integrator, 1920x1080 1024spp"),
}


def frame_params(name, scene_dir):
    cfg = FRAMES[name]
    sc = nart_amd.Scene(cfg["scene"](scene_dir))
    p = nart_amd.load_sessions(sc.path)[0]
    p.image_width, p.image_height, p.spp = cfg["w"], cfg["h"], cfg["spp"]
    return sc, p


def tile_digests(tiles):
    """uint64 BLAKE2b-64 of each bucket's float32 tile bytes, tiles shaped (buckets, px, 5)."""
    tiles = np.ascontiguousarray(tiles, np.float32)
    out = np.empty(len(tiles), np.uint64)
    for i in range(len(tiles)):
        out[i] = np.frombuffer(hashlib.blake2b(tiles[i].tobytes(), digest_size=8).digest(), np.uint64)[0]
    return out
