"""Whole-frame golden digests of the BASELINE configs, made with the oracle (CPU restatement of
RenderSession::Render, render.cpp:114-206).  TEST INFRASTRUCTURE: run in the build container
(no GPU); the committed output is data only.

For each config the oracle renders every bucket of the full frame (RenderTile + AddSample,
render.cpp:72-112, 23-70) and the script stores, per bucket, a 64-bit BLAKE2b digest of the
bucket's float32 tile (`tileSize^2 x 5` floats, the reference's `Pixel` AoS) plus a digest of the
combined framebuffer (render.cpp:183-203) and of its finalised float32 RGBA
(WriteImageToEXR's contribution / filterWeightSum, render.cpp:220-226).  tests/test_gpu_frames.py
renders the same frames on the HIP path and compares the digests bucket by bucket.

    python tests/golden/make_frame_digests.py c3 [threads]        -> tests/golden/frame_c3.npz

Work is checkpointed per chunk of buckets under /tmp/nart_frame_golden/, so an interrupted run
resumes where it stopped.
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402

import nart_amd  # noqa: E402
import oracle  # noqa: E402
from frame_configs import FRAMES, frame_params, tile_digests  # noqa: E402

SCRATCH = "/tmp/nart_frame_golden"


def main():
    name = sys.argv[1]
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else oracle.default_threads()
    sc, p = frame_params(name, os.path.join(SCRATCH, "scene_" + name))
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    tpx = g.tile_size * g.tile_size
    orc = oracle.Oracle(sc)
    chunk = FRAMES[name]["chunk"]
    os.makedirs(SCRATCH, exist_ok=True)
    t0 = time.time()
    parts = []
    for c0 in range(0, nb, chunk):
        ids = np.arange(c0, min(nb, c0 + chunk), dtype=np.uint32)
        f = os.path.join(SCRATCH, "%s_%d_%06d.npy" % (name, p.spp, c0))
        if not os.path.exists(f):
            t = time.time()
            tiles = orc.render_buckets(p, ids, threads)
            np.save(f + ".tmp.npy", tiles)
            os.replace(f + ".tmp.npy", f)
            print("%s buckets %d/%d  %.0f s (chunk %.0f s)" % (name, ids[-1] + 1, nb, time.time() - t0,
                                                                time.time() - t), flush=True)
        parts.append(f)
    tiles = np.concatenate([np.load(f) for f in parts])
    assert tiles.shape == (nb, tpx, 5)
    img = nart_amd.combine_tiles(p, tiles)
    fin = nart_amd.finalize(p, img)
    out = os.path.join(HERE, "frame_%s.npz" % name)
    meta = {"config": name, "workload": FRAMES[name]["workload"], "image": [p.image_width, p.image_height],
            "spp": p.spp, "buckets": nb, "tile_pixels": tpx, "digest": "blake2b-64 of the float32 bytes",
            "oracle_threads": threads, "oracle_source_sha": oracle_sha(),
            "generated_by": "tests/golden/make_frame_digests.py", "host": os.uname().nodename,
            "finalized_rgb_mean": [float(fin[..., c].astype(np.float64).mean()) for c in range(3)]}
    np.savez_compressed(out, tile_digests=tile_digests(tiles),
                        image_digest=np.frombuffer(hashlib.blake2b(img.tobytes(), digest_size=8).digest(), np.uint64),
                        final_digest=np.frombuffer(hashlib.blake2b(fin.astype(np.float32).tobytes(),
                                                                   digest_size=8).digest(), np.uint64),
                        meta=np.array(json.dumps(meta)))
    print(json.dumps(meta), flush=True)


def oracle_sha():
    h = hashlib.sha256()
    for f in ("nart_oracle.c", "nart_oracle.h", "Makefile"):
        h.update(open(os.path.join(REPO, "oracle", f), "rb").read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    main()
