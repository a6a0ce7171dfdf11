"""Work and latency of single buckets vs a whole shard (development aid).

For each bucket id: render it alone (one launch of 256 pixels = 4 waves, so its time is the
serial chain of its costliest pixels) with and without counters, and print its per-sample
work next to the shard's average.  Used to tell a long chain made of many ordinary queries
from one made of a few pathological ones (octree replays, long traversals).
    python tools/chain_probe.py [--spp 256] [--ids 5338 5339 100] [--shard 8]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import nart_amd  # noqa: E402
from nart_amd import scenes  # noqa: E402


def per_sample(d):
    n = max(1, d["traced_samples"])
    return {k: round(d[k] / n, 3) for k in ("rays_extend", "rays_shadow", "node_visits", "tri_tests", "bounces",
                                            "octree_checks", "octree_replays")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--ids", type=int, nargs="*", default=[5338, 5339, 5218, 5458, 100, 8000])
    ap.add_argument("--shard", type=int, default=8)
    a = ap.parse_args()
    path = scenes.glass_sphere(os.path.join("/tmp", "nart_chain_%d" % os.getpid()))
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height, p.spp = 1920, 1080, a.spp
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    tpx = g.tile_size * g.tile_size
    gpu = nart_amd.HipRenderer(scene, device=0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()

    def run(ids, counters):
        tiles = torch.zeros((len(ids), tpx, 5), dtype=torch.float32, device=dev)
        gpu.set_counters(counters)
        st = nart_amd.RenderStats()
        torch.cuda.synchronize()
        t = time.perf_counter()
        gpu.render_buckets_async(p, np.asarray(ids, dtype=np.uint32), tiles.data_ptr(), stream.cuda_stream, st)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) * 1e3
        gpu.set_counters(False)
        return dt, st.as_dict()

    run([0], False)
    for b in a.ids:
        dt, d = run([b], False)
        _, c = run([b], True)
        print(json.dumps({"bucket": b, "xy": [b % g.n_buckets_x * 16, b // g.n_buckets_x * 16], "wall_ms": round(dt, 2),
                          "kernel_ms": round(d["kernel_ms"], 2), "per_sample": per_sample(c)}), flush=True)
    mine = list(range(0, nb, a.shard))
    dt, d = run(mine, False)
    _, c = run(mine, True)
    print(json.dumps({"shard": "1/%d" % a.shard, "buckets": len(mine), "wall_ms": round(dt, 2),
                      "kernel_ms": round(d["kernel_ms"], 2), "per_sample": per_sample(c)}), flush=True)


if __name__ == "__main__":
    main()
