"""Per-rank shard timing on one GPU (development aid for the N-GPU strong-scaling path).

Renders rank 0's bucket share of an N-rank C3 frame (the same interleaved ownership as
nart_amd.dist.BucketShard) for N in --ns and prints the device times, so the tail of a small
shard can be measured without an N-GPU node:  python tools/shard_perf.py --ns 1 2 4 8
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
from nart_amd.dist import BucketShard  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("-s", type=int, default=0)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--rank", type=int, default=-1, help="-1: every rank of each N (all reported, worst and spread)")
    ap.add_argument("--config", default="c3", help="bench.py config (c2, c3, c4, c5); -s overrides its spp")
    ap.add_argument("--spec", type=int, default=2, help="path-kernel builds: 0 generic, 1 specialised, 2 + lean")
    a = ap.parse_args()
    sys.path.insert(0, REPO)
    import bench
    cfg = bench.CONFIGS[a.config]
    path = cfg["scene"](os.path.join("/tmp", "nart_shard_%d" % os.getpid()))
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height = cfg["w"], cfg["h"]
    p.spp = a.s if a.s > 0 else cfg["spp"]
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    tpx = g.tile_size * g.tile_size
    gpu = nart_amd.HipRenderer(scene, device=0)
    gpu.set_specialize(a.spec)
    stream = torch.cuda.current_stream()
    dev = torch.device("cuda", 0)
    for n in a.ns:
        ranks = range(n) if a.rank < 0 else [a.rank]
        per = []
        for r in ranks:
            shard = BucketShard(g.n_buckets_x, nb, tpx, r, n, dev)
            best = None
            for _ in range(a.reps):
                st = nart_amd.RenderStats()
                torch.cuda.synchronize()
                t = time.perf_counter()
                gpu.render_buckets_async(p, shard.mine, shard.tiles.data_ptr(), stream.cuda_stream, st)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t) * 1e3
                d = {"wall_ms": dt, "kernel_ms": st.kernel_ms, "splat_ms": st.splat_ms, "latin_ms": st.latin_ms}
                if best is None or dt < best["wall_ms"]:
                    best = d
            best["rank"] = r
            per.append(best)
        worst = max(per, key=lambda d: d["wall_ms"])
        walls = [d["wall_ms"] for d in per]
        print(json.dumps({"n": n, "buckets_per_rank": len(BucketShard(g.n_buckets_x, nb, tpx, 0, n, "cpu").mine),
                          "worst": {k: round(v, 3) for k, v in worst.items()},
                          "spread": {"min_ms": round(min(walls), 3), "max_ms": round(max(walls), 3),
                                     "mean_ms": round(sum(walls) / len(walls), 3)},
                          "ranks": [{k: round(v, 3) for k, v in d.items()} for d in per]}), flush=True)


if __name__ == "__main__":
    main()
