"""A/B of the split launch on small shards (development aid, GPU box):
    python tools/split_ab.py [--config c3] [--n 8] [--ranks 0 3] [--spp S]
For each setting (env NART_RQ_SPLIT / _Q / _PER / _PROBE, read per render call) renders rank r's
bucket share of an n-rank frame and prints the wall and path-kernel times (best of --reps)."""
import argparse
import itertools
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import nart_amd  # noqa: E402
from nart_amd.dist import BucketShard  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--ranks", type=int, nargs="+", default=[0, 3])
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--ks", default="0,128,256,512,1024")
    ap.add_argument("--qs", default="4,2")
    ap.add_argument("--pers", default="1,2")
    ap.add_argument("--probe", default="1")
    a = ap.parse_args()
    import bench
    cfg = bench.CONFIGS[a.config]
    path = cfg["scene"](os.path.join("/tmp", "nart_split_%d" % os.getpid()))
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height = cfg["w"], cfg["h"]
    p.spp = a.spp or cfg["spp"]
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    tpx = g.tile_size * g.tile_size
    gpu = nart_amd.HipRenderer(scene, device=0)
    stream = torch.cuda.current_stream()
    dev = torch.device("cuda", 0)
    shards = {r: BucketShard(g.n_buckets_x, nb, tpx, r, a.n, dev) for r in a.ranks}
    ref = {}
    settings = [(0, 0, 0, 0)] + [(k, q, per, pr) for k, q, per, pr in itertools.product(
        [int(x) for x in a.ks.split(",") if int(x) > 0], [int(x) for x in a.qs.split(",")],
        [int(x) for x in a.pers.split(",")], [int(x) for x in a.probe.split(",")]) if q * per <= 64]
    for k, q, per, pr in settings:
        for key, v in (("NART_RQ_SPLIT", k), ("NART_RQ_SPLIT_Q", q), ("NART_RQ_SPLIT_PER", per),
                       ("NART_RQ_SPLIT_PROBE", pr)):
            os.environ[key] = str(v)
        for r, shard in shards.items():
            best = None
            for _ in range(a.reps):
                st = nart_amd.RenderStats()
                torch.cuda.synchronize()
                t = time.perf_counter()
                gpu.render_buckets_async(p, shard.mine, shard.tiles.data_ptr(), stream.cuda_stream, st)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t) * 1e3
                if best is None or dt < best[0]:
                    best = (dt, st.kernel_ms, st.splat_ms)
            h = torch.sum(shard.tiles.view(torch.int32).to(torch.int64) * 1000003 % 2147483647).item()
            same = ref.setdefault(r, h) == h
            print(json.dumps({"K": k, "Q": q, "per": per, "probe": pr, "rank": r, "wall_ms": round(best[0], 2),
                              "kernel_ms": round(best[1], 2), "splat_ms": round(best[2], 2),
                              "same_tiles_as_default": same}), flush=True)


if __name__ == "__main__":
    main()
