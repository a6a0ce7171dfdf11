"""Critical-path split of the last-finishing pixel chains of an N-rank shard (development aid,
VERDICT r04 next #1): needs the NART_WAVEPROF build (tools/build_variant.sh wprof -DNART_WAVEPROF).

  NART_HIP_LIB=abbuild/wprof/libnart_hip.so python tools/chain_breakdown.py --config c3 --n 8 --rank 2

1. renders rank R's bucket share of an N-rank frame with k_render_rq's chain records on
   (NART_CHAIN_REPORT): per lane's first pixel, shader cycles with its own rays outstanding, with
   its rays resolved while the traversal phase serves other lanes, in path phases where it shaded,
   in path phases of other lanes, idle;
2. renders the last-finishing chains' pixels again alone (nart_hip_render_samples, one pixel, one
   lane, no speculation), which gives the same split without contention.
Both runs are subprocesses (the records are printed by the library on stderr)."""
import argparse
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

LAST = re.compile(r"CHAIN last#(\d+) lane (\d+) slot (\d+) px \((\d+),(\d+)\) prio (\d) pair (\d) finish ([\d.]+) ms "
                  r"cycles: own_rays (\d+) wait_others (\d+) shade (\d+) other_path (\d+) idle (\d+) total (\d+)")
MEAN = re.compile(r"CHAIN (priority mean|records \d+ \(priority \d+\) mean) cycles: own_rays ([\d.]+) wait_others "
                  r"([\d.]+) shade ([\d.]+) other_path ([\d.]+) idle ([\d.]+) total ([\d.]+)")


def child_shard(a):
    import torch
    import nart_amd
    import bench
    from nart_amd.dist import BucketShard
    cfg = bench.CONFIGS[a.config]
    path = cfg["scene"](os.path.join("/tmp", "nart_chain_%d" % os.getpid()))
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height, p.spp = cfg["w"], cfg["h"], cfg["spp"]
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    tpx = g.tile_size * g.tile_size
    gpu = nart_amd.HipRenderer(scene, device=0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    shard = BucketShard(g.n_buckets_x, nb, tpx, a.rank, a.n, dev)
    os.environ.pop("NART_CHAIN_REPORT", None)
    gpu.render_buckets_async(p, shard.mine, shard.tiles.data_ptr(), stream.cuda_stream)  # warm-up
    torch.cuda.synchronize()
    os.environ["NART_CHAIN_REPORT"] = "1"
    st = nart_amd.RenderStats()
    gpu.render_buckets_async(p, shard.mine, shard.tiles.data_ptr(), stream.cuda_stream, st)
    torch.cuda.synchronize()
    print(json.dumps({"kernel_ms": st.kernel_ms, "splat_ms": st.splat_ms, "schedule": st.schedule_names()}),
          flush=True)


def child_alone(a):
    import nart_amd
    import bench
    cfg = bench.CONFIGS[a.config]
    path = cfg["scene"](os.path.join("/tmp", "nart_chain_%d" % os.getpid()))
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height, p.spp = cfg["w"], cfg["h"], cfg["spp"]
    gpu = nart_amd.HipRenderer(scene, device=0)
    gpu.render_samples(p, a.x, a.y, 1, 1)  # warm-up
    os.environ["NART_CHAIN_REPORT"] = "1"
    gpu.render_samples(p, a.x, a.y, 1, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--alone", type=int, default=3, help="last-finishing chains to re-render alone")
    ap.add_argument("--child", default=None)
    ap.add_argument("-x", type=int, default=0)
    ap.add_argument("-y", type=int, default=0)
    a = ap.parse_args()
    if a.child == "shard":
        return child_shard(a)
    if a.child == "alone":
        return child_alone(a)
    me = [sys.executable, os.path.abspath(__file__), "--config", a.config, "--n", str(a.n), "--rank", str(a.rank)]
    r = subprocess.run(me + ["--child", "shard"], capture_output=True, text=True, timeout=300)
    sys.stderr.write(r.stderr[-2000:] if r.returncode else "")
    assert r.returncode == 0, r.returncode
    out = {"config": a.config, "n": a.n, "rank": a.rank, "shard": json.loads(r.stdout.strip().splitlines()[-1])}
    for m in MEAN.finditer(r.stderr):
        out["mean_" + ("priority" if m.group(1) == "priority mean" else "all")] = dict(
            zip(["own_rays", "wait_others", "shade", "other_path", "idle", "total"], map(float, m.groups()[1:])))
    lasts = []
    for m in LAST.finditer(r.stderr):
        g = m.groups()
        lasts.append({"rank_last": int(g[0]), "lane": int(g[1]), "px": [int(g[3]), int(g[4])], "prio": int(g[5]),
                      "pair": int(g[6]), "finish_ms": float(g[7]),
                      "cycles": dict(zip(["own_rays", "wait_others", "shade", "other_path", "idle", "total"],
                                         map(int, g[8:])))})
    out["last_chains"] = lasts
    seen = set()
    for c in lasts:
        if len(seen) >= a.alone or tuple(c["px"]) in seen:
            continue
        seen.add(tuple(c["px"]))
        r2 = subprocess.run(me + ["--child", "alone", "-x", str(c["px"][0]), "-y", str(c["px"][1])],
                            capture_output=True, text=True, timeout=300)
        m = LAST.search(r2.stderr)
        c["alone"] = dict(zip(["own_rays", "wait_others", "shade", "other_path", "idle", "total"],
                              map(int, m.groups()[8:]))) if m else None
        c["alone_finish_ms"] = float(m.group(8)) if m else None
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
