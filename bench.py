"""Bench: Msamples/s of nart's render path on glassSphere.json at 1920x1080, 256 spp (C3).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

A step renders the whole frame once: every rank renders an interleaved share of the
reference's 16x16 buckets (all spp of their pixels) into device tiles, the tiles are gathered
to rank 0 over RCCL, and rank 0 combines them in bucket raster order (render.cpp:183-203),
so the image is bit-identical for any N.  Total work is fixed as N grows ("strong").

value = W*H*spp*K / T (Msamples/s, camera samples, render.cpp:164-168 extra rows excluded),
T = max over ranks of the barrier-bracketed wall time of the K steps.
roofline: the path-tracing kernel's algorithmic bytes per launch (counter pass: BVH node and
triangle records, winner attributes, per-sample I/O) / its HIP-event duration.
cpu_baseline: the oracle (line-faithful C restatement of the TBB tile renderer, oracle/) on a
bounded bucket sample of the same frame, timed on this host (rank 0, N=1 only).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import nart_amd  # noqa: E402
from nart_amd import scenes  # noqa: E402
from nart_amd.dist import BucketShard  # noqa: E402

WIDTH, HEIGHT, SPP = 1920, 1080, 256
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md, chip-level parameters)


def bytes_per_sample(c):
    """Algorithmic bytes per traced sample of the path-tracing kernel, SURVEY.md 8(d) minus the
    splat term (the splat is its own kernel): per extension ray 64 B ray record + 32 B hit
    record + 64 B winner attributes, per shadow ray 64 B ray + 4 B result, 64 B per BVH2 node
    visit, 48 B per triangle test, 256 B path state per shaded hit, 40 B camera-ray generation
    per sample."""
    n = max(1, c["traced_samples"])
    return (160.0 * c["rays_extend"] + 68.0 * c["rays_shadow"] + 64.0 * c["node_visits"] + 48.0 * c["tri_tests"]
            + 256.0 * c["bounces"]) / n + 40.0


def cpu_baseline(scene, p):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    stride = int(os.environ.get("NART_CPU_BUCKET_STRIDE", "29"))
    ids = np.arange(0, nb, stride, dtype=np.uint32)
    threads = oracle.default_threads()
    orc = oracle.Oracle(scene)
    t = time.time()
    orc.render_buckets(p, ids, threads)
    dt = time.time() - t
    samples = 0
    for i in ids:
        bx, by = int(i) % g.n_buckets_x, int(i) // g.n_buckets_x
        x1 = min(p.bucket_size * (bx + 1), p.image_width)
        y1 = min(p.bucket_size * (by + 1), p.image_height)
        samples += max(0, x1 - p.bucket_size * bx) * max(0, y1 - p.bucket_size * by) * p.spp
    return {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": "%d of %d buckets (every %dth in raster order, 29 coprime to the 120 bucket columns) of the same %dx%d %dspp frame, %d samples, %.1f s"
                      % (len(ids), nb, stride, p.image_width, p.image_height, p.spp, samples, dt)}


def load_traffic(kernel_avg_ms):
    """HBM bytes per launch of the render kernel from the committed rocprofv3 PMC summary."""
    path = os.path.join(REPO, "profiles", "pmc_latest.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        if d.get("config") == "%dx%dx%d" % (WIDTH, HEIGHT, SPP):
            return d.get("hbm_bytes_per_launch")
    except Exception:
        return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    torch.cuda.set_device(local)
    if dist:
        import torch.distributed as td
        td.init_process_group("nccl", device_id=torch.device("cuda", local))

    scene_dir = os.path.join("/tmp", "nart_bench_scene_%d" % os.getpid())
    path = scenes.glass_sphere(scene_dir)
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height, p.spp = WIDTH, HEIGHT, SPP
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    tpx = g.tile_size * g.tile_size
    gpu = nart_amd.HipRenderer(scene, device=local)
    stream = torch.cuda.current_stream()
    dev = torch.device("cuda", local)
    shard = BucketShard(nb, tpx, rank, world, dev)  # interleaved buckets, gather to rank 0
    mine = shard.mine
    if rank == 0:
        image = torch.zeros((g.total_height, g.total_width, 5), dtype=torch.float32, device=dev)

    def step(stats):
        gpu.render_buckets_async(p, mine, shard.tiles.data_ptr(), stream.cuda_stream, stats)
        by_id = shard.gather()
        if rank == 0:
            gpu.combine_async(p, by_id.data_ptr(), image.data_ptr(), stream.cuda_stream)

    def barrier():
        torch.cuda.synchronize()
        if dist:
            import torch.distributed as td
            td.barrier()

    # counter pass (not timed): algorithmic bytes per sample of this rank's buckets
    cp = p.copy()
    cp.spp = 16
    gpu.set_counters(True)
    cst = nart_amd.RenderStats()
    ctiles = torch.zeros((len(mine), tpx, 5), dtype=torch.float32, device=dev)
    gpu.render_buckets_async(cp, mine, ctiles.data_ptr(), stream.cuda_stream, cst)
    gpu.set_counters(False)
    counters = cst.as_dict()
    del ctiles

    for _ in range(a.warmup):
        step(nart_amd.RenderStats())
    barrier()
    st = nart_amd.RenderStats()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(st)
    barrier()
    dt = time.perf_counter() - t0
    if dist:
        import torch.distributed as td
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        td.all_reduce(tt, op=td.ReduceOp.MAX)
        dt = float(tt.item())

    samples_total = WIDTH * HEIGHT * SPP * a.steps
    value = samples_total / dt / 1e6
    kernel_avg_ms = st.kernel_ms / max(1, st.kernel_launches)
    bps = bytes_per_sample(counters)
    per_launch_samples = st.traced_samples / max(1, st.kernel_launches)
    achieved = bps * per_launch_samples / (kernel_avg_ms * 1e-3) / 1e9
    if rank == 0:
        img_ok = bool(torch.isfinite(image).all().item())
        out = {
            "metric": "Msamples/s at 1920x1080x256spp (glassSphere.json)",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "reference scene input/scenes/glassSphere.json (+ sphere.geo, backdrop.geo) packed in assets/",
            "config": {"workload": "C3 glassSphere.json 1920x1080 256spp, bucket 16, bounces 10, filterWidth 2, "
                                   "roughening 0.2", "image": [WIDTH, HEIGHT], "spp": SPP, "buckets": nb,
                       "parallelism": "buckets interleaved over %d rank(s), RCCL gather to rank 0" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": load_traffic(kernel_avg_ms),
                         "kernel": "k_render", "kernel_avg_ms": round(kernel_avg_ms, 3),
                         "bytes_per_sample": round(bps, 1)},
            "kernel_ms_per_step": round(st.kernel_ms / a.steps, 3),
            "splat_ms_per_step": round(st.splat_ms / a.steps, 3),
            "latin_ms_per_step": round(st.latin_ms / a.steps, 3),
            "image_finite": img_ok,
            "counters_per_sample": {k: round(counters[k] / max(1, counters["traced_samples"]), 3)
                                    for k in ("rays_extend", "rays_shadow", "node_visits", "tri_tests",
                                              "bounces")},
        }
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(scene, p)
            out["vs_cpu_baseline"] = round(value / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    if dist:
        import torch.distributed as td
        td.destroy_process_group()


if __name__ == "__main__":
    main()
