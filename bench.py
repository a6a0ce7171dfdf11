"""Bench: Msamples/s of nart's render path on glassSphere.json at 1920x1080, 256 spp (C3).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Without a launcher, --gpus N > 1 spawns the N rank processes itself (nart_amd.dist.spawn_ranks,
before any GPU call); under a launcher, --gpus must equal WORLD_SIZE or the bench exits non-zero.
NART_DIST_BACKEND=gloo (host-staged tiles) and NART_BENCH_SAME_DEVICE=1 (every rank on GPU 0)
rehearse the multi-rank path on a one-GPU box; the default is RCCL ("nccl"), one GPU per rank.

A step renders the whole frame once: every rank renders an interleaved share of the
reference's 16x16 buckets (all spp of their pixels) into device tiles, the tiles are gathered
to rank 0 over RCCL, and rank 0 combines them in bucket raster order (render.cpp:183-203),
so the image is bit-identical for any N.  Total work is fixed as N grows ("strong").

value = W*H*spp*K / T (Msamples/s, camera samples, render.cpp:164-168 extra rows excluded),
T = max over ranks of the barrier-bracketed wall time of the K steps.
roofline: the path-tracing kernel's algorithmic bytes per launch (counter pass, SURVEY.md 8(d)
per-sample figure) / its HIP-event duration.
cpu_baseline: the oracle (line-faithful C restatement of the TBB tile renderer, oracle/) on a
bounded bucket sample of the same frame, timed on this host (rank 0, N=1 only).  The GPU's
tiles of those buckets are compared with the oracle's bit for bit ("parity").
The other BASELINE.json configs (C2 Cornell, C4 environment-lit textured scene, C5 volume) run
with --config; the default (C3) is the metric BASELINE.json names.
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
from nart_amd.dist import BucketShard, spawn_ranks  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    "c3": dict(scene=lambda d: scenes.glass_sphere(d), w=1920, h=1080, spp=256, stride=29,
               workload="C3 glassSphere.json 1920x1080 256spp, bucket 16, bounces 10, filterWidth 2, roughening 0.2",
               data="reference scene input/scenes/glassSphere.json (+ sphere.geo, backdrop.geo) packed in assets/"),
    "c2": dict(scene=lambda d: scenes.cornell(d), w=1920, h=1080, spp=64, stride=7,
               workload="C2 synthesized Lambert Cornell box, one disk light, 1920x1080 64spp, bounces 10",
               data="synthesized scene (nart_amd/scenes.py cornell)"),
    "c4": dict(scene=lambda d: scenes.c4_teapot(d), w=3840, h=2160, spp=512, stride=211,
               workload="C4 reference teapot.geo (15,704 triangles) as plastic with input/textures/uv.exr rho_d and "
                        "noise.exr roughness map + a generated tangent-space normal map on a lambert plane.geo, "
                        "generated 1024x512 environment light, "
                        "3840x2160 512spp",
               data="reference meshes/textures packed in assets/ + generated sky EXR (nart_amd/scenes.py c4_teapot)"),
    "c4env": dict(scene=lambda d: scenes.environment(d), w=3840, h=2160, spp=512, stride=211,
                  workload="C4-style environment-lit textured, normal-mapped plastic + rough glass (UV spheres), "
                           "3840x2160 512spp (round-2 C4 scene)",
                  data="synthesized scene + generated sky EXR (nart_amd/scenes.py environment)"),
    "c5": dict(scene=lambda d: scenes.volume(d, kind="c5"), w=1920, h=1080, spp=1024, stride=7,
               workload="C5 homogeneous medium (density 1, sigma_s 8), volume integrator, 1920x1080 1024spp, 32 bounces",
               data="synthesized .vol + generated sky EXR (nart_amd/scenes.py volume)"),
}


def bytes_per_sample(c):
    """Algorithmic bytes per traced sample of the path-tracing kernel, SURVEY.md 8(d) minus the
    splat term (the splat is its own kernel): per extension ray 64 B ray record + 32 B hit
    record + 64 B winner attributes, per shadow ray 64 B ray + 4 B result, 64 B per BVH2 node
    visit, 48 B per triangle test, 256 B path state per shaded hit, 40 B camera-ray generation
    per sample."""
    n = max(1, c["traced_samples"])
    return (160.0 * c["rays_extend"] + 68.0 * c["rays_shadow"] + 64.0 * c["node_visits"] + 48.0 * c["tri_tests"]
            + 256.0 * c["bounces"]) / n + 40.0


def cpu_sample_ids(p, stride):
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    stride = int(os.environ.get("NART_CPU_BUCKET_STRIDE", str(stride)))
    return np.arange(0, nb, stride, dtype=np.uint32), stride


def cpu_baseline(scene, p, ids, stride):
    """Oracle on the sampled buckets (timed), returning the rate and the oracle's tiles."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    threads = oracle.default_threads()
    orc = oracle.Oracle(scene)
    t = time.time()
    tiles = orc.render_buckets(p, ids, threads)
    dt = time.time() - t
    samples = 0
    for i in ids:
        bx, by = int(i) % g.n_buckets_x, int(i) // g.n_buckets_x
        x1 = min(p.bucket_size * (bx + 1), p.image_width)
        y1 = min(p.bucket_size * (by + 1), p.image_height)
        samples += max(0, x1 - p.bucket_size * bx) * max(0, y1 - p.bucket_size * by) * p.spp
    out = {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
           "sample": "%d of %d buckets (every %dth in raster order, coprime to the %d bucket columns) of the same "
                     "%dx%d %dspp frame, %d samples, %.1f s" % (len(ids), nb, stride, g.n_buckets_x, p.image_width,
                                                              p.image_height, p.spp, samples, dt)}
    return out, tiles


def load_profile(tag):
    """The committed rocprofv3 summary of this bench command (tools/profile.sh +
    tools/summarize_prof.py: FETCH_SIZE x 2 + WRITE_SIZE per launch, SQ lane utilisation), and
    where it comes from.  A bench cannot run rocprofv3 on itself, so the figures are read from
    the committed summary, and only if it was measured on the current kernel sources
    (hip_source_sha); otherwise None and the source says why."""
    from nart_amd.build import hip_source_sha
    path = os.path.join(REPO, "profiles", "pmc_latest_%s.json" % tag)
    if not os.path.exists(path):
        path = os.path.join(REPO, "profiles", "pmc_latest.json")
    if not os.path.exists(path):
        return None, "no committed PMC summary"
    try:
        d = json.load(open(path))
    except Exception as e:  # noqa: BLE001
        return None, "unreadable PMC summary: %s" % e
    if d.get("config") != tag:
        return None, "PMC summary is for %s, not %s" % (d.get("config"), tag)
    sha = hip_source_sha()
    if d.get("hip_source_sha") != sha:
        return None, "PMC summary %s predates the current kernel sources (%s vs %s)" % (
            d.get("profile"), d.get("hip_source_sha"), sha)
    return d, "profiles/%s_pmc.json (rocprofv3: 2 x FETCH_SIZE + WRITE_SIZE, SQ counters; kernel sources %s)" % (
        d.get("profile"), sha)


def kernel_ratios(prof, samples, tiles_bytes):
    """Counter bytes against algorithmic bytes for the splat and the LatinSquare (per launch):
    splat input 24 B per sample (sample + radiance) + its tiles; LatinSquare 8 B per sample written."""
    if not prof:
        return None
    out = {}
    for k, e in prof.get("kernels", {}).items():
        if "hbm_bytes" not in e:
            continue
        if "k_splat" in k:
            alg = 24.0 * samples + tiles_bytes
        elif "k_latin" in k:
            alg = 8.0 * samples
        else:
            continue
        out[k] = {"algorithmic_bytes": alg, "counter_bytes": e["hbm_bytes"],
                  "counter_over_algorithmic": round(e["hbm_bytes"] / alg, 2),
                  "lane_utilization": e.get("lane_utilization")}
    return out or None


def workload_name(cfg, a, W, H, SPP):
    if not a.size:
        return cfg["workload"]
    return "%s, resized to %dx%d %dspp (rehearsal, not the bench workload)" % (cfg["workload"], W, H, SPP)


def one_process_main(a, cfg, W, H, SPP):
    """--one-process: the whole frame through nart_hip_render_device on a multi-device context
    (the path the C ABI and the `nart` CLI ship): per-device host threads render their lattice
    share of the buckets, the tiles are gathered to device 0 with the library's RCCL
    ncclSend/ncclRecv group (device copies where RCCL is unavailable or the devices repeat), and
    device 0 combines them.  The image stays on device 0 (no PCIe copy)."""
    if "WORLD_SIZE" in os.environ and os.environ["WORLD_SIZE"] != "1":
        print("bench.py: --one-process runs without a launcher", file=sys.stderr)
        sys.exit(2)
    same = os.environ.get("NART_BENCH_SAME_DEVICE", "0") not in ("", "0")
    devices = [0] * a.gpus if same else list(range(a.gpus))
    scene_dir = os.path.join("/tmp", "nart_bench_scene_%s_%d" % (a.config, os.getpid()))
    path = cfg["scene"](scene_dir)
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height, p.spp = W, H, SPP
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    torch.cuda.set_device(0)
    gpu = nart_amd.HipRenderer(scene, devices=devices) if a.gpus > 1 else nart_amd.HipRenderer(scene, device=0)
    gather = gpu.gather_mode() if a.gpus > 1 else "none"
    for _ in range(a.warmup):
        gpu.render_device(p)
    torch.cuda.synchronize()
    st = nart_amd.RenderStats()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        dptr = gpu.render_device(p, st)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    value = W * H * SPP * a.steps / dt / 1e6
    n_img = g.total_height * g.total_width * 5
    image = torch.empty(n_img, dtype=torch.float32, device="cuda:0")
    # copy the context's device image into a torch tensor (device to device, after the timed steps)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    rc = hip.hipMemcpy(ctypes.c_void_p(image.data_ptr()), ctypes.c_void_p(dptr), ctypes.c_size_t(n_img * 4),
                       ctypes.c_int(3))  # hipMemcpyDeviceToDevice
    assert rc == 0, rc
    image = image.view(g.total_height, g.total_width, 5)
    out = {
        "metric": "Msamples/s at %dx%dx%dspp (%s)" % (W, H, SPP, os.path.basename(path)),
        "value": round(value, 3), "unit": "Msamples/s", "n_gpus": a.gpus, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32", "data": cfg["data"],
        "config": {"workload": workload_name(cfg, a, W, H, SPP), "image": [W, H], "spp": SPP, "buckets": nb,
                   "parallelism": "buckets on a lattice over %d device(s) of one process (nart_hip_create_multi)"
                                  % a.gpus},
        "gather": {"rccl": "library ncclSend/ncclRecv group to device 0 (nart_hip_create_multi, INTEGRATION.md 3a)",
                   "copy": "device-to-device copies to device 0 (NART_GATHER=copy or repeated devices)",
                   "copy-fallback": "device-to-device copies to device 0 (RCCL unavailable)",
                   "none": "none (one device)"}[gather],
        "devices": devices,
        "kernel_ms_per_step": round(st.kernel_ms / a.steps, 3),
        "splat_ms_per_step": round(st.splat_ms / a.steps, 3),
        "latin_ms_per_step": round(st.latin_ms / a.steps, 3),
        "schedule": st.schedule_names(),
        "image_finite": bool(torch.isfinite(image).all().item()),
    }
    if a.dump_image:
        np.save(a.dump_image, image.cpu().numpy())
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # smaller frames of the same scene (multi-rank rehearsals and tests; not a bench line)
    ap.add_argument("--size", default=None, help="WxHxSPP override, e.g. 320x180x8")
    ap.add_argument("--dump-image", default=None, help="rank 0 saves the combined float32 image (.npy)")
    ap.add_argument("--one-process", action="store_true",
                    help="one process drives all --gpus devices through the library's multi-device context "
                         "(nart_hip_create_multi: per-device threads, RCCL ncclSend/ncclRecv gather to device 0, "
                         "INTEGRATION.md 3a) instead of one rank per GPU")
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    W, H, SPP = cfg["w"], cfg["h"], cfg["spp"]
    if a.size:
        W, H, SPP = (int(v) for v in a.size.lower().split("x"))
    if a.one_process:
        return one_process_main(a, cfg, W, H, SPP)

    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # no launcher: start the N ranks here, before this process touches a GPU
        sys.exit(spawn_ranks(a.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print("bench.py: --gpus %d but the job has %d rank(s) (WORLD_SIZE); refusing to report a %d-GPU number"
              % (a.gpus, world, a.gpus), file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    backend = os.environ.get("NART_DIST_BACKEND", "nccl")
    if os.environ.get("NART_BENCH_SAME_DEVICE", "0") not in ("", "0"):
        local = 0  # rehearsal: every rank on GPU 0 (RCCL needs distinct GPUs, so use gloo)
    torch.cuda.set_device(local)
    if dist:
        import torch.distributed as td
        if backend == "nccl":
            td.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            td.init_process_group(backend)
        world = td.get_world_size()
        print("bench.py: rank %d of %d on %s (%s), backend %s" % (rank, world, torch.cuda.get_device_name(local),
                                                                  "cuda:%d" % local, backend), file=sys.stderr)

    scene_dir = os.path.join("/tmp", "nart_bench_scene_%s_%d" % (a.config, os.getpid()))
    path = cfg["scene"](scene_dir)
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height, p.spp = W, H, SPP
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    tpx = g.tile_size * g.tile_size
    gpu = nart_amd.HipRenderer(scene, device=local)
    stream = torch.cuda.current_stream()
    dev = torch.device("cuda", local)
    shard = BucketShard(g.n_buckets_x, nb, tpx, rank, world, dev)  # interleaved buckets, gather to rank 0
    mine = shard.mine
    by_id = None
    if rank == 0:
        image = torch.zeros((g.total_height, g.total_width, 5), dtype=torch.float32, device=dev)
        # Render() returns the framebuffer on the host (render.cpp:114-206): each
        # timed step ends with the combined image copied into this pinned host buffer
        image_host = torch.empty((g.total_height, g.total_width, 5), dtype=torch.float32, pin_memory=True)

    ev = []  # per step: (start, rendered, gathered, combined, on host) events on the render stream

    def step(stats):
        nonlocal by_id
        e = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        e[0].record(stream)
        gpu.render_buckets_async(p, mine, shard.tiles.data_ptr(), stream.cuda_stream, stats)
        e[1].record(stream)
        by_id = shard.gather()
        e[2].record(stream)
        if rank == 0:
            gpu.combine_async(p, by_id.data_ptr(), image.data_ptr(), stream.cuda_stream)
            e[3].record(stream)
            with torch.cuda.stream(stream):
                image_host.copy_(image, non_blocking=True)
        else:
            e[3].record(stream)
        e[4].record(stream)
        ev.append(e)

    def barrier():
        torch.cuda.synchronize()
        if dist:
            import torch.distributed as td
            td.barrier()

    # counter passes (not timed): algorithmic bytes per sample.  The figure priced in the roofline
    # comes from the timed configuration itself (full spp) on the cpu_baseline bucket sample of this
    # rank's share; a 16-spp pass over the whole share is reported beside it as a cross-check.
    def counter_pass(ids, spp):
        cp = p.copy()
        cp.spp = spp
        gpu.set_counters(True)
        cst = nart_amd.RenderStats()
        ctiles = torch.zeros((max(1, len(ids)), tpx, 5), dtype=torch.float32, device=dev)
        gpu.render_buckets_async(cp, ids, ctiles.data_ptr(), stream.cuda_stream, cst)
        torch.cuda.synchronize()
        gpu.set_counters(False)
        del ctiles
        return cst.as_dict()

    sample_ids, sample_stride = cpu_sample_ids(p, cfg["stride"])
    mine_sample = np.intersect1d(mine, sample_ids).astype(np.uint32)
    if len(mine_sample) == 0:
        mine_sample = mine[:1]
    counters = counter_pass(mine_sample, SPP)
    counters16 = counter_pass(mine, min(16, SPP))

    for _ in range(a.warmup):
        step(nart_amd.RenderStats())
    barrier()
    ev.clear()
    st = nart_amd.RenderStats()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(st)
    barrier()
    dt = time.perf_counter() - t0
    render_ms = [e[0].elapsed_time(e[1]) for e in ev]
    gather_ms = [e[1].elapsed_time(e[2]) for e in ev]
    host_copy_ms = [e[3].elapsed_time(e[4]) for e in ev]
    mine_t = torch.tensor([dt, sum(render_ms) / len(ev), sum(gather_ms) / len(ev)], dtype=torch.float64)
    per_rank = [mine_t]
    if dist:
        import torch.distributed as td
        tt = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        td.all_reduce(tt, op=td.ReduceOp.MAX)
        dt = float(tt.item())
        src = mine_t.to(dev) if backend == "nccl" else mine_t
        per_rank = [torch.zeros_like(src) for _ in range(world)]
        td.all_gather(per_rank, src)

    samples_total = W * H * SPP * a.steps
    value = samples_total / dt / 1e6
    kernel_avg_ms = st.kernel_ms / max(1, st.kernel_launches)  # k_primary + k_render_rq per launch
    primary_avg_ms = st.primary_ms / max(1, st.kernel_launches)
    bps = bytes_per_sample(counters)
    bps16 = bytes_per_sample(counters16)
    per_launch_samples = st.traced_samples / max(1, st.kernel_launches)
    achieved = bps * per_launch_samples / (kernel_avg_ms * 1e-3) / 1e9
    prof, prof_src = load_profile("%dx%dx%d" % (W, H, SPP))
    traffic = prof.get("hbm_bytes_per_launch") if prof else None
    # The path kernels are latency/issue-bound, not HBM-bound: achieved/frac price the contract's
    # ALGORITHMIC bytes (BVH nodes, triangles, rays, path state per sample) against
    # the HBM ceiling, but those bytes are served from LDS/L1/L2 (a ~0.5 MB scene).  What HBM really
    # moves is `traffic` (rocprofv3 2 x FETCH_SIZE + WRITE_SIZE per launch) -> measured_frac, and
    # what limits the kernel shows in lane_utilization (SQ_THREAD_CYCLES_VALU / 64
    # SQ_ACTIVE_INST_VALU: divergent lanes) and valu_busy.
    # `bound` is the contract's ceiling class (no MFMA on this path, so "hbm"); `frac` is the
    # contract's algorithmic fraction and is restated as `algorithmic_frac`, beside the measured
    # `measured_frac`, so neither reads as the other.
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "frac_kind": "algorithmic: contract bytes (SURVEY.md 8(d)) / kernel time / HBM peak; most of those "
                             "bytes are served by LDS/L1/L2, so this is NOT measured HBM utilisation "
                             "(that is measured_frac)",
                "algorithmic_frac": round(achieved / HBM_PEAK_GBPS, 4),
                "achieved_kind": "algorithmic bytes per launch (SURVEY.md 8(d) per-sample model x traced samples)",
                "limiter_class": "latency",
                "limiter": "latency/issue: dependent LDS/L2 loads in BVH traversal and divergent lanes "
                           "(DESIGN.md section 4), not HBM bandwidth",
                "measured_frac": (round(traffic / (kernel_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
                                  if traffic else None),
                "lane_utilization": prof.get("lane_utilization") if prof else None,
                "valu_busy": prof.get("valu_busy") if prof else None,
                # issue-rate ceiling of the path kernel: issue_frac =
                # (SQ_ACTIVE_INST_VALU + SQ_INSTS_SALU) / SQ_WAVE_CYCLES, the fraction of a wave's
                # issue slots (one per quad-cycle) it used; simd_valu_frac = the SIMD's VALU pipe
                # (two wave64 instructions per quad-cycle) over its resident waves
                "issue_frac": prof.get("issue_frac") if prof else None,
                "simd_valu_frac": prof.get("simd_valu_frac") if prof else None,
                "waves_per_simd": prof.get("waves_per_simd") if prof else None,
                "traffic_source": prof_src,
                "kernel": "k_render_volume_sm" if p.integrator == 1 else "k_primary + k_render_rq",
                "kernel_avg_ms": round(kernel_avg_ms, 3), "bytes_per_sample": round(bps, 1),
                "bytes_per_sample_source": {
                    "spp": SPP, "sample": "counter pass at the timed spp over %d buckets of this rank's share (the "
                                          "cpu_baseline sample: every %dth bucket)" % (len(mine_sample), sample_stride),
                    "cross_check_16spp_whole_share": round(bps16, 1),
                    "ratio_16spp_over_timed": round(bps16 / bps, 4)},
                "rays_per_s": round((counters["rays_extend"] + counters["rays_shadow"]) /
                                    max(1, counters["traced_samples"]) * per_launch_samples /
                                    (kernel_avg_ms * 1e-3), 1)}
    ratios = kernel_ratios(prof, per_launch_samples, nb * tpx * 20.0)
    if ratios:
        roofline["other_kernels"] = ratios
    if p.integrator != 1:
        # the path tracing is two launches (camera rays, then the path kernel); the counters and
        # the time above cover both, the rocprofv3 summary lists them separately
        roofline["kernel_split_ms"] = {"k_primary": round(primary_avg_ms, 3),
                                       "k_render_rq": round(kernel_avg_ms - primary_avg_ms, 3)}
    if rank == 0:
        img_ok = bool(torch.isfinite(image).all().item()) and bool(torch.equal(image.cpu(), image_host))
        out = {
            "metric": "Msamples/s at %dx%dx%dspp (%s)" % (W, H, SPP, os.path.basename(path)),
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
            "data": cfg["data"],
            "config": {"workload": workload_name(cfg, a, W, H, SPP), "image": [W, H], "spp": SPP, "buckets": nb,
                       "parallelism": "buckets interleaved over %d rank(s), %s gather to rank 0" % (
                           world, {"nccl": "RCCL"}.get(backend, backend))},
            "gather": ("none (one rank)" if world == 1 else
                       "torch.distributed gather of the ranks' device tiles to rank 0 over %s, one process per GPU "
                       "(nart_amd/dist.py BucketShard); the C ABI's multi-device context gathers with its own "
                       "ncclSend/ncclRecv group instead (bench.py --one-process)" % {"nccl": "RCCL"}.get(backend, backend)),
            "roofline": roofline,
            "kernel_ms_per_step": round(st.kernel_ms / a.steps, 3),
            "splat_ms_per_step": round(st.splat_ms / a.steps, 3),
            "latin_ms_per_step": round(st.latin_ms / a.steps, 3),
            "host_copy_ms": round(sum(host_copy_ms) / len(ev), 3),
            "timing_boundary": "framebuffer on the host: each timed step ends with rank 0's combined float32 image "
                               "(%d x %d Pixels) copied to pinned host memory (host_copy_ms), as Render() returns "
                               "std::vector<Pixel> (render.cpp:114-206)" % (g.total_width, g.total_height),
            "image_finite": img_ok,
            "per_rank_ms": [{"rank": r, "step_wall_ms": round(float(v[0]) / a.steps * 1e3, 3),
                             "render_ms": round(float(v[1]), 3), "gather_ms": round(float(v[2]), 3)}
                            for r, v in enumerate(t.cpu() for t in per_rank)],
            "counters_per_sample": {k: round(counters[k] / max(1, counters["traced_samples"]), 3)
                                    for k in ("rays_extend", "rays_shadow", "node_visits", "tri_tests",
                                              "bounces", "octree_checks", "octree_replays")},
        }
        if world == 1 and not a.no_cpu_baseline:
            ids, stride = cpu_sample_ids(p, cfg["stride"])
            out["cpu_baseline"], ref_tiles = cpu_baseline(scene, p, ids, stride)
            out["vs_cpu_baseline"] = round(value / out["cpu_baseline"]["value"], 1)
            gt = by_id[torch.from_numpy(ids.astype(np.int64)).to(dev)].cpu().numpy()
            diff = np.abs(gt.astype(np.float64) - ref_tiles.astype(np.float64))
            out["parity"] = {"buckets_compared": int(len(ids)), "tile_floats": int(gt.size),
                             "bit_identical": bool(np.array_equal(gt.view(np.uint32), ref_tiles.view(np.uint32))),
                             "max_abs_diff": float(diff.max()), "rmse": float(np.sqrt((diff ** 2).mean()))}
        if a.dump_image:
            np.save(a.dump_image, image.cpu().numpy())
        print(json.dumps(out), flush=True)
    if dist:
        import torch.distributed as td
        td.destroy_process_group()


if __name__ == "__main__":
    main()
