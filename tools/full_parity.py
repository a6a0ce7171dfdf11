"""Whole-frame parity of a BASELINE config: every bucket rendered on the GPU and by the oracle
(in chunks, with a progress line per chunk), tiles compared bit for bit, then both tile sets
combined and finalised (WriteImageToEXR's contribution / filterWeightSum) and compared per
pixel: the metric's "per-pixel RMSE vs CPU ref" over all W x H x RGB.  GPU box, repo root:

    python tools/full_parity.py c3 [spp]      -> profiles/parity_<config>.json
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import nart_amd  # noqa: E402
import oracle  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    cfg = bench.CONFIGS[name]
    path = cfg["scene"]("/tmp/nart_parity_%s" % name)
    sc = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height = cfg["w"], cfg["h"]
    p.spp = int(sys.argv[2]) if len(sys.argv) > 2 else cfg["spp"]
    g = nart_amd.session_geometry(p)
    nb = g.n_buckets_x * g.n_buckets_y
    tpx = g.tile_size * g.tile_size
    ids = np.arange(nb, dtype=np.uint32)
    gpu = nart_amd.HipRenderer(sc)
    t = torch.zeros((nb, tpx, 5), dtype=torch.float32, device="cuda")
    t0 = time.time()
    gpu.render_buckets_async(p, ids, t.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    gpu_s = time.time() - t0
    gt = t.cpu().numpy()
    del t
    orc = oracle.Oracle(sc)
    rt = np.zeros_like(gt)
    chunk = max(1, nb // 12)
    t0 = time.time()
    for c0 in range(0, nb, chunk):
        rt[c0:c0 + chunk] = orc.render_buckets(p, ids[c0:c0 + chunk], oracle.default_threads())
        print("oracle buckets %d/%d  %.0f s" % (min(nb, c0 + chunk), nb, time.time() - t0), flush=True)
    cpu_s = time.time() - t0
    tile_bits = bool(np.array_equal(gt.view(np.uint32), rt.view(np.uint32)))
    ndiff = int((gt.view(np.uint32) != rt.view(np.uint32)).any(axis=2).sum())
    gi = nart_amd.combine_tiles(p, gt)
    ri = nart_amd.combine_tiles(p, rt)
    gf = nart_amd.finalize(p, gi)[..., :3].astype(np.float64)
    rf = nart_amd.finalize(p, ri)[..., :3].astype(np.float64)
    d = gf - rf
    out = {"config": name, "workload": cfg["workload"], "spp": p.spp, "image": [p.image_width, p.image_height],
           "buckets": nb, "tiles_bit_identical": tile_bits, "differing_tile_pixels": ndiff,
           "framebuffer_bit_identical": bool(np.array_equal(gi.view(np.uint32), ri.view(np.uint32))),
           "per_pixel_rmse_rgb": float(np.sqrt((d ** 2).mean())), "max_abs_diff_rgb": float(np.abs(d).max()),
           "gpu_render_s": round(gpu_s, 3), "oracle_s": round(cpu_s, 1), "oracle_threads": oracle.default_threads()}
    print(json.dumps(out), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "parity_%s_%d.json" % (name, p.spp)), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
