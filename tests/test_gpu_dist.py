"""Multi-rank data path on the GPU: two ranks on one MI355X, each rendering its interleaved bucket
share with nart_hip_render_buckets_async into device tiles, the tiles gathered to rank 0
(nart_amd.dist.BucketShard; gloo staging through host memory, since RCCL needs one GPU per
rank) and combined on the device.  The image must equal the single-rank render bit for bit.
This covers everything bench.py's N-GPU path runs except the RCCL transport itself."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, scene_path, w, h, spp, out_path):
    sys.path[:0] = [REPO]
    import torch
    import torch.distributed as td
    import nart_amd
    from nart_amd.dist import BucketShard
    td.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        scene = nart_amd.Scene(scene_path)
        p = nart_amd.load_sessions(scene_path)[0]
        p.image_width, p.image_height, p.spp = w, h, spp
        g = nart_amd.session_geometry(p)
        nb = g.n_buckets_x * g.n_buckets_y
        gpu = nart_amd.HipRenderer(scene, device=0)
        stream = torch.cuda.current_stream()
        shard = BucketShard(g.n_buckets_x, nb, g.tile_size * g.tile_size, rank, world, dev)
        gpu.render_buckets_async(p, shard.mine, shard.tiles.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        by_id = shard.gather()
        if rank == 0:
            image = torch.zeros((g.total_height, g.total_width, 5), dtype=torch.float32, device=dev)
            gpu.combine_async(p, by_id.data_ptr(), image.data_ptr(), stream.cuda_stream)
            torch.cuda.synchronize()
            np.save(out_path, image.cpu().numpy())
        td.barrier()
    finally:
        td.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_on_one_gpu_match_single_rank(gpu, glass_scene, tmp_path, world):
    import nart_amd
    w, h, spp = 200, 120, 8  # 13 x 8 buckets: uneven shares
    out = str(tmp_path / "img.npy")
    mp.start_processes(_worker, args=(world, _free_port(), glass_scene.path, w, h, spp, out), nprocs=world,
                       start_method="spawn")
    img = np.load(out)
    p = nart_amd.load_sessions(glass_scene.path)[0]
    p.image_width, p.image_height, p.spp = w, h, spp
    ref = nart_amd.HipRenderer(glass_scene).render(p)
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))


def test_bench_spawned_ranks_on_one_gpu(gpu, glass_scene, tmp_path):
    """bench.py --gpus 2 without a launcher: it spawns both ranks itself (here both on GPU 0 with
    the gloo backend; the driver's 8-GPU runs use RCCL), reports n_gpus 2, and rank 0's combined
    image equals the single-rank render bit for bit."""
    import json
    import subprocess
    import nart_amd
    out = str(tmp_path / "bench_img.npy")
    env = dict(os.environ, NART_DIST_BACKEND="gloo", NART_BENCH_SAME_DEVICE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--size", "200x120x8",
                        "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--dump-image", out],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2
    ranks = line["per_rank_ms"]
    assert [r["rank"] for r in ranks] == [0, 1]
    assert all(r["render_ms"] > 0 and r["gather_ms"] >= 0 for r in ranks)
    assert line["roofline"]["bytes_per_sample_source"]["spp"] == 8
    img = np.load(out)
    p = nart_amd.load_sessions(glass_scene.path)[0]
    p.image_width, p.image_height, p.spp = 200, 120, 8
    ref = nart_amd.HipRenderer(glass_scene).render(p)
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    assert line["gather"].startswith("torch.distributed gather")


@pytest.mark.parametrize("n", [1, 2, 3])
def test_bench_one_process_multi_device(gpu, glass_scene, tmp_path, n):
    """bench.py --one-process --gpus N: the path the C ABI ships (nart_hip_create_multi +
    nart_hip_render_device: per-device threads, library gather to device 0, combine there).  On the
    one-GPU box the N devices are GPU 0 repeated (device-copy gather); the line names the gather it
    timed, and the combined image equals the single-device render bit for bit."""
    import json
    import subprocess
    import nart_amd
    out = str(tmp_path / "bench1p_img.npy")
    env = dict(os.environ, NART_BENCH_SAME_DEVICE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--one-process", "--gpus", str(n),
                        "--size", "200x120x8", "--steps", "2", "--warmup", "1", "--dump-image", out],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == n and line["devices"] == [0] * n and line["image_finite"]
    assert line["gather"].startswith("none" if n == 1 else "device-to-device copies")
    img = np.load(out)
    p = nart_amd.load_sessions(glass_scene.path)[0]
    p.image_width, p.image_height, p.spp = 200, 120, 8
    ref = nart_amd.HipRenderer(glass_scene).render(p)
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
