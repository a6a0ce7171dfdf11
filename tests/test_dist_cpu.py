"""Multi-rank render path on CPU (gloo, world_size 2 and 3): the bucket sharding, tile gather and
combine of nart_amd.dist (used by bench.py over RCCL) reproduce the single-process image bit
for bit (render.cpp:152-203).  Tiles come from the oracle, which stands in for each rank's GPU."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, scene_path, w, h, spp, out_path):
    sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]
    import torch
    import torch.distributed as td
    import nart_amd
    import oracle
    from nart_amd.dist import BucketShard
    td.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    try:
        scene = nart_amd.Scene(scene_path)
        p = nart_amd.load_sessions(scene_path)[0]
        p.image_width, p.image_height, p.spp = w, h, spp
        g = nart_amd.session_geometry(p)
        nb = g.n_buckets_x * g.n_buckets_y
        shard = BucketShard(g.n_buckets_x, nb, g.tile_size * g.tile_size, rank, world, torch.device("cpu"))
        t = oracle.Oracle(scene).render_buckets(p, shard.mine, 2)
        shard.tiles[:len(shard.mine)] = torch.from_numpy(t)
        by_id = shard.gather()
        if rank == 0:
            np.save(out_path, nart_amd.combine_tiles(p, by_id.numpy()))
    finally:
        td.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gather_matches_single_process(built, glass_scene, tmp_path, world):
    import nart_amd
    import oracle
    w, h, spp = 72, 40, 2  # 5 x 3 buckets: uneven shares for world 2 and 3
    out = str(tmp_path / "img.npy")
    mp.start_processes(_worker, args=(world, _free_port(), glass_scene.path, w, h, spp, out), nprocs=world,
                       start_method="spawn")
    img = np.load(out)
    p = nart_amd.load_sessions(glass_scene.path)[0]
    p.image_width, p.image_height, p.spp = w, h, spp
    ref = oracle.Oracle(glass_scene).render(p)
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))


def test_bucket_ownership_partitions():
    from nart_amd.dist import BucketShard
    import torch
    for nbx, nb, world in [(120, 8160, 8), (5, 15, 2), (7, 7, 4), (3, 3, 8), (13, 104, 3)]:
        parts = [BucketShard(nbx, nb, 4, r, world, torch.device("cpu")).mine for r in range(world)]
        owned = np.concatenate(parts)
        assert np.array_equal(np.sort(owned), np.arange(nb))
        sizes = [len(x) for x in parts]
        assert max(sizes) - min(sizes) <= (nb // nbx + 1), sizes
