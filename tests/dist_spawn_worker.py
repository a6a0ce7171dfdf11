"""One rank of tests/test_bench_spawn.py: started by nart_amd.dist.spawn_ranks (the launcher bench.py
uses for --gpus N without torch.distributed.run), rendezvous from the environment it sets, gloo.
The oracle's tiles stand in for the rank's GPU (CPU test); rank 0 combines and saves the image.

    python tests/dist_spawn_worker.py <scene.json> <W> <H> <SPP> <out.npy>
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as td  # noqa: E402


def main():
    scene_path, w, h, spp, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    import nart_amd
    import oracle
    from nart_amd.dist import BucketShard
    assert os.environ["MASTER_ADDR"] == "127.0.0.1"
    td.init_process_group("gloo")  # env:// rendezvous (RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT)
    try:
        rank, world = td.get_rank(), td.get_world_size()
        assert rank == int(os.environ["LOCAL_RANK"])
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
            np.save(out, nart_amd.combine_tiles(p, by_id.numpy()))
        td.barrier()
    finally:
        td.destroy_process_group()


if __name__ == "__main__":
    main()
