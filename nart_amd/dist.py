"""Multi-GPU render: one process per GPU, buckets sharded across ranks, tiles gathered to rank 0.

The reference renders the 16x16 buckets of a session with a tbb::task_group and sums their
tiles into the image in bucket raster order (render.cpp:152-203).  Across ranks:
  * rank r renders buckets r, r + N, r + 2N, ... (interleaved: the costly sphere region spreads
    evenly over ranks, with no host work queue);
  * each rank's tiles (tileSize^2 Pixels per bucket) are gathered to rank 0 with one
    torch.distributed gather (RCCL over xGMI on GPUs; gloo in the CPU tests, and in the
    one-GPU multi-rank test, where device tiles are staged through host memory);
  * rank 0 scatters them into bucket-id order and combines in bucket raster order, so the
    image is bit-identical for any N.
No other collective is on the data path.

spawn_ranks starts the one-process-per-GPU job itself when a script is run with --gpus N and no
launcher (torch.distributed.run) set up the rendezvous: N children with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT, started before the parent touches any GPU.
"""
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv, env=None):
    """Run `python argv...` as ranks 0..n-1 of one job (rendezvous on 127.0.0.1) and return the
    first non-zero exit code, or 0.  If a rank fails, the ranks still running are stopped (they
    would wait for it at the next collective)."""
    port = free_port()
    base = dict(os.environ if env is None else env)
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=e))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:  # exact children of this call, never a pattern
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


class BucketShard:
    """Bucket ownership and the tile gather for one rank of an N-rank render."""

    def __init__(self, n_buckets, tile_pixels, rank, world, device):
        self.nb, self.tpx, self.rank, self.world = n_buckets, tile_pixels, rank, world
        self.mine = np.arange(rank, n_buckets, world, dtype=np.uint32)
        self.per_rank = (n_buckets + world - 1) // world
        self.tiles = torch.zeros((self.per_rank, tile_pixels, 5), dtype=torch.float32, device=device)
        self.gathered = self.by_id = None
        if rank == 0:
            self.gathered = torch.zeros((world, self.per_rank, tile_pixels, 5), dtype=torch.float32, device=device)
            self.by_id = torch.zeros((n_buckets, tile_pixels, 5), dtype=torch.float32, device=device)
            owned = [np.arange(r, n_buckets, world) for r in range(world)]
            self.order = torch.from_numpy(np.concatenate(owned).astype(np.int64)).to(device)
            self.slots = torch.from_numpy(np.concatenate(
                [r * self.per_rank + np.arange(len(o)) for r, o in enumerate(owned)]).astype(np.int64)).to(device)

    def gather(self):
        """Collective: rank 0 returns the (n_buckets, tileSize^2, 5) tiles in bucket-id order."""
        if self.world > 1:
            import torch.distributed as td
            # gloo gathers host tensors only: stage device tiles through host memory
            stage = self.tiles.is_cuda and td.get_backend() == "gloo"
            mine = self.tiles.cpu() if stage else self.tiles
            if self.rank == 0:
                dst = self.gathered.cpu() if stage else self.gathered
                td.gather(mine, gather_list=list(dst.unbind(0)), dst=0)
                if stage:
                    self.gathered.copy_(dst)
            else:
                td.gather(mine, dst=0)
                return None
            src = self.gathered.view(self.world * self.per_rank, self.tpx, 5)
        else:
            src = self.tiles
        self.by_id[self.order] = src[self.slots]
        return self.by_id
