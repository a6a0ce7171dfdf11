"""Multi-GPU render: one process per GPU, buckets sharded across ranks, tiles gathered to rank 0.

The reference renders the 16x16 buckets of a session with a tbb::task_group and sums their
tiles into the image in bucket raster order (render.cpp:152-203).  Across ranks:
  * rank r renders the buckets bucket_owners assigns it (diagonal-lattice interleave: the
    costly sphere region spreads evenly over ranks, with no host work queue);
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
import math
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


def lattice_step(world):
    """Row shift s of the diagonal lattice: the s in [1, world) coprime to world closest to 0.382
    world (golden section: neighbouring rows' owners are far apart), 0 for one rank."""
    cands = [s for s in range(1, world) if math.gcd(s, world) == 1]
    return min(cands, key=lambda s: abs(s - 0.382 * world)) if cands else 0


def bucket_owners(n_buckets_x, n_buckets, world, scheme="lattice"):
    """Owner rank of every bucket id (by * n_buckets_x + bx).  "lattice" (default): a diagonal
    lattice, owner = (bx + s * by) % world with s = lattice_step(world): every run of `world`
    buckets along a row or column holds each rank once, so every region of the frame -- the costly
    glass of C3 -- splits evenly over the ranks.  "mod": b % world, which with a bucket-column count
    divisible by world gives each rank whole vertical stripes (C3 1/8 shards 86-101 ms).  Must
    match shard_ids in host/multi_gpu.h (nart_hip_shard_buckets)."""
    b = np.arange(n_buckets, dtype=np.int64)
    if scheme == "mod" or world == 1:
        return b % world
    return (b % n_buckets_x + lattice_step(world) * (b // n_buckets_x)) % world


class BucketShard:
    """Bucket ownership and the tile gather for one rank of an N-rank render."""

    def __init__(self, n_buckets_x, n_buckets, tile_pixels, rank, world, device, scheme=None):
        self.nb, self.tpx, self.rank, self.world = n_buckets, tile_pixels, rank, world
        scheme = scheme or os.environ.get("NART_SHARD", "lattice")
        owners = bucket_owners(n_buckets_x, n_buckets, world, scheme)
        self.mine = np.nonzero(owners == rank)[0].astype(np.uint32)
        self.per_rank = int(max(np.bincount(owners, minlength=world).max(), 1))
        self.tiles = torch.zeros((self.per_rank, tile_pixels, 5), dtype=torch.float32, device=device)
        self.gathered = self.by_id = None
        if rank == 0:
            self.gathered = torch.zeros((world, self.per_rank, tile_pixels, 5), dtype=torch.float32, device=device)
            self.by_id = torch.zeros((n_buckets, tile_pixels, 5), dtype=torch.float32, device=device)
            owned = [np.nonzero(owners == r)[0] for r in range(world)]
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
