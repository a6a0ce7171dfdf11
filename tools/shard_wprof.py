"""WAVEPROF split of rank 0's C3 shard at N (development aid; NART_HIP_LIB = a -DNART_WAVEPROF
build): per-wave cycle percentiles and the path/traversal split, printed by the library."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import nart_amd  # noqa: E402
from nart_amd import scenes  # noqa: E402
from nart_amd.dist import BucketShard  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    path = scenes.glass_sphere(os.path.join("/tmp", "nart_sw_%d" % os.getpid()))
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height, p.spp = 1920, 1080, spp
    g = nart_amd.session_geometry(p)
    gpu = nart_amd.HipRenderer(scene, device=0)
    gpu.set_counters(True)
    dev = torch.device("cuda", 0)
    shard = BucketShard(g.n_buckets_x * g.n_buckets_y, g.tile_size * g.tile_size, 0, n, dev)
    st = nart_amd.RenderStats()
    gpu.render_buckets_async(p, shard.mine, shard.tiles.data_ptr(), torch.cuda.current_stream().cuda_stream, st)
    torch.cuda.synchronize()
    print("kernel_ms %.1f" % st.kernel_ms, flush=True)


if __name__ == "__main__":
    main()
