"""bench.py's multi-rank entry (CPU): --gpus N without a launcher spawns N ranks itself
(nart_amd.dist.spawn_ranks), and --gpus N inside a job of another size exits non-zero instead of
reporting a number for the wrong GPU count."""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_flag_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "--gpus 2 but the job has 1 rank" in r.stderr
    assert r.stdout.strip() == ""  # no JSON line


def test_spawn_ranks_gloo_matches_single_process(built, glass_scene, tmp_path):
    """The spawn launcher bench.py uses: 2 ranks, env:// rendezvous on 127.0.0.1, gloo gather of
    host tiles, rank-0 combine -- bit-identical to the single-process render."""
    import nart_amd
    import oracle
    from nart_amd.dist import spawn_ranks
    w, h, spp = 72, 40, 2
    out = str(tmp_path / "img.npy")
    rc = spawn_ranks(2, [os.path.join(REPO, "tests", "dist_spawn_worker.py"), glass_scene.path, str(w), str(h),
                         str(spp), out])
    assert rc == 0
    img = np.load(out)
    p = nart_amd.load_sessions(glass_scene.path)[0]
    p.image_width, p.image_height, p.spp = w, h, spp
    ref = oracle.Oracle(glass_scene).render(p)
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))


def test_spawn_ranks_reports_failure():
    from nart_amd.dist import spawn_ranks
    code = "import os, sys, time; r = int(os.environ['RANK']); time.sleep(0 if r else 30); sys.exit(3 if r == 0 else 0)"
    rc = spawn_ranks(2, ["-c", code])
    assert rc == 3
