"""The `nart` CLI drop-in end to end on the GPU: src/core/main.cpp:12-61's surface
(two positionals + the reference's flags, "Loading / Rendering / Writing to / Completed in",
<out>.exr for one session and <out>_<n>.exr for several, main.cpp:44-49) with
RenderSession::Render() on the MI355X.  Each written EXR is decoded by the independent reader
(tests/exr_py.py) and must equal finalize(oracle framebuffer) as halves, bit for bit
(WriteImageToEXR, render.cpp:208-234: crop, divide by the weight sum, Imath RNE half)."""
import os
import re
import subprocess

import numpy as np
import pytest

import exr_py
import nart_amd
import oracle

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NART = os.path.join(REPO, "nart_amd", "bin", "nart")


def _run(args, timeout=300):
    r = subprocess.run([NART] + args, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    return r.stdout


def _expected_halves(scene, p):
    with np.errstate(over="ignore"):
        return nart_amd.finalize(p, oracle.Oracle(scene).render(p)).astype(np.float16).view(np.uint16)


@pytest.mark.parametrize("devices", [None, "0,0"], ids=["one-gpu", "two-device-rehearsal"])
def test_cli_glass_sphere(gpu, glass_scene, tmp_path, devices):
    out = str(tmp_path / "glass")
    args = [glass_scene.path, out, "-w", "64", "-h", "48", "-s", "4"] + (["--devices", devices] if devices else [])
    log = _run(args)
    lines = log.strip().splitlines()
    assert lines[0] == "Loading %s..." % glass_scene.path
    assert lines[1] == "Rendering..."
    assert lines[2] == "Writing to %s.exr..." % out
    assert re.fullmatch(r"Completed in [0-9.e+-]+s", lines[3])
    p = nart_amd.parse_args(["nart", glass_scene.path, out, "-w", "64", "-h", "48", "-s", "4"])
    p = nart_amd.load_sessions(glass_scene.path, p)[0]
    halves, hdr = exr_py.read_rgba_halves(out + ".exr")
    assert hdr["compression"] == exr_py.ZIP  # the reference's RgbaOutputFile default
    assert halves.shape == (48, 64, 4)
    assert np.array_equal(halves, _expected_halves(glass_scene, p))


def test_cli_ring_sessions(gpu, ref_scenes, tmp_path):
    """ring.json holds three sessions (roughening 0 / 0.2 / 0.3): out_0.exr .. out_2.exr."""
    sc = ref_scenes["ring"]
    out = str(tmp_path / "ring")
    flags = ["-w", "64", "-h", "36", "-s", "2"]
    log = _run([sc.path, out] + flags)
    assert log.count("Rendering...") == 3 and log.count("Completed in") == 3
    cli = nart_amd.parse_args(["nart", sc.path, out] + flags)
    sessions = nart_amd.load_sessions(sc.path, cli)
    assert len(sessions) == 3
    for k, p in enumerate(sessions):
        path = "%s_%d.exr" % (out, k)
        assert ("Writing to %s..." % path) in log
        halves, _ = exr_py.read_rgba_halves(path)
        assert np.array_equal(halves, _expected_halves(sc, p)), "session %d" % k
    assert not os.path.exists(out + ".exr")


def test_cli_rejects_bad_device_flags(gpu, glass_scene, tmp_path):
    r = subprocess.run([NART, glass_scene.path, str(tmp_path / "x"), "--gpus", "0"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode != 0 and "--gpus 0" in r.stderr
