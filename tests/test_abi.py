"""C ABI surface: both libraries load on a CPU-only host and export every function that
include/*.h declares (no compute calls: those need a GPU)."""
import ctypes
import os
import re

import nart_amd
from nart_amd import build as nb

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    text = open(os.path.join(REPO, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nart_\w+)\s*\(", text)))


def test_scene_lib_exports_header(built):
    lib = ctypes.CDLL(nb.build_scene_lib())
    names = declared("nart_scene.h")
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_hip_lib_exports_header(built):
    lib = ctypes.CDLL(nb.build_hip_lib())
    names = declared("nart_hip.h")
    assert len(names) >= 10
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_python_bindings_cover_abi(built):
    assert set(declared("nart_scene.h")) == set(nart_amd.SCENE_SYMBOLS)
    assert set(declared("nart_hip.h")) == set(nart_amd.HIP_SYMBOLS)


def test_hip_create_without_gpu_fails_cleanly(built, glass_scene):
    import torch
    if torch.cuda.is_available():
        return
    try:
        nart_amd.HipRenderer(glass_scene)
    except nart_amd.NartError as e:
        assert e.code == -3  # NART_E_HIP, no abort
    else:
        raise AssertionError("render context created without a GPU")
