import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")


@pytest.fixture(scope="session")
def built():
    from nart_amd import build as nb
    nb.build_scene_lib()
    import oracle
    oracle.build()
    return True


@pytest.fixture(scope="session")
def glass_scene(built, tmp_path_factory):
    import nart_amd
    from nart_amd import scenes
    return nart_amd.Scene(scenes.glass_sphere(str(tmp_path_factory.mktemp("glassSphere"))))


@pytest.fixture(scope="session")
def cornell_scene(built, tmp_path_factory):
    import nart_amd
    from nart_amd import scenes
    return nart_amd.Scene(scenes.cornell(str(tmp_path_factory.mktemp("cornell"))))


@pytest.fixture(scope="session")
def materials_scene(built, tmp_path_factory):
    import nart_amd
    from nart_amd import scenes
    return nart_amd.Scene(scenes.materials(str(tmp_path_factory.mktemp("materials"))))


@pytest.fixture(scope="session")
def env_scene(built, tmp_path_factory):
    import nart_amd
    from nart_amd import scenes
    return nart_amd.Scene(scenes.environment(str(tmp_path_factory.mktemp("env"))))


@pytest.fixture(scope="session")
def env_const_scene(built, tmp_path_factory):
    import nart_amd
    from nart_amd import scenes
    return nart_amd.Scene(scenes.environment(str(tmp_path_factory.mktemp("envc")), textured_env=False))


@pytest.fixture(scope="session")
def volume_scenes(built, tmp_path_factory):
    import nart_amd
    from nart_amd import scenes
    return {k: nart_amd.Scene(scenes.volume(str(tmp_path_factory.mktemp("vol_" + k)), kind=k))
            for k in ("c5", "emissive")}


@pytest.fixture(scope="session")
def ref_scenes(built, tmp_path_factory):
    """Reference scenes packed in assets/ (ring: ring light + 3 sessions; veach: 4 disk lights)."""
    import nart_amd
    from nart_amd import scenes
    return {n: nart_amd.Scene(scenes.reference_scene(n, str(tmp_path_factory.mktemp(n)))) for n in ("ring", "veach")}


@pytest.fixture(scope="session")
def gpu(built):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    from nart_amd import build as nb
    nb.build_hip_lib()
    return True
