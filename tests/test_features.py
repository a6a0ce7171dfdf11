"""Scene feature masks (host only, no GPU): nart_hip_scene_features_of -- the mask that selects the
scene-specialised path-kernel build (render.hip scene_features / dispatch_megakernel) -- against an
independent reading of each suite scene's JSON: material kinds, light kinds, textured patterns,
normal maps (glass ignores its normal map, glassmaterial.cpp:3-9).  The GPU suite
(tests/test_gpu_specialize.py) checks that every build renders the same bits; this checks which
build a scene gets."""
import json

import pytest

import nart_amd
from nart_amd import scenes
from nart_amd.api import FEATURES as FT, FT_ALL

MAT = {"lambert": FT["lambert"], "specular": FT["specular"], "glass": FT["glass"], "glossy": FT["glossy"],
       "plastic": FT["plastic"]}
LIGHT = {"disk": FT["disk"], "ring": FT["ring"], "environment": FT["environment"]}
FM_DIFFUSE = FT["lambert"] | FT["disk"]
FM_GLASS = FT["lambert"] | FT["glass"] | FT["disk"]
FM_ENVTEX = FT["lambert"] | FT["plastic"] | FT["environment"] | FT["texture"] | FT["normal_map"]
# pattern fields each material kind reads (src/materials/*.cpp; the loader keeps only these)
FIELDS = {"lambert": ("rho_d", "normal"), "specular": ("rho_s", "eta", "normal"),
          "glass": ("rho_s", "tau", "eta", "roughness"), "glossy": ("rho_s", "eta", "roughness", "normal"),
          "plastic": ("rho_d", "rho_s", "eta", "roughness", "normal")}


def _textured(v):
    return isinstance(v, dict) and v.get("type") == "texture"


def json_features(path):
    js = json.load(open(path))
    f = 0
    for m in js.get("meshes", []):
        mat = m["material"]
        kind = mat["type"]
        f |= MAT[kind]
        for k in FIELDS[kind]:
            if k in mat and _textured(mat[k]):
                f |= FT["texture"]
        if kind != "glass" and "normal" in mat:
            f |= FT["normal_map"]
    for lt in js.get("lights", []):
        f |= LIGHT[lt["type"]]
        if _textured(lt.get("Le")):
            f |= FT["texture"]
    return f


def expected_build(f):
    """dispatch_megakernel's choice (bounces <= 10, not the counter pass)."""
    if f & FT["environment"]:
        return FM_ENVTEX if (f & ~FM_ENVTEX) == 0 else FT_ALL
    for m in (FM_DIFFUSE, FM_GLASS):
        if (f & ~m) == 0:
            return m
    return FT_ALL


SCENES = {
    "glassSphere": (lambda d: scenes.glass_sphere(d), FM_GLASS),
    "cornell": (lambda d: scenes.cornell(d), FM_DIFFUSE),
    "c4_teapot": (lambda d: scenes.c4_teapot(d), FM_ENVTEX),
    "materials": (lambda d: scenes.materials(d), FT_ALL),
    "environment": (lambda d: scenes.environment(d), FT_ALL),
    "nested_glass": (lambda d: scenes.nested_glass(d, bounces=10), FM_GLASS),
    "ring": (lambda d: scenes.reference_scene("ring", d), FT_ALL),
    "veach": (lambda d: scenes.reference_scene("veach", d), FT_ALL),
}


@pytest.mark.parametrize("name", sorted(SCENES))
def test_scene_feature_mask_and_build(built, tmp_path, name):
    make, build = SCENES[name]
    path = make(str(tmp_path))
    sc = nart_amd.Scene(path)
    got = nart_amd.api.scene_features(sc)
    assert got == json_features(path), (name, hex(got), hex(json_features(path)))
    assert expected_build(got) == build, (name, hex(got))
    sc.close()
