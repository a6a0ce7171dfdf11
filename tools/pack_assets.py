"""Pack reference scenes (input/scenes/<name>.json + the .geo meshes they use) into
assets/<name>.npz, because /root/reference does not exist on the GPU box: glassSphere (C1/C3),
ring (ring light, three sessions) and veach (four disk lights of different sizes over plastic
plates, the MIS test scene).

Numbers are stored as values, not text: .geo floats are parsed with the C library's strtof
(what `std::istream >> float` does in LoadMeshFromFile, scene.cpp:132-139) and JSON numbers as
Python doubles (nlohmann parses doubles, scene.cpp).  nart_amd/scenes.py writes them back as
'%.9g' (round-trips every float32 through strtof) and repr(double) respectively, so the
materialised files load to bit-identical scene data.

Run in the build container:  python tools/pack_assets.py /root/reference
"""
import ctypes
import json
import os
import sys

import numpy as np

libc = ctypes.CDLL(None)
libc.strtof.restype = ctypes.c_float
libc.strtof.argtypes = [ctypes.c_char_p, ctypes.c_void_p]


def parse_geo(path):
    toks = open(path).read().split()
    ints, floats, kinds = [], [], []
    for t in toks:
        if all(c.isdigit() for c in t):
            kinds.append(0)
            ints.append(int(t))
        else:
            kinds.append(1)
            floats.append(libc.strtof(t.encode(), None))
    return (np.array(kinds, np.uint8), np.array(ints, np.uint32), np.array(floats, np.float32))


def main(ref, scene_name="glassSphere"):
    scene_path = os.path.join(ref, "input", "scenes", scene_name + ".json")
    scene = json.load(open(scene_path))
    arrays = {}
    for m in scene["meshes"]:
        fp = m["filePath"]
        name = os.path.basename(fp.replace("//", "/"))
        if "geo_" + name + "_kinds" not in arrays:
            k, i, f = parse_geo(os.path.join(ref, fp.replace("//", "/")))
            arrays["geo_" + name + "_kinds"] = k
            arrays["geo_" + name + "_ints"] = i
            arrays["geo_" + name + "_floats"] = f
        m["filePath"] = name
    arrays["scene_json"] = np.frombuffer(json.dumps(scene).encode(), np.uint8)
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets", scene_name + ".npz")
    np.savez_compressed(out, **arrays)
    print("wrote", out, os.path.getsize(out), "bytes")


MESHES = ("teapot", "monkey", "cube", "plane")  # C4 assets + ingestion checks
TEXTURES = ("uv", "noise")                     # C4 rho_d / normal map (ZIPS EXRs, copied as-is)


def pack_meshes(ref):
    """assets/meshes.npz: the reference's loose .geo meshes that no packed scene carries, stored
    like the scene meshes (token kinds, ints, strtof floats); input/textures/{uv,noise}.exr are
    copied unchanged to assets/textures/ (data files, read by the drop-in's own EXR reader)."""
    import shutil
    arrays = {}
    for name in MESHES:
        k, i, f = parse_geo(os.path.join(ref, "input", "meshes", name + ".geo"))
        arrays["geo_%s.geo_kinds" % name] = k
        arrays["geo_%s.geo_ints" % name] = i
        arrays["geo_%s.geo_floats" % name] = f
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")
    out = os.path.join(root, "meshes.npz")
    np.savez_compressed(out, **arrays)
    print("wrote", out, os.path.getsize(out), "bytes")
    os.makedirs(os.path.join(root, "textures"), exist_ok=True)
    for t in TEXTURES:
        dst = os.path.join(root, "textures", t + ".exr")
        shutil.copyfile(os.path.join(ref, "input", "textures", t + ".exr"), dst)
        print("copied", dst, os.path.getsize(dst), "bytes")


if __name__ == "__main__":
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    names = sys.argv[2:] or ["glassSphere"]
    for name in names:
        if name == "meshes":
            pack_meshes(ref)
        else:
            main(ref, name)
