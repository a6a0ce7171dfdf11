"""Benchmark scenes materialised in the reference's own input formats (JSON + .geo).

    glassSphere  the reference's input/scenes/glassSphere.json with sphere.geo and backdrop.geo,
                 unpacked from assets/glassSphere.npz (packed by tools/pack_assets.py because
                 /root/reference is not present on the GPU box).  C1 / C3 of BASELINE.json.
    cornell      a synthesized Lambert-only Cornell box lit by one disk light (C2 of
                 BASELINE.json; the reference ships no Cornell box).  Walls are 8x8-quad
                 grids and two boxes, so the reference octree gets many chunks (Q14).

Both are written to a directory and loaded through the drop-in's normal ingestion path.
"""
import json
import os
import tempfile

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
ASSETS = os.path.join(os.path.dirname(_HERE), "assets")


def _fmt(x):
    return "%.9g" % float(np.float32(x))


def _write_geo(path, kinds, ints, floats):
    toks = []
    ii = fi = 0
    for k in kinds:
        if k == 0:
            toks.append(str(int(ints[ii])))
            ii += 1
        else:
            toks.append(_fmt(floats[fi]))
            fi += 1
    with open(path, "w") as f:
        f.write(" ".join(toks) + "\n")


def write_geo(path, faces, verts, normals, face_normals, uvs=None, face_uvs=None):
    """Write a .geo mesh (LoadMeshFromFile layout, scene.cpp:91-223)."""
    toks = [str(len(faces))] + [str(len(f)) for f in faces]
    toks += [str(i) for f in faces for i in f]
    toks += [_fmt(c) for v in verts for c in v]
    toks += [str(i) for f in face_normals for i in f]
    toks += [_fmt(c) for n in normals for c in n]
    if uvs is not None:
        toks += [str(i) for f in face_uvs for i in f]
        toks += [_fmt(c) for uv in uvs for c in uv]
    with open(path, "w") as f:
        f.write(" ".join(toks) + "\n")


def glass_sphere(directory=None):
    """Unpack glassSphere into `directory`; returns the JSON path."""
    d = directory or tempfile.mkdtemp(prefix="nart_glassSphere_")
    os.makedirs(d, exist_ok=True)
    z = np.load(os.path.join(ASSETS, "glassSphere.npz"), allow_pickle=False)
    scene = json.loads(bytes(z["scene_json"]).decode())
    for m in scene["meshes"]:
        name = m["filePath"]
        p = os.path.join(d, name)
        if not os.path.exists(p):
            _write_geo(p, z["geo_" + name + "_kinds"], z["geo_" + name + "_ints"], z["geo_" + name + "_floats"])
        m["filePath"] = p
    path = os.path.join(d, "glassSphere.json")
    with open(path, "w") as f:
        json.dump(scene, f, indent=1)
    return path


def _grid_quad(origin, u, v, n, res):
    """res x res quads spanning origin + [0,1]u + [0,1]v, facing n."""
    o, u, v = (np.asarray(a, np.float64) for a in (origin, u, v))
    verts = [tuple(o + u * (i / res) + v * (j / res)) for j in range(res + 1) for i in range(res + 1)]
    faces = []
    for j in range(res):
        for i in range(res):
            a = j * (res + 1) + i
            faces.append([a, a + 1, a + res + 2, a + res + 1])
    return faces, verts, [tuple(n)], [[0] * 4 for _ in faces]


def _box(center, size, angle_deg):
    c, s = np.asarray(center, np.float64), np.asarray(size, np.float64) / 2
    a = np.radians(angle_deg)
    rot = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
    corners = [np.array([x, y, z]) for z in (-1, 1) for y in (-1, 1) for x in (-1, 1)]
    verts = [tuple(c + rot @ (s * k)) for k in corners]
    quads = [([0, 2, 3, 1], (0, 0, -1)), ([4, 5, 7, 6], (0, 0, 1)), ([0, 1, 5, 4], (0, -1, 0)),
             ([2, 6, 7, 3], (0, 1, 0)), ([0, 4, 6, 2], (-1, 0, 0)), ([1, 3, 7, 5], (1, 0, 0))]
    faces = [q for q, _ in quads]
    normals = [tuple(rot @ np.array(n, np.float64)) for _, n in quads]
    return faces, verts, normals, [[i] * 4 for i in range(6)]


def cornell(directory=None, width=1920, height=1080, spp=64):
    """Synthesized Lambert Cornell box with one disk light; returns the JSON path."""
    d = directory or tempfile.mkdtemp(prefix="nart_cornell_")
    os.makedirs(d, exist_ok=True)
    white, red, green = [0.73, 0.73, 0.73], [0.63, 0.065, 0.05], [0.14, 0.45, 0.091]
    walls = [("floor", (-1, -1, 0), (2, 0, 0), (0, 2, 0), (0, 0, 1), white),
             ("ceiling", (-1, -1, 2), (0, 2, 0), (2, 0, 0), (0, 0, -1), white),
             ("back", (-1, 1, 0), (0, 0, 2), (2, 0, 0), (0, -1, 0), white),
             ("left", (-1, -1, 0), (0, 2, 0), (0, 0, 2), (1, 0, 0), red),
             ("right", (1, -1, 0), (0, 0, 2), (0, 2, 0), (-1, 0, 0), green)]
    meshes = []
    for name, o, u, v, n, rho in walls:
        p = os.path.join(d, name + ".geo")
        write_geo(p, *_grid_quad(o, u, v, n, 8))
        meshes.append({"filePath": p, "material": {"type": "lambert", "rho_d": rho}})
    for name, c, s, a in [("tall", (-0.35, 0.3, 0.6), (0.6, 0.6, 1.2), 17.0), ("short", (0.38, -0.25, 0.3),
                                                                              (0.6, 0.6, 0.6), -18.0)]:
        p = os.path.join(d, name + ".geo")
        write_geo(p, *_box(c, s, a))
        meshes.append({"filePath": p, "material": {"type": "lambert", "rho_d": white}})
    scene = {
        "renderSessions": [{"imageWidth": width, "imageHeight": height, "bucketSize": 16, "spp": spp, "bounces": 10,
                            "filterWidth": 2, "rougheningFactor": 0}],
        "camera": {"fov": 16.5, "transform": [1, 0, 0, 0, 0, 0, -1, -3.9, 0, 1, 0, 1, 0, 0, 0, 1]},
        "meshes": meshes,
        "lights": [{"type": "disk", "radius": 0.35, "Le": [1, 1, 1], "intensity": 40.0,
                    "transform": [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 1.98, 0, 0, 0, 1]}],
    }
    path = os.path.join(d, "cornell.json")
    with open(path, "w") as f:
        json.dump(scene, f, indent=1)
    return path
