"""Benchmark scenes materialised in the reference's own input formats (JSON + .geo).

    glassSphere  the reference's input/scenes/glassSphere.json with sphere.geo and backdrop.geo,
                 unpacked from assets/glassSphere.npz (packed by tools/pack_assets.py because
                 /root/reference is not present on the GPU box).  C1 / C3 of BASELINE.json.
    ring, veach  the reference's ring.json (three sessions) and veach.json, packed the same way.
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
    """Write a .geo mesh (LoadMeshFromFile layout, scene.cpp:91-223).  The reader sizes each
    coordinate array by the largest index referencing it, so arrays are cut to that length."""
    verts = verts[:max(i for f in faces for i in f) + 1]
    normals = normals[:max(i for f in face_normals for i in f) + 1]
    if uvs is not None:
        uvs = uvs[:max(i for f in face_uvs for i in f) + 1]
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


REFERENCE_SCENES = ("glassSphere", "ring", "veach")


def reference_scene(name, directory=None):
    """Materialise a packed reference scene (assets/<name>.npz, tools/pack_assets.py) into
    `directory`; returns the JSON path."""
    d = directory or tempfile.mkdtemp(prefix="nart_%s_" % name)
    os.makedirs(d, exist_ok=True)
    z = np.load(os.path.join(ASSETS, name + ".npz"), allow_pickle=False)
    scene = json.loads(bytes(z["scene_json"]).decode())
    for m in scene["meshes"]:
        fname = m["filePath"]
        p = os.path.join(d, fname)
        if not os.path.exists(p):
            _write_geo(p, z["geo_" + fname + "_kinds"], z["geo_" + fname + "_ints"], z["geo_" + fname + "_floats"])
        m["filePath"] = p
    path = os.path.join(d, name + ".json")
    with open(path, "w") as f:
        json.dump(scene, f, indent=1)
    return path


def glass_sphere(directory=None):
    """glassSphere (C1 / C3 of BASELINE.json); returns the JSON path."""
    return reference_scene("glassSphere", directory)


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


def write_texture(path, rgba, compression=3):
    """Write an (H, W, 4) float array as a half-RGBA EXR through the drop-in's own writer
    (WriteImageToEXR layout: a Pixel framebuffer with a 1-pixel border and unit weights)."""
    from . import api
    rgba = np.asarray(rgba, np.float32)
    h, w = rgba.shape[:2]
    p = api.default_params()
    p.image_width, p.image_height, p.filter_width = w, h, 1.0
    img = np.zeros((h + 2, w + 2, 5), np.float32)
    img[1:h + 1, 1:w + 1, :4] = rgba
    img[..., 4] = 1.0
    api.write_exr(path, p, img, compression)


def _uv_sphere(center, radius, n_lat=12, n_lon=24):
    """Lat-long sphere with per-vertex normals and UVs (quads, triangle caps)."""
    c = np.asarray(center, np.float64)
    verts, normals, uvs = [], [], []
    for j in range(n_lat + 1):
        th = np.pi * j / n_lat
        for i in range(n_lon + 1):
            ph = 2 * np.pi * i / n_lon
            n = np.array([np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)])
            verts.append(tuple(c + radius * n))
            normals.append(tuple(n))
            uvs.append((i / n_lon, 1 - j / n_lat))
    faces = []
    for j in range(n_lat):
        for i in range(n_lon):
            a, b = j * (n_lon + 1) + i, (j + 1) * (n_lon + 1) + i
            if j == 0:
                faces.append([a, b, b + 1])
            elif j == n_lat - 1:
                faces.append([a, b, a + 1])
            else:
                faces.append([a, b, b + 1, a + 1])
    return faces, verts, normals, faces, uvs, faces


def _uv_grid(origin, u, v, n, res):
    faces, verts, normals, fn = _grid_quad(origin, u, v, n, res)
    uvs = [(i / res, j / res) for j in range(res + 1) for i in range(res + 1)]
    return faces, verts, normals, fn, uvs, faces


def materials(directory=None, width=320, height=240, spp=16):
    """Every material type, textured / roughness-textured / normal-mapped patterns, a ring and
    a disk light and nested dielectric priorities -- the device paths glassSphere and the
    Cornell box leave untouched.  Textures are generated (no RNG) and written as ZIP EXRs."""
    d = directory or tempfile.mkdtemp(prefix="nart_materials_")
    os.makedirs(d, exist_ok=True)
    n = 64
    yy, xx = np.mgrid[0:n, 0:n].astype(np.float32) / (n - 1)
    check = ((np.floor(xx * 8) + np.floor(yy * 8)) % 2).astype(np.float32)
    albedo = np.stack([0.2 + 0.6 * xx, 0.15 + 0.5 * check, 0.7 - 0.5 * yy, np.ones_like(xx)], -1)
    bump = np.stack([0.5 + 0.35 * np.sin(xx * 12.0), 0.5 + 0.35 * np.cos(yy * 9.0),
                     np.full_like(xx, 0.9), np.ones_like(xx)], -1)
    rough = np.stack([0.05 + 0.6 * xx, 0.05 + 0.6 * xx, 0.05 + 0.6 * xx, np.ones_like(xx)], -1)
    tex = {}
    for name, arr in (("albedo", albedo), ("bump", bump), ("rough", rough)):
        tex[name] = os.path.join(d, name + ".exr")
        write_texture(tex[name], arr)
    geo = {}
    geo["ground"] = _uv_grid((-3, -3, 0), (6, 0, 0), (0, 6, 0), (0, 0, 1), 6)
    geo["back"] = _uv_grid((-3, 2.5, 0), (6, 0, 0), (0, 0, 4), (0, -1, 0), 4)
    geo["glossy"] = _uv_sphere((-1.4, 0.4, 0.6), 0.6)
    geo["mirror"] = _uv_sphere((0.0, 0.9, 0.6), 0.6)
    geo["plastic"] = _uv_sphere((1.4, 0.4, 0.6), 0.6)
    geo["glass"] = _uv_sphere((0.2, -0.8, 0.45), 0.45)
    geo["inner"] = _uv_sphere((0.2, -0.8, 0.45), 0.25, 8, 16)
    for k, g in geo.items():
        write_geo(os.path.join(d, k + ".geo"), *g)
    T = lambda p: {"type": "texture", "filePath": p}  # noqa: E731
    meshes = [
        ("ground", {"type": "plastic", "rho_d": T(tex["albedo"]), "rho_s": [0.9, 0.9, 0.9], "eta": 1.5,
                    "roughness": 0.2, "normal": T(tex["bump"])}, None),
        ("back", {"type": "lambert", "rho_d": T(tex["albedo"]), "normal": T(tex["bump"])}, None),
        ("glossy", {"type": "glossy", "rho_s": [0.95, 0.64, 0.54], "eta": 1.8, "roughness": T(tex["rough"])}, None),
        ("mirror", {"type": "specular", "rho_s": [0.9, 0.9, 0.9], "eta": 8192}, None),
        ("plastic", {"type": "plastic", "rho_d": [0.1, 0.3, 0.6], "rho_s": [1, 1, 1], "eta": 1.5,
                     "roughness": 0.0}, None),
        ("glass", {"type": "glass", "rho_s": [1, 1, 1], "tau": [0.9, 0.95, 1.0], "eta": 1.5,
                   "roughness": 0.15}, 2),
        ("inner", {"type": "glass", "rho_s": [1, 1, 1], "tau": [1.0, 0.6, 0.6], "eta": 1.33,
                   "roughness": 0.0}, 3),
    ]
    jm = []
    for name, mat, prio in meshes:
        e = {"filePath": os.path.join(d, name + ".geo"), "material": mat}
        if prio is not None:
            e["priority"] = prio
        jm.append(e)
    scene = {
        "renderSessions": [{"imageWidth": width, "imageHeight": height, "bucketSize": 16, "spp": spp,
                            "bounces": 12, "filterWidth": 1.5, "rougheningFactor": 0.3}],
        "camera": {"fov": 24.0, "transform": [1, 0, 0, 0, 0, 0.2588190, -0.9659258, -6.2, 0, 0.9659258, 0.2588190, 2.0,
                                              0, 0, 0, 1]},
        "meshes": jm,
        "lights": [
            {"type": "ring", "radius": 0.8, "innerRadius": 0.4, "Le": [1.0, 0.9, 0.8], "intensity": 30.0,
             "transform": [1, 0, 0, 0.5, 0, 1, 0, -0.5, 0, 0, 1, 3.2, 0, 0, 0, 1]},
            {"type": "disk", "radius": 0.3, "Le": [0.6, 0.7, 1.0], "intensity": 60.0,
             "transform": [1, 0, 0, -2.0, 0, 0, 1, 1.5, 0, -1, 0, 1.2, 0, 0, 0, 1]},
        ],
    }
    path = os.path.join(d, "materials.json")
    with open(path, "w") as f:
        json.dump(scene, f, indent=1)
    return path


def nested_glass(directory=None, width=48, height=36, spp=4, n=14, bounces=32):
    """n concentric smooth glass spheres (radius 0.1 k, priority rising inward, eta alternating
    1.5 / 1.2) in front of a lambert backdrop, lit by a disk light: a camera ray through the
    middle crosses n interfaces inward, so the nested-dielectric list (pathintegrator.h:9-19)
    grows to n entries -- beyond the 10 the path kernels keep in registers."""
    d = directory or tempfile.mkdtemp(prefix="nart_nested_")
    os.makedirs(d, exist_ok=True)
    jm = []
    for k in range(n):
        name = "shell%02d" % k
        write_geo(os.path.join(d, name + ".geo"), *_uv_sphere((0.0, 0.0, 1.0), 0.1 * (n - k), 10, 20))
        jm.append({"filePath": os.path.join(d, name + ".geo"), "priority": k + 1,
                   "material": {"type": "glass", "rho_s": [1, 1, 1], "tau": [1, 1, 1],
                                "eta": 1.5 if k % 2 == 0 else 1.2, "roughness": 0}})
    write_geo(os.path.join(d, "back.geo"), *_uv_grid((-4, 3, -2), (8, 0, 0), (0, 0, 6), (0, -1, 0), 4))
    jm.append({"filePath": os.path.join(d, "back.geo"), "material": {"type": "lambert", "rho_d": [0.6, 0.5, 0.4]}})
    scene = {
        "renderSessions": [{"imageWidth": width, "imageHeight": height, "bucketSize": 8, "spp": spp,
                            "bounces": bounces, "filterWidth": 1.5, "rougheningFactor": 0.0}],
        "camera": {"fov": 20.0, "transform": [1, 0, 0, 0, 0, 0, -1, -7.0, 0, 1, 0, 1.0, 0, 0, 0, 1]},
        "meshes": jm,
        "lights": [{"type": "disk", "radius": 0.8, "Le": [1.0, 0.95, 0.9], "intensity": 40.0,
                    "transform": [1, 0, 0, 0.0, 0, 0, 1, -3.0, 0, -1, 0, 3.0, 0, 0, 0, 1]}],
    }
    path = os.path.join(d, "nested.json")
    with open(path, "w") as f:
        json.dump(scene, f, indent=1)
    return path


def sky_texture(width=128, height=64, sun=(0.3, 0.35), sun_size=0.035, sun_power=60.0):
    """Equirect sky (row 0 = zenith): blue-to-white gradient, dark ground, Gaussian sun.  Fixed
    formula, no RNG."""
    v, u = np.mgrid[0:height, 0:width].astype(np.float32)
    u, v = (u + 0.5) / width, (v + 0.5) / height
    up = np.clip(1.0 - 2.0 * v, 0.0, 1.0)
    sky = np.stack([0.55 + 0.3 * (1 - up), 0.7 + 0.2 * (1 - up), np.full_like(up, 1.0)], -1) * (v < 0.5)[..., None]
    ground = np.stack([0.18, 0.15, 0.12]) * np.ones_like(u)[..., None] * (v >= 0.5)[..., None]
    d2 = (u - sun[0]) ** 2 + ((v - sun[1]) * 0.5) ** 2
    s = sun_power * np.exp(-d2 / (2 * sun_size ** 2))
    rgb = sky + ground + np.stack([s, 0.9 * s, 0.75 * s], -1)
    return np.concatenate([rgb, np.ones_like(u)[..., None]], -1).astype(np.float32)


def environment(directory=None, width=320, height=180, spp=16, textured_env=True):
    """C4-style scene: a textured, normal-mapped plastic mesh, a rough glass sphere and a
    textured Lambert ground lit only by an importance-sampled environment light
    (environmentlight.cpp, Piecewise2DDistribution) built from sky_texture()."""
    d = directory or tempfile.mkdtemp(prefix="nart_env_")
    os.makedirs(d, exist_ok=True)
    n = 64
    yy, xx = np.mgrid[0:n, 0:n].astype(np.float32) / (n - 1)
    check = ((np.floor(xx * 6) + np.floor(yy * 6)) % 2).astype(np.float32)
    albedo = np.stack([0.25 + 0.5 * check, 0.3 + 0.4 * xx, 0.6 - 0.4 * yy, np.ones_like(xx)], -1)
    bump = np.stack([0.5 + 0.3 * np.sin(xx * 20.0), 0.5 + 0.3 * np.sin(yy * 17.0), np.full_like(xx, 0.95),
                     np.ones_like(xx)], -1)
    paths = {k: os.path.join(d, k + ".exr") for k in ("albedo", "bump", "sky")}
    write_texture(paths["albedo"], albedo)
    write_texture(paths["bump"], bump)
    write_texture(paths["sky"], sky_texture())
    write_geo(os.path.join(d, "ground.geo"), *_uv_grid((-4, -4, 0), (8, 0, 0), (0, 8, 0), (0, 0, 1), 4))
    write_geo(os.path.join(d, "ball.geo"), *_uv_sphere((-0.7, 0.2, 0.8), 0.8, 16, 32))
    write_geo(os.path.join(d, "glass.geo"), *_uv_sphere((1.0, -0.4, 0.5), 0.5))
    T = lambda p: {"type": "texture", "filePath": p}  # noqa: E731
    scene = {
        "renderSessions": [{"imageWidth": width, "imageHeight": height, "bucketSize": 16, "spp": spp,
                            "bounces": 8, "filterWidth": 2, "rougheningFactor": 0.2}],
        "camera": {"fov": 22.0, "transform": [1, 0, 0, 0, 0, 0.2588190, -0.9659258, -6.0, 0, 0.9659258, 0.2588190,
                                              2.0, 0, 0, 0, 1]},
        "meshes": [
            {"filePath": os.path.join(d, "ground.geo"), "material": {"type": "lambert", "rho_d": T(paths["albedo"])}},
            {"filePath": os.path.join(d, "ball.geo"),
             "material": {"type": "plastic", "rho_d": T(paths["albedo"]), "rho_s": [1, 1, 1], "eta": 1.5,
                          "roughness": 0.25, "normal": T(paths["bump"])}},
            {"filePath": os.path.join(d, "glass.geo"),
             "material": {"type": "glass", "rho_s": [1, 1, 1], "tau": [1, 1, 1], "eta": 1.5, "roughness": 0.1}},
        ],
        "lights": [{"type": "environment", "Le": T(paths["sky"]) if textured_env else [0.8, 0.85, 1.0],
                    "intensity": 1.5}],
    }
    path = os.path.join(d, "environment.json")
    with open(path, "w") as f:
        json.dump(scene, f, indent=1)
    return path


def write_vol(path, bounds_min, bounds_max, density):
    """.vol medium (scene.cpp:826-864): boundsMin, boundsMax, resolution, density (x fastest)."""
    d = np.asarray(density, np.float32)
    rz, ry, rx = d.shape
    toks = [_fmt(v) for v in list(bounds_min) + list(bounds_max)] + [str(rx), str(ry), str(rz)]
    toks += [_fmt(v) for v in d.reshape(-1)]
    with open(path, "w") as f:
        f.write(" ".join(toks) + "\n")


def volume(directory=None, width=320, height=180, spp=16, kind="c5"):
    """Volume-integrator scenes (volumeintegrator.cpp, media.cpp): the camera sits in a medium
    box lit by the synthetic sky.  kind "c5": BASELINE C5 (constant density 1, 2x2x2 grid, unit
    cube, sigma_a 0, sigma_s 8, Le 0, 32 bounces).  kind "emissive": a 4x3x5 density gradient
    with absorption and emission (every branch of the collision callback)."""
    d = directory or tempfile.mkdtemp(prefix="nart_vol_")
    os.makedirs(d, exist_ok=True)
    sky = os.path.join(d, "sky.exr")
    write_texture(sky, sky_texture())
    vol = os.path.join(d, "medium.vol")
    if kind == "c5":
        write_vol(vol, (-0.5, -0.5, -0.5), (0.5, 0.5, 0.5), np.ones((2, 2, 2), np.float32))
        medium = {"filePath": vol, "Le": [0, 0, 0], "sigma_a": 0.0, "sigma_s": 8.0}
        cam = [1, 0, 0, 0, 0, 0, -1, -2.5, 0, 1, 0, 0, 0, 0, 0, 1]
        bounces = 32
    else:
        z, y, x = np.mgrid[0:5, 0:3, 0:4].astype(np.float32)
        dens = 0.2 + 0.8 * (x / 3.0) * (1.0 - 0.5 * y / 2.0) + 0.3 * (z / 4.0)
        write_vol(vol, (-1.0, -0.8, -0.6), (1.2, 0.9, 1.0), dens)
        medium = {"filePath": vol, "Le": [2.0, 1.2, 0.4], "sigma_a": 1.5, "sigma_s": 3.0}
        cam = [1, 0, 0, 0.1, 0, 0, -1, -0.5, 0, 1, 0, 0.2, 0, 0, 0, 1]
        bounces = 6
    scene = {
        "renderSessions": [{"imageWidth": width, "imageHeight": height, "bucketSize": 16, "spp": spp,
                            "bounces": bounces, "filterWidth": 2, "integrator": "volume"}],
        "camera": {"fov": 30.0, "transform": cam, "medium": medium},
        "meshes": [],
        "lights": [{"type": "environment", "Le": {"type": "texture", "filePath": sky}, "intensity": 1.0}],
    }
    path = os.path.join(d, "volume_%s.json" % kind)
    with open(path, "w") as f:
        json.dump(scene, f, indent=1)
    return path


def reference_mesh(name, directory):
    """Materialise one of the reference's loose meshes (assets/meshes.npz: teapot, monkey, cube,
    plane; tools/pack_assets.py) as `directory/<name>.geo`; returns the path."""
    os.makedirs(directory, exist_ok=True)
    p = os.path.join(directory, name + ".geo")
    if not os.path.exists(p):
        z = np.load(os.path.join(ASSETS, "meshes.npz"), allow_pickle=False)
        key = "geo_%s.geo" % name
        _write_geo(p, z[key + "_kinds"], z[key + "_ints"], z[key + "_floats"])
    return p


def reference_texture(name):
    """The reference's input/textures/<name>.exr (uv, noise), shipped unchanged in assets/textures."""
    return os.path.join(ASSETS, "textures", name + ".exr")


def tangent_normal_map(n=1024, amp=0.35):
    """Tangent-space normal map of a smooth height field (fixed formula, no RNG), encoded as
    (normal + 1) / 2; every normal has z > 0.49, so no texel decodes to a zero vector."""
    v, u = np.mgrid[0:n, 0:n].astype(np.float64)
    u, v = (u + 0.5) / n, (v + 0.5) / n
    dhu = amp * 2 * np.pi * 8 * np.cos(2 * np.pi * 8 * u) * np.cos(2 * np.pi * 6 * v) * 0.1
    dhv = -amp * 2 * np.pi * 6 * np.sin(2 * np.pi * 8 * u) * np.sin(2 * np.pi * 6 * v) * 0.1
    nrm = np.stack([-dhu, -dhv, np.ones_like(u)], -1)
    nrm /= np.linalg.norm(nrm, axis=-1, keepdims=True)
    rgb = (nrm + 1.0) * 0.5
    return np.concatenate([rgb, np.ones_like(u)[..., None]], -1).astype(np.float32)


def c4_teapot(directory=None, width=3840, height=2160, spp=512, env_size=(1024, 512)):
    """C4 of BASELINE.json on the assets SURVEY 8(d) names: the reference's teapot.geo (15,704
    triangles; the reference reads it without UVs, scene.cpp:183-188) as "plastic" with
    input/textures/uv.exr (512^2, ZIPS) as rho_d, input/textures/noise.exr (1024^2, ZIPS) as the
    roughness map and a generated 1024^2 tangent-space normal map (SURVEY's alternative to
    noise.exr, which is gray noise: as a normal map 32 of its texels give 2t - 1 = 0, a NaN shading
    frame, and NaN texture coordinates that the reference's (int) texel index turns into an
    out-of-bounds read -- undefined behaviour, not a parity target), on a Lambert plane.geo
    ground, lit only by an importance-sampled environment light built from a generated 1024x512
    equirect sky (sky_texture: gradient + Gaussian sun, fixed formula, no RNG).  4K / 512 spp."""
    d = directory or tempfile.mkdtemp(prefix="nart_c4_")
    os.makedirs(d, exist_ok=True)
    teapot = reference_mesh("teapot", d)
    plane = reference_mesh("plane", d)
    sky = os.path.join(d, "sky.exr")
    write_texture(sky, sky_texture(env_size[0], env_size[1]))
    bump = os.path.join(d, "bump.exr")
    write_texture(bump, tangent_normal_map(1024))
    T = lambda p: {"type": "texture", "filePath": p}  # noqa: E731
    scene = {
        "renderSessions": [{"imageWidth": width, "imageHeight": height, "bucketSize": 16, "spp": spp,
                            "bounces": 8, "filterWidth": 2, "rougheningFactor": 0.2}],
        "camera": {"fov": 16.0, "transform": [1, 0, 0, 0.1, 0, 0.2588190, -0.9659258, -5.5, 0, 0.9659258, 0.2588190,
                                              1.1, 0, 0, 0, 1]},
        "meshes": [
            {"filePath": plane, "transform": [6, 0, 0, 0, 0, 6, 0, 0, 0, 0, 1, -1.168334, 0, 0, 0, 1],
             "material": {"type": "lambert", "rho_d": [0.45, 0.42, 0.38]}},
            {"filePath": teapot,
             "material": {"type": "plastic", "rho_d": T(reference_texture("uv")), "rho_s": [1, 1, 1], "eta": 1.5,
                          "roughness": T(reference_texture("noise")), "normal": T(bump)}},
        ],
        "lights": [{"type": "environment", "Le": T(sky), "intensity": 1.5}],
    }
    path = os.path.join(d, "c4_teapot.json")
    with open(path, "w") as f:
        json.dump(scene, f, indent=1)
    return path
