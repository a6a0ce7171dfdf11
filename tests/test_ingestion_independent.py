"""Ingestion checked against independent test-side restatements.  The oracle
renders from the product's own scene blob, so these are what make JSON/.geo/EXR ingestion more
than self-compared:
  * tests/geo_py.py restates LoadMeshFromFile (scene.cpp:77-343) and the mesh transforms
    (scene.cpp:754-767) in numpy float32 with istream extraction semantics;
  * tests/exr_py.py restates the OpenEXR scanline container and its ZIP/ZIPS/RLE codecs (zlib +
    predictor + interleave) that Imf::RgbaInputFile applies to the reference's textures
    (texturepattern.cpp:111-128) -- and decodes the product's own EXR writer output.
Both are compared bit for bit with what nart_scene_load put into the blob."""
import json
import os

import numpy as np
import pytest

import exr_py
import geo_py

REF_MESH_SCENES = ("glassSphere", "ring", "veach")


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _assert_tris_equal(got, want):
    assert got.shape == want.shape, (got.shape, want.shape)
    ne = _bits(got) != _bits(want)
    assert not ne.any(), "%d of %d floats differ (first row %d)" % (int(ne.sum()), ne.size, int(np.argwhere(ne)[0][0]))


@pytest.mark.parametrize("name", REF_MESH_SCENES)
def test_reference_scene_triangles(built, tmp_path, name):
    import nart_amd
    from nart_amd import scenes
    path = scenes.reference_scene(name, str(tmp_path))
    _assert_tris_equal(nart_amd.Scene(path).triangles(), geo_py.load_scene_triangles(path))


def _single_mesh_scene(tmp_path, mesh_path, transform=None, material=None):
    m = {"filePath": mesh_path, "material": material or {"type": "lambert", "rho_d": [0.5, 0.5, 0.5]}}
    if transform is not None:
        m["transform"] = transform
    sc = {"renderSessions": [{"imageWidth": 8, "imageHeight": 8}],
          "camera": {"fov": 20, "transform": [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1]},
          "meshes": [m],
          "lights": [{"type": "disk", "radius": 1, "Le": [1, 1, 1], "intensity": 1,
                      "transform": [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1]}]}
    p = str(tmp_path / "scene.json")
    with open(p, "w") as f:
        json.dump(sc, f)
    return p


# rotation about (1, 2, 3) by 0.7 rad, non-uniform scale (1.5, 0.4, 2.2), translation: every
# entry of inverse(M) is non-trivial, so normals exercise GLM's cofactor inverse
_c, _s = np.cos(0.7), np.sin(0.7)
_k = np.array([1.0, 2.0, 3.0]) / np.sqrt(14.0)
_K = np.array([[0, -_k[2], _k[1]], [_k[2], 0, -_k[0]], [-_k[1], _k[0], 0]])
_R = np.eye(3) + _s * _K + (1 - _c) * (_K @ _K)
_A = _R @ np.diag([1.5, 0.4, 2.2])
SKEWED = [float(_A[0, 0]), float(_A[0, 1]), float(_A[0, 2]), 0.25,
          float(_A[1, 0]), float(_A[1, 1]), float(_A[1, 2]), -1.5,
          float(_A[2, 0]), float(_A[2, 1]), float(_A[2, 2]), 3.0, 0.0, 0.0, 0.0, 1.0]


@pytest.mark.parametrize("mesh", ["teapot", "monkey", "cube", "plane"])
@pytest.mark.parametrize("transform", [None, SKEWED], ids=["identity", "skewed"])
def test_reference_mesh_triangles(built, tmp_path, mesh, transform):
    import nart_amd
    from nart_amd import scenes
    p = _single_mesh_scene(tmp_path, scenes.reference_mesh(mesh, str(tmp_path)), transform)
    _assert_tris_equal(nart_amd.Scene(p).triangles(), geo_py.load_scene_triangles(p))


def test_teapot_has_no_uvs(built, tmp_path):
    """teapot.geo's section after the normals starts with "0.418112": `>> uint32` reads 0 and the
    next read fails on ".418112" while still on the first face, so the reference loads the teapot
    without UVs (scene.cpp:183-188) and every triangle gets (0,0), (0,1), (1,0)."""
    import nart_amd
    from nart_amd import scenes
    p = _single_mesh_scene(tmp_path, scenes.reference_mesh("teapot", str(tmp_path)))
    t = nart_amd.Scene(p).triangles()
    assert t.shape[0] == 15704
    assert np.array_equal(t[:, 18:], np.tile(np.float32([0, 0, 0, 1, 1, 0]), (t.shape[0], 1)))


def test_c4_scene_triangles_and_textures(built, tmp_path):
    """The C4 scene (teapot + plane with a JSON transform, uv.exr, noise.exr, generated sky)."""
    import nart_amd
    from nart_amd import scenes
    path = scenes.c4_teapot(str(tmp_path))
    sc = nart_amd.Scene(path)
    _assert_tris_equal(sc.triangles(), geo_py.load_scene_triangles(path))
    texs = sc.textures()
    want = [exr_py.read_rgba_halves(p)[0] for p in (scenes.reference_texture("uv"), scenes.reference_texture("noise"),
                                                   os.path.join(str(tmp_path), "bump.exr"),
                                                   os.path.join(str(tmp_path), "sky.exr"))]
    assert len(texs) == len(want) == 4
    for w in want:  # each file's texels appear in the blob (load order is the JSON's pattern order)
        assert any(g.shape == w.shape and np.array_equal(g, w) for g in texs)


@pytest.mark.parametrize("name", ["uv", "noise"])
def test_reference_textures_decode(built, name):
    """The reference's ZIPS textures (input/textures/uv.exr 512^2, noise.exr 1024^2), decoded by the
    product's reader and by the independent restatement: texel for texel, as half bits."""
    import nart_amd
    from nart_amd import scenes
    path = scenes.reference_texture(name)
    halves, hdr = exr_py.read_rgba_halves(path)
    assert hdr["compression"] == exr_py.ZIPS
    mine = nart_amd.read_exr(path).astype(np.float16).view(np.uint16)
    assert np.array_equal(mine, halves)


@pytest.mark.parametrize("compression", [0, 3], ids=["none", "zip"])
def test_writer_output_decodes_independently(built, tmp_path, compression):
    """WriteImageToEXR (render.cpp:208-234) output, decoded by the restatement: crop, divide by the
    weight sum, float -> half round-to-nearest-even (numpy's float16 cast is RNE too)."""
    import nart_amd
    rng = np.random.default_rng(7)
    p = nart_amd.default_params()
    p.image_width, p.image_height, p.filter_width = 37, 21, 2.0
    g = nart_amd.session_geometry(p)
    img = rng.uniform(-3, 70000, (g.total_height, g.total_width, 5)).astype(np.float32)
    img[..., 4] = rng.uniform(0.5, 3.0, img.shape[:2]).astype(np.float32)
    out = str(tmp_path / "w.exr")
    nart_amd.write_exr(out, p, img, compression)
    halves, hdr = exr_py.read_rgba_halves(out)
    assert hdr["compression"] == (exr_py.ZIP if compression == 3 else exr_py.NONE)
    with np.errstate(over="ignore"):  # values above 65504 round to inf, as Imath does
        want = nart_amd.finalize(p, img).astype(np.float16).view(np.uint16)
    assert np.array_equal(halves, want)


REF_TEX = "/root/reference/input/textures"


@pytest.mark.skipif(not os.path.isdir(REF_TEX), reason="reference checkout not present")
@pytest.mark.parametrize("rel,rows", [("glassIceWater/iceCube_normal.exr", 512),
                                      ("glassIceWater/iceCube_roughness.exr", 512),
                                      ("glassIceWater/glass_roughness.exr", 64),
                                      ("cameraLens/lens_roughness.exr", 64)])
def test_piz_textures_independently(built, rel, rows):
    """The reference's PIZ textures (texturepattern.cpp:111-128 through Imf::RgbaInputFile: HALF
    BGR, HALF Y, FLOAT Y -> halves) decoded by the product's reader (host/exr_piz.cpp) and by the
    test-side PIZ restatement (tests/exr_piz_py.py: canonical Huffman by code length, numpy
    wavelet levels, reverse LUT) must agree half for half -- the whole 512^2 textures, the first
    PIZ chunks of the 4096^2 ones (pure Python is slow)."""
    import nart_amd
    path = os.path.join(REF_TEX, rel)
    mine, hdr = exr_py.read_rgba_halves(path, max_rows=rows)
    assert hdr["compression"] == exr_py.PIZ
    prod = nart_amd.read_exr(path).astype(np.float16).view(np.uint16)
    assert prod.shape == mine.shape
    assert np.array_equal(prod[:rows], mine[:rows]), int((prod[:rows] != mine[:rows]).sum())
