"""Independent (test-side) restatement of the reference's mesh ingestion, in numpy float32:
Scene::LoadMeshes' per-mesh transform (scene.cpp:754-767, MatrixFromVector 64-75) and
Scene::LoadMeshFromFile (scene.cpp:77-343):
  * whitespace tokens read with `istream >> uint32 / float` (libstdc++ -> strtof: glibc's strtof
    is called through ctypes);
  * vertices = transpose(M) * vec4(v, 1), normals = normalize(vec3(inverse(M) * vec4(n, 0))),
    with GLM 0.9.9.8's operation order (mat4 * vec4 = (m0 v0 + m1 v1) + (m2 v2 + m3 v3); the
    cofactor inverse of func_matrix.inl; dot3 = (x + y) + z; normalize = v * (1 / sqrt(dot)));
  * fan triangulation (0, j+1, j+2) per face, optional UVs (default (0,0), (0,1), (1,0)).
It shares no code with the product's loader (nart_amd/csrc/host/scene_host.cpp); the tests compare
the two triangle by triangle, bit for bit.  GLM is not in this image, so its operation order is
the published source's as recalled (an assumption DESIGN.md records).
"""
import ctypes
import json
import os

import numpy as np

_libc = ctypes.CDLL(None)
_libc.strtof.restype = ctypes.c_float
_libc.strtof.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
f32 = np.float32


def _strtof(tok):
    return f32(_libc.strtof(tok.encode(), None))


def matrix_from_vector(v):
    """MatrixFromVector: column i = v[4i .. 4i+3]; m[col][row] as float32 (JSON double -> float)."""
    a = np.array([f32(x) for x in v], np.float32)
    return a.reshape(4, 4)  # m[c] = column c


def mat_mul_vec(m, v):
    """GLM mat4 * vec4: (m[0] v0 + m[1] v1) + (m[2] v2 + m[3] v3), columns m[c], float32."""
    with np.errstate(all="ignore"):
        return ((m[0] * v[0] + m[1] * v[1]) + (m[2] * v[2] + m[3] * v[3])).astype(np.float32)


def transpose(m):
    return np.ascontiguousarray(m.T)


def inverse(m):
    """GLM compute_inverse<4,4> (cofactors, then * (1 / det)), float32 throughout."""
    with np.errstate(all="ignore"):
        c00 = m[2][2] * m[3][3] - m[3][2] * m[2][3]
        c02 = m[1][2] * m[3][3] - m[3][2] * m[1][3]
        c03 = m[1][2] * m[2][3] - m[2][2] * m[1][3]
        c04 = m[2][1] * m[3][3] - m[3][1] * m[2][3]
        c06 = m[1][1] * m[3][3] - m[3][1] * m[1][3]
        c07 = m[1][1] * m[2][3] - m[2][1] * m[1][3]
        c08 = m[2][1] * m[3][2] - m[3][1] * m[2][2]
        c10 = m[1][1] * m[3][2] - m[3][1] * m[1][2]
        c11 = m[1][1] * m[2][2] - m[2][1] * m[1][2]
        c12 = m[2][0] * m[3][3] - m[3][0] * m[2][3]
        c14 = m[1][0] * m[3][3] - m[3][0] * m[1][3]
        c15 = m[1][0] * m[2][3] - m[2][0] * m[1][3]
        c16 = m[2][0] * m[3][2] - m[3][0] * m[2][2]
        c18 = m[1][0] * m[3][2] - m[3][0] * m[1][2]
        c19 = m[1][0] * m[2][2] - m[2][0] * m[1][2]
        c20 = m[2][0] * m[3][1] - m[3][0] * m[2][1]
        c22 = m[1][0] * m[3][1] - m[3][0] * m[1][1]
        c23 = m[1][0] * m[2][1] - m[2][0] * m[1][1]
        A = lambda *x: np.array(x, np.float32)  # noqa: E731
        fac0, fac1, fac2 = A(c00, c00, c02, c03), A(c04, c04, c06, c07), A(c08, c08, c10, c11)
        fac3, fac4, fac5 = A(c12, c12, c14, c15), A(c16, c16, c18, c19), A(c20, c20, c22, c23)
        vec0 = A(m[1][0], m[0][0], m[0][0], m[0][0])
        vec1 = A(m[1][1], m[0][1], m[0][1], m[0][1])
        vec2 = A(m[1][2], m[0][2], m[0][2], m[0][2])
        vec3 = A(m[1][3], m[0][3], m[0][3], m[0][3])
        inv0 = (vec1 * fac0 - vec2 * fac1) + vec3 * fac2
        inv1 = (vec0 * fac0 - vec2 * fac3) + vec3 * fac4
        inv2 = (vec0 * fac1 - vec1 * fac3) + vec3 * fac5
        inv3 = (vec0 * fac2 - vec1 * fac4) + vec2 * fac5
        sa, sb = A(1, -1, 1, -1), A(-1, 1, -1, 1)
        inv = np.stack([inv0 * sa, inv1 * sb, inv2 * sa, inv3 * sb]).astype(np.float32)
        row0 = A(inv[0][0], inv[1][0], inv[2][0], inv[3][0])
        dot0 = m[0] * row0
        dot1 = f32((dot0[0] + dot0[1]) + (dot0[2] + dot0[3]))
        one_over_det = f32(f32(1) / dot1)
        return (inv * one_over_det).astype(np.float32)


def normalize3(v):
    with np.errstate(all="ignore"):
        d = f32(f32(v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])
        return (v * f32(f32(1) / np.sqrt(d))).astype(np.float32)


class IStream:
    """`std::istream >> uint32_t / float` (libstdc++ num_get): skip white space, take the longest
    prefix of the number's grammar; a read that takes no digits fails."""

    def __init__(self, text):
        self.s, self.p = text, 0

    def _ws(self):
        while self.p < len(self.s) and self.s[self.p].isspace():
            self.p += 1

    def u32(self):
        self._ws()
        s, neg = self.s, False
        if self.p < len(s) and s[self.p] in "+-":
            neg = s[self.p] == "-"
            self.p += 1
        b = self.p
        while self.p < len(s) and s[self.p].isdigit():
            self.p += 1
        if self.p == b or int(s[b:self.p]) > 0xFFFFFFFF:
            return None
        x = int(s[b:self.p])
        return (-x) & 0xFFFFFFFF if neg else x

    def f32(self):
        self._ws()
        s, b = self.s, self.p
        if self.p < len(s) and s[self.p] in "+-":
            self.p += 1
        any_d = False
        while self.p < len(s) and s[self.p].isdigit():
            self.p += 1
            any_d = True
        if self.p < len(s) and s[self.p] == ".":
            self.p += 1
            while self.p < len(s) and s[self.p].isdigit():
                self.p += 1
                any_d = True
        if any_d and self.p < len(s) and s[self.p] in "eE":
            self.p += 1
            if self.p < len(s) and s[self.p] in "+-":
                self.p += 1
            while self.p < len(s) and s[self.p].isdigit():
                self.p += 1
        tok = s[b:self.p]
        if not any_d:
            return None
        return _strtof(tok)


def load_geo(path, m):
    """LoadMeshFromFile(path, objectToWorld = m): (n_tris, 24) float32 rows in nart_triangle order
    (v0 v1 v2 n0 n1 n2 uv0 uv1 uv2)."""
    st = IStream(open(path).read())

    def need(x):
        assert x is not None, "Mesh file could not be read"
        return x

    nf = need(st.u32())
    faces = [need(st.u32()) for _ in range(nf)]
    nvi = sum(faces)
    vidx = [need(st.u32()) for _ in range(nvi)]
    vc = np.array([need(st.f32()) for _ in range((max(vidx) + 1) * 3)], np.float32)
    nidx = [need(st.u32()) for _ in range(nvi)]
    nc = np.array([need(st.f32()) for _ in range((max(nidx) + 1) * 3)], np.float32)
    # UVs: absent when a read fails while still on the first face (scene.cpp:179-205)
    uvidx = []
    for k in range(nvi):
        x = st.u32()
        if x is None:
            assert k < faces[0], "Mesh file could not be read"
            uvidx = None
            break
        uvidx.append(x)
    if uvidx is not None:
        uc = np.array([need(st.f32()) for _ in range((max(uvidx) + 1) * 2)], np.float32)
    tm = transpose(m)
    im = inverse(m)
    verts = [mat_mul_vec(tm, np.array([vc[3 * i], vc[3 * i + 1], vc[3 * i + 2], 1], np.float32))[:3]
             for i in range(len(vc) // 3)]
    norms = [normalize3(mat_mul_vec(im, np.array([nc[3 * i], nc[3 * i + 1], nc[3 * i + 2], 0], np.float32))[:3])
             for i in range(len(nc) // 3)]
    uvs = [uc[2 * i:2 * i + 2] for i in range(len(uc) // 2)] if uvidx is not None else None
    rows = []
    l = 0
    for f in faces:
        for j in range(f - 2):
            k = (l, l + j + 1, l + j + 2)
            v = [verts[vidx[q]] for q in k]
            n = [norms[nidx[q]] for q in k]
            if uvs is not None:
                t = [uvs[uvidx[q]] for q in k]
            else:
                t = [np.float32([0, 0]), np.float32([0, 1]), np.float32([1, 0])]
            rows.append(np.concatenate(v + n + t))
        l += f
    return np.array(rows, np.float32).reshape(-1, 24)


def load_scene_triangles(json_path):
    """Every mesh of a scene in JSON order (LoadMeshes): the triangles the reference builds."""
    scene = json.load(open(json_path))
    out = []
    for m in scene.get("meshes", []):
        tr = m.get("transform", [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1])
        path = m["filePath"]
        if not os.path.isabs(path):
            path = os.path.join(os.path.dirname(json_path), path)
        out.append(load_geo(path, matrix_from_vector(tr)))
    return np.concatenate(out) if out else np.zeros((0, 24), np.float32)
