// Host-side scene ingestion, session resolution, filter table, tile combine and EXR I/O
// for the nart drop-in.  Every function states the reference code it reproduces.
//
// Arithmetic that reaches the renderer (vertex/normal transforms, constant clamps, the
// filter table) follows GLM 0.9.9.8's scalar code paths operation by operation:
//   mat4 * vec4 = (m0*v0 + m1*v1) + (m2*v2 + m3*v3)      (type_mat4x4.inl operator*)
//   normalize(v) = v * (1 / sqrt(dot(v, v)))             (func_geometric.inl, inversesqrt)
//   vec3 dot = (x*x' + y*y') + z*z'                      (compute_dot<vec3>)
//   inverse  = cofactor form of compute_inverse<4,4>     (func_matrix.inl)
// and is compiled with -ffp-contract=off so no multiply-add is fused.
#include <algorithm>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include <zlib.h>

#include "../../../include/nart_scene.h"
#include "exr_piz.h"
#include "json.h"

namespace {

thread_local std::string g_error;

int set_error(int code, const std::string& msg) {
    g_error = msg;
    return code;
}

const float kOneMinusEps = 1.f - 1.1920928955078125e-07f;  // 1 - glm::epsilon<float>()

inline float glm_min(float a, float b) { return (b < a) ? b : a; }
inline float glm_max(float a, float b) { return (a < b) ? b : a; }

// glm::inverse for mat4 (compute_inverse<4,4,float>), m[c*4+r].
void glm_inverse(const float* m, float* out) {
    auto M = [&](int c, int r) { return m[c * 4 + r]; };
    float Coef00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3);
    float Coef02 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
    float Coef03 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3);
    float Coef04 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
    float Coef06 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3);
    float Coef07 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
    float Coef08 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2);
    float Coef10 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
    float Coef11 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2);
    float Coef12 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
    float Coef14 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3);
    float Coef15 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
    float Coef16 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2);
    float Coef18 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
    float Coef19 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2);
    float Coef20 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
    float Coef22 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1);
    float Coef23 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
    float Fac0[4] = {Coef00, Coef00, Coef02, Coef03};
    float Fac1[4] = {Coef04, Coef04, Coef06, Coef07};
    float Fac2[4] = {Coef08, Coef08, Coef10, Coef11};
    float Fac3[4] = {Coef12, Coef12, Coef14, Coef15};
    float Fac4[4] = {Coef16, Coef16, Coef18, Coef19};
    float Fac5[4] = {Coef20, Coef20, Coef22, Coef23};
    float Vec0[4] = {M(1, 0), M(0, 0), M(0, 0), M(0, 0)};
    float Vec1[4] = {M(1, 1), M(0, 1), M(0, 1), M(0, 1)};
    float Vec2[4] = {M(1, 2), M(0, 2), M(0, 2), M(0, 2)};
    float Vec3[4] = {M(1, 3), M(0, 3), M(0, 3), M(0, 3)};
    float Inv[4][4];
    const float SignA[4] = {+1.f, -1.f, +1.f, -1.f};
    const float SignB[4] = {-1.f, +1.f, -1.f, +1.f};
    for (int k = 0; k < 4; ++k) {
        float i0 = (Vec1[k] * Fac0[k] - Vec2[k] * Fac1[k]) + Vec3[k] * Fac2[k];
        float i1 = (Vec0[k] * Fac0[k] - Vec2[k] * Fac3[k]) + Vec3[k] * Fac4[k];
        float i2 = (Vec0[k] * Fac1[k] - Vec1[k] * Fac3[k]) + Vec3[k] * Fac5[k];
        float i3 = (Vec0[k] * Fac2[k] - Vec1[k] * Fac4[k]) + Vec2[k] * Fac5[k];
        Inv[0][k] = i0 * SignA[k];
        Inv[1][k] = i1 * SignB[k];
        Inv[2][k] = i2 * SignA[k];
        Inv[3][k] = i3 * SignB[k];
    }
    float Row0[4] = {Inv[0][0], Inv[1][0], Inv[2][0], Inv[3][0]};
    float Dot0[4];
    for (int k = 0; k < 4; ++k) Dot0[k] = M(0, k) * Row0[k];
    float Dot1 = (Dot0[0] + Dot0[1]) + (Dot0[2] + Dot0[3]);
    float OneOverDeterminant = 1.f / Dot1;
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out[c * 4 + r] = Inv[c][r] * OneOverDeterminant;
}

// glm mat4 * vec4 (column-vector form).
void glm_mat_vec(const float* m, const float* v, float* out) {
    for (int r = 0; r < 4; ++r)
        out[r] = (m[0 * 4 + r] * v[0] + m[1 * 4 + r] * v[1]) + (m[2 * 4 + r] * v[2] + m[3 * 4 + r] * v[3]);
}

void glm_normalize3(float* v) {
    float d = (v[0] * v[0] + v[1] * v[1]) + v[2] * v[2];
    float s = 1.f / std::sqrt(d);
    v[0] *= s;
    v[1] *= s;
    v[2] *= s;
}

bool read_file(const std::string& path, std::string& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

// Whitespace token reader reproducing `std::istream >> uint32_t / float` on .geo files.
struct TokenReader {
    const std::string& s;
    size_t p = 0;
    explicit TokenReader(const std::string& str) : s(str) {}
    bool next(std::string& tok) {
        while (p < s.size() && std::isspace(static_cast<unsigned char>(s[p]))) ++p;
        if (p >= s.size()) return false;
        size_t b = p;
        while (p < s.size() && !std::isspace(static_cast<unsigned char>(s[p]))) ++p;
        tok = s.substr(b, p - b);
        return true;
    }
    // `std::istream >> uint32_t` / `>> float` as libstdc++'s num_get extracts them: skip white
    // space, then take the longest prefix that fits the number's grammar -- NOT the whole
    // white-space-delimited token.  "0.418112" read as an integer gives 0 and leaves ".418112",
    // whose next integer read fails (teapot.geo's UV section: scene.cpp:179-205 then decides the
    // mesh has no UVs).
    void skip_ws() {
        while (p < s.size() && std::isspace(static_cast<unsigned char>(s[p]))) ++p;
    }
    static bool digit(char c) { return c >= '0' && c <= '9'; }
    bool u32(uint32_t& v) {
        skip_ws();
        bool neg = false;
        if (p < s.size() && (s[p] == '+' || s[p] == '-')) neg = s[p++] == '-';
        const size_t b = p;
        uint64_t x = 0;
        bool overflow = false;
        while (p < s.size() && digit(s[p])) {
            x = x * 10 + (uint64_t)(s[p++] - '0');
            if (x > 0xFFFFFFFFull) overflow = true, x = 0xFFFFFFFFull;
        }
        if (p == b || overflow) return false;  // failbit (no digits / out of range)
        v = neg ? (uint32_t)(0u - (uint32_t)x) : (uint32_t)x;  // num_get negates unsigned values
        return true;
    }
    bool f32(float& v) {
        skip_ws();
        const size_t b = p;
        if (p < s.size() && (s[p] == '+' || s[p] == '-')) ++p;
        bool any = false;
        while (p < s.size() && digit(s[p])) ++p, any = true;
        if (p < s.size() && s[p] == '.') {
            ++p;
            while (p < s.size() && digit(s[p])) ++p, any = true;
        }
        if (any && p < s.size() && (s[p] == 'e' || s[p] == 'E')) {
            ++p;
            if (p < s.size() && (s[p] == '+' || s[p] == '-')) ++p;
            while (p < s.size() && digit(s[p])) ++p;
        }
        const std::string t = s.substr(b, p - b);
        char* end = nullptr;
        v = std::strtof(t.c_str(), &end);  // num_get<float> -> __convert_to_v -> strtof
        return !t.empty() && end == t.c_str() + t.size();
    }
};

}  // namespace

struct nart_scene {
    nart_scene_blob blob;
    std::vector<nart_triangle> triangles;
    std::vector<nart_mesh> meshes;
    std::vector<nart_material> materials;
    std::vector<nart_light> lights;
    std::vector<nart_texture> textures;
    std::vector<std::vector<uint16_t>> texture_data;
    std::vector<std::string> texture_paths;
    std::vector<float> density;
};

namespace {

// MatrixFromVector (scene.cpp:64-75): column i = elements 4i..4i+3.
bool matrix_from_vector(const std::vector<float>& v, float* m) {
    if (v.size() < 16) return false;
    for (int i = 0; i < 16; ++i) m[i] = v[i];
    return true;
}

int load_texture(nart_scene* sc, const std::string& path, bool is_roughness, nart_pattern& ptn) {
    ptn.type = NART_PTN_TEXTURE;
    ptn.is_roughness = is_roughness ? 1 : 0;
    for (size_t i = 0; i < sc->texture_paths.size(); ++i) {
        if (sc->texture_paths[i] == path) {
            ptn.texture = static_cast<int32_t>(i);
            return NART_OK;
        }
    }
    uint32_t w = 0, h = 0;
    uint16_t* data = nullptr;
    int rc = nart_read_exr_rgba(path.c_str(), &w, &h, &data);
    if (rc != NART_OK) return rc;
    sc->texture_data.emplace_back(data, data + size_t(w) * h * 4);
    nart_free(data);
    nart_texture t;
    t.width = w;
    t.height = h;
    t.rgba = nullptr;
    sc->textures.push_back(t);
    sc->texture_paths.push_back(path);
    ptn.texture = static_cast<int32_t>(sc->textures.size() - 1);
    return NART_OK;
}

nart_pattern constant_pattern(float x, float y, float z) {
    nart_pattern p;
    std::memset(&p, 0, sizeof(p));
    p.type = NART_PTN_CONSTANT;
    p.value[0] = x;
    p.value[1] = y;
    p.value[2] = z;
    p.texture = -1;
    return p;
}

// Shared shape of GetRho_s / GetTau / GetLe (scene.cpp:388-431, 468-510, 549-590):
// object -> only "texture" is accepted (the "constant" branch falls into the else-abort,
// scene.cpp:352-374); array -> each component clamped to 1 - epsilon.
int get_vec_pattern(nart_scene* sc, const nartjson::Value& mat, const char* key, bool clamp,
                    bool roughness_tex, nart_pattern& out) {
    const nartjson::Value& v = mat[key];
    if (v.is_object()) {
        std::string type = v["type"].str();
        if (type == "texture") return load_texture(sc, v["filePath"].str(), roughness_tex, out);
        return set_error(NART_E_INVALID, "Error: '" + type + "' is not a pattern type (scene.cpp:352-374 aborts)");
    }
    std::vector<float> g = v.floats();
    if (g.size() < 3) return set_error(NART_E_INVALID, std::string("pattern '") + key + "' needs 3 values");
    if (clamp)
        out = constant_pattern(glm_min(g[0], kOneMinusEps), glm_min(g[1], kOneMinusEps), glm_min(g[2], kOneMinusEps));
    else
        out = constant_pattern(g[0], g[1], g[2]);
    return NART_OK;
}

// GetEta (scene.cpp:433-466)
int get_eta(nart_scene* sc, const nartjson::Value& mat, nart_pattern& out) {
    const nartjson::Value& v = mat["eta"];
    if (v.is_object()) {
        std::string type = v["type"].str();
        if (type == "texture") return load_texture(sc, v["filePath"].str(), false, out);
        return set_error(NART_E_INVALID, "Error: '" + type + "' is not a pattern type (scene.cpp:439-456 aborts)");
    }
    float eta = v.num<float>();
    out = constant_pattern(eta, eta, eta);
    return NART_OK;
}

// GetAlpha (scene.cpp:512-546): alpha = roughness^2; textures square per fetch.
int get_alpha(nart_scene* sc, const nartjson::Value& mat, nart_pattern& out) {
    const nartjson::Value& v = mat["roughness"];
    if (v.is_object()) {
        std::string type = v["type"].str();
        if (type == "texture") return load_texture(sc, v["filePath"].str(), true, out);
        return set_error(NART_E_INVALID, "Error: '" + type + "' is not a pattern type (scene.cpp:518-536 aborts)");
    }
    float r = v.num<float>();
    float a = r * r;
    out = constant_pattern(a, a, a);
    return NART_OK;
}

// GetNormal (scene.cpp:592-642)
int get_normal(nart_scene* sc, const nartjson::Value& mat, nart_pattern& out, int32_t& has) {
    has = 0;
    if (!mat.contains("normal")) return NART_OK;
    const nartjson::Value& v = mat["normal"];
    if (v.is_object()) {
        std::string type = v["type"].str();
        if (type == "texture") {
            has = 1;
            return load_texture(sc, v["filePath"].str(), false, out);
        }
        return set_error(NART_E_INVALID, "Error: '" + type + "' is not a pattern type (scene.cpp:599-621 aborts)");
    }
    if (v.is_array()) {
        std::vector<float> g = v.floats();
        if (g.size() < 3) return set_error(NART_E_INVALID, "normal needs 3 values");
        out = constant_pattern(glm_min(g[0], kOneMinusEps), glm_min(g[1], kOneMinusEps), glm_min(g[2], kOneMinusEps));
        has = 1;
    }
    return NART_OK;
}

// LoadMeshFromFile (scene.cpp:77-343)
int load_geo(nart_scene* sc, const std::string& path, const float* objectToWorld, uint32_t mesh_id,
             uint32_t material, uint32_t priority) {
    std::string text;
    if (!read_file(path, text)) return set_error(NART_E_IO, "Error: Mesh file " + path + " could not be opened.");
    TokenReader rd(text);
    uint32_t numFaces = 0;
    if (!rd.u32(numFaces)) return set_error(NART_E_IO, "Error: Mesh file could not be read: " + path);
    std::vector<uint32_t> faces(numFaces);
    uint32_t numVertIndices = 0;
    for (uint32_t i = 0; i < numFaces; ++i) {
        if (!rd.u32(faces[i])) return set_error(NART_E_IO, "Error: Mesh file could not be read: " + path);
        if (faces[i] < 3) return set_error(NART_E_INVALID, "face with fewer than 3 vertices in " + path);
        numVertIndices += faces[i];
    }
    std::vector<uint32_t> vertIndices(numVertIndices);
    uint32_t maxVertIndex = 0;
    for (uint32_t k = 0; k < numVertIndices; ++k) {
        if (!rd.u32(vertIndices[k])) return set_error(NART_E_IO, "Error: Mesh file could not be read: " + path);
        maxVertIndex = vertIndices[k] > maxVertIndex ? vertIndices[k] : maxVertIndex;
    }
    uint32_t numVertCoords = (maxVertIndex + 1) * 3;
    std::vector<float> vertCoords(numVertCoords);
    for (uint32_t i = 0; i < numVertCoords; ++i)
        if (!rd.f32(vertCoords[i])) return set_error(NART_E_IO, "Error: Mesh file could not be read: " + path);
    std::vector<uint32_t> normIndices(numVertIndices);
    uint32_t maxNormIndex = 0;
    for (uint32_t k = 0; k < numVertIndices; ++k) {
        if (!rd.u32(normIndices[k])) return set_error(NART_E_IO, "Error: Mesh file could not be read: " + path);
        maxNormIndex = normIndices[k] > maxNormIndex ? normIndices[k] : maxNormIndex;
    }
    uint32_t numNormCoords = (maxNormIndex + 1) * 3;
    std::vector<float> normCoords(numNormCoords);
    for (uint32_t i = 0; i < numNormCoords; ++i)
        if (!rd.f32(normCoords[i])) return set_error(NART_E_IO, "Error: Mesh file could not be read: " + path);
    // UVs (optional): absent if the very first UV index cannot be read (scene.cpp:174-205)
    std::vector<uint32_t> UVIndices(numVertIndices);
    bool noUVs = false;
    uint32_t maxUVIndex = 0;
    for (uint32_t k = 0; k < numVertIndices; ++k) {
        if (!rd.u32(UVIndices[k])) {
            if (k < faces[0]) {
                noUVs = true;
                break;
            }
            return set_error(NART_E_IO, "Error: Mesh file could not be read: " + path);
        }
        maxUVIndex = UVIndices[k] > maxUVIndex ? UVIndices[k] : maxUVIndex;
    }
    std::vector<float> UVCoords;
    if (!noUVs) {
        uint32_t numUVCoords = (maxUVIndex + 1) * 2;
        UVCoords.resize(numUVCoords);
        for (uint32_t i = 0; i < numUVCoords; ++i)
            if (!rd.f32(UVCoords[i])) return set_error(NART_E_IO, "Error: Mesh file could not be read: " + path);
    }

    // verts = transpose(objectToWorld) * vec4(v, 1)   (scene.cpp:236-243)
    float T[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) T[c * 4 + r] = objectToWorld[r * 4 + c];
    std::vector<float> verts((maxVertIndex + 1) * 3);
    for (uint32_t i = 0; i <= maxVertIndex; ++i) {
        float v4[4] = {vertCoords[3 * i], vertCoords[3 * i + 1], vertCoords[3 * i + 2], 1.f}, o[4];
        glm_mat_vec(T, v4, o);
        verts[3 * i] = o[0];
        verts[3 * i + 1] = o[1];
        verts[3 * i + 2] = o[2];
    }
    // norms = normalize(vec3(inverse(objectToWorld) * vec4(n, 0)))   (scene.cpp:245-256)
    float I[16];
    glm_inverse(objectToWorld, I);
    std::vector<float> norms((maxNormIndex + 1) * 3);
    for (uint32_t i = 0; i <= maxNormIndex; ++i) {
        float n4[4] = {normCoords[3 * i], normCoords[3 * i + 1], normCoords[3 * i + 2], 0.f}, o[4];
        glm_mat_vec(I, n4, o);
        glm_normalize3(o);
        norms[3 * i] = o[0];
        norms[3 * i + 1] = o[1];
        norms[3 * i + 2] = o[2];
    }

    nart_mesh mesh;
    mesh.first_tri = static_cast<uint32_t>(sc->triangles.size());
    mesh.material = material;
    mesh.priority = priority;
    // Fan triangulation (scene.cpp:270-339); default UVs (0,0),(0,1),(1,0) (geometry.h:56-58)
    uint32_t l = 0;
    for (uint32_t f = 0; f < numFaces; ++f) {
        for (uint32_t j = 0; j + 2 < faces[f]; ++j) {
            uint32_t idx[3] = {l, l + j + 1, l + j + 2};
            nart_triangle t;
            float* vp[3] = {t.v0, t.v1, t.v2};
            float* np[3] = {t.n0, t.n1, t.n2};
            float* up[3] = {t.uv0, t.uv1, t.uv2};
            const float defuv[3][2] = {{0.f, 0.f}, {0.f, 1.f}, {1.f, 0.f}};
            for (int c = 0; c < 3; ++c) {
                uint32_t vi = vertIndices[idx[c]], ni = normIndices[idx[c]];
                std::memcpy(vp[c], &verts[3 * vi], 12);
                std::memcpy(np[c], &norms[3 * ni], 12);
                if (noUVs) {
                    up[c][0] = defuv[c][0];
                    up[c][1] = defuv[c][1];
                } else {
                    uint32_t ui = UVIndices[idx[c]];
                    up[c][0] = UVCoords[2 * ui];
                    up[c][1] = UVCoords[2 * ui + 1];
                }
            }
            sc->triangles.push_back(t);
        }
        l += faces[f];
    }
    mesh.num_tris = static_cast<uint32_t>(sc->triangles.size()) - mesh.first_tri;
    (void)mesh_id;
    sc->meshes.push_back(mesh);
    return NART_OK;
}

int load_scene(nart_scene* sc, const std::string& json_path) {
    std::string text;
    if (!read_file(json_path, text)) return set_error(NART_E_IO, "Error: Scene file could not be opened.");
    nartjson::Value json;
    try {
        json = nartjson::Parser(text).parse();
    } catch (std::exception& e) {
        return set_error(NART_E_INVALID, std::string("Error parsing scene: ") + e.what());
    }
    try {
        // LoadCamera (scene.cpp:782-875)
        float camM[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        float fov = 11.f;
        std::memset(&sc->blob.medium, 0, sizeof(sc->blob.medium));
        if (json.contains("camera")) {
            const nartjson::Value& cam = json["camera"];
            fov = cam["fov"].num<float>();
            if (!matrix_from_vector(cam["transform"].floats(), camM))
                return set_error(NART_E_INVALID, "Error in camera: transform needs 16 values");
            if (cam.contains("medium")) {
                const nartjson::Value& med = cam["medium"];
                std::string vpath = med["filePath"].str();
                std::vector<float> le = med["Le"].floats();
                nart_medium& m = sc->blob.medium;
                m.Le[0] = le.at(0);
                m.Le[1] = le.at(1);
                m.Le[2] = le.at(2);
                m.sigma_a = med["sigma_a"].num<float>();
                m.sigma_s = med["sigma_s"].num<float>();
                std::string vtext;
                if (!read_file(vpath, vtext)) return set_error(NART_E_IO, "Error: Volume file " + vpath + " could not be opened.");
                TokenReader rd(vtext);
                for (int i = 0; i < 3; ++i)
                    if (!rd.f32(m.bounds_min[i])) return set_error(NART_E_IO, "Error: Volume file could not be read.");
                for (int i = 0; i < 3; ++i)
                    if (!rd.f32(m.bounds_max[i])) return set_error(NART_E_IO, "Error: Volume file could not be read.");
                for (int i = 0; i < 3; ++i)
                    if (!rd.u32(m.res[i])) return set_error(NART_E_IO, "Error: Volume file could not be read.");
                uint64_t npts = uint64_t(m.res[0]) * m.res[1] * m.res[2];
                sc->density.assign(npts, 0.f);
                for (uint64_t i = 0; i < npts; ++i)
                    if (!rd.f32(sc->density[i])) return set_error(NART_E_IO, "Error: Volume file could not be read.");
                m.present = 1;
            }
        }
        sc->blob.camera.fov = fov;
        std::memcpy(sc->blob.camera.m, camM, sizeof(camM));

        // LoadMeshes (scene.cpp:644-780)
        if (json.contains("meshes")) {
            const nartjson::Value& meshes = json["meshes"];
            uint32_t id = 0;
            for (const nartjson::Value& elem : meshes.arr) {
                std::string path = elem["filePath"].str();
                const nartjson::Value& mat = elem["material"];
                std::string type = mat["type"].str();
                nart_material m;
                std::memset(&m, 0, sizeof(m));
                m.rho_d = m.rho_s = m.tau = m.eta = m.alpha = m.normal = constant_pattern(0, 0, 0);
                int rc = NART_OK;
                if (type == "lambert") {
                    m.type = NART_MAT_LAMBERT;
                    // plain-array rho_d is NOT clamped (scene.cpp:377-383)
                    rc = get_vec_pattern(sc, mat, "rho_d", false, false, m.rho_d);
                    if (!rc) rc = get_normal(sc, mat, m.normal, m.has_normal);
                } else if (type == "specular") {
                    m.type = NART_MAT_SPECULAR;
                    rc = get_vec_pattern(sc, mat, "rho_s", true, false, m.rho_s);
                    if (!rc) rc = get_eta(sc, mat, m.eta);
                    if (!rc) rc = get_normal(sc, mat, m.normal, m.has_normal);
                } else if (type == "glass") {
                    m.type = NART_MAT_GLASS;
                    rc = get_vec_pattern(sc, mat, "rho_s", true, false, m.rho_s);
                    if (!rc) rc = get_vec_pattern(sc, mat, "tau", true, false, m.tau);
                    if (!rc) rc = get_eta(sc, mat, m.eta);
                    if (!rc) rc = get_alpha(sc, mat, m.alpha);
                    if (!rc) rc = get_normal(sc, mat, m.normal, m.has_normal);
                    m.has_normal = 0;  // GlassMaterial self-moves normalPtn: always null (glassmaterial.cpp:3-9)
                } else if (type == "glossy") {
                    m.type = NART_MAT_GLOSSY;
                    rc = get_vec_pattern(sc, mat, "rho_s", true, false, m.rho_s);
                    if (!rc) rc = get_eta(sc, mat, m.eta);
                    if (!rc) rc = get_alpha(sc, mat, m.alpha);
                    if (!rc) rc = get_normal(sc, mat, m.normal, m.has_normal);
                } else if (type == "plastic") {
                    m.type = NART_MAT_PLASTIC;
                    rc = get_vec_pattern(sc, mat, "rho_d", false, false, m.rho_d);
                    if (!rc) rc = get_vec_pattern(sc, mat, "rho_s", true, false, m.rho_s);
                    if (!rc) rc = get_eta(sc, mat, m.eta);
                    if (!rc) rc = get_alpha(sc, mat, m.alpha);
                    if (!rc) rc = get_normal(sc, mat, m.normal, m.has_normal);
                } else {
                    return set_error(NART_E_INVALID, "Error: '" + type + "' is not a material type.");
                }
                if (rc) return rc;
                sc->materials.push_back(m);
                // priority: get<uint8_t>() (scene.cpp:739-752)
                uint32_t priority = 0;
                if (!elem["priority"].is_null()) priority = static_cast<uint8_t>(elem["priority"].num<uint8_t>());
                // transform (scene.cpp:755-767), default identity
                float M[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
                if (!elem["transform"].is_null() && !matrix_from_vector(elem["transform"].floats(), M))
                    return set_error(NART_E_INVALID, "Error in mesh transform");
                rc = load_geo(sc, path, M, id, static_cast<uint32_t>(sc->materials.size() - 1), priority);
                if (rc) return rc;
                ++id;
            }
        }

        // LoadLights (scene.cpp:877-932).  Unknown types are skipped; no "distant" branch.
        if (!json["lights"].is_null()) {
            for (const nartjson::Value& elem : json["lights"].arr) {
                nart_light L;
                std::memset(&L, 0, sizeof(L));
                float M[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
                if (!elem["transform"].is_null() && !matrix_from_vector(elem["transform"].floats(), M))
                    return set_error(NART_E_INVALID, "Error in light transform");
                std::memcpy(L.m, M, sizeof(M));
                std::string type = elem["type"].str();
                int rc = NART_OK;
                if (type == "disk") {
                    L.type = NART_LIGHT_DISK;
                    L.radius = elem["radius"].num<float>();
                    rc = get_vec_pattern(sc, elem, "Le", true, false, L.Le);
                    L.intensity = elem["intensity"].num<float>();
                } else if (type == "ring") {
                    L.type = NART_LIGHT_RING;
                    L.radius = elem["radius"].num<float>();
                    L.inner_radius = elem["innerRadius"].num<float>();
                    rc = get_vec_pattern(sc, elem, "Le", true, false, L.Le);
                    L.intensity = elem["intensity"].num<float>();
                } else if (type == "environment") {
                    L.type = NART_LIGHT_ENVIRONMENT;
                    rc = get_vec_pattern(sc, elem, "Le", true, false, L.Le);
                    L.intensity = elem["intensity"].num<float>();
                } else {
                    continue;
                }
                if (rc) return rc;
                sc->lights.push_back(L);
            }
        }
    } catch (std::exception& e) {
        return set_error(NART_E_INVALID, std::string("Error in scene: ") + e.what());
    }
    if (sc->lights.size() > 255) return set_error(NART_E_INVALID, "more than 255 lights (uint8 light index)");

    for (size_t i = 0; i < sc->textures.size(); ++i) sc->textures[i].rgba = sc->texture_data[i].data();
    nart_scene_blob& b = sc->blob;
    b.num_triangles = static_cast<uint32_t>(sc->triangles.size());
    b.num_meshes = static_cast<uint32_t>(sc->meshes.size());
    b.num_materials = static_cast<uint32_t>(sc->materials.size());
    b.num_lights = static_cast<uint32_t>(sc->lights.size());
    b.num_textures = static_cast<uint32_t>(sc->textures.size());
    b.reserved = 0;
    b.triangles = sc->triangles.data();
    b.meshes = sc->meshes.data();
    b.materials = sc->materials.data();
    b.lights = sc->lights.data();
    b.textures = sc->textures.data();
    b.medium.density = sc->density.empty() ? nullptr : sc->density.data();
    return NART_OK;
}

// std::stoi / std::stof front ends (render.cpp:236-325): leading integer/float prefix,
// invalid_argument when no conversion is possible.
bool stoi_like(const char* s, int& out) {
    char* end = nullptr;
    errno = 0;
    long v = std::strtol(s, &end, 10);
    if (end == s || errno == ERANGE || v < INT32_MIN || v > INT32_MAX) return false;
    out = static_cast<int>(v);
    return true;
}
bool stof_like(const char* s, float& out) {
    char* end = nullptr;
    errno = 0;
    float v = std::strtof(s, &end);
    if (end == s || errno == ERANGE) return false;
    out = v;
    return true;
}

// ---- EXR helpers -------------------------------------------------------------------
void put_u8(std::vector<uint8_t>& b, uint8_t v) { b.push_back(v); }
void put_i32(std::vector<uint8_t>& b, int32_t v) {
    for (int i = 0; i < 4; ++i) b.push_back(uint8_t((uint32_t(v) >> (8 * i)) & 0xFF));
}
void put_u64(std::vector<uint8_t>& b, uint64_t v) {
    for (int i = 0; i < 8; ++i) b.push_back(uint8_t((v >> (8 * i)) & 0xFF));
}
void put_f32(std::vector<uint8_t>& b, float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    put_i32(b, int32_t(u));
}
void put_str(std::vector<uint8_t>& b, const char* s) {
    while (*s) b.push_back(uint8_t(*s++));
    b.push_back(0);
}
void put_attr(std::vector<uint8_t>& b, const char* name, const char* type, const std::vector<uint8_t>& v) {
    put_str(b, name);
    put_str(b, type);
    put_i32(b, int32_t(v.size()));
    b.insert(b.end(), v.begin(), v.end());
}

}  // namespace

extern "C" {

int nart_scene_load(const char* json_path, nart_scene** out) {
    if (!json_path || !out) return set_error(NART_E_INVALID, "null argument");
    nart_scene* sc = new (std::nothrow) nart_scene();
    if (!sc) return set_error(NART_E_OOM, "out of memory");
    std::memset(&sc->blob, 0, sizeof(sc->blob));
    int rc = load_scene(sc, json_path);
    if (rc != NART_OK) {
        delete sc;
        return rc;
    }
    *out = sc;
    return NART_OK;
}

const nart_scene_blob* nart_scene_blob_of(const nart_scene* scene) { return scene ? &scene->blob : nullptr; }

void nart_scene_free(nart_scene* scene) { delete scene; }

const char* nart_scene_last_error(void) { return g_error.c_str(); }

void nart_render_params_init(nart_render_params* p) {
    p->integrator = NART_INTEGRATOR_PATH;
    p->image_width = 0;
    p->image_height = 0;
    p->bucket_size = 0;
    p->spp = 0;
    p->bounces = 0;
    p->filter_width = -1.f;
    p->roughening_factor = -1.f;
}

// ParseRenderParamArguments (render.cpp:236-325)
int nart_parse_args(int argc, char** argv, nart_render_params* params) {
    for (int i = 3; i < argc; ++i) {
        std::string arg = argv[i];
        bool has_value = i + 1 < argc;  // reference reads argv[argc] here (Q29); we reject
        int iv = 0;
        float fv = 0.f;
        if (arg == "--imageWidth" || arg == "-w") {
            if (!has_value || !stoi_like(argv[++i], iv)) return set_error(NART_E_INVALID, "Invalid width");
            params->image_width = static_cast<uint32_t>(iv);
        } else if (arg == "--imageHeight" || arg == "-h") {
            if (!has_value || !stoi_like(argv[++i], iv)) return set_error(NART_E_INVALID, "Invalid height");
            params->image_height = static_cast<uint32_t>(iv);
        } else if (arg == "--bucketSize" || arg == "-b") {
            if (!has_value || !stoi_like(argv[++i], iv)) return set_error(NART_E_INVALID, "Invalid bucket size");
            params->bucket_size = static_cast<uint32_t>(iv);
        } else if (arg == "--spp" || arg == "-s") {
            if (!has_value || !stoi_like(argv[++i], iv)) return set_error(NART_E_INVALID, "Invalid spp");
            params->spp = static_cast<uint32_t>(iv);
        } else if (arg == "--bounces" || arg == "-o") {
            if (!has_value || !stoi_like(argv[++i], iv)) return set_error(NART_E_INVALID, "Invalid bounces");
            params->bounces = static_cast<uint32_t>(iv);
        } else if (arg == "--filterWidth" || arg == "-f") {
            if (!has_value || !stof_like(argv[++i], fv)) return set_error(NART_E_INVALID, "Invalid filter width");
            params->filter_width = fv;
        } else if (arg == "--rougheningFactor" || arg == "-r") {
            if (!has_value || !stof_like(argv[++i], fv)) return set_error(NART_E_INVALID, "Invalid roughening factor");
            params->roughening_factor = fv;  // CLI value is not clamped (Q29)
        } else {
            return set_error(NART_E_INVALID, "Invalid input: " + arg);
        }
    }
    return NART_OK;
}

// LoadSessions (render.cpp:327-414)
int nart_load_sessions(const char* json_path, const nart_render_params* cli, nart_render_params* out, int max) {
    std::string text;
    if (!read_file(json_path, text)) return set_error(NART_E_IO, "Error: Scene file could not be opened.");
    nartjson::Value json;
    try {
        json = nartjson::Parser(text).parse();
    } catch (std::exception& e) {
        return set_error(NART_E_INVALID, std::string("Error parsing scene: ") + e.what());
    }
    int n = 0;
    try {
        if (!json["renderSessions"].is_null()) {
            for (const nartjson::Value& elem : json["renderSessions"].arr) {
                nart_render_params p = *cli;
                if (!elem["integrator"].is_null() && p.integrator == NART_INTEGRATOR_PATH) {
                    std::string s = elem["integrator"].str();
                    if (s == "path") p.integrator = NART_INTEGRATOR_PATH;
                    if (s == "volume") p.integrator = NART_INTEGRATOR_VOLUME;
                }
                if (!elem["imageWidth"].is_null() && p.image_width == 0) p.image_width = elem["imageWidth"].num<uint32_t>();
                if (!elem["imageHeight"].is_null() && p.image_height == 0) p.image_height = elem["imageHeight"].num<uint32_t>();
                if (!elem["bucketSize"].is_null() && p.bucket_size == 0) p.bucket_size = elem["bucketSize"].num<uint32_t>();
                if (!elem["spp"].is_null() && p.spp == 0) p.spp = elem["spp"].num<uint32_t>();
                if (!elem["bounces"].is_null() && p.bounces == 0) p.bounces = elem["bounces"].num<uint32_t>();
                if (!elem["filterWidth"].is_null() && p.filter_width < 0.f) p.filter_width = elem["filterWidth"].num<float>();
                if (!elem["rougheningFactor"].is_null() && p.roughening_factor < 0.f)
                    p.roughening_factor = glm_min(glm_max(elem["rougheningFactor"].num<float>(), 0.f), 1.f);
                if (elem["imageWidth"].is_null() && p.image_width == 0) p.image_width = 64;
                if (elem["imageHeight"].is_null() && p.image_height == 0) p.image_height = 64;
                if (elem["bucketSize"].is_null() && p.bucket_size == 0) p.bucket_size = 16;
                if (elem["spp"].is_null() && p.spp == 0) p.spp = 1;
                if (elem["bounces"].is_null() && p.bounces == 0) p.bounces = 10;
                if (elem["filterWidth"].is_null() && p.filter_width < 0.f) p.filter_width = 1.f;
                if (elem["rougheningFactor"].is_null() && p.roughening_factor < 0.f) p.roughening_factor = 0.f;
                if (n < max) out[n] = p;
                ++n;
            }
        }
    } catch (std::exception& e) {
        return set_error(NART_E_INVALID, std::string("Error in renderSessions: ") + e.what());
    }
    return n;
}

// RenderSession ctor (render.cpp:14-21) and bucket counts (render.cpp:117-123)
void nart_session_geometry_of(const nart_render_params* p, nart_session_geometry* g) {
    g->filter_bounds = static_cast<uint32_t>(std::ceil(p->filter_width));
    g->tile_size = p->bucket_size + g->filter_bounds * 2;
    g->total_width = p->image_width + g->filter_bounds * 2;
    g->total_height = p->image_height + g->filter_bounds * 2;
    g->n_buckets_x = uint32_t(std::ceil(static_cast<float>(p->image_width) / static_cast<float>(p->bucket_size)));
    g->n_buckets_y = uint32_t(std::ceil(static_cast<float>(p->image_height) / static_cast<float>(p->bucket_size)));
}

// filterTable[i] = Gaussian(63, i)  (render.cpp:125-130; render.h:23-32)
void nart_filter_table(float table[64]) {
    const float pi = 3.14159265358979323846264338327950288f;
    for (int i = 0; i < 64; ++i) {
        float width = 63.f, x = static_cast<float>(i);
        if (x >= width) {
            table[i] = 0.f;
            continue;
        }
        float sigma = width / 3.f;
        table[i] = (1.f / std::sqrt(2.f * pi * sigma * sigma)) * std::exp(-(x * x) / (2.f * sigma * sigma));
    }
}

// Tile combine in bucket raster order (render.cpp:183-203)
void nart_combine_tiles(const nart_render_params* p, const nart_pixel* tiles, nart_pixel* image) {
    nart_session_geometry g;
    nart_session_geometry_of(p, &g);
    size_t npx = size_t(g.total_width) * g.total_height;
    std::memset(image, 0, npx * sizeof(nart_pixel));
    size_t tpx = size_t(g.tile_size) * g.tile_size;
    for (uint32_t j = 0; j < g.n_buckets_y; ++j)
        for (uint32_t i = 0; i < g.n_buckets_x; ++i) {
            const nart_pixel* v = tiles + (size_t(j) * g.n_buckets_x + i) * tpx;
            for (uint32_t y = 0; y < g.tile_size; ++y)
                for (uint32_t x = 0; x < g.tile_size; ++x) {
                    uint32_t pX = x + i * p->bucket_size, pY = y + j * p->bucket_size;
                    if (pX < p->image_width + g.filter_bounds && pY < p->image_height + g.filter_bounds) {
                        nart_pixel& d = image[size_t(pY) * g.total_width + pX];
                        const nart_pixel& s = v[size_t(y) * g.tile_size + x];
                        for (int c = 0; c < 4; ++c) d.contribution[c] += s.contribution[c];
                        d.filter_weight_sum += s.filter_weight_sum;
                    }
                }
        }
}

// Imath 3.1 imath_float_to_half (software path, round to nearest even)
uint16_t nart_float_to_half(float f) {
    uint32_t vi;
    std::memcpy(&vi, &f, 4);
    uint32_t ui = vi & ~0x80000000u;
    uint16_t ret = uint16_t((vi >> 16) & 0x8000u);
    if (ui >= 0x38800000u) {
        if (ui >= 0x7f800000u) {
            ret |= 0x7c00;
            if (ui == 0x7f800000u) return ret;
            uint32_t m = (ui & 0x7fffffu) >> 13;
            return uint16_t(ret | uint16_t(m) | uint16_t(m == 0));
        }
        if (ui > 0x477fefffu) return uint16_t(ret | 0x7c00);
        ui -= 0x38000000u;
        ui = ((ui + 0x00000fffu + ((ui >> 13) & 1u)) >> 13);
        return uint16_t(ret | uint16_t(ui));
    }
    if (ui < 0x33000001u) return ret;
    uint32_t e = ui >> 23;
    uint32_t shift = 0x7eu - e;
    uint32_t m = 0x800000u | (ui & 0x7fffffu);
    uint32_t r = m << (32 - shift);
    ret |= uint16_t(m >> shift);
    if (r > 0x80000000u || (r == 0x80000000u && (ret & 0x1u) != 0)) ++ret;
    return ret;
}

// Imath imath_half_to_float (exact)
float nart_half_to_float(uint16_t h) {
    uint32_t hexpmant = (uint32_t(h) << 17) >> 4;
    uint32_t v = (uint32_t(h) >> 15) << 31;
    if (hexpmant >= 0x00800000u) {
        v |= hexpmant;
        if (hexpmant >= 0x0f800000u) v |= 0x7f800000u;
        else v += 0x38000000u;
    } else if (hexpmant != 0) {
        uint32_t lc = 0;
        for (uint32_t x = hexpmant; !(x & 0x80000000u); x <<= 1) ++lc;
        lc -= 8;
        v |= 0x38800000u;
        v |= (hexpmant << lc);
        v -= (lc << 23);
    }
    float f;
    std::memcpy(&f, &v, 4);
    return f;
}

// WriteImageToEXR (render.cpp:208-234): RGBA half scanline file (channels A,B,G,R).
int nart_write_exr(const char* path, const nart_render_params* p, const nart_pixel* image, int compression) {
    nart_session_geometry g;
    nart_session_geometry_of(p, &g);
    const uint32_t W = p->image_width, H = p->image_height;
    if (W == 0 || H == 0) return set_error(NART_E_INVALID, "empty image");
    if (compression != 0 && compression != 3) return set_error(NART_E_INVALID, "compression must be 0 (none) or 3 (zip)");
    // result = contribution / filterWeightSum per channel (render.cpp:220-221)
    std::vector<uint16_t> px(size_t(W) * H * 4);
    for (uint32_t y = g.filter_bounds; y < H + g.filter_bounds; ++y)
        for (uint32_t x = g.filter_bounds; x < W + g.filter_bounds; ++x) {
            const nart_pixel& s = image[size_t(y) * g.total_width + x];
            uint16_t* d = &px[(size_t(y - g.filter_bounds) * W + (x - g.filter_bounds)) * 4];
            for (int c = 0; c < 4; ++c) d[c] = nart_float_to_half(s.contribution[c] / s.filter_weight_sum);
        }
    std::vector<uint8_t> f;
    put_i32(f, 20000630);
    put_i32(f, 2);
    std::vector<uint8_t> ch;
    const char* names[4] = {"A", "B", "G", "R"};
    for (const char* n : names) {
        put_str(ch, n);
        put_i32(ch, 1);  // HALF
        put_u8(ch, 0);
        put_u8(ch, 0);
        put_u8(ch, 0);
        put_u8(ch, 0);
        put_i32(ch, 1);
        put_i32(ch, 1);
    }
    put_u8(ch, 0);
    put_attr(f, "channels", "chlist", ch);
    put_attr(f, "compression", "compression", std::vector<uint8_t>{uint8_t(compression)});
    std::vector<uint8_t> box;
    put_i32(box, 0);
    put_i32(box, 0);
    put_i32(box, int32_t(W) - 1);
    put_i32(box, int32_t(H) - 1);
    put_attr(f, "dataWindow", "box2i", box);
    put_attr(f, "displayWindow", "box2i", box);
    put_attr(f, "lineOrder", "lineOrder", std::vector<uint8_t>{0});
    std::vector<uint8_t> one;
    put_f32(one, 1.f);
    put_attr(f, "pixelAspectRatio", "float", one);
    std::vector<uint8_t> v2;
    put_f32(v2, 0.f);
    put_f32(v2, 0.f);
    put_attr(f, "screenWindowCenter", "v2f", v2);
    put_attr(f, "screenWindowWidth", "float", one);
    put_u8(f, 0);
    const uint32_t lines_per_chunk = compression == 3 ? 16 : 1;
    const uint32_t nchunks = (H + lines_per_chunk - 1) / lines_per_chunk;
    size_t table_pos = f.size();
    for (uint32_t i = 0; i < nchunks; ++i) put_u64(f, 0);
    const int order[4] = {3, 2, 1, 0};  // A,B,G,R from r,g,b,a storage
    for (uint32_t cidx = 0; cidx < nchunks; ++cidx) {
        uint32_t y0 = cidx * lines_per_chunk, y1 = y0 + lines_per_chunk < H ? y0 + lines_per_chunk : H;
        std::vector<uint8_t> raw;
        for (uint32_t y = y0; y < y1; ++y)
            for (int c = 0; c < 4; ++c)
                for (uint32_t x = 0; x < W; ++x) {
                    uint16_t h = px[(size_t(y) * W + x) * 4 + order[c]];
                    raw.push_back(uint8_t(h & 0xFF));
                    raw.push_back(uint8_t(h >> 8));
                }
        std::vector<uint8_t> data = raw;
        if (compression == 3) {
            // OpenEXR ZIP: interleave even/odd bytes, delta predictor, zlib
            std::vector<uint8_t> t(raw.size());
            size_t half = (raw.size() + 1) / 2, a = 0, b = half;
            for (size_t i = 0; i < raw.size(); ++i) {
                if (i % 2 == 0) t[a++] = raw[i];
                else t[b++] = raw[i];
            }
            for (size_t i = t.size(); i-- > 1;) t[i] = uint8_t(int(t[i]) - int(t[i - 1]) + 128);
            uLongf clen = compressBound(t.size());
            std::vector<uint8_t> comp(clen);
            if (compress(comp.data(), &clen, t.data(), t.size()) != Z_OK) return set_error(NART_E_IO, "zlib error");
            comp.resize(clen);
            if (comp.size() < raw.size()) data.swap(comp);
        }
        uint64_t pos = f.size();
        for (int i = 0; i < 8; ++i) f[table_pos + 8 * cidx + i] = uint8_t((pos >> (8 * i)) & 0xFF);
        put_i32(f, int32_t(y0));
        put_i32(f, int32_t(data.size()));
        f.insert(f.end(), data.begin(), data.end());
    }
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return set_error(NART_E_IO, std::string("cannot open ") + path);
    size_t wr = std::fwrite(f.data(), 1, f.size(), fp);
    std::fclose(fp);
    return wr == f.size() ? NART_OK : set_error(NART_E_IO, "short write");
}

// RgbaInputFile-style reader: scanline files, NONE / RLE / ZIPS / ZIP / PIZ, HALF or FLOAT channels,
// R/G/B/A or Y (luminance -> gray).  Returns halves, row 0 = first scanline of the data window.
int nart_read_exr_rgba(const char* path, uint32_t* width, uint32_t* height, uint16_t** rgba) {
    std::string s;
    if (!read_file(path, s)) return set_error(NART_E_IO, std::string("cannot open texture ") + path);
    const uint8_t* b = reinterpret_cast<const uint8_t*>(s.data());
    size_t n = s.size(), p = 8;
    auto rd32 = [&](size_t at) -> uint32_t {
        return uint32_t(b[at]) | (uint32_t(b[at + 1]) << 8) | (uint32_t(b[at + 2]) << 16) | (uint32_t(b[at + 3]) << 24);
    };
    if (n < 8 || rd32(0) != 20000630u) return set_error(NART_E_INVALID, "not an EXR file");
    if (rd32(4) & 0x200u) return set_error(NART_E_UNSUPPORTED, "tiled EXR not supported");
    int compression = -1;
    int32_t dw[4] = {0, 0, -1, -1};
    struct Chan { std::string name; int type; };
    std::vector<Chan> chans;
    while (p < n && b[p] != 0) {
        std::string name(reinterpret_cast<const char*>(b + p));
        p += name.size() + 1;
        std::string type(reinterpret_cast<const char*>(b + p));
        p += type.size() + 1;
        uint32_t sz = rd32(p);
        p += 4;
        if (p + sz > n) return set_error(NART_E_INVALID, "truncated EXR header");
        if (name == "compression") compression = b[p];
        if (name == "dataWindow")
            for (int i = 0; i < 4; ++i) dw[i] = int32_t(rd32(p + 4 * i));
        if (name == "channels") {
            size_t q = p;
            while (q < p + sz && b[q] != 0) {
                std::string cn(reinterpret_cast<const char*>(b + q));
                q += cn.size() + 1;
                chans.push_back({cn, int(rd32(q))});
                q += 16;
            }
        }
        p += sz;
    }
    ++p;
    uint32_t W = uint32_t(dw[2] - dw[0] + 1), H = uint32_t(dw[3] - dw[1] + 1);
    if (dw[2] < dw[0] || dw[3] < dw[1]) return set_error(NART_E_INVALID, "bad dataWindow");
    uint32_t lpc;
    switch (compression) {
        case 0: case 1: case 2: lpc = 1; break;
        case 3: lpc = 16; break;
        case 4: lpc = 32; break;  // PIZ (exr_piz.cpp)
        default: return set_error(NART_E_UNSUPPORTED, std::string("EXR compression ") + std::to_string(compression) + " not supported (PXR24/B44/DWA)");
    }
    size_t bpp_line = 0;
    for (auto& c : chans) bpp_line += (c.type == 1 ? 2 : 4) * size_t(W);
    uint32_t nchunks = (H + lpc - 1) / lpc;
    std::vector<uint16_t> out(size_t(W) * H * 4, 0);
    uint16_t one_half = 0x3c00;
    for (size_t i = 0; i < size_t(W) * H; ++i) out[i * 4 + 3] = one_half;  // A = 1 when absent
    for (uint32_t ci = 0; ci < nchunks; ++ci) {
        uint64_t off = 0;
        for (int k = 0; k < 8; ++k) off |= uint64_t(b[p + 8 * ci + k]) << (8 * k);
        if (off + 8 > n) return set_error(NART_E_INVALID, "bad chunk offset");
        int32_t y = int32_t(rd32(off));
        uint32_t dsz = rd32(off + 4);
        if (off + 8 + dsz > n) return set_error(NART_E_INVALID, "truncated chunk");
        uint32_t lines = uint32_t(std::min<int64_t>(lpc, int64_t(dw[3]) - y + 1));
        size_t rawsz = bpp_line * lines;
        std::vector<uint8_t> raw(rawsz);
        const uint8_t* src = b + off + 8;
        if (dsz == rawsz) {
            std::memcpy(raw.data(), src, rawsz);
        } else if (compression == 4) {
            std::vector<int> types;
            for (auto& c : chans) types.push_back(c.type);
            if (!nart::piz_decode(src, dsz, types.data(), int(types.size()), W, lines, raw) || raw.size() != rawsz)
                return set_error(NART_E_INVALID, "PIZ chunk decode failed");
        } else if (compression == 1) {
            std::vector<uint8_t> t;
            size_t q = 0;
            while (q < dsz) {
                int8_t c = int8_t(src[q++]);
                if (c < 0) {
                    for (int k = 0; k < -c && q < dsz; ++k) t.push_back(src[q++]);
                } else if (q < dsz) {
                    for (int k = 0; k < c + 1; ++k) t.push_back(src[q]);
                    ++q;
                }
            }
            if (t.size() != rawsz) return set_error(NART_E_INVALID, "RLE size mismatch");
            for (size_t i = 1; i < t.size(); ++i) t[i] = uint8_t(int(t[i - 1]) + int(t[i]) - 128);
            size_t h2 = (rawsz + 1) / 2;
            for (size_t i = 0; i < rawsz; ++i) raw[i] = (i % 2 == 0) ? t[i / 2] : t[h2 + i / 2];
        } else {
            std::vector<uint8_t> t(rawsz);
            uLongf dl = rawsz;
            if (uncompress(t.data(), &dl, src, dsz) != Z_OK || dl != rawsz) return set_error(NART_E_INVALID, "zlib inflate failed");
            for (size_t i = 1; i < t.size(); ++i) t[i] = uint8_t(int(t[i - 1]) + int(t[i]) - 128);
            size_t h2 = (rawsz + 1) / 2;
            for (size_t i = 0; i < rawsz; ++i) raw[i] = (i % 2 == 0) ? t[i / 2] : t[h2 + i / 2];
        }
        size_t q = 0;
        for (uint32_t l = 0; l < lines; ++l) {
            uint32_t row = uint32_t(y - dw[1]) + l;
            for (auto& c : chans) {
                int slot = -1;
                bool lum = false;
                if (c.name == "R") slot = 0;
                else if (c.name == "G") slot = 1;
                else if (c.name == "B") slot = 2;
                else if (c.name == "A") slot = 3;
                else if (c.name == "Y") lum = true;
                for (uint32_t x = 0; x < W; ++x) {
                    uint16_t hv;
                    if (c.type == 1) {
                        hv = uint16_t(raw[q] | (raw[q + 1] << 8));
                        q += 2;
                    } else {
                        uint32_t u = uint32_t(raw[q]) | (uint32_t(raw[q + 1]) << 8) | (uint32_t(raw[q + 2]) << 16) | (uint32_t(raw[q + 3]) << 24);
                        q += 4;
                        float fv;
                        if (c.type == 2) std::memcpy(&fv, &u, 4);
                        else fv = float(u);
                        hv = nart_float_to_half(fv);
                    }
                    size_t o = (size_t(row) * W + x) * 4;
                    if (lum) { out[o] = out[o + 1] = out[o + 2] = hv; }
                    else if (slot >= 0) out[o + slot] = hv;
                }
            }
        }
    }
    uint16_t* mem = static_cast<uint16_t*>(std::malloc(out.size() * sizeof(uint16_t)));
    if (!mem) return set_error(NART_E_OOM, "out of memory");
    std::memcpy(mem, out.data(), out.size() * sizeof(uint16_t));
    *width = W;
    *height = H;
    *rgba = mem;
    return NART_OK;
}

void nart_free(void* p) { std::free(p); }

}  // extern "C"
