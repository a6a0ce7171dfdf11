/*
 * nart_scene.h — host-side scene ingestion and session configuration (C ABI).
 *
 * This is the host half of the drop-in for nart's tiled renderer.  It keeps the
 * reference's input surface (JSON scene, .geo meshes, EXR textures, CLI flags)
 * and hands the render path a flat, POD scene blob.
 *
 * Reference interfaces each entry point replaces (file:line in shanesimmsart/nart):
 *   nart_scene_load          <- Scene::Scene(std::string)            src/core/scene.cpp:3-26
 *                               (LoadCamera 782-875, LoadMeshes 644-780, LoadLights 877-932,
 *                                LoadMeshFromFile 77-343, Get{Rho_d,...,Normal} 345-642)
 *   nart_parse_args          <- ParseRenderParamArguments             src/core/render.cpp:236-325
 *   nart_load_sessions       <- LoadSessions                          src/core/render.cpp:327-414
 *   nart_write_exr           <- RenderSession::WriteImageToEXR        src/core/render.cpp:208-234
 *   nart_render_params       <- struct RenderParams                   include/nart/core/scene.h:25-36
 *   nart_pixel               <- struct Pixel                          include/nart/core/render.h:18-21
 *
 * Ownership: nart_scene_load allocates; nart_scene_free releases.  The blob returned by
 * nart_scene_blob_of points into the scene and stays valid until nart_scene_free.
 * Errors: functions return 0 on success, a negative NART_E_* code on failure, and
 * never abort the process (the reference aborts: scene.cpp:17-18, 371-373).
 */
#ifndef NART_SCENE_H
#define NART_SCENE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NART_OK 0
#define NART_E_INVALID (-1)
#define NART_E_IO (-2)
#define NART_E_HIP (-3)
#define NART_E_OOM (-4)
#define NART_E_RCCL (-5)
#define NART_E_UNSUPPORTED (-6)

/* IntegratorFlag (scene.h:23) */
#define NART_INTEGRATOR_PATH 0
#define NART_INTEGRATOR_VOLUME 1

/* RenderParams (scene.h:25-36); 0 / negative = "not set" sentinels as in the reference. */
typedef struct nart_render_params {
    int32_t integrator;
    uint32_t image_width;
    uint32_t image_height;
    uint32_t bucket_size;
    uint32_t spp;
    uint32_t bounces;
    float filter_width;
    float roughening_factor;
} nart_render_params;

/* Pixel (render.h:18-21): float4 contribution + filter weight sum, 20 B AoS. */
typedef struct nart_pixel {
    float contribution[4];
    float filter_weight_sum;
} nart_pixel;

/* Triangle (geometry.h:53-65): 96 B, world space, exactly as the reference stores it. */
typedef struct nart_triangle {
    float v0[3], v1[3], v2[3];
    float n0[3], n1[3], n2[3];
    float uv0[2], uv1[2], uv2[2];
} nart_triangle;

/* Pattern (pattern.h:5-18) */
#define NART_PTN_CONSTANT 0
#define NART_PTN_TEXTURE 1
typedef struct nart_pattern {
    int32_t type;         /* NART_PTN_* */
    float value[3];       /* constant value (after the reference's clamps / squaring) */
    int32_t texture;      /* texture index for NART_PTN_TEXTURE */
    int32_t is_roughness; /* TexturePattern isRoughness: squares each channel */
} nart_pattern;

/* Material types (src/materials/<type>material.cpp) */
#define NART_MAT_LAMBERT 0  /* DiffuseMaterial */
#define NART_MAT_SPECULAR 1 /* SpecularMaterial */
#define NART_MAT_GLASS 2    /* GlassMaterial */
#define NART_MAT_GLOSSY 3   /* GlossyDielectricMaterial */
#define NART_MAT_PLASTIC 4  /* PlasticMaterial */
typedef struct nart_material {
    int32_t type;
    int32_t has_normal; /* normal pattern present (ignored by glass: glassmaterial.cpp:3-9) */
    nart_pattern rho_d, rho_s, tau, eta, alpha, normal;
} nart_material;

/* Mesh (TriMesh, geometry.h:68-91): triangles [first_tri, first_tri+num_tris) */
typedef struct nart_mesh {
    uint32_t first_tri;
    uint32_t num_tris;
    uint32_t material;
    uint32_t priority; /* uint8 in the reference */
} nart_mesh;

/* Lights (src/lights/<type>light.cpp).  m is glm::mat4 storage: m[col*4+row]. */
#define NART_LIGHT_DISK 0
#define NART_LIGHT_RING 1
#define NART_LIGHT_ENVIRONMENT 2
typedef struct nart_light {
    int32_t type;
    float radius;
    float inner_radius;
    float intensity;
    nart_pattern Le;
    float m[16];
} nart_light;

/* Half-float RGBA texture, row 0 = top (Imf::Array2D<Imf::Rgba> layout). */
typedef struct nart_texture {
    uint32_t width;
    uint32_t height;
    const uint16_t* rgba; /* width*height*4 halves */
} nart_texture;

/* Camera medium (media.h / scene.cpp:801-871), C5 only. */
typedef struct nart_medium {
    int32_t present;
    float bounds_min[3], bounds_max[3];
    float sigma_a, sigma_s;
    float Le[3];
    uint32_t res[3];
    const float* density; /* res[0]*res[1]*res[2], x fastest */
} nart_medium;

/* Pinhole camera (pinholecamera.cpp:3-40).  m is glm::mat4 storage. */
typedef struct nart_camera {
    float fov;
    float m[16];
} nart_camera;

/* Flat POD view of a loaded scene. */
typedef struct nart_scene_blob {
    uint32_t num_triangles;
    uint32_t num_meshes;
    uint32_t num_materials;
    uint32_t num_lights;
    uint32_t num_textures;
    uint32_t reserved;
    const nart_triangle* triangles;
    const nart_mesh* meshes;
    const nart_material* materials;
    const nart_light* lights;
    const nart_texture* textures;
    nart_camera camera;
    nart_medium medium;
} nart_scene_blob;

typedef struct nart_scene nart_scene;

int nart_scene_load(const char* json_path, nart_scene** out);
const nart_scene_blob* nart_scene_blob_of(const nart_scene* scene);
void nart_scene_free(nart_scene* scene);
const char* nart_scene_last_error(void);

/* CLI: argv[0] program, argv[1] scene, argv[2] output, flags from argv[3] (render.cpp:236). */
void nart_render_params_init(nart_render_params* p); /* sentinels of scene.h:27-35 */
int nart_parse_args(int argc, char** argv, nart_render_params* params);

/* Resolve renderSessions[] against CLI params (render.cpp:327-414).  Writes up to max
   sessions into out and returns the number of sessions found (may exceed max). */
int nart_load_sessions(const char* json_path, const nart_render_params* cli,
                       nart_render_params* out, int max);

/* Derived session geometry (RenderSession ctor, render.cpp:14-21). */
typedef struct nart_session_geometry {
    uint32_t filter_bounds;
    uint32_t tile_size;
    uint32_t total_width;
    uint32_t total_height;
    uint32_t n_buckets_x;
    uint32_t n_buckets_y;
} nart_session_geometry;
void nart_session_geometry_of(const nart_render_params* p, nart_session_geometry* g);

/* Gaussian filter table (render.cpp:125-130, render.h:23-32). */
void nart_filter_table(float table[64]);

/* Combine per-bucket tiles into the totalW x totalH image in bucket raster order
   (render.cpp:183-203).  tiles: n_buckets * tile_size^2 Pixels indexed by bucket id. */
void nart_combine_tiles(const nart_render_params* p, const nart_pixel* tiles, nart_pixel* image);

/* WriteImageToEXR (render.cpp:208-234): crop, divide by weight sum, float->half (Imath RNE),
   RGBA scanline EXR.  compression: 0 = none, 3 = ZIP (the reference's default). */
int nart_write_exr(const char* path, const nart_render_params* p, const nart_pixel* image,
                   int compression);

/* Imath float->half (half.h imath_float_to_half, round-to-nearest-even). */
uint16_t nart_float_to_half(float f);
float nart_half_to_float(uint16_t h);

/* Read an RGBA EXR (NONE/RLE/ZIPS/ZIP/PIZ) as Imf::RgbaInputFile would, into halves. */
int nart_read_exr_rgba(const char* path, uint32_t* width, uint32_t* height, uint16_t** rgba);
void nart_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
