// Device-resident scene layout for the nart render path.  Built once per context by the
// host (api.cpp) from the nart_scene_blob; every derived constant that the reference
// recomputes per call (light frames, triangle normals) is precomputed on the host with the
// identical float operations, so the device reads bit-identical values.
//
// HBM layout (all arrays 16-B aligned, read-only during a render):
//   nodes     : BVH2, 64 B per node (two child AABBs + two child codes), depth-first order
//   tri_isect : 64 B per triangle in BVH leaf order: {n.xyz, dot(v0,n)}, {v0.xyz, v1.x},
//               {v1.yz, v2.xy}, {v2.z, global index, -, -}
//   tris      : the reference's 96-B Triangle records in scene order (winner attributes)
//   tri_mesh  : mesh id per triangle (scene order)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/nart_scene.h"

namespace nd {

// Child code: >= 0 inner node index; < 0 leaf = ~(first << 5 | (count - 1)).
struct BVHNode {
    float lo0[3], hi0[3];
    float lo1[3], hi1[3];
    int32_t child[2];
    int32_t pad[2];
};
static_assert(sizeof(BVHNode) == 64, "BVHNode must be 64 B");

#define NART_LEAF_MAX 32
#define NART_STACK_DEPTH 20

struct DPattern {
    int32_t type;  // NART_PTN_*
    int32_t tex;
    int32_t rough;
    float v[3];
};

struct DMaterial {
    int32_t type;  // NART_MAT_*
    int32_t has_normal;
    DPattern rho_d, rho_s, tau, eta, alpha, normal;
};

// Light with the per-call constants of disklight.cpp / ringlight.cpp precomputed.
struct DLight {
    int32_t type;  // NART_LIGHT_*
    float radius, inner, intensity;
    DPattern Le;
    float m[16];         // LightToWorld (glm storage)
    float center[3];     // vec3(vec4(0,0,0,1) * M)
    float n[3];          // vec3(vec4(0,0,-1,0) * M)
    float D;             // dot(center, n)
    float axu[4];        // vec4(1,0,0,0) * M
    float axv[4];        // vec4(0,1,0,0) * M
    float pdf_area;      // 1/(pi r r) (disk) or 1/(pi (1 - ri^2/r^2) r r) (ring)
    float r2, ri2;       // radius^2, innerRadius^2
    float inner_ratio;   // innerRadius / radius
    int32_t env;         // index into env distribution table, -1 if none
};

struct DTexture {
    uint32_t w, h;
    uint64_t offset;  // into tex_pool (halves, RGBA)
};

// Piecewise2DDistribution (texturepattern.cpp:3-109) for a texture-lit environment light.
struct DEnvDist {
    uint32_t w, h;
    float invW, invH;
    const float *mpdf, *cpdf, *mcdf, *ccdf;
    // guide tables of the two CDF searches (build_env; null: full searches): cell c of K (values
    // in [c/K, (c+1)/K)) holds a | b << 16, the range of BinarySearch's upper bound, relative to
    // the search start -- mguide[K] for the marginal, cguide[row * K + c] for the conditionals
    const uint32_t *mguide, *cguide;
};
#define NART_ENV_GUIDE_K 64u

struct DMesh {
    uint32_t material;
    uint32_t priority;
};

// Camera medium (media.h:98-120).  maj[] mirrors the reference's Medium layout after
// MajorantGrid::majorants[1]: {majorant * sigma_maj, sigma_maj, boundsMin, boundsMax}, because
// RayMajorantIterator::Next indexes past the 1-entry majorant array (media.cpp:241, 250-251).
struct DMedium {
    int32_t present;
    uint32_t rx, ry, rz;  // uint8_t resolutions of DensityGrid (truncated as in scene.cpp:866)
    float bmin[3], bmax[3];
    float sigma_a, sigma_s;
    float Le[3];
    float maj[8];
    const float* density;
    // exact strength reductions (host-checked, build_medium): x / d == x * (1/d) bit for bit when d
    // is a power of two whose reciprocal is a normal float (both are the correctly rounded x * 2^-k)
    float inv_bs[3];       // 1 / (bmax - bmin) per axis, valid where bit i of bs_pow2 is set
    uint32_t bs_pow2;
    float inv_maj[8];      // 1 / maj[j], valid where bit j of maj_pow2 is set
    uint32_t maj_pow2;
    // 2x2x2 grids: the 8 densities in the kernel arguments (DensityGrid::LookUp then always reads
    // corners 0/1 of each axis: no memory access, same arithmetic)
    uint32_t grid2;
    float dens8[8];
};

// Reference octree (bvh.cpp:115-250), kept beside the device BVH so that the render path can
// reproduce Octree::Intersect's reachability exactly (path.h, oc_resolve).  Node indices are
// the reference's creation order; bmin/bmax are the BoundingVolume extents (axis dot products,
// bvh.cpp:81-113, extended bottom-up as bvh.cpp:235-250).
struct OcNode {
    float bmin[3], bmax[3];
    int32_t parent;        // -1 at the root
    uint32_t chunk_first;  // leaves: first (tri_first, tri_count) pair in oc_chunks
    uint32_t chunk_count;  // leaves: chunks in InsertChunk order; 0 for inner nodes
    int32_t children[8];   // -1 where absent
    int32_t is_leaf;
};
static_assert(sizeof(OcNode) == 72, "OcNode must be 72 B");

// Scene tables are read-only while a render kernel runs.  cst(p) returns p through the constant
// address space, so that a read at a wave-uniform index becomes a scalar load (a read at a per-lane
// index stays a vector load).
template <typename T>
__host__ __device__ inline const T* cst(const T* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef const __attribute__((address_space(4))) T cT;
    return (const T*)(const cT*)(uintptr_t)p;
#else
    return p;
#endif
}

struct DScene {
    const BVHNode* nodes;
    const float4* tri_isect;
    // tri_isect's vertices pre-permuted per ray major axis (Triangle::Intersect's
    // (kx, ky, kz) = (m+1, m+2, m) mod 3, geometry.cpp:48-56): [major][leaf-order tri] 64 B =
    // {v0p.xyz, v1p.x}, {v1p.yz, v2p.xy}, {v2p.z, global index, info, grazing threshold},
    // {n, dot(v0, n)} (tri_isect words 0-3)
    const float4* tri_perm;
    const nart_triangle* tris;
    const uint32_t* tri_mesh;
    const DMesh* meshes;
    const DMaterial* mats;
    // [mesh] bxdf_eta of the one-lobe BSDF a hit on the mesh creates when the material's patterns
    // are constant: 0 (Lambert) or the material's eta (kernels.h IList COMPACT)
    const float* mesh_eta;
    const DLight* lights;
    const DTexture* texs;
    const uint16_t* tex_pool;
    const DEnvDist* envs;
    uint32_t num_lights;
    uint32_t num_tris;
    uint32_t num_leaf_tris;  // test records in leaf order (tri_isect, one tri_perm block)
    int32_t root;            // root code (inner node index or leaf code)
    int32_t geometry_visible;// 0 when the reference octree's root is a leaf (bvh.cpp:131, Q14)
    float cam_m[16];
    float cam_tan;           // tan(radians(fov)) (host libm, as the reference)
    DMedium medium;
    // reference octree + replay heap pool (oc_resolve in path.h)
    const OcNode* oc_nodes;
    const uint32_t* oc_chunks;  // (tri_first, tri_count) into oc_tris
    const uint32_t* oc_tris;    // global triangle ids, chunk insertion order
    const int32_t* tri_leaf;    // leaf node of each triangle, -1 if unreachable
    uint32_t* oc_lock;          // [oc_pool] replay heap ownership (a wave's 64 heaps per entry)
    unsigned long long* oc_heap;// [oc_pool][64][oc_cap] (key bits | node << 32)
    int32_t oc_root;
    uint32_t oc_cap, oc_pool;
    int32_t oc_exact;           // 0 disables the emulation (A/B only; not reference behaviour), 2 replays every query
    float oc_scale;             // max |coordinate| of the scene and camera (margins)
};

}  // namespace nd
