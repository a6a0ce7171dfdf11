/*
 * nart_oracle.c — TEST INFRASTRUCTURE ONLY (see nart_oracle.h).  PARITY UNPINNED.
 *
 * Plain-C restatement of shanesimmsart/nart's render path, following the reference sources
 * operation by operation (file:line cited per function, paths relative to the reference root).
 * GLM 0.9.9.8 scalar semantics are spelled out in the helpers below; every float expression
 * keeps the reference's association order and is compiled with -ffp-contract=off.
 * Transcendentals are glibc's (glm::sin -> sinf, glm::cos -> cosf, ...), exactly as the
 * reference links them on Linux.
 */
#define _GNU_SOURCE
#include "nart_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- GLM-equivalent math */
typedef struct { float x, y; } v2;
typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;

#define INF_F (__builtin_inff())
/* glm::pi<float>() etc.: genType(<double literal>) */
static const float PI_F = (float)3.14159265358979323846264338327950288;
static const float TWO_PI_F = (float)6.28318530717958647692528676655900576;
static const float ONE_OVER_PI_F = (float)0.318309886183790671537767526745028724;
static const float ONE_OVER_TWO_PI_F = (float)0.159154943091895335768883763372514362;
static const float EPS_F = FLT_EPSILON; /* glm::epsilon<float>() */

static inline v2 V2(float x, float y) { v2 r = {x, y}; return r; }
static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v4 V4(float x, float y, float z, float w) { v4 r = {x, y, z, w}; return r; }
static inline v3 add3(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub3(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul3(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls3(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 divs3(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 div3(v3 a, v3 b) { return V3(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline v3 neg3(v3 a) { return V3(-a.x, -a.y, -a.z); }
/* compute_dot<vec3>: tmp = a*b; tmp.x + tmp.y + tmp.z */
static inline float dot3(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
/* compute_dot<vec4>: (tmp.x + tmp.y) + (tmp.z + tmp.w) */
static inline float dot4(v4 a, v4 b) { return (a.x * b.x + a.y * b.y) + (a.z * b.z + a.w * b.w); }
static inline v3 cross3(v3 x, v3 y) {
    return V3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
/* normalize(v) = v * inversesqrt(dot(v,v)), inversesqrt(x) = 1 / sqrt(x) */
static inline v3 normalize3(v3 v) { float s = 1.f / sqrtf(dot3(v, v)); return muls3(v, s); }
static inline v4 normalize4(v4 v) {
    float s = 1.f / sqrtf(dot4(v, v));
    return V4(v.x * s, v.y * s, v.z * s, v.w * s);
}
/* glm::min / max / abs for floats (func_common.inl) */
static inline float gmin(float a, float b) { return (b < a) ? b : a; }
static inline float gmax(float a, float b) { return (a < b) ? b : a; }
static inline float gabs(float x) { return x >= 0.f ? x : -x; }
static inline float gfract(float x) { return x - floorf(x); }
static inline float gmod(float a, float b) { return a - b * floorf(a / b); }
static inline float gmix(float x, float y, float a) { return x * (1.f - a) + y * a; }
static inline v3 vmin3(v3 a, v3 b) { return V3(gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z)); }
static inline v3 vmax3(v3 a, v3 b) { return V3(gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z)); }
static inline float v3get(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
/* row vector * mat4: result[i] = m[i][0]*v0 + m[i][1]*v1 + m[i][2]*v2 + m[i][3]*v3 */
static inline v4 vec_mul_mat(v4 v, const float* m) {
    float r[4];
    for (int i = 0; i < 4; ++i)
        r[i] = ((m[i * 4 + 0] * v.x + m[i * 4 + 1] * v.y) + m[i * 4 + 2] * v.z) + m[i * 4 + 3] * v.w;
    return V4(r[0], r[1], r[2], r[3]);
}
static inline v3 xyz(v4 v) { return V3(v.x, v.y, v.z); }
/* static_cast<uint32_t>(float) as clang emits it on x86-64 (cvttss2si to 64 bit, low half). */
static inline uint32_t f2u32(float f) {
    if (!(f > -9.2233715e18f && f < 9.2233715e18f)) return 0u;
    return (uint32_t)(int64_t)f;
}
static inline uint8_t f2u8(float f) { return (uint8_t)f2u32(f); }

/* ---------------------------------------------------------------- RNG (rng.h:8-59) */
typedef struct { uint32_t y; } rng_t;
static inline void rng_seed(rng_t* r, uint32_t s) { r->y = s + 2463534242u; }
static inline float rng_float(rng_t* r) {
    r->y ^= (r->y << 13);
    r->y ^= (r->y >> 17);
    r->y ^= (r->y << 5);
    float f = (float)(uint32_t)(r->y * 0x9E3779BBu) * 2.3283064365386963e-10f;
    return gmin(1.f - EPS_F, f);
}
static inline uint32_t rng_int(rng_t* r, uint32_t max) {
    r->y ^= (r->y << 13);
    r->y ^= (r->y >> 17);
    r->y ^= (r->y << 5);
    return (uint32_t)(((uint64_t)(uint32_t)(r->y * 0x9E3779B9u) * ((uint64_t)max + 1)) >> 32);
}

/* ---------------------------------------------------------------- sampling.cpp */
static v2 uniform_sample_disk(v2 s) { /* sampling.cpp:5-16 */
    float r = sqrtf(s.x);
    float theta = s.y * TWO_PI_F;
    float c = cosf(theta), sn = sinf(theta);
    return V2(r * c, r * sn);
}
static v2 uniform_sample_ring(v2 s, float* pdf, float inner) { /* sampling.cpp:18-31 */
    float r = sqrtf(gmix(inner, 1.f, s.x));
    float theta = s.y * TWO_PI_F;
    float c = cosf(theta), sn = sinf(theta);
    *pdf = 1.f / (PI_F * (1.f - inner));
    return V2(r * c, r * sn);
}
static v3 cosine_sample_hemisphere(v2 s, float* pdf) { /* sampling.cpp:47-58 */
    v2 d = uniform_sample_disk(s);
    float z = sqrtf(1.f - (d.x * d.x + d.y * d.y));
    *pdf = z * ONE_OVER_PI_F;
    return V3(d.x, d.y, z);
}
static float stratified_1d(rng_t* rng, uint32_t n, uint32_t ns) { /* sampling.cpp:64-67 */
    float inv = 1.f / (float)ns;
    return ((float)n + rng_float(rng)) * inv;
}
/* LatinSquare (sampling.cpp:72-86); vec2(a(), b()) evaluated left to right (Clang, Q2). */
static void latin_square(rng_t* rng, uint32_t n, v2* s) {
    for (uint32_t i = 0; i < n; ++i) {
        float a = stratified_1d(rng, i, n);
        float b = stratified_1d(rng, i, n);
        s[i] = V2(a, b);
    }
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t c = rng_int(rng, n - 1 - i);
        float t = s[i].x; s[i].x = s[c].x; s[c].x = t;
        c = rng_int(rng, n - 1 - i);
        t = s[i].y; s[i].y = s[c].y; s[c].y = t;
    }
}

/* ---------------------------------------------------------------- geometry.cpp */
typedef struct {
    v3 o, d;
    uint8_t major;
    float Sx, Sy, Sz;
} ray_t;
static ray_t make_ray(v3 o, v3 d) { /* geometry.cpp:3-15 */
    ray_t r;
    r.o = o;
    r.d = d;
    v3 a = V3(gabs(d.x), gabs(d.y), gabs(d.z));
    r.major = (a.x > a.y) ? ((a.x > a.z) ? 0 : 2) : ((a.y > a.z) ? 1 : 2);
    r.Sz = 1.f / v3get(d, r.major);
    uint8_t m0 = (uint8_t)(r.major + 1);
    if (m0 == 3) m0 = 0;
    uint8_t m1 = (uint8_t)(r.major + 2);
    if (m1 >= 3) m1 -= 3;
    r.Sx = -v3get(d, m0) * r.Sz;
    r.Sy = -v3get(d, m1) * r.Sz;
    return r;
}

typedef struct { /* Intersection (geometry.h:29-51) */
    int32_t mat;
    float u, v;
    v3 p, gn, sn, dpds, dpdt;
    v2 st;
    float tMin, tMax;
    uint32_t meshID;
    uint32_t priority;
} isect_t;
static inline void isect_init(isect_t* i) {
    memset(i, 0, sizeof(*i));
    i->mat = -1;
    i->tMin = 0.f;
    i->tMax = INF_F;
    i->meshID = 0xFFFFFFFFu;
    i->priority = 0;
}
static inline v3 tv(const float* a) { return V3(a[0], a[1], a[2]); }

static int triangle_intersect(const nart_triangle* T, const ray_t* ray, isect_t* is) { /* geometry.cpp:32-115 */
    v3 v0 = tv(T->v0), v1 = tv(T->v1), v2_ = tv(T->v2);
    v3 n = cross3(sub3(v1, v0), sub3(v2_, v0));
    float t = (dot3(v0, n) - dot3(ray->o, n)) / dot3(ray->d, n);
    if (t <= is->tMin || t >= is->tMax) return 0;
    v3 p0 = sub3(v0, ray->o), p1 = sub3(v1, ray->o), p2 = sub3(v2_, ray->o);
    uint8_t M = ray->major;
    uint8_t m0 = (uint8_t)(M + 1);
    if (m0 == 3) m0 = 0;
    uint8_t m1 = (uint8_t)(M + 2);
    if (m1 >= 3) m1 -= 3;
    p0 = V3(v3get(p0, m0), v3get(p0, m1), v3get(p0, M));
    p1 = V3(v3get(p1, m0), v3get(p1, m1), v3get(p1, M));
    p2 = V3(v3get(p2, m0), v3get(p2, m1), v3get(p2, M));
    p0.x += p0.z * ray->Sx;
    p0.y += p0.z * ray->Sy;
    p1.x += p1.z * ray->Sx;
    p1.y += p1.z * ray->Sy;
    p2.x += p2.z * ray->Sx;
    p2.y += p2.z * ray->Sy;
    float e0 = (p1.x * p2.y) - (p1.y * p2.x);
    float e1 = (p2.x * p0.y) - (p2.y * p0.x);
    float e2 = (p0.x * p1.y) - (p0.y * p1.x);
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return 0;
    if (gabs(e0) + gabs(e1) + gabs(e2) == 0.f) return 0;
    float invDet = 1.f / (e0 + e1 + e2);
    v3 p = muls3(add3(add3(muls3(v0, e0), muls3(v1, e1)), muls3(v2_, e2)), invDet);
    float u = e0 * invDet;
    float v = e1 * invDet;
    n = normalize3(n);
    is->tMax = t;
    is->u = u;
    is->v = v;
    is->gn = n;
    float w = 1 - is->u - is->v;
    is->sn = add3(add3(muls3(tv(T->n0), is->u), muls3(tv(T->n1), is->v)), muls3(tv(T->n2), w));
    is->p = p;
    is->st = V2((T->uv0[0] * is->u + T->uv1[0] * is->v) + T->uv2[0] * w,
                (T->uv0[1] * is->u + T->uv1[1] * is->v) + T->uv2[1] * w);
    float UVDet = ((T->uv0[0] - T->uv2[0]) * (T->uv1[1] - T->uv2[1])) - ((T->uv0[1] - T->uv2[1]) * (T->uv1[0] - T->uv2[0]));
    float invUVDet = 1.f / UVDet;
    is->dpds = muls3(add3(muls3(sub3(v0, v2_), T->uv1[1] - T->uv2[1]), muls3(sub3(v1, v2_), T->uv2[1] - T->uv0[1])), invUVDet);
    is->dpdt = muls3(add3(muls3(sub3(v0, v2_), T->uv2[0] - T->uv1[0]), muls3(sub3(v1, v2_), T->uv0[0] - T->uv2[0])), invUVDet);
    return 1;
}

/* ---------------------------------------------------------------- BVH (bvh.cpp) */
typedef struct { float bmin[3], bmax[3]; } bv_t;
static void bv_init(bv_t* b) {
    for (int i = 0; i < 3; ++i) { b->bmin[i] = INF_F; b->bmax[i] = -INF_F; }
}
static void bv_extend(bv_t* b, const bv_t* o) { /* bvh.cpp:16-21 */
    for (int i = 0; i < 3; ++i) {
        b->bmin[i] = gmin(b->bmin[i], o->bmin[i]);
        b->bmax[i] = gmax(b->bmax[i], o->bmax[i]);
    }
}
static const v3 AXIS[3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
static int bv_intersect(const bv_t* b, const ray_t* ray, float* tEntry) { /* bvh.cpp:23-60 */
    float tMin = -INF_F, tMax = INF_F;
    for (int i = 0; i < 3; ++i) {
        float slabMin = (b->bmin[i] - dot3(ray->o, AXIS[i])) / dot3(ray->d, AXIS[i]);
        float slabMax = (b->bmax[i] - dot3(ray->o, AXIS[i])) / dot3(ray->d, AXIS[i]);
        if (slabMin > slabMax) { float t = slabMin; slabMin = slabMax; slabMax = t; }
        if (slabMin > tMax || tMin > slabMax) return 0;
        tMin = gmax(tMin, slabMin);
        tMax = gmin(tMax, slabMax);
    }
    *tEntry = tMin;
    return 1;
}

typedef struct {
    uint32_t* tris; /* global triangle indices, insertion order */
    uint32_t n, cap;
    v3 bboxMin, bboxMax;
    bv_t bv;
} chunk_t;

typedef struct {
    int32_t children[8];
    int32_t* chunks; /* chunk ids */
    uint32_t nchunks, cap;
    int isLeaf;
    v3 nodeMin, nodeMax;
    bv_t bv;
} onode_t;

struct oracle_scene {
    const nart_scene_blob* blob;
    uint32_t* tri_mesh;  /* mesh of each triangle */
    chunk_t* chunks;
    uint32_t nchunks_total; /* numChunks + 1 slots */
    onode_t* nodes;
    uint32_t nnodes, capnodes;
    int root;
    uint32_t grid_res[3];
    float* tex_f; /* textures converted to float rgb (row-major, 3 floats) */
    size_t* tex_off;
    /* environment distributions per light (Piecewise2DDistribution) */
    struct pw2d { int present; uint32_t w, h; float invW, invH; float *mpdf, *cpdf, *mcdf, *ccdf; } * env;
    uint32_t nenv; /* entries of env: oracle_destroy must not read the caller's blob, which may be gone */
    /* camera medium (media.h:98-120): the majorant table is laid out as the reference's Medium
       members after MajorantGrid::majorants[1] -- {majorant * sigma_maj, sigma_maj, boundsMin,
       boundsMax} -- because RayMajorantIterator::Next can index past the 1-entry array. */
    int has_medium;
    float maj[8];
};

static int new_node(oracle_scene* s, v3 mn, v3 mx) {
    if (s->nnodes == s->capnodes) {
        s->capnodes = s->capnodes ? s->capnodes * 2 : 64;
        s->nodes = (onode_t*)realloc(s->nodes, s->capnodes * sizeof(onode_t));
    }
    onode_t* n = &s->nodes[s->nnodes];
    memset(n, 0, sizeof(*n));
    for (int i = 0; i < 8; ++i) n->children[i] = -1;
    n->isLeaf = 1;
    n->nodeMin = mn;
    n->nodeMax = mx;
    bv_init(&n->bv);
    return (int)s->nnodes++;
}
static void node_push_chunk(onode_t* n, int32_t c) {
    if (n->nchunks == n->cap) {
        n->cap = n->cap ? n->cap * 2 : 4;
        n->chunks = (int32_t*)realloc(n->chunks, n->cap * sizeof(int32_t));
    }
    n->chunks[n->nchunks++] = c;
}
/* OctreeNode::InsertChunk (bvh.cpp:178-233), including the post-increment depth quirk. */
static void insert_chunk(oracle_scene* s, int node, int32_t chunk, uint8_t depth) {
    onode_t* n = &s->nodes[node];
    if (n->isLeaf) {
        if (n->nchunks == 0 || depth >= 5) {
            node_push_chunk(n, chunk);
        } else {
            n->isLeaf = 0;
            for (uint32_t i = 0; i < s->nodes[node].nchunks; ++i) {
                int32_t back = s->nodes[node].chunks[s->nodes[node].nchunks - 1];
                insert_chunk(s, node, back, depth++);
                s->nodes[node].nchunks--; /* pop_back */
            }
            insert_chunk(s, node, chunk, depth++);
        }
    } else {
        const chunk_t* c = &s->chunks[chunk];
        uint8_t idx = 0;
        v3 cc = add3(c->bboxMin, muls3(sub3(c->bboxMax, c->bboxMin), 0.5f));
        v3 nc = add3(n->nodeMin, muls3(sub3(n->nodeMax, n->nodeMin), 0.5f));
        if (cc.x > nc.x) idx |= 1;
        if (cc.y > nc.y) idx |= 2;
        if (cc.z > nc.z) idx |= 4;
        if (n->children[idx] < 0) {
            v3 size = muls3(sub3(n->nodeMax, n->nodeMin), 0.5f);
            v3 cmin = nc, cmax = nc;
            if (idx & 1) cmax.x += size.x; else cmin.x -= size.x;
            if (idx & 2) cmax.y += size.y; else cmin.y -= size.y;
            if (idx & 4) cmax.z += size.z; else cmin.z -= size.z;
            int child = new_node(s, cmin, cmax);
            s->nodes[node].children[idx] = child;
        }
        insert_chunk(s, s->nodes[node].children[idx], chunk, depth++);
    }
}
static void build_bvs(oracle_scene* s, int node) { /* bvh.cpp:235-250 */
    onode_t* n = &s->nodes[node];
    if (n->isLeaf) {
        for (uint32_t i = 0; i < n->nchunks; ++i) bv_extend(&n->bv, &s->chunks[n->chunks[i]].bv);
    } else {
        for (int c = 0; c < 8; ++c) {
            int ch = s->nodes[node].children[c];
            if (ch >= 0) {
                build_bvs(s, ch);
                bv_extend(&s->nodes[node].bv, &s->nodes[ch].bv);
            }
        }
    }
}
static void chunk_push(chunk_t* c, uint32_t t) {
    if (c->n == c->cap) {
        c->cap = c->cap ? c->cap * 2 : 8;
        c->tris = (uint32_t*)realloc(c->tris, c->cap * sizeof(uint32_t));
    }
    c->tris[c->n++] = t;
}
static void chunk_bounds(oracle_scene* s, chunk_t* c) { /* bvh.cpp:81-113 */
    c->bboxMin = V3(INF_F, INF_F, INF_F);
    c->bboxMax = V3(-INF_F, -INF_F, -INF_F);
    bv_init(&c->bv);
    for (uint32_t k = 0; k < c->n; ++k) {
        const nart_triangle* T = &s->blob->triangles[c->tris[k]];
        v3 vs[3] = {tv(T->v0), tv(T->v1), tv(T->v2)};
        for (int j = 0; j < 3; ++j) {
            c->bboxMin = vmin3(c->bboxMin, vs[j]);
            c->bboxMax = vmax3(c->bboxMax, vs[j]);
        }
        for (int i = 0; i < 3; ++i) {
            for (int j = 0; j < 3; ++j) {
                float d = dot3(vs[j], AXIS[i]);
                c->bv.bmin[i] = gmin(d, c->bv.bmin[i]);
                c->bv.bmax[i] = gmax(d, c->bv.bmax[i]);
            }
        }
    }
}
static void build_bvh(oracle_scene* s) { /* BVH::BVH (bvh.cpp:252-326) */
    const nart_scene_blob* b = s->blob;
    uint32_t numTriangles = 0;
    v3 sceneMax = V3(-INF_F, -INF_F, -INF_F), sceneMin = V3(INF_F, INF_F, INF_F);
    for (uint32_t m = 0; m < b->num_meshes; ++m) {
        numTriangles += b->meshes[m].num_tris;
        for (uint32_t i = 0; i < b->meshes[m].num_tris; ++i) {
            const nart_triangle* T = &b->triangles[b->meshes[m].first_tri + i];
            v3 vs[3] = {tv(T->v0), tv(T->v1), tv(T->v2)};
            for (int j = 0; j < 3; ++j) {
                sceneMax = vmax3(vs[j], sceneMax);
                sceneMin = vmin3(vs[j], sceneMin);
            }
        }
    }
    v3 sceneSize = sub3(sceneMax, sceneMin);
    float lambda = 3.f;
    float sceneVolume = sceneSize.x * sceneSize.y * sceneSize.z;
    v3 q = muls3(divs3(V3((float)numTriangles, (float)numTriangles, (float)numTriangles), sceneVolume), lambda);
    float third = 1.f / 3.f;
    v3 res = V3(floorf(sceneSize.x * powf(q.x, third)), floorf(sceneSize.y * powf(q.y, third)),
                floorf(sceneSize.z * powf(q.z, third)));
    res = V3(gmin(gmax(res.x, 1.f), 128.f), gmin(gmax(res.y, 1.f), 128.f), gmin(gmax(res.z, 1.f), 128.f));
    uint32_t numChunks = f2u32(res.x * res.y * res.z);
    s->grid_res[0] = f2u32(res.x);
    s->grid_res[1] = f2u32(res.y);
    s->grid_res[2] = f2u32(res.z);
    s->nchunks_total = numChunks + 1;
    s->chunks = (chunk_t*)calloc(s->nchunks_total, sizeof(chunk_t));
    for (uint32_t m = 0; m < b->num_meshes; ++m) {
        for (uint32_t i = 0; i < b->meshes[m].num_tris; ++i) {
            uint32_t g = b->meshes[m].first_tri + i;
            const nart_triangle* T = &b->triangles[g];
            v3 tmin = sub3(vmin3(vmin3(tv(T->v0), tv(T->v1)), tv(T->v2)), sceneMin);
            v3 cc = mul3(div3(tmin, sceneSize), res);
            cc = V3(floorf(cc.x), floorf(cc.y), floorf(cc.z));
            /* chunk index bug: cx*ry*rz + cy*rz + cx (bvh.cpp:304-306) */
            uint32_t ci = f2u32(floorf(cc.x * res.y * res.z + cc.y * res.z + cc.x));
            ci = (numChunks < ci) ? numChunks : ci;
            chunk_push(&s->chunks[ci], g);
        }
    }
    s->root = new_node(s, sceneMin, sceneMax);
    for (uint32_t c = 0; c < s->nchunks_total; ++c) {
        if (s->chunks[c].n) {
            chunk_bounds(s, &s->chunks[c]);
            insert_chunk(s, s->root, (int32_t)c, 0);
        }
    }
    build_bvs(s, s->root);
}

/* Chunk::Intersect (bvh.cpp:66-79) */
static int chunk_intersect(const oracle_scene* s, const chunk_t* c, const ray_t* ray, isect_t* is) {
    int hit = 0;
    for (uint32_t k = 0; k < c->n; ++k) {
        uint32_t g = c->tris[k];
        if (triangle_intersect(&s->blob->triangles[g], ray, is)) {
            hit = 1;
            const nart_mesh* m = &s->blob->meshes[s->tri_mesh[g]];
            is->mat = (int32_t)m->material;
            is->meshID = s->tri_mesh[g];
            is->priority = m->priority;
        }
    }
    return hit;
}

/* Octree::Intersect (bvh.cpp:132-176): best-first with a binary min-heap of (tEntry, node).
   Equal keys are ordered by node creation index (the reference orders by node address). */
typedef struct { float key; int32_t node; } qent_t;
static inline int qless(qent_t a, qent_t b) { return a.key < b.key || (!(b.key < a.key) && a.node < b.node); }
typedef struct { qent_t* e; uint32_t n, cap; } heap_t;
static void heap_push(heap_t* h, qent_t x) {
    if (h->n == h->cap) {
        h->cap = h->cap ? h->cap * 2 : 64;
        h->e = (qent_t*)realloc(h->e, h->cap * sizeof(qent_t));
    }
    uint32_t i = h->n++;
    while (i > 0) {
        uint32_t p = (i - 1) / 2;
        if (!qless(x, h->e[p])) break;
        h->e[i] = h->e[p];
        i = p;
    }
    h->e[i] = x;
}
static qent_t heap_pop(heap_t* h) {
    qent_t top = h->e[0];
    qent_t x = h->e[--h->n];
    uint32_t i = 0;
    for (;;) {
        uint32_t l = 2 * i + 1, r = l + 1, m = i;
        qent_t best = x;
        if (l < h->n && qless(h->e[l], best)) { m = l; best = h->e[l]; }
        if (r < h->n && qless(h->e[r], best)) { m = r; }
        if (m == i) break;
        h->e[i] = h->e[m];
        i = m;
    }
    if (h->n) h->e[i] = x;
    return top;
}
static int bvh_intersect(const oracle_scene* s, const ray_t* ray, isect_t* is, heap_t* q) {
    q->n = 0;
    qent_t r0 = {INF_F, s->root};
    heap_push(q, r0);
    int hit = 0;
    while (q->n) {
        qent_t cur = heap_pop(q);
        const onode_t* node = &s->nodes[cur.node];
        for (int c = 0; c < 8; ++c) {
            int ch = node->children[c];
            if (ch < 0) continue;
            const onode_t* child = &s->nodes[ch];
            float te;
            if (bv_intersect(&child->bv, ray, &te)) {
                qent_t e = {te, ch};
                heap_push(q, e);
                if (child->isLeaf) {
                    for (uint32_t k = 0; k < child->nchunks; ++k) {
                        isect_t tri;
                        isect_init(&tri);
                        if (chunk_intersect(s, &s->chunks[child->chunks[k]], ray, &tri)) {
                            if (tri.tMax < is->tMax) {
                                *is = tri;
                                hit = 1;
                            }
                        }
                    }
                }
            }
        }
        if (q->n && is->tMax < q->e[0].key) break;
    }
    return hit;
}

/* ---------------------------------------------------------------- patterns */
static v3 tex_fetch(const oracle_scene* s, int tex, float su, float sv, int rough) { /* texturepattern.cpp:172-187 */
    const nart_texture* t = &s->blob->textures[tex];
    float u = gmin(gmax(su, 0.0001f), 0.9999f);
    float v = gmin(gmax(1.f - sv, 0.0001f), 0.9999f);
    int iu = (int)((float)t->width * u);
    int iv = (int)((float)t->height * v);
    const float* px = &s->tex_f[s->tex_off[tex] + ((size_t)iv * t->width + (size_t)iu) * 3];
    float r = px[0], g = px[1], b = px[2];
    if (rough) { r *= r; g *= g; b *= b; }
    return V3(r, g, b);
}
static v3 ptn_value(const oracle_scene* s, const nart_pattern* p, v2 st) {
    if (p->type == NART_PTN_CONSTANT) return V3(p->value[0], p->value[1], p->value[2]);
    return tex_fetch(s, p->texture, st.x, st.y, p->is_roughness);
}

/* ---------------------------------------------------------------- BxDFs */
enum { B_LAMBERT, B_SPECULAR, B_SPECDIEL, B_DIEL, B_TS };
enum { F_SPECULAR = 1, F_GLOSSY = 2, F_DIFFUSE = 4, F_TRANSMISSIVE = 8 };
typedef struct {
    int type;
    uint8_t flags; /* BxDF::flags member (set in ctor) */
    v3 rho, tau;
    float eta, alpha_0, alpha_prime;
} bxdf_t;

static float fresnel(float eta_o, float eta_i, float cosTheta) { /* bxdf.cpp:3-22 */
    if (eta_o == eta_i) return 0.f;
    float cos_o = gmin(gabs(cosTheta), 1.f);
    float sin_o = sqrtf(1.f - (cos_o * cos_o));
    float sin_i = (eta_o / eta_i) * sin_o;
    if (sin_i > 1.f) return 1.f;
    float cos_i = sqrtf(1.f - (sin_i * sin_i));
    if (gabs(cos_o + cos_i) < 0.00001f) return 0.f;
    float fPara = ((eta_i * cos_o) - (eta_o * cos_i)) / ((eta_i * cos_o) + (eta_o * cos_i));
    float fPerp = ((eta_o * cos_o) - (eta_i * cos_i)) / ((eta_o * cos_o) + (eta_i * cos_i));
    return ((fPara * fPara) + (fPerp * fPerp)) * 0.5f;
}
static inline v3 reflect3(v3 w1, v3 w2) { return sub3(muls3(w2, 2.f * dot3(w1, w2)), w1); } /* bxdf.h:14-16 */

/* Smith Lambda / GGX D shared by DielectricBRDF and TorranceSparrowBRDF */
static float lambda_(float alpha, v3 w) {
    float sinT = sqrtf(1.f - (w.z * w.z));
    float tanT = (sinT / w.z);
    return (-1.f + sqrtf(1.f + (alpha * alpha * tanT * tanT))) * 0.5f;
}
static float G_(float a, v3 wo, v3 wi) { return 1.f / (1.f + lambda_(a, wo) + lambda_(a, wi)); }
static float G1_(float a, v3 w) { return 1.f / (1.f + lambda_(a, w)); }
static float D_ggx(float alpha, v3 wh) { /* torrancesparrowbrdf.cpp:19-30 (no wh.z==0 test) */
    float sinT = sqrtf(1.f - (wh.z * wh.z));
    float tanT = (sinT / wh.z);
    float tan2 = tanT * tanT;
    return 1.f / ((PI_F * alpha * alpha * ((wh.z * wh.z) * (wh.z * wh.z))) * (1.f + (tan2 / (alpha * alpha))) *
                  (1.f + (tan2 / (alpha * alpha))));
}
static float D_diel(float alpha, v3 wh) { /* dielectricbrdf.cpp:19-29 */
    if (wh.z == 0.f) return 0.f;
    return D_ggx(alpha, wh);
}

/* VNDF sample shared by both microfacet lobes (dielectricbrdf.cpp:106-139,
   torrancesparrowbrdf.cpp:68-96).  diel selects the wo.x==wo.y==0 and wo.z<0 handling. */
static v3 sample_wh(v3 wo, float alpha, v2 sample, int diel) {
    v3 wo_h = normalize3(V3(wo.x * alpha, wo.y * alpha, wo.z));
    if (diel && wo.z < 0.f) wo_h = muls3(wo_h, -1.f);
    v3 T1;
    if (diel && wo.x == 0.f && wo.y == 0.f) T1 = V3(1.f, 0.f, 0.f);
    else T1 = V3(wo_h.y, -wo_h.x, 0.f);
    T1 = normalize3(T1);
    v3 T2 = normalize3(cross3(T1, wo_h));
    v2 vh = uniform_sample_disk(sample);
    float s = (1.f + wo_h.z) * 0.5f;
    vh.y = (s * vh.y) + ((1.f - s) * sqrtf(1.f - (vh.x * vh.x)));
    v3 wh = V3(sqrtf(1.f - (vh.x * vh.x) - (vh.y * vh.y)), vh.x, vh.y);
    wh = add3(add3(muls3(wo_h, wh.x), muls3(T1, wh.y)), muls3(T2, wh.z));
    wh = normalize3(V3(wh.x * alpha, wh.y * alpha, wh.z));
    return wh;
}

static v3 bxdf_f(const bxdf_t* b, v3 wo, v3 wi, int uap, float eta_outer) {
    switch (b->type) {
        case B_LAMBERT: return muls3(b->rho, ONE_OVER_PI_F); /* lambertbrdf.cpp:7-11 */
        case B_SPECULAR:
        case B_SPECDIEL: return V3(0.f, 0.f, 0.f);
        case B_DIEL: { /* dielectricbrdf.cpp:31-80 */
            float alpha = uap ? b->alpha_prime : b->alpha_0;
            float eta_o = eta_outer, eta_i = b->eta;
            if (wo.z < 0.f) { float t = eta_o; eta_o = eta_i; eta_i = t; }
            if (wo.z * wi.z >= 0.f) {
                v3 wh = normalize3(add3(wo, wi));
                if (wh.z < 0.f) wh = muls3(wh, -1.f);
                float g = G_(alpha, wo, wi);
                float d = D_diel(alpha, wh);
                float Fr = fresnel(eta_o, eta_i, gabs(dot3(wh, wo)));
                if (wo.z * wi.z == 0.f) return V3(0.f, 0.f, 0.f);
                return divs3(muls3(muls3(muls3(b->rho, g), d), Fr), (4.f * wo.z * wi.z));
            } else {
                v3 wh = normalize3(add3(muls3(wo, eta_o), muls3(wi, eta_i)));
                if (wh.z < 0.f) wh = muls3(wh, -1.f);
                float Fr = fresnel(eta_o, eta_i, gabs(dot3(wh, wo)));
                if (Fr >= 1.f) return V3(0.f, 0.f, 0.f);
                float g = G_(alpha, wo, wi);
                float d = D_diel(alpha, wh);
                float wiDotWh = dot3(wi, wh);
                float woDotWh = dot3(wo, wh);
                float num = g * d * (1.f - Fr) * gabs(wiDotWh) * gabs(woDotWh) * eta_o * eta_o;
                float x = ((eta_i * wiDotWh) + (eta_o * woDotWh));
                float denom = x * x * gabs(wo.z * wi.z);
                float q = num / denom;
                return mul3(V3(q, q, q), b->tau);
            }
        }
        case B_TS: { /* torrancesparrowbrdf.cpp:32-51 */
            float alpha = uap ? b->alpha_prime : b->alpha_0;
            if (wo.z < 0.f || wi.z < 0.f) return V3(0.f, 0.f, 0.f);
            v3 wh = normalize3(add3(wo, wi));
            float g = G_(alpha, wo, wi);
            float d = D_ggx(alpha, wh);
            float fr = fresnel(eta_outer, b->eta, dot3(wh, wi));
            if (wo.z * wi.z == 0.f) return V3(0.f, 0.f, 0.f);
            return divs3(muls3(muls3(muls3(b->rho, g), d), fr), (4.f * wo.z * wi.z));
        }
    }
    return V3(0.f, 0.f, 0.f);
}

static float bxdf_pdf(const bxdf_t* b, v3 wo, v3 wi, int uap, float eta_outer) {
    switch (b->type) {
        case B_LAMBERT: return wi.z * ONE_OVER_PI_F;
        case B_SPECULAR:
        case B_SPECDIEL: return 0.f;
        case B_DIEL: { /* dielectricbrdf.cpp:187-225 */
            float eta_o = eta_outer, eta_i = b->eta;
            if (eta_o == eta_i) return 0.f;
            float alpha = uap ? b->alpha_prime : b->alpha_0;
            if (wo.z * wi.z >= 0.f) {
                v3 wh = normalize3(add3(wo, wi));
                if (wh.z < 0.f) wh = muls3(wh, -1.f);
                float cosThetaH = gabs(gmin(dot3(wo, wh), 1.f));
                float pdf = (D_diel(alpha, wh) * gmin(dot3(wo, wh), 1.f) * G1_(alpha, wo)) / wo.z;
                return gmax(0.f, pdf / (4.f * cosThetaH));
            }
            if (wo.z < 0.f) { float t = eta_o; eta_o = eta_i; eta_i = t; }
            v3 wh = normalize3(add3(muls3(wo, eta_o), muls3(wi, eta_i)));
            if (wh.z < 0.f) wh = muls3(wh, -1.f);
            float pdf = (D_diel(alpha, wh) * gmin(gabs(dot3(wo, wh)), 1.f) * G1_(alpha, wo)) / gabs(wo.z);
            float dotWiWh = dot3(wi, wh);
            float dotWoWh = dot3(wo, wh);
            float denom = (eta_i * dotWiWh + eta_o * dotWoWh);
            float JDet = (fabsf(dotWiWh) * eta_i * eta_i) / (denom * denom);
            return pdf * JDet;
        }
        case B_TS: { /* torrancesparrowbrdf.cpp:109-124 */
            float alpha = uap ? b->alpha_prime : b->alpha_0;
            v3 wh = normalize3(add3(wo, wi));
            if (wh.z < 0.f) return 0.f;
            float cosThetaH = gmin(dot3(wo, wh), 1.f);
            float pdf = (D_ggx(alpha, wh) * gmin(dot3(wo, wh), 1.f) * G1_(alpha, wo)) / wo.z;
            return gmax(0.f, pdf / (4.f * cosThetaH));
        }
    }
    return 0.f;
}

static float bxdf_eta(const bxdf_t* b) { return b->type == B_LAMBERT ? 0.f : b->eta; }

/* BxDF::Sample_f for each lobe.  alpha_i may be NULL. */
static v3 bxdf_sample_f(const bxdf_t* b, v3 wo, v3* wi, float s1, v2 sample, float* pdf, uint8_t* flags,
                        float* alpha_i, int uap, float eta_outer) {
    (void)s1;
    switch (b->type) {
        case B_LAMBERT: /* lambertbrdf.cpp:13-22 */
            if (alpha_i) *alpha_i = 1.f;
            *flags = F_DIFFUSE;
            *wi = cosine_sample_hemisphere(sample, pdf);
            return bxdf_f(b, wo, *wi, uap, eta_outer);
        case B_SPECULAR: /* specularbrdf.cpp:14-36 */
            if (alpha_i) *alpha_i = 0.f;
            *flags = F_SPECULAR;
            *wi = V3(-wo.x, -wo.y, wo.z);
            *pdf = 1.f;
            if (wi->z == 0.f) return V3(1.f, 1.f, 1.f);
            return divs3(muls3(b->rho, fresnel(eta_outer, b->eta, wi->z)), gabs(wi->z));
        case B_SPECDIEL: { /* speculardielectricbrdf.cpp:15-89 */
            float eta_o = eta_outer, eta_i = b->eta;
            if (eta_o == eta_i) {
                *wi = neg3(wo);
                *pdf = 0.f;
                *flags |= F_TRANSMISSIVE;
                return b->tau;
            }
            if (alpha_i) *alpha_i = 0.f;
            *flags = F_SPECULAR;
            if (wo.z < 0.f) { float t = eta_o; eta_o = eta_i; eta_i = t; }
            float Fr = fresnel(eta_o, eta_i, gabs(wo.z));
            if (sample.x < Fr) {
                *pdf = Fr;
                *wi = V3(-wo.x, -wo.y, wo.z);
                if (wi->z == 0.f) return V3(1.f, 1.f, 1.f);
                float q = Fr / gabs(wi->z);
                return mul3(V3(q, q, q), b->rho);
            }
            *pdf = 1.f - Fr;
            float sinT_o = sqrtf(1.f - (wo.z * wo.z));
            float sinT_i = ((eta_o / eta_i) * sinT_o);
            if (sinT_i >= 1.f) {
                *wi = V3(-wo.x, -wo.y, wo.z);
                return mul3(V3(1.f, 1.f, 1.f), b->rho);
            }
            *flags |= F_TRANSMISSIVE;
            v3 n = V3(0.f, 0.f, 1.f);
            v3 bb = muls3(n, wo.z);
            v3 a = sub3(wo, bb);
            v3 c = muls3(neg3(a), (eta_o / eta_i));
            v3 d = muls3(neg3(n), sqrtf(1.f - (sinT_i * sinT_i)));
            if (wo.z < 0.f) d = muls3(d, -1.f);
            *wi = normalize3(add3(c, d));
            float q = ((eta_o / eta_i) * (eta_o / eta_i) * (1.f - Fr)) / gabs(wi->z);
            v3 f = V3(q, q, q);
            return mul3(f, b->tau);
        }
        case B_DIEL: { /* dielectricbrdf.cpp:82-183 */
            float eta_o = eta_outer, eta_i = b->eta;
            if (eta_o == eta_i) {
                *wi = neg3(wo);
                *pdf = 0.f;
                *flags |= F_TRANSMISSIVE;
                return b->tau;
            }
            float alpha = uap ? b->alpha_prime : b->alpha_0;
            if (alpha_i) *alpha_i = alpha;
            *flags = F_SPECULAR;
            if (alpha > 0.0001f) *flags = F_GLOSSY;
            if (alpha >= 1.0f) *flags = F_DIFFUSE;
            v3 wh = sample_wh(wo, alpha, sample, 1);
            if (wo.z < 0.f) { float t = eta_o; eta_o = eta_i; eta_i = t; }
            float Fr = fresnel(eta_o, eta_i, gabs(dot3(wh, wo)));
            if (s1 < Fr) {
                *wi = normalize3(reflect3(wo, wh));
                *pdf = bxdf_pdf(b, wo, *wi, uap, eta_outer) * Fr;
                return bxdf_f(b, wo, *wi, uap, eta_outer);
            }
            float cos_o = gmin(1.f, gmax(-1.f, dot3(wo, wh)));
            float sin_o = sqrtf(1.f - (cos_o * cos_o));
            float sin_i = ((eta_o / eta_i) * sin_o);
            if (sin_i >= 1.f) {
                *wi = normalize3(reflect3(wo, wh));
                *pdf = bxdf_pdf(b, wo, *wi, uap, eta_outer) * (1.f - Fr);
                return bxdf_f(b, wo, *wi, uap, eta_outer);
            }
            *flags |= F_TRANSMISSIVE;
            v3 bb = muls3(wh, cos_o);
            v3 a = sub3(wo, bb);
            v3 c = muls3(neg3(a), (eta_o / eta_i));
            v3 d = muls3(neg3(wh), sqrtf(1.f - (sin_i * sin_i)));
            if (dot3(wo, wh) < 0.f) d = muls3(d, -1.f);
            *wi = normalize3(add3(c, d));
            *pdf = bxdf_pdf(b, wo, *wi, uap, eta_outer) * (1.f - Fr);
            return bxdf_f(b, wo, *wi, uap, eta_outer);
        }
        case B_TS: { /* torrancesparrowbrdf.cpp:53-105 */
            float alpha = uap ? b->alpha_prime : b->alpha_0;
            if (alpha_i) *alpha_i = alpha;
            *flags = F_SPECULAR;
            if (alpha > 0.001f) *flags = F_GLOSSY;
            if (alpha >= 1.0f) *flags = F_DIFFUSE;
            v3 wh = sample_wh(wo, alpha, sample, 0);
            *wi = normalize3(reflect3(wo, wh));
            *pdf = bxdf_pdf(b, wo, *wi, uap, eta_outer);
            return bxdf_f(b, wo, *wi, uap, eta_outer);
        }
    }
    return V3(0.f, 0.f, 0.f);
}

/* ---------------------------------------------------------------- BSDF (bxdf.cpp:24-115) */
typedef struct {
    v3 n_t, n_b, n;
    uint8_t num;
    bxdf_t b[2];
} bsdf_t;
static inline v3 to_local(const bsdf_t* s, v3 v) { return normalize3(V3(dot3(v, s->n_t), dot3(v, s->n_b), dot3(v, s->n))); }
static inline v3 to_world(const bsdf_t* s, v3 v) {
    return normalize3(add3(add3(muls3(s->n_t, v.x), muls3(s->n_b, v.y)), muls3(s->n, v.z)));
}
static void build_coord_sys(bsdf_t* s, const isect_t* is, const v3* nn) { /* bxdf.cpp:27-45 */
    s->n_t = normalize3(sub3(is->dpds, muls3(s->n, dot3(is->dpds, s->n))));
    s->n_b = normalize3(cross3(is->sn, s->n_t));
    if (nn) {
        s->n = normalize3(to_world(s, *nn));
        s->n_t = normalize3(sub3(is->dpds, muls3(s->n, dot3(is->dpds, s->n))));
        s->n_b = normalize3(cross3(is->sn, s->n_t));
    }
}
static v3 bsdf_f(const bsdf_t* s, v3 wo, v3 wi, int uap, float eta_outer) {
    v3 f = V3(0.f, 0.f, 0.f);
    for (uint8_t i = 0; i < s->num; ++i) f = add3(f, bxdf_f(&s->b[i], wo, wi, uap, eta_outer));
    return f;
}
static v3 bsdf_sample_f(const bsdf_t* s, v3 wo, v3* wi, float s1, v2 sample, float* pdf, uint8_t* flags, int uap,
                        float eta_outer, float* alpha_i, float* eta_i) {
    uint8_t idx = f2u8(s1 * (float)s->num);
    s1 = gfract(s1 * (float)s->num);
    v3 f = bxdf_sample_f(&s->b[idx], wo, wi, s1, sample, pdf, flags, alpha_i, uap, eta_outer);
    if (eta_i && (*flags & F_TRANSMISSIVE)) *eta_i = bxdf_eta(&s->b[idx]);
    if (!(*flags & F_SPECULAR)) {
        for (uint8_t i = 0; i < s->num; ++i) {
            if (i != idx && !(s->b[i].flags & F_SPECULAR)) {
                float bp = bxdf_pdf(&s->b[i], wo, *wi, uap, eta_outer);
                if (bp > 0.f) {
                    *pdf += bxdf_pdf(&s->b[i], wo, *wi, uap, eta_outer);
                    f = add3(f, bxdf_f(&s->b[i], wo, *wi, uap, eta_outer));
                }
            }
        }
        *pdf /= (float)s->num;
    }
    return f;
}
static float bsdf_sample_eta(const bsdf_t* s, float s1) { return bxdf_eta(&s->b[f2u8(s1 * (float)s->num)]); }
static float bsdf_pdf(const bsdf_t* s, v3 wo, v3 wi, int uap, float eta_outer) {
    float pdf = 0.f;
    for (uint8_t i = 0; i < s->num; ++i) pdf += bxdf_pdf(&s->b[i], wo, wi, uap, eta_outer);
    return pdf / (float)s->num;
}

/* ---------------------------------------------------------------- materials */
static void mk_lambert(bxdf_t* b, v3 rho) { memset(b, 0, sizeof(*b)); b->type = B_LAMBERT; b->flags = F_DIFFUSE; b->rho = rho; }
static void mk_specular(bxdf_t* b, v3 rho_s, float eta) { memset(b, 0, sizeof(*b)); b->type = B_SPECULAR; b->flags = F_SPECULAR; b->rho = rho_s; b->eta = eta; }
static void mk_specdiel(bxdf_t* b, v3 rho_s, v3 tau, float eta) { memset(b, 0, sizeof(*b)); b->type = B_SPECDIEL; b->flags = F_SPECULAR; b->rho = rho_s; b->tau = tau; b->eta = eta; }
static void mk_diel(bxdf_t* b, v3 rho_s, v3 tau, float eta, float a0, float ap) { memset(b, 0, sizeof(*b)); b->type = B_DIEL; b->flags = F_GLOSSY; b->rho = rho_s; b->tau = tau; b->eta = eta; b->alpha_0 = a0; b->alpha_prime = ap; }
static void mk_ts(bxdf_t* b, v3 rho_s, float eta, float a0, float ap) { memset(b, 0, sizeof(*b)); b->type = B_TS; b->flags = F_GLOSSY; b->rho = rho_s; b->eta = eta; b->alpha_0 = a0; b->alpha_prime = ap; }

static void create_bsdf(const oracle_scene* s, const isect_t* is, float alphaTweak, bsdf_t* bs) {
    const nart_material* m = &s->blob->materials[is->mat];
    memset(bs, 0, sizeof(*bs));
    bs->n = is->sn;
    bs->num = m->type == NART_MAT_PLASTIC ? 2 : 1;
    if (m->has_normal && m->type != NART_MAT_GLASS) {
        v3 n = ptn_value(s, &m->normal, is->st);
        n = muls3(n, 2.f);
        n = sub3(n, V3(1.f, 1.f, 1.f));
        build_coord_sys(bs, is, &n);
    } else {
        build_coord_sys(bs, is, NULL);
    }
    switch (m->type) {
        case NART_MAT_LAMBERT: /* diffusematerial.cpp:6-27 */
            mk_lambert(&bs->b[0], ptn_value(s, &m->rho_d, is->st));
            break;
        case NART_MAT_SPECULAR: { /* specularmaterial.cpp:9-43 */
            float alpha = 0.f;
            float ap = 1.f - ((1.f - alpha) * alphaTweak);
            v3 rho_s = ptn_value(s, &m->rho_s, is->st);
            float eta = ptn_value(s, &m->eta, is->st).x;
            if (ap > 0.0001f) mk_ts(&bs->b[0], rho_s, eta, gmax(0.0001f, alpha), ap);
            else mk_specular(&bs->b[0], rho_s, eta);
            break;
        }
        case NART_MAT_GLASS: { /* glassmaterial.cpp:11-47 */
            float alpha = ptn_value(s, &m->alpha, is->st).x;
            float ap = 1.f - ((1.f - ptn_value(s, &m->alpha, is->st).x) * alphaTweak);
            v3 rho_s = ptn_value(s, &m->rho_s, is->st);
            v3 tau = ptn_value(s, &m->tau, is->st);
            float eta = ptn_value(s, &m->eta, is->st).x;
            if (ap > 0.0001f) mk_diel(&bs->b[0], rho_s, tau, eta, gmax(0.0001f, alpha), ap);
            else mk_specdiel(&bs->b[0], rho_s, tau, eta);
            break;
        }
        case NART_MAT_GLOSSY: { /* glossydielectricmaterial.cpp:12-47 */
            float alpha = ptn_value(s, &m->alpha, is->st).x;
            float ap = 1.f - ((1.f - alpha) * alphaTweak);
            v3 rho_s = ptn_value(s, &m->rho_s, is->st);
            float eta = ptn_value(s, &m->eta, is->st).x;
            if (ap > 0.0001f) mk_ts(&bs->b[0], rho_s, eta, gmax(0.0001f, alpha), ap);
            else mk_specular(&bs->b[0], rho_s, eta);
            break;
        }
        case NART_MAT_PLASTIC: { /* plasticmaterial.cpp:12-51 */
            float alpha = ptn_value(s, &m->alpha, is->st).x;
            float ap = 1.f - ((1.f - alpha) * alphaTweak);
            v3 rho_d = ptn_value(s, &m->rho_d, is->st);
            v3 rho_s = ptn_value(s, &m->rho_s, is->st);
            float eta = ptn_value(s, &m->eta, is->st).x;
            mk_lambert(&bs->b[0], rho_d);
            if (ap > 0.001f) mk_ts(&bs->b[1], rho_s, eta, gmax(0.0001f, alpha), ap);
            else mk_specular(&bs->b[1], rho_s, eta);
            break;
        }
    }
}

/* ---------------------------------------------------------------- lights */
static uint32_t binary_search(float value, const float* v, uint32_t start, uint32_t end) { /* util.cpp:4-20 */
    uint32_t i = start;
    while (start < end) {
        i = start + ((end - start) / 2);
        if (v[i] > value) {
            end = i;
            i -= 1;
        } else {
            start = i + 1;
        }
    }
    return i;
}
static float pw_pdf(const struct pw2d* d, v2 s) { /* texturepattern.cpp:104-109 */
    uint32_t u = f2u32(s.x * (float)d->w);
    uint32_t v = f2u32(s.y * (float)d->h);
    return d->mpdf[v] * d->cpdf[v * d->w + u];
}
static v2 pw_sample(const struct pw2d* d, v2 s, float* pdf) { /* texturepattern.cpp:72-102 */
    uint32_t lb = binary_search(s.y, d->mcdf, 0, d->h);
    float uc = 0.f;
    float vc = ((s.y - d->mcdf[lb]) / d->mpdf[lb]) + ((float)lb * d->invH);
    vc = gmin(vc, 0.9999999f);
    uint32_t v = f2u32(vc * (float)d->h);
    if (d->mpdf[v] > 0.f) {
        lb = binary_search(s.x, d->ccdf, v * (d->w + 1), v * (d->w + 1) + d->w);
        lb %= (d->w + 1);
        uc = ((s.x - d->ccdf[v * (d->w + 1) + lb]) / d->cpdf[v * d->w + lb]) + ((float)lb * d->invW);
        uc = gmin(uc, 0.9999999f);
        uint32_t u = f2u32(uc * (float)d->w);
        *pdf = d->mpdf[v] * d->cpdf[v * d->w + u];
    }
    /* else: `pdf == 0.f;` is a no-op (texturepattern.cpp:99): pdf keeps its value */
    return V2(uc, vc);
}
/* Pattern::Sample / Pdf for the env light's Le (constantpattern.cpp:3-14, texturepattern.cpp:130-170) */
static v3 ptn_sample(const oracle_scene* s, int light, const nart_pattern* p, v2 sample, v2* ps, float* pdf) {
    if (p->type == NART_PTN_CONSTANT) {
        *ps = sample;
        *pdf = 1.f;
        return V3(p->value[0], p->value[1], p->value[2]);
    }
    *ps = sample;
    if (!s->env[light].present) *pdf = 1.f;
    else *ps = pw_sample(&s->env[light], sample, pdf);
    return tex_fetch(s, p->texture, ps->x, ps->y, p->is_roughness);
}
static float ptn_pdf(const oracle_scene* s, int light, const nart_pattern* p, v2 st) {
    if (p->type == NART_PTN_CONSTANT || !s->env[light].present) return 1.f;
    v2 q = V2(gmin(st.x, 0.9999f), gmin(st.y, 0.9999f));
    return pw_pdf(&s->env[light], q);
}

typedef struct { v3 p; v2 st; float tMax; } lisect_t;

static float area_pdf(const nart_light* L, lisect_t* li, v3 p, v3 wi) { /* disklight.cpp:62-104, ringlight.cpp:66-112 */
    v3 center = xyz(vec_mul_mat(V4(0.f, 0.f, 0.f, 1.f), L->m));
    v3 n = xyz(vec_mul_mat(V4(0.f, 0.f, -1.f, 0.f), L->m));
    if (dot3(wi, n) >= 0.f) return 0.f;
    float D = dot3(center, n);
    float t = (D - dot3(p, n)) / dot3(wi, n);
    if (t < 0.f) return 0.f;
    v3 pHit = add3(p, muls3(wi, t));
    v3 c2p = sub3(pHit, center);
    float u = dot4(V4(c2p.x, c2p.y, c2p.z, 0.f), vec_mul_mat(V4(1.f, 0.f, 0.f, 0.f), L->m)) / L->radius;
    float v = dot4(V4(c2p.x, c2p.y, c2p.z, 0.f), vec_mul_mat(V4(0.f, 1.f, 0.f, 0.f), L->m)) / L->radius;
    u = (u + 1.f) * 0.5f;
    v = (v + 1.f) * 0.5f;
    li->st = V2(u, 1.f - v);
    float dist = c2p.x * c2p.x + c2p.y * c2p.y + c2p.z * c2p.z;
    if (dist > L->radius * L->radius) return 0.f;
    float pdf;
    if (L->type == NART_LIGHT_RING) {
        if (dist < L->inner_radius * L->inner_radius) return 0.f;
        pdf = 1.f / (PI_F * (1.f - ((L->inner_radius * L->inner_radius) / (L->radius * L->radius))) * L->radius * L->radius);
    } else {
        pdf = 1.f / (PI_F * L->radius * L->radius);
    }
    pdf = pdf * ((t * t) / dot3(neg3(wi), n));
    li->tMax = t;
    return pdf;
}

static void env_dir(v3 wi, float* theta, float* phi) {
    *theta = acosf(wi.z);
    *phi = atan2f(wi.y, wi.x) + PI_F;
    if (*phi > TWO_PI_F) *phi -= TWO_PI_F;
    if (*phi < 0.f) *phi += TWO_PI_F;
}

/* Light::Li (disklight.cpp:12-23, ringlight.cpp:13-24, environmentlight.cpp:9-28) */
static v3 light_li(const oracle_scene* s, int li_idx, lisect_t* li, v3 p, v3 wi, float* pdf) {
    const nart_light* L = &s->blob->lights[li_idx];
    if (L->type == NART_LIGHT_ENVIRONMENT) {
        float theta, phi;
        env_dir(wi, &theta, &phi);
        li->st = V2(1.f - (phi * ONE_OVER_TWO_PI_F), 1.f - (theta * ONE_OVER_PI_F));
        if (pdf) {
            *pdf = ptn_pdf(s, li_idx, &L->Le, li->st);
            *pdf *= ONE_OVER_PI_F * 0.25f / gabs(sinf(theta));
        }
        li->tMax = (float)0x7f7fffff;
        return muls3(ptn_value(s, &L->Le, li->st), L->intensity);
    }
    float lp = area_pdf(L, li, p, wi);
    if (lp > 0.f) {
        if (pdf) *pdf = lp;
        return muls3(ptn_value(s, &L->Le, li->st), L->intensity);
    }
    return V3(0.f, 0.f, 0.f);
}

/* Light::Sample_Li (disklight.cpp:25-60, ringlight.cpp:26-64, environmentlight.cpp:30-61) */
static v3 light_sample_li(const oracle_scene* s, int li_idx, lisect_t* li, v3 p, v3* wi, v2 sample, float* pdf) {
    const nart_light* L = &s->blob->lights[li_idx];
    if (L->type == NART_LIGHT_ENVIRONMENT) {
        v2 ps = V2(0.f, 0.f);
        v3 Lv = muls3(ptn_sample(s, li_idx, &L->Le, sample, &ps, pdf), L->intensity);
        float theta = (1.f - ps.y) * PI_F;
        float phi = (1.f - ps.x) * 2.f * PI_F;
        phi += PI_F;
        if (phi > TWO_PI_F) phi -= TWO_PI_F;
        if (phi < 0.f) phi += TWO_PI_F;
        float x = cosf(phi) * sinf(theta);
        float y = sinf(phi) * sinf(theta);
        float z = cosf(theta);
        *wi = V3(x, y, z);
        *pdf *= ONE_OVER_PI_F * 0.25f / gabs(sinf(theta));
        li->tMax = (float)0x7f7fffff;
        return Lv;
    }
    v4 ds;
    if (L->type == NART_LIGHT_RING) {
        v2 r = uniform_sample_ring(sample, pdf, L->inner_radius / L->radius);
        ds = V4(r.x * L->radius, r.y * L->radius, 0.f, 1.f);
    } else {
        v2 r = uniform_sample_disk(sample);
        ds = V4(r.x * L->radius, r.y * L->radius, 0.f, 1.f);
    }
    float u = ((ds.x + 1.f) * 0.5f) / L->radius;
    float v = ((ds.y + 1.f) * 0.5f) / L->radius;
    li->st = V2(u, 1.f - v);
    ds = vec_mul_mat(ds, L->m);
    v3 n = xyz(vec_mul_mat(V4(0.f, 0.f, -1.f, 0.f), L->m));
    *wi = sub3(xyz(ds), p);
    float dist = sqrtf(wi->x * wi->x + wi->y * wi->y + wi->z * wi->z);
    *wi = normalize3(*wi);
    if (L->type == NART_LIGHT_RING) *pdf /= (PI_F * L->radius * L->radius);
    else *pdf = 1.f / (PI_F * L->radius * L->radius);
    float wiDotN = dot3(neg3(*wi), n);
    if (wiDotN <= 0.f) {
        *pdf = 0.f;
        return V3(0.f, 0.f, 0.f);
    }
    *pdf = *pdf * ((dist * dist) / wiDotN);
    li->p = xyz(ds);
    li->tMax = dist;
    return muls3(ptn_value(s, &L->Le, li->st), L->intensity);
}

/* ---------------------------------------------------------------- path integrator */
typedef struct { uint32_t meshID; uint32_t priority; float eta; } iinfo_t;
#define SHADOW_BIAS 0.001f

typedef struct { heap_t heap; } worker_t;

static int isect_is_valid(const isect_t* is, const iinfo_t* list, uint32_t n, float* eta_outer) { /* pathintegrator.cpp:7-36 */
    *eta_outer = 1.f;
    if (n) {
        if (list[n - 1].meshID != is->meshID) *eta_outer = list[n - 1].eta;
        else if (n >= 2) *eta_outer = list[n - 2].eta;
    }
    for (uint32_t k = 0; k < n; ++k)
        if ((uint8_t)is->priority < (uint8_t)list[k].priority) return 0;
    return 1;
}
static void update_isect_list(iinfo_t* list, uint32_t* n, const isect_t* is, float eta_sampled) { /* 123-142 */
    for (uint32_t k = *n; k-- > 0;) {
        if (list[k].meshID == is->meshID) {
            for (uint32_t j = k; j + 1 < *n; ++j) list[j] = list[j + 1];
            --*n;
            return;
        }
    }
    list[*n].meshID = is->meshID;
    list[*n].priority = is->priority;
    list[*n].eta = eta_sampled;
    ++*n;
}

/* EstimateDirect (pathintegrator.cpp:38-121) */
static v3 estimate_direct(const oracle_scene* s, worker_t* w, v3 wo, const bsdf_t* bsdf, const isect_t* is, rng_t* rng,
                          uint8_t* flags, float eta_outer) {
    v3 L = V3(0.f, 0.f, 0.f);
    v3 wi, Li;
    float scatteringPdf = 0.f, lightingPdf = 0.f;
    float numLights = (float)s->blob->num_lights;
    uint8_t lightIndex = f2u8(gmin(rng_float(rng), 1.f - EPS_F) * numLights);
    /* BSDF sampling */
    scatteringPdf = 0.f;
    float sx = rng_float(rng);
    float sy = rng_float(rng);
    v2 scatterSample = V2(sx, sy);
    float bsdfSample = rng_float(rng);
    v3 f = bsdf_sample_f(bsdf, wo, &wi, bsdfSample, scatterSample, &scatteringPdf, flags, 1, eta_outer, NULL, NULL);
    if (scatteringPdf > 0.f) {
        float flip = wi.z > 0.f ? 1.f : -1.f;
        ray_t shadow = make_ray(add3(is->p, muls3(muls3(is->gn, SHADOW_BIAS), flip)), to_world(bsdf, wi));
        lisect_t li;
        li.tMax = INF_F;
        Li = light_li(s, lightIndex, &li, is->p, to_world(bsdf, wi), &lightingPdf);
        isect_t sh;
        isect_init(&sh);
        sh.tMax = li.tMax;
        if (!bvh_intersect(s, &shadow, &sh, &w->heap)) {
            float weight = 1.f;
            if (!(*flags & F_SPECULAR)) {
                weight = (scatteringPdf * scatteringPdf) / (scatteringPdf * scatteringPdf + lightingPdf * lightingPdf);
                if (lightingPdf > 0.f) L = add3(L, divs3(muls3(muls3(mul3(f, Li), gabs(wi.z)), weight), scatteringPdf));
            } else {
                L = add3(L, divs3(muls3(muls3(mul3(f, Li), gabs(wi.z)), weight), scatteringPdf));
            }
        }
    }
    /* light sampling */
    v3 wiWorld;
    lightingPdf = 0.f;
    float lx = rng_float(rng);
    float ly = rng_float(rng);
    v2 lightSample = V2(lx, ly);
    lisect_t li;
    li.tMax = INF_F;
    Li = light_sample_li(s, lightIndex, &li, is->p, &wiWorld, lightSample, &lightingPdf);
    wi = to_local(bsdf, wiWorld);
    float flip = wi.z > 0.f ? 1.f : -1.f;
    ray_t shadow = make_ray(add3(is->p, muls3(muls3(is->gn, SHADOW_BIAS), flip)), wiWorld);
    isect_t sh;
    isect_init(&sh);
    sh.tMax = li.tMax;
    if (!bvh_intersect(s, &shadow, &sh, &w->heap) && lightingPdf > 0.f) {
        float weight = 1.f;
        scatteringPdf = bsdf_pdf(bsdf, wo, wi, 1, eta_outer);
        if (scatteringPdf > 0.f) {
            v3 f2 = bsdf_f(bsdf, wo, wi, 1, eta_outer);
            weight = (lightingPdf * lightingPdf) / (scatteringPdf * scatteringPdf + lightingPdf * lightingPdf);
            L = add3(L, divs3(muls3(muls3(mul3(f2, Li), gabs(wi.z)), weight), lightingPdf));
        }
    }
    return muls3(L, numLights);
}

/* test statistic: the longest IntersectionInfo list any path reached (oracle_max_list) */
static uint32_t g_max_list = 0;
uint32_t oracle_max_list(int reset) {
    const uint32_t v = __atomic_load_n(&g_max_list, __ATOMIC_RELAXED);
    if (reset) __atomic_store_n(&g_max_list, 0u, __ATOMIC_RELAXED);
    return v;
}

/* PathIntegrator::Li_alpha (pathintegrator.cpp:144-259) */
static v4 li_alpha(const oracle_scene* s, worker_t* w, rng_t* rng, ray_t ray, const nart_render_params* p) {
    iinfo_t list[64];
    uint32_t nlist = 0;
    v3 L = V3(0.f, 0.f, 0.f);
    float alpha = 0.f;
    float eta_sampled = 1.f, eta_outer = 1.f;
    isect_t is;
    isect_init(&is);
    v3 beta = V3(1.f, 1.f, 1.f);
    uint8_t flags = 0;
    float gamma = p->roughening_factor * p->roughening_factor;
    float alphaTweak = 1.f;
    for (uint32_t bounce = 0; bounce < p->bounces; ++bounce) {
        float lightTMax = is.tMax;
        int lightHit = 0;
        v3 Le = V3(0.f, 0.f, 0.f);
        for (uint8_t j = 0; j < s->blob->num_lights; ++j) {
            lisect_t li;
            li.tMax = INF_F;
            v3 Li = light_li(s, j, &li, ray.o, ray.d, NULL);
            if (li.tMax < lightTMax) {
                Le = Li;
                lightTMax = li.tMax;
                is.tMax = li.tMax;
                lightHit = 1;
                alpha = 1.f;
            }
        }
        if (bvh_intersect(s, &ray, &is, &w->heap)) {
            bsdf_t bsdf;
            create_bsdf(s, &is, alphaTweak, &bsdf);
            if (isect_is_valid(&is, list, nlist, &eta_outer)) {
                if (bounce == 0) alpha = 1.f;
                v3 wo = to_local(&bsdf, neg3(ray.d));
                uint8_t directFlags = 0;
                L = add3(L, mul3(estimate_direct(s, w, wo, &bsdf, &is, rng, &directFlags, eta_outer), beta));
                float a = rng_float(rng);
                float b = rng_float(rng);
                v2 scatteringSample = V2(a, b);
                float bsdfSample = rng_float(rng);
                float scatteringPdf = 0.f;
                float alpha_i = 0.f;
                v3 wi;
                v3 f = bsdf_sample_f(&bsdf, wo, &wi, bsdfSample, scatteringSample, &scatteringPdf, &flags, 0, eta_outer,
                                     &alpha_i, &eta_sampled);
                if (scatteringPdf <= 0.f) break;
                alphaTweak = (1.f - (gamma * alpha_i)) * alphaTweak;
                beta = mul3(beta, muls3(divs3(f, scatteringPdf), gabs(wi.z)));
                float flip = wi.z > 0.f ? 1.f : -1.f;
                ray = make_ray(add3(is.p, muls3(muls3(is.gn, SHADOW_BIAS), flip)), to_world(&bsdf, wi));
            } else {
                ray = make_ray(add3(is.p, muls3(ray.d, SHADOW_BIAS)), ray.d);
                flags = F_TRANSMISSIVE;
                float bsdfSample = rng_float(rng);
                eta_sampled = bsdf_sample_eta(&bsdf, bsdfSample);
            }
            if (flags & F_TRANSMISSIVE) {
                update_isect_list(list, &nlist, &is, eta_sampled);
                uint32_t m = __atomic_load_n(&g_max_list, __ATOMIC_RELAXED);
                while (nlist > m && !__atomic_compare_exchange_n(&g_max_list, &m, nlist, 1, __ATOMIC_RELAXED,
                                                                 __ATOMIC_RELAXED)) {
                }
            }
            float q = gmax((beta.x + beta.y + beta.z) * 0.33333f, 0.f);
            if (bounce > 3) {
                if (q >= rng_float(rng)) beta = divs3(beta, q);
                else break;
            }
            isect_init(&is);
        } else if (bounce == 0) {
            if (lightHit) L = Le;
            break;
        } else {
            /* escaped at bounce > 0: the remaining iterations repeat the same miss with no
               RNG draws and no state change (Q6) */
            break;
        }
    }
    return V4(L.x, L.y, L.z, alpha);
}

/* ---------------------------------------------------------------- volume integrator */
static v3 uniform_sample_sphere(v2 smp) { /* sampling.cpp:33-45 (pdf = 1/(4 pi) is unused) */
    float theta = acosf(1.f - (2.f * smp.x));
    float phi = smp.y * TWO_PI_F;
    float cosTheta = cosf(theta);
    float sinTheta = sinf(theta);
    float cosPhi = cosf(phi);
    float sinPhi = sinf(phi);
    return V3(sinTheta * cosPhi, sinTheta * sinPhi, cosTheta);
}

static float dg_at(const nart_medium* m, uint8_t x, uint8_t y, uint8_t z) { /* media.cpp:3-7 */
    uint8_t rx = (uint8_t)m->res[0], ry = (uint8_t)m->res[1];
    uint32_t index = (uint32_t)((rx * ry * z) + (rx * y) + x);
    return m->density[index];
}
static float dg_lookup(const nart_medium* m, v3 p) { /* media.cpp:10-45, trilinear */
    uint8_t rx = (uint8_t)m->res[0], ry = (uint8_t)m->res[1], rz = (uint8_t)m->res[2];
    float x = gmin(gmax(0.f, p.x), 0.999f) * (float)(rx - 1);
    uint8_t loX = (uint8_t)x, hiX = (uint8_t)(loX + 1);
    float xD = (x - (float)loX);
    float y = gmin(gmax(0.f, p.y), 0.999f) * (float)(ry - 1);
    uint8_t loY = (uint8_t)y, hiY = (uint8_t)(loY + 1);
    float yD = (y - (float)loY);
    float z = gmin(gmax(0.f, p.z), 0.999f) * (float)(rz - 1);
    uint8_t loZ = (uint8_t)z, hiZ = (uint8_t)(loZ + 1);
    float zD = (z - (float)loZ);
    float x0 = gmix(dg_at(m, loX, loY, loZ), dg_at(m, hiX, loY, loZ), xD);
    float x1 = gmix(dg_at(m, loX, loY, hiZ), dg_at(m, hiX, loY, hiZ), xD);
    float x2 = gmix(dg_at(m, loX, hiY, loZ), dg_at(m, hiX, hiY, loZ), xD);
    float x3 = gmix(dg_at(m, loX, hiY, hiZ), dg_at(m, hiX, hiY, hiZ), xD);
    float y0 = gmix(x0, x2, yD);
    float y1 = gmix(x1, x3, yD);
    return gmix(y0, y1, zD);
}
static uint8_t u8min(uint8_t a, uint8_t b) { return b < a ? b : a; }
static void build_medium(oracle_scene* s) { /* MajorantGrid ctor, width 1 (media.cpp:47-130) */
    const nart_medium* m = &s->blob->medium;
    s->has_medium = m->present;
    if (!m->present) return;
    uint8_t rx = (uint8_t)m->res[0], ry = (uint8_t)m->res[1], rz = (uint8_t)m->res[2];
    float sigma_maj = m->sigma_a + m->sigma_s;
    float mx = ((float)rx - 1.f) / 1.f, my = ((float)ry - 1.f) / 1.f, mz = ((float)rz - 1.f) / 1.f;
    uint8_t x1 = u8min((uint8_t)f2u32(ceilf(mx)), rx);
    uint8_t y1 = u8min((uint8_t)f2u32(ceilf(my)), ry);
    uint8_t z1 = u8min((uint8_t)f2u32(ceilf(mz)), rz);
    float majorant = 0.f;
    for (uint8_t k = 0; k < z1; ++k)
        for (uint8_t j = 0; j < y1; ++j)
            for (uint8_t i = 0; i < x1; ++i) majorant = gmax(majorant, dg_at(m, i, j, k));
    for (int c = 0; c < 8; ++c) {
        float px = (c & 4) ? 1.f : 0.f, py = (c & 2) ? 1.f : 0.f, pz = (c & 1) ? 1.f : 0.f;
        majorant = gmax(majorant, dg_lookup(m, V3(px, py, pz)));
    }
    s->maj[0] = majorant * sigma_maj;
    s->maj[1] = sigma_maj;
    s->maj[2] = m->bounds_min[0]; s->maj[3] = m->bounds_min[1]; s->maj[4] = m->bounds_min[2];
    s->maj[5] = m->bounds_max[0]; s->maj[6] = m->bounds_max[1]; s->maj[7] = m->bounds_max[2];
}

typedef struct { /* RayMajorantIterator (media.cpp:138-255), width-1 majorant grid */
    float tCurrent, tMax;
    uint32_t currentIndex;
    v3 nextCrossing, crossDistance;
    int stepAxis[3];
} maj_iter_t;

static int medium_sample_ray(const oracle_scene* s, v3 o, v3 d, maj_iter_t* it) { /* media.cpp:281-324 */
    const nart_medium* m = &s->blob->medium;
    float tMin = -INF_F, tMax = INF_F;
    for (int i = 0; i < 3; ++i) {
        v3 n = V3(i == 0 ? 1.f : 0.f, i == 1 ? 1.f : 0.f, i == 2 ? 1.f : 0.f);
        float slabMin = (m->bounds_min[i] - dot3(o, n)) / dot3(d, n);
        float slabMax = (m->bounds_max[i] - dot3(o, n)) / dot3(d, n);
        if (slabMin > slabMax) { float t = slabMin; slabMin = slabMax; slabMax = t; }
        if (slabMin > tMax || tMin > slabMax) return 0;
        tMin = gmax(tMin, slabMin);
        tMax = gmin(tMax, slabMax);
    }
    v3 bmin = V3(m->bounds_min[0], m->bounds_min[1], m->bounds_min[2]);
    v3 bmax = V3(m->bounds_max[0], m->bounds_max[1], m->bounds_max[2]);
    it->tMax = tMax;
    it->tCurrent = gmax(0.f, tMin);
    v3 pE = add3(o, muls3(d, it->tCurrent));
    v3 pX = add3(o, muls3(d, tMax));
    v3 bs = sub3(bmax, bmin);
    pE = div3(sub3(pE, bmin), bs);
    pE = V3(gmax(gmin(pE.x, 0.999999f), 0.f), gmax(gmin(pE.y, 0.999999f), 0.f), gmax(gmin(pE.z, 0.999999f), 0.f));
    pE = muls3(pE, 1.f);
    it->currentIndex = 0; /* ivec3(pEntering) is 0 in a width-1 grid */
    pX = div3(sub3(pX, bmin), bs);
    pX = V3(gmax(gmin(pX.x, 0.999999f), 0.f), gmax(gmin(pX.y, 0.999999f), 0.f), gmax(gmin(pX.z, 0.999999f), 0.f));
    pX = muls3(pX, 1.f);
    v3 gD = normalize3(sub3(pX, pE));
    if (pX.x == pE.x && pX.y == pE.y && pX.z == pE.z) gD = V3(1.f, 0.f, 0.f);
    v3 cd = V3(gabs(((1.f / gD.x) * 1.f) * bs.x), gabs(((1.f / gD.y) * 1.f) * bs.y), gabs(((1.f / gD.z) * 1.f) * bs.z));
    if (gD.x == 0.f) cd.x = INF_F;
    if (gD.y == 0.f) cd.y = INF_F;
    if (gD.z == 0.f) cd.z = INF_F;
    it->crossDistance = cd;
    float t3[3];
    for (int i = 0; i < 3; ++i) {
        float pe = v3get(pE, i), g = v3get(gD, i);
        if (v3get(d, i) >= 0.f) t3[i] = gabs((ceilf(pe + 0.00001f) - pe) / g);
        else t3[i] = gabs((floorf(pe - 0.00001f) - pe) / g);
        if (g == 0.f) t3[i] = INF_F;
    }
    it->nextCrossing = muls3(mul3(V3(t3[0], t3[1], t3[2]), bs), 1.f);
    it->stepAxis[0] = gD.x < 0.f ? -1 : 1;
    it->stepAxis[1] = gD.y < 0.f ? -1 : 1;
    it->stepAxis[2] = gD.z < 0.f ? -1 : 1;
    return 1;
}
static int maj_next(const oracle_scene* s, maj_iter_t* it, float* sigma, float* t0, float* t1) {
    if (it->tCurrent + 0.0001f > it->tMax) return 0;
    static const uint8_t choiceMap[8] = {2, 1, 0, 1, 2, 0, 0, 0};
    uint8_t choice = 0;
    if (it->nextCrossing.x < it->nextCrossing.y) choice += 4;
    if (it->nextCrossing.x < it->nextCrossing.z) choice += 2;
    if (it->nextCrossing.y < it->nextCrossing.z) choice += 1;
    int index = choiceMap[choice];
    float dt = v3get(it->nextCrossing, index);
    if (it->currentIndex > 7) return 0; /* beyond the Medium object: undefined in the reference */
    *sigma = s->maj[it->currentIndex];
    *t0 = it->tCurrent;
    *t1 = it->tCurrent + dt;
    it->nextCrossing = sub3(it->nextCrossing, V3(dt, dt, dt));
    if (index == 0) it->nextCrossing.x = it->crossDistance.x;
    else if (index == 1) it->nextCrossing.y = it->crossDistance.y;
    else it->nextCrossing.z = it->crossDistance.z;
    it->currentIndex += (uint32_t)(it->stepAxis[index] > 0 ? 1 : 0);
    it->tCurrent += dt;
    return 1;
}

/* VolumeIntegrator::Li_alpha (volumeintegrator.cpp:3-84) with SampleT_maj (media.h:128-181) */
static v4 li_volume(const oracle_scene* s, rng_t* rng, ray_t ray, const nart_render_params* p) {
    const nart_medium* m = &s->blob->medium;
    v3 L = V3(0.f, 0.f, 0.f), beta = V3(1.f, 1.f, 1.f);
    uint32_t bounce = 0;
    for (;;) {
        int scattered = 0, terminated = 0;
        (void)rng_float(rng); /* u: passed to SampleT_maj, unused there */
        float uMode = rng_float(rng);
        maj_iter_t it;
        if (s->has_medium && medium_sample_ray(s, ray.o, ray.d, &it)) {
            const v3 o = ray.o, d = ray.d; /* SampleT_maj's copy of the ray */
            int done = 0;
            while (!done) {
                float sigma, t0, t1;
                if (!maj_next(s, &it, &sigma, &t0, &t1)) break;
                float tMin = t0;
                for (;;) {
                    float t = tMin + (-logf(1.f - rng_float(rng)) / sigma);
                    if (t < t1) {
                        v3 pp = add3(o, muls3(d, t));
                        if (pp.x < m->bounds_min[0] || pp.y < m->bounds_min[1] || pp.z < m->bounds_min[2] ||
                            pp.x > m->bounds_max[0] || pp.y > m->bounds_max[1] || pp.z > m->bounds_max[2]) {
                            done = 1;
                            break;
                        }
                        v3 q = div3(sub3(pp, V3(m->bounds_min[0], m->bounds_min[1], m->bounds_min[2])),
                                    sub3(V3(m->bounds_max[0], m->bounds_max[1], m->bounds_max[2]),
                                         V3(m->bounds_min[0], m->bounds_min[1], m->bounds_min[2])));
                        float density = dg_lookup(m, q);
                        float sa = m->sigma_a * density, ss = m->sigma_s * density;
                        v3 mLe = muls3(V3(m->Le[0], m->Le[1], m->Le[2]), density);
                        float pAbsorb = sa / sigma;
                        float pScatter = ss / sigma;
                        if (uMode < pAbsorb) {
                            terminated = 1;
                            L = add3(L, mul3(mLe, beta));
                            done = 1;
                            break;
                        } else if (uMode < pAbsorb + pScatter) {
                            if (bounce++ > p->bounces) {
                                terminated = 1;
                                done = 1;
                                break;
                            }
                            float a = rng_float(rng);
                            float b = rng_float(rng);
                            ray.o = pp;
                            ray.d = uniform_sample_sphere(V2(a, b));
                            scattered = 1;
                            done = 1;
                            break;
                        } else {
                            uMode = rng_float(rng);
                        }
                        tMin = t; /* null collision: continue from here (T_maj only feeds the unused callback argument) */
                    } else {
                        break;
                    }
                }
            }
        }
        if (terminated) break;
        if (scattered) continue;
        float lightTMax = INF_F;
        v3 Le = V3(0.f, 0.f, 0.f);
        for (uint8_t j = 0; j < s->blob->num_lights; ++j) {
            lisect_t li;
            li.tMax = INF_F;
            v3 Li = light_li(s, j, &li, ray.o, ray.d, NULL);
            if (li.tMax < lightTMax) {
                Le = Li;
                lightTMax = li.tMax;
            }
        }
        L = add3(L, mul3(Le, beta));
        break;
    }
    return V4(L.x, L.y, L.z, 1.f);
}

/* ---------------------------------------------------------------- camera */
static ray_t cast_ray(const oracle_scene* s, v2 smp, uint32_t W, uint32_t H, uint32_t x, uint32_t y) { /* pinholecamera.cpp:9-40 */
    const nart_camera* c = &s->blob->camera;
    float aspect = (float)W / (float)H;
    float tanv = tanf(c->fov * (float)0.01745329251994329576923690768489);
    float px = ((((float)x + smp.x) / (float)W) * 2.f - 1.f) * tanv * aspect;
    float py = ((((float)y + smp.y) / (float)H) * -2.f + 1.f) * tanv;
    v4 o = V4(0.f, 0.f, 0.f, 1.f);
    v4 d = normalize4(V4(px, py, -1.f, 0.f));
    o = vec_mul_mat(o, c->m);
    d = vec_mul_mat(d, c->m);
    return make_ray(xyz(o), xyz(d));
}

/* ---------------------------------------------------------------- render session */
typedef struct {
    uint32_t fb, tileSize, totalW, totalH, nbx, nby;
    float table[64];
} sess_t;

static void session_of(const nart_render_params* p, sess_t* ss) { /* render.cpp:14-21, 117-130 */
    ss->fb = f2u32(ceilf(p->filter_width));
    ss->tileSize = p->bucket_size + ss->fb * 2;
    ss->totalW = p->image_width + ss->fb * 2;
    ss->totalH = p->image_height + ss->fb * 2;
    ss->nbx = f2u32(ceilf((float)p->image_width / (float)p->bucket_size));
    ss->nby = f2u32(ceilf((float)p->image_height / (float)p->bucket_size));
    for (uint8_t i = 0; i < 64; ++i) { /* Gaussian(63, i) (render.h:23-32) */
        float width = 63.f, x = (float)i;
        if (x >= width) { ss->table[i] = 0.f; continue; }
        float sigma = width / 3.f;
        ss->table[i] = (1.f / sqrtf(2.f * PI_F * sigma * sigma)) * expf(-(x * x) / (2.f * sigma * sigma));
    }
}

/* AddSample (render.cpp:23-70) */
static void add_sample(const sess_t* ss, const nart_render_params* p, v2 sc, v4 L, nart_pixel* px) {
    float fw = p->filter_width;
    uint32_t x0 = f2u32(floorf(sc.x - fw)), x1 = f2u32(ceilf(sc.x + fw));
    uint32_t y0 = f2u32(floorf(sc.y - fw)), y1 = f2u32(ceilf(sc.y + fw));
    for (uint32_t y = y0; y < y1; ++y) {
        for (uint32_t x = x0; x < x1; ++x) {
            float distX = ((float)x + 0.5f) - sc.x;
            float distY = ((float)y + 0.5f) - sc.y;
            float dist = sqrtf(distX * distX + distY * distY);
            uint8_t fi = f2u8((dist / fw) * 64);
            fi = ((uint8_t)63 < fi) ? (uint8_t)63 : fi;
            float wgt = ss->table[fi];
            uint32_t tileX = f2u32(floorf(distX + gmod(sc.x - (float)ss->fb, (float)p->bucket_size) + (float)ss->fb));
            uint32_t tileY = f2u32(floorf(distY + gmod(sc.y - (float)ss->fb, (float)p->bucket_size) + (float)ss->fb));
            uint32_t ti = (tileY * ss->tileSize) + tileX;
            px[ti].contribution[0] += L.x * wgt;
            px[ti].contribution[1] += L.y * wgt;
            px[ti].contribution[2] += L.z * wgt;
            px[ti].contribution[3] += L.w * wgt;
            px[ti].filter_weight_sum += wgt;
        }
    }
}

/* RenderTile (render.cpp:72-112) */
static void render_tile(const oracle_scene* s, worker_t* w, const nart_render_params* p, const sess_t* ss, uint32_t bx,
                        uint32_t by, nart_pixel* tile, v2* smp) {
    memset(tile, 0, sizeof(nart_pixel) * ss->tileSize * ss->tileSize);
    uint32_t x0 = p->bucket_size * bx, y0 = p->bucket_size * by;
    uint32_t x1 = p->bucket_size * (bx + 1), y1 = p->bucket_size * (by + 1);
    if (ss->totalW < x1) x1 = ss->totalW;
    if (ss->totalH < y1) y1 = ss->totalH;
    for (uint32_t y = y0; y < y1; ++y) {
        for (uint32_t x = x0; x < x1; ++x) {
            rng_t rng;
            rng_seed(&rng, y * ss->totalW + x);
            latin_square(&rng, p->spp, smp);
            for (uint32_t i = 0; i < p->spp; ++i) {
                ray_t ray = cast_ray(s, smp[i], p->image_width, p->image_height, x, y);
                v4 L = p->integrator == NART_INTEGRATOR_VOLUME ? li_volume(s, &rng, ray, p) : li_alpha(s, w, &rng, ray, p);
                v2 sc = V2((float)(x + ss->fb) + smp[i].x, (float)(y + ss->fb) + smp[i].y);
                add_sample(ss, p, sc, L, tile);
            }
        }
    }
}

typedef struct {
    const oracle_scene* s;
    const nart_render_params* p;
    const sess_t* ss;
    const uint32_t* ids;
    uint32_t n;
    nart_pixel* tiles;
    atomic_uint next;
} job_t;

static void* worker_main(void* arg) {
    job_t* j = (job_t*)arg;
    worker_t w;
    memset(&w, 0, sizeof(w));
    v2* smp = (v2*)malloc(sizeof(v2) * (j->p->spp ? j->p->spp : 1));
    size_t tpx = (size_t)j->ss->tileSize * j->ss->tileSize;
    for (;;) {
        uint32_t k = atomic_fetch_add(&j->next, 1u);
        if (k >= j->n) break;
        uint32_t id = j->ids[k];
        render_tile(j->s, &w, j->p, j->ss, id % j->ss->nbx, id / j->ss->nbx, j->tiles + tpx * k, smp);
    }
    free(smp);
    free(w.heap.e);
    return NULL;
}

static int check_params(const oracle_scene* s, const nart_render_params* p) {
    if (!p->image_width || !p->image_height || !p->bucket_size || !p->spp) return NART_E_INVALID;
    if (p->filter_width <= 0.f) return NART_E_INVALID;
    if (p->integrator == NART_INTEGRATOR_VOLUME && s->has_medium && (s->blob->medium.res[0] % 256 < 2 || s->blob->medium.res[1] % 256 < 2 || s->blob->medium.res[2] % 256 < 2))
        return NART_E_UNSUPPORTED; /* DensityGrid::LookUp reads past the grid below 2 points per axis */
    if (p->bounces > 64) return NART_E_UNSUPPORTED;
    if (s->blob->num_lights == 0) return NART_E_INVALID; /* reference throws in GetLight */
    return NART_OK;
}

int oracle_render_buckets(oracle_scene* s, const nart_render_params* p, const uint32_t* ids, uint32_t n,
                          nart_pixel* tiles, int threads) {
    int rc = check_params(s, p);
    if (rc) return rc;
    sess_t ss;
    session_of(p, &ss);
    job_t j;
    j.s = s;
    j.p = p;
    j.ss = &ss;
    j.ids = ids;
    j.n = n;
    j.tiles = tiles;
    atomic_init(&j.next, 0u);
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, worker_main, &j);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(th);
    return NART_OK;
}

int oracle_render(oracle_scene* s, const nart_render_params* p, nart_pixel* image, int threads) {
    int rc = check_params(s, p);
    if (rc) return rc;
    sess_t ss;
    session_of(p, &ss);
    uint32_t nb = ss.nbx * ss.nby;
    size_t tpx = (size_t)ss.tileSize * ss.tileSize;
    nart_pixel* tiles = (nart_pixel*)malloc(sizeof(nart_pixel) * tpx * nb);
    uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * nb);
    if (!tiles || !ids) { free(tiles); free(ids); return NART_E_OOM; }
    for (uint32_t i = 0; i < nb; ++i) ids[i] = i;
    rc = oracle_render_buckets(s, p, ids, nb, tiles, threads);
    if (!rc) {
        /* combine in bucket raster order (render.cpp:183-203) */
        memset(image, 0, sizeof(nart_pixel) * ss.totalW * ss.totalH);
        for (uint32_t j = 0; j < ss.nby; ++j)
            for (uint32_t i = 0; i < ss.nbx; ++i) {
                const nart_pixel* v = tiles + tpx * (j * ss.nbx + i);
                for (uint32_t y = 0; y < ss.tileSize; ++y)
                    for (uint32_t x = 0; x < ss.tileSize; ++x) {
                        uint32_t pX = x + i * p->bucket_size, pY = y + j * p->bucket_size;
                        if (pX < p->image_width + ss.fb && pY < p->image_height + ss.fb) {
                            nart_pixel* d = &image[pY * ss.totalW + pX];
                            const nart_pixel* q = &v[y * ss.tileSize + x];
                            for (int c = 0; c < 4; ++c) d->contribution[c] += q->contribution[c];
                            d->filter_weight_sum += q->filter_weight_sum;
                        }
                    }
            }
    }
    free(tiles);
    free(ids);
    return rc;
}

int oracle_render_samples(oracle_scene* s, const nart_render_params* p, uint32_t x0, uint32_t y0, uint32_t w,
                          uint32_t h, float* out, float* uv) {
    int rc = check_params(s, p);
    if (rc) return rc;
    sess_t ss;
    session_of(p, &ss);
    worker_t wk;
    memset(&wk, 0, sizeof(wk));
    v2* smp = (v2*)malloc(sizeof(v2) * p->spp);
    for (uint32_t y = y0; y < y0 + h; ++y)
        for (uint32_t x = x0; x < x0 + w; ++x) {
            rng_t rng;
            rng_seed(&rng, y * ss.totalW + x);
            latin_square(&rng, p->spp, smp);
            size_t base = ((size_t)(y - y0) * w + (x - x0)) * p->spp;
            for (uint32_t i = 0; i < p->spp; ++i) {
                ray_t ray = cast_ray(s, smp[i], p->image_width, p->image_height, x, y);
                v4 L = p->integrator == NART_INTEGRATOR_VOLUME ? li_volume(s, &rng, ray, p) : li_alpha(s, &wk, &rng, ray, p);
                float* o = out + (base + i) * 4;
                o[0] = L.x; o[1] = L.y; o[2] = L.z; o[3] = L.w;
                if (uv) { uv[(base + i) * 2] = smp[i].x; uv[(base + i) * 2 + 1] = smp[i].y; }
            }
        }
    free(smp);
    free(wk.heap.e);
    return NART_OK;
}

/* ---------------------------------------------------------------- create / destroy */
static void build_env(oracle_scene* s) { /* Piecewise2DDistribution ctor (texturepattern.cpp:3-70) */
    const nart_scene_blob* b = s->blob;
    s->env = (struct pw2d*)calloc(b->num_lights ? b->num_lights : 1, sizeof(struct pw2d));
    s->nenv = s->env ? b->num_lights : 0;
    for (uint32_t l = 0; l < b->num_lights; ++l) {
        const nart_light* L = &b->lights[l];
        if (L->Le.type != NART_PTN_TEXTURE) continue;
        struct pw2d* d = &s->env[l];
        const nart_texture* t = &b->textures[L->Le.texture];
        const float* px = &s->tex_f[s->tex_off[L->Le.texture]];
        uint32_t W = t->width, H = t->height;
        d->present = 1;
        d->w = W;
        d->h = H;
        d->invW = 1.f / (float)W;
        d->invH = 1.f / (float)H;
        d->mpdf = (float*)calloc(H, sizeof(float));
        d->cpdf = (float*)calloc((size_t)W * H, sizeof(float));
        d->mcdf = (float*)calloc(H + 1, sizeof(float));
        d->ccdf = (float*)calloc((size_t)W * H + H, sizeof(float));
        float fInt = 0.f;
        for (uint32_t j = 0; j < H; ++j) {
            d->mpdf[j] = 0.f;
            for (uint32_t i = 0; i < W; ++i) {
                const float* q = &px[((size_t)(H - j - 1) * W + i) * 3];
                d->mpdf[j] += fabsf(q[0]) + fabsf(q[1]) + fabsf(q[2]);
            }
            d->mpdf[j] *= d->invW;
            fInt += d->mpdf[j];
        }
        fInt *= d->invH;
        for (uint32_t j = 0; j < H; ++j) {
            if (d->mpdf[j] != 0.f) {
                for (uint32_t i = 0; i < W; ++i) {
                    const float* q = &px[((size_t)(H - j - 1) * W + i) * 3];
                    d->cpdf[j * W + i] = fabsf(q[0]) + fabsf(q[1]) + fabsf(q[2]);
                    d->cpdf[j * W + i] /= d->mpdf[j];
                }
            } else {
                for (uint32_t i = 0; i < W; ++i) d->cpdf[j * W + i] = 1.f;
            }
        }
        float invFInt = 1.f / fInt;
        for (uint32_t j = 0; j < H; ++j) d->mpdf[j] *= invFInt;
        d->mcdf[0] = 0.f;
        d->mcdf[H] = 1.f;
        for (uint32_t i = 1; i < H; ++i) d->mcdf[i] = d->mcdf[i - 1] + (d->mpdf[i - 1] * d->invH);
        for (uint32_t i = 0; i < H; ++i) {
            d->ccdf[i * (W + 1)] = 0.f;
            d->ccdf[i * (W + 1) + W] = 1.f;
        }
        for (uint32_t j = 0; j < H; ++j)
            for (uint32_t i = 1; i < W; ++i)
                d->ccdf[j * (W + 1) + i] = d->ccdf[j * (W + 1) + i - 1] + (d->cpdf[j * W + i - 1] * d->invW);
    }
}

static float half_to_float(uint16_t h) {
    uint32_t hexpmant = ((uint32_t)h << 17) >> 4;
    uint32_t v = ((uint32_t)h >> 15) << 31;
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
    memcpy(&f, &v, 4);
    return f;
}

int oracle_create(const nart_scene_blob* blob, oracle_scene** out) {
    if (!blob || !out) return NART_E_INVALID;
    oracle_scene* s = (oracle_scene*)calloc(1, sizeof(oracle_scene));
    if (!s) return NART_E_OOM;
    s->blob = blob;
    s->tri_mesh = (uint32_t*)malloc(sizeof(uint32_t) * (blob->num_triangles ? blob->num_triangles : 1));
    for (uint32_t m = 0; m < blob->num_meshes; ++m)
        for (uint32_t i = 0; i < blob->meshes[m].num_tris; ++i) s->tri_mesh[blob->meshes[m].first_tri + i] = m;
    size_t total = 0;
    s->tex_off = (size_t*)calloc(blob->num_textures + 1, sizeof(size_t));
    for (uint32_t t = 0; t < blob->num_textures; ++t) {
        s->tex_off[t] = total;
        total += (size_t)blob->textures[t].width * blob->textures[t].height * 3;
    }
    s->tex_f = (float*)malloc(sizeof(float) * (total ? total : 1));
    for (uint32_t t = 0; t < blob->num_textures; ++t) {
        const nart_texture* tx = &blob->textures[t];
        for (size_t i = 0; i < (size_t)tx->width * tx->height; ++i)
            for (int c = 0; c < 3; ++c) s->tex_f[s->tex_off[t] + i * 3 + c] = half_to_float(tx->rgba[i * 4 + c]);
    }
    build_bvh(s);
    build_env(s);
    build_medium(s);
    *out = s;
    return NART_OK;
}

void oracle_destroy(oracle_scene* s) {
    if (!s) return;
    for (uint32_t c = 0; c < s->nchunks_total; ++c) free(s->chunks[c].tris);
    free(s->chunks);
    for (uint32_t n = 0; n < s->nnodes; ++n) free(s->nodes[n].chunks);
    free(s->nodes);
    free(s->tri_mesh);
    free(s->tex_f);
    free(s->tex_off);
    if (s->env) {
        for (uint32_t l = 0; l < s->nenv; ++l) {
            free(s->env[l].mpdf);
            free(s->env[l].cpdf);
            free(s->env[l].mcdf);
            free(s->env[l].ccdf);
        }
        free(s->env);
    }
    free(s);
}

int oracle_bvh_stats(const oracle_scene* s, uint32_t* n_chunks, uint32_t* max_chunk_tris, uint32_t* root_is_leaf,
                     uint32_t* grid_res) {
    uint32_t nc = 0, mx = 0;
    for (uint32_t c = 0; c < s->nchunks_total; ++c)
        if (s->chunks[c].n) {
            ++nc;
            if (s->chunks[c].n > mx) mx = s->chunks[c].n;
        }
    /* triangles reachable by traversal: chunks held by leaves (a leaf that splits while
       holding several chunks re-inserts only one of them, bvh.cpp:187-190) */
    uint32_t reach = 0;
    for (uint32_t n = 0; n < s->nnodes; ++n)
        if (s->nodes[n].isLeaf)
            for (uint32_t k = 0; k < s->nodes[n].nchunks; ++k) reach += s->chunks[s->nodes[n].chunks[k]].n;
    if (s->nodes[s->root].isLeaf) reach = 0; /* root leaf: children never exist (bvh.cpp:131) */
    *n_chunks = nc;
    *max_chunk_tris = mx;
    grid_res[3] = reach;
    *root_is_leaf = (uint32_t)s->nodes[s->root].isLeaf;
    for (int i = 0; i < 3; ++i) grid_res[i] = s->grid_res[i];
    return NART_OK;
}

void oracle_rng_stream(uint32_t seed, uint32_t n, float* out) {
    rng_t r;
    rng_seed(&r, seed);
    for (uint32_t i = 0; i < n; ++i) out[i] = rng_float(&r);
}

void oracle_latin_square(uint32_t seed, uint32_t spp, float* out_xy, uint32_t* state_after) {
    rng_t r;
    rng_seed(&r, seed);
    latin_square(&r, spp, (v2*)out_xy);
    if (state_after) *state_after = r.y;
}

float oracle_fresnel(float eta_o, float eta_i, float c) { return fresnel(eta_o, eta_i, c); }
uint32_t oracle_binary_search(float value, const float* v, uint32_t start, uint32_t end) {
    return binary_search(value, v, start, end);
}

/* ---------------------------------------------------------------- debugging aids (tests/tools only) */
/* Camera ray of pixel (x, y) with image sample (u, v) (pinholecamera.cpp:9-40). */
void oracle_camera_ray(const oracle_scene* s, uint32_t W, uint32_t H, uint32_t x, uint32_t y, float u, float v,
                       float* o, float* d) {
    ray_t r = cast_ray(s, V2(u, v), W, H, x, y);
    o[0] = r.o.x; o[1] = r.o.y; o[2] = r.o.z;
    d[0] = r.d.x; d[1] = r.d.y; d[2] = r.d.z;
}
/* Closest hit of one ray: the reference octree (out[0] = triangle or -1, out[1] = t bits) and a
   brute-force pass over every triangle with Triangle::Intersect, keeping the strictly closest
   (out[2], out[3]).  tmax presets Intersection::tMax as the light loop does. */
void oracle_trace(const oracle_scene* s, const float* o, const float* d, float tmax, int32_t* out) {
    ray_t r = make_ray(V3(o[0], o[1], o[2]), V3(d[0], d[1], d[2]));
    heap_t q = {0, 0, 0};
    isect_t is;
    isect_init(&is);
    is.tMax = tmax;
    int32_t best = -1;
    if (bvh_intersect(s, &r, &is, &q)) {
        /* find which triangle produced is.tMax */
        for (uint32_t g = 0; g < s->blob->num_triangles; ++g) {
            isect_t t1;
            isect_init(&t1);
            if (triangle_intersect(&s->blob->triangles[g], &r, &t1) && memcmp(&t1.tMax, &is.tMax, 4) == 0) {
                best = (int32_t)g;
                break;
            }
        }
    }
    free(q.e);
    out[0] = best;
    memcpy(&out[1], &is.tMax, 4);
    isect_t bf;
    isect_init(&bf);
    bf.tMax = tmax;
    int32_t bg = -1;
    for (uint32_t g = 0; g < s->blob->num_triangles; ++g) {
        isect_t t1;
        isect_init(&t1);
        t1.tMax = bf.tMax;
        if (triangle_intersect(&s->blob->triangles[g], &r, &t1)) {
            bf.tMax = t1.tMax;
            bg = (int32_t)g;
        }
    }
    out[2] = bg;
    memcpy(&out[3], &bf.tMax, 4);
}
