// Device path integrator for nart (gfx950).  Mirrors, function by function and operation by
// operation, src/integrators/pathintegrator.cpp, src/core/{geometry,bxdf}.cpp,
// src/bxdfs/*, src/materials/*, src/lights/{disk,ring,environment}light.cpp,
// src/patterns/*, src/cameras/pinholecamera.cpp.  Only the acceleration structure differs:
// the reference's octree of triangle chunks (bvh.cpp) is replaced by a binned-SAH BVH2 that
// returns the same closest hit (ties broken by scene order).
#pragma once

#include "dmath.h"
#include "dscene.h"

namespace nd {

enum { F_SPECULAR = 1, F_GLOSSY = 2, F_DIFFUSE = 4, F_TRANSMISSIVE = 8 };
#define SHADOW_BIAS 0.001f

// Scene feature mask (template parameter FM of the shading functions and k_render_rq): the
// material, light and pattern kinds a scene holds (scene_features, render.hip).  A kernel built
// for a mask compiles only those kinds' code -- no plastic lobes, ring lights, texture fetches or
// normal-map frames in glassSphere's build -- and serves every scene whose mask it covers; FT_ALL
// is the generic build.  Each kind's operations are unchanged, so every build renders the same bits.
enum : uint32_t {
    FT_LAMBERT = 1u << 0,   // diffusematerial.cpp
    FT_SPECMAT = 1u << 1,   // specularmaterial.cpp
    FT_GLASS = 1u << 2,     // glassmaterial.cpp
    FT_GLOSSY = 1u << 3,    // glossydielectricmaterial.cpp
    FT_PLASTIC = 1u << 4,   // plasticmaterial.cpp (the only two-lobe BSDF)
    FT_DISK = 1u << 5,      // disklight.cpp
    FT_RING = 1u << 6,      // ringlight.cpp
    FT_ENV = 1u << 7,       // environmentlight.cpp
    FT_TEX = 1u << 8,       // any TexturePattern (materials or light Le)
    FT_NMAP = 1u << 9,      // any material with a normal map
    FT_ALL = (1u << 10) - 1u
};
// BxDF kinds a mask can create (the roughening factor moves a material between its two kinds)
NHD constexpr bool ft_lambert(uint32_t FM) { return (FM & (FT_LAMBERT | FT_PLASTIC)) != 0u; }
NHD constexpr bool ft_ts(uint32_t FM) { return (FM & (FT_SPECMAT | FT_GLOSSY | FT_PLASTIC)) != 0u; }
NHD constexpr bool ft_spec(uint32_t FM) { return ft_ts(FM); }
NHD constexpr bool ft_diel(uint32_t FM) { return (FM & FT_GLASS) != 0u; }
#define NO_HIT 0xFFFFFFFFu

// ---------------------------------------------------------------- Ray (geometry.cpp:3-15)
struct Ray {
    f3 o, d;
    int major;
    float Sx, Sy, Sz;
};
ND Ray make_ray(f3 o, f3 d) {
    Ray r;
    r.o = o;
    r.d = d;
    f3 a = F3(gabs(d.x), gabs(d.y), gabs(d.z));
    r.major = (a.x > a.y) ? ((a.x > a.z) ? 0 : 2) : ((a.y > a.z) ? 1 : 2);
    int m0 = r.major + 1;
    if (m0 == 3) m0 = 0;
    int m1 = r.major + 2;
    if (m1 >= 3) m1 -= 3;
    r.Sz = 1.f / comp(d, r.major);
    r.Sx = -comp(d, m0) * r.Sz;
    r.Sy = -comp(d, m1) * r.Sz;
    return r;
}
// (p[m0], p[m1], p[major]) permutation of Triangle::Intersect (geometry.cpp:48-56)
ND f3 permute(f3 p, int major) {  // selects, not branches: major differs across lanes
    const bool m0 = major == 0, m1 = major == 1;
    return F3(m0 ? p.y : (m1 ? p.z : p.x), m0 ? p.z : (m1 ? p.x : p.y), m0 ? p.x : (m1 ? p.y : p.z));
}

// Sheared-space edge functions (geometry.cpp:42-75)
ND void edge_functions(const Ray& r, f3 v0, f3 v1, f3 v2, float& e0, float& e1, float& e2) {
    f3 p0 = permute(sub(v0, r.o), r.major);
    f3 p1 = permute(sub(v1, r.o), r.major);
    f3 p2 = permute(sub(v2, r.o), r.major);
    p0.x += p0.z * r.Sx;
    p0.y += p0.z * r.Sy;
    p1.x += p1.z * r.Sx;
    p1.y += p1.z * r.Sy;
    p2.x += p2.z * r.Sx;
    p2.y += p2.z * r.Sy;
    e0 = (p1.x * p2.y) - (p1.y * p2.x);
    e1 = (p2.x * p0.y) - (p2.y * p0.x);
    e2 = (p0.x * p1.y) - (p0.y * p1.x);
}
ND bool edges_accept(float e0, float e1, float e2) {  // geometry.cpp:78-81
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return false;
    if (gabs(e0) + gabs(e1) + gabs(e2) == 0.f) return false;
    return true;
}

// ---------------------------------------------------------------- BVH traversal
struct TraceCounters {
    uint32_t nodes, tris;
    uint32_t oc_checks, oc_replays;  // octree.h: exact ancestor checks, octree replays
};

// Closest hit (ANY=false): minimum (t, scene index) over triangles with 0 < t < tmax whose
// sheared edge test passes -- the set Octree::Intersect selects from (bvh.cpp:132-176).
// Any hit (ANY=true): shadow query, true iff such a triangle exists.
// The stack lives in LDS: sc/st point at this lane's column, stride = lanes per block.
// lnodes / nl: the first nl nodes (breadth-first order: the top of the tree) staged in LDS.
//
// The traversal is resumable (Trav + trav_step); kernels that refill finished lanes with new rays
// between steps keep more lanes of a wave busy than a loop that runs each ray to completion.
struct Trav {
    f3 inv, oi;        // slab-test reciprocals and -o * inv
    float tmax, bestT;
    float cullT;       // boxes entered beyond cullT are skipped (oc_cull(bestT); tmax for any-hit)
    float t2;          // closest accepted hit other than the winner (or tmax)
    uint32_t bestG;
    uint32_t bestInfo; // tri_isect word 14 of the winner: octree leaf | inside-leaf bit
    int code, sp;
    bool any, risky;   // risky: a NaN plane distance or an exact tie with the winner was seen
};

// Closest-hit culling distance.  Boxes are kept up to a little beyond the best hit so that every
// hit within oc_cull(t*) of the winner is tested: then min(t2, oc_cull(t*)) bounds every other
// hit from below, which octree.h needs (oc_resolve).  Monotone in b, so a box culled when the
// best was b >= t* holds no hit below oc_cull(t*).
ND float oc_cull(const DScene& S, float b) { return b + (b * 0x1p-12f + S.oc_scale * 0x1p-20f); }

// Box tests need not be exact (boxes are padded on the host), so use fast reciprocals.  They are
// clamped to +-1e20: for a zero direction component 1/d = inf would make fma(lo, inv, -o * inv) =
// inf - inf = NaN and reject a box the ray runs inside (a camera ray of the C3 frame has d.z == 0
// exactly).  With the clamp the slab distances keep their signs and stay far beyond any scene
// distance unless the origin lies within float rounding of a padded face -- where the box holds no
// triangle the ray can reach.
ND void trav_slab(const Ray& r, Trav& t) {
    const float BIG = 1e20f;
    t.inv = F3(fminf(fmaxf(__builtin_amdgcn_rcpf(r.d.x), -BIG), BIG),
               fminf(fmaxf(__builtin_amdgcn_rcpf(r.d.y), -BIG), BIG),
               fminf(fmaxf(__builtin_amdgcn_rcpf(r.d.z), -BIG), BIG));
    t.oi = F3(-r.o.x * t.inv.x, -r.o.y * t.inv.y, -r.o.z * t.inv.z);
}
ND void trav_begin(const DScene& S, const Ray& r, float tmax, bool ANY, Trav& t) {
    trav_slab(r, t);
    t.tmax = tmax;
    t.bestT = tmax;
    t.cullT = ANY ? tmax : oc_cull(S, tmax);
    t.t2 = tmax;
    t.bestG = NO_HIT;
    t.bestInfo = 0u;
    t.code = S.root;
    t.sp = 0;
    t.any = ANY;
    t.risky = false;
}

// Traversal stack entry: one 8-B LDS word (node code, entry distance), so a pop is one
// ds_read_b64 (sc points at this lane's int2 column, laid out [depth][lane]).  C3 at 64 spp:
// 134.3 -> 133.9 ms vs two 4-B arrays.
// SHORT (the lean ray-queue build, kernels.h WV = 3): only entries [0, sk) live in LDS; deeper
// ones go to the lane's own global column gs[sp - sk] (rare: the LDS of a 768-lane block holds
// too few levels for the deeper BVHs).  The same entries in the same order either way.
template <bool SHORT = false>
ND void stk_push(int* sc, int2* gs, int stride, int sp, int code, float tn, int sk = 0) {
    const int2 v = make_int2(code, __float_as_int(tn));
    if (!SHORT || sp < sk) reinterpret_cast<int2*>(sc)[sp * stride] = v;
    else gs[sp - sk] = v;
}
template <bool SHORT = false>
ND int2 stk_read(const int* sc, const int2* gs, int stride, int sp, int sk) {
    if (!SHORT || sp < sk) return reinterpret_cast<const int2*>(sc)[sp * stride];
    return gs[sp - sk];
}

// pop the next subtree that can still contain a closer hit
template <bool SHORT = false>
ND bool trav_pop(Trav& t, const int* sc, const int2* gs, int stride, int sk = 0) {
    while (t.sp > 0) {
        --t.sp;
        const int2 e = stk_read<SHORT>(sc, gs, stride, t.sp, sk);
        if (__int_as_float(e.y) <= t.cullT) {
            t.code = e.x;
            return true;
        }
    }
    return false;
}

// trav_pop with its first iteration peeled: the top entry is usually kept, and a lane then pays
// one LDS read and a compare instead of the loop's exec-mask bookkeeping (the same pops in the
// same order; C3 316 -> 306 ms, C4 3,287 -> 3,210 ms, profiles/r04z2_pop_peel_ab.log)
template <bool SHORT = false>
ND bool trav_pop1(Trav& t, const int* sc, const int2* gs, int stride, int sk = 0) {
    if (t.sp <= 0) return false;
    --t.sp;
    const int2 e = stk_read<SHORT>(sc, gs, stride, t.sp, sk);
    if (__int_as_float(e.y) <= t.cullT) {
        t.code = e.x;
        return true;
    }
    return trav_pop<SHORT>(t, sc, gs, stride, sk);
}

// One step: descend to the next leaf, test all its triangles, pop the next subtree.  Returns
// true when the query is resolved (t.bestG = winner or NO_HIT).  (A one-node-or-one-triangle
// "if-if" step measured slower on C3: 123 vs 95 ms per frame in the wavefront trace kernel.)
// LDS-staged nodes, 64 B each (a 16-B pad after every 4 nodes measured C3 276.3 -> 282.5 ms,
// C4 51.9 -> 51.6 ms and was retired, profiles/r05ae_node_pad_ab.txt).  node_slot: first float4 of
// node i.
NHD uint32_t node_slot(uint32_t i) { return 4u * i; }
NHD size_t node_lds_bytes(uint32_t n) { return (size_t)16 * (n ? node_slot(n - 1u) + 4u : 0u); }
// LDS quarter of 16-B part k of BVH node i (stage_nodes, kernels.h).  ROT: rotate by (i >> 2) & 3,
// in the environment-light builds, whose larger BVHs gain from the bank spread (C4 path kernel
// 52.1 -> 51.3 ms at 1080p/32; C3 276.2 -> 279.4 ms, so the other builds do not rotate:
// profiles/r05ad_node_swz_ab.txt, r05aj_c4_node_rot_ab.log)
template <bool ROT = false>
NHD uint32_t node_quarter(uint32_t i, uint32_t k) {
    return ROT ? (k + (i >> 2)) & 3u : k;
}
#ifndef NART_TRI_PF
#define NART_TRI_PF 2  // triangle records loaded per group in the leaf loop (0: one at a time)
#endif
#define NART_TRI_PAD 3  // padding records after tri_perm (a group of up to 4 may read past a leaf)
template <bool COUNT, bool ROT = false, bool SHORT = false>
ND bool trav_step(const DScene& S, const Ray& r, Trav& t, int* sc, int2* gs, int stride, TraceCounters& cnt,
                  const float4* lnodes, int nl, int sk = 0) {
    // (a wave-uniform node loop -- ballot per iteration, stopping once at most 0/2/4/8 lanes still
    // descend -- measured 13 % slower in k_render_rq than this per-lane loop: 114 vs 101 ms)
    while (t.code >= 0) {
        if (COUNT) cnt.nodes++;
        float4 a, b, c;
        int4 k;
        if (t.code < nl) {
#if defined(__HIP_DEVICE_COMPILE__)
            // explicit LDS address space: ds_read_b128, not a flat load through the generic aperture.
            // A flat load counts against both the vector-memory and the LDS counters, and the
            // compiler serialised the node's four flat loads behind waits for earlier triangle
            // loads; the LDS loads issue together.  k_render_rq, C3: 346.3 -> 336.5 ms per frame,
            // 1/8 shard 85.9 -> 81.9 ms (profiles/r04_node_ds_ab.log; round 1's k_render measured
            // 577 vs 570 ms the other way).
            typedef float v4f __attribute__((ext_vector_type(4)));
            typedef const __attribute__((address_space(3))) v4f lds_v4f;
            lds_v4f* np = (lds_v4f*)lnodes + node_slot((uint32_t)t.code);
            const uint32_t r = node_quarter<ROT>((uint32_t)t.code, 0u);
            const v4f qa = np[r], qb = np[(r + 1u) & 3u], qc = np[(r + 2u) & 3u], qk = np[(r + 3u) & 3u];
            a = make_float4(qa.x, qa.y, qa.z, qa.w);
            b = make_float4(qb.x, qb.y, qb.z, qb.w);
            c = make_float4(qc.x, qc.y, qc.z, qc.w);
            k = make_int4(__float_as_int(qk.x), __float_as_int(qk.y), __float_as_int(qk.z), __float_as_int(qk.w));
#else
            const float4* np = lnodes + node_slot((uint32_t)t.code);
            const uint32_t r = node_quarter<ROT>((uint32_t)t.code, 0u);
            a = np[r];
            b = np[(r + 1u) & 3u];
            c = np[(r + 2u) & 3u];
            k = reinterpret_cast<const int4*>(np)[(r + 3u) & 3u];
#endif
        } else {
            const float4* np = reinterpret_cast<const float4*>(S.nodes + t.code);
            a = np[0];
            b = np[1];
            c = np[2];
            k = reinterpret_cast<const int4*>(np)[3];
        }
        const f3 inv = t.inv, oi = t.oi;
        // child 0: lo (a.x a.y a.z) hi (a.w b.x b.y); child 1: lo (b.z b.w c.x) hi (c.y c.z c.w)
        float tx0 = fmaf(a.x, inv.x, oi.x), tx1 = fmaf(a.w, inv.x, oi.x);
        float ty0 = fmaf(a.y, inv.y, oi.y), ty1 = fmaf(b.x, inv.y, oi.y);
        float tz0 = fmaf(a.z, inv.z, oi.z), tz1 = fmaf(b.y, inv.z, oi.z);
        float n0 = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
        float f0 = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
        float ux0 = fmaf(b.z, inv.x, oi.x), ux1 = fmaf(c.y, inv.x, oi.x);
        float uy0 = fmaf(b.w, inv.y, oi.y), uy1 = fmaf(c.z, inv.y, oi.y);
        float uz0 = fmaf(c.x, inv.z, oi.z), uz1 = fmaf(c.w, inv.z, oi.z);
        float n1 = fmaxf(fmaxf(fminf(ux0, ux1), fminf(uy0, uy1)), fminf(uz0, uz1));
        float f1 = fminf(fminf(fmaxf(ux0, ux1), fmaxf(uy0, uy1)), fmaxf(uz0, uz1));
        bool h0 = (n0 <= f0) && (f0 >= 0.f) && (n0 <= t.cullT);
        bool h1 = (n1 <= f1) && (f1 >= 0.f) && (n1 <= t.cullT);
        // the child choice as selects: the far child is written to the free slot at sp on every step
        // and kept (sp + 1) only when both children are entered (sp <= max_stack < stack_depth, so
        // the write stays inside the lane's stack); the nearer child (by entry distance) first.
        // Against the branch form (push when both, else take the one hit, else pop): the same
        // entries, order and codes with fewer exec-mask instructions per node: C3 321 -> 316 ms,
        // 1/8 shard 81 -> 77 ms (profiles/r04t_*)
        const bool both = h0 && h1, swap = n1 < n0;
        // (a short stack's global column is written only when the entry is kept)
        if (!SHORT || t.sp < sk || both) stk_push<SHORT>(sc, gs, stride, t.sp, swap ? k.x : k.y, swap ? n0 : n1, sk);
        t.sp += both ? 1 : 0;
        t.code = both ? (swap ? k.y : k.x) : (h0 ? k.x : k.y);
        if (!h0 && !h1 && !trav_pop1<SHORT>(t, sc, gs, stride, sk)) return true;
    }
    const uint32_t lc = ~(uint32_t)t.code;
    const uint32_t first = lc >> 5, count = (lc & 31u) + 1u;
    // Vertices pre-permuted for this ray's major axis (DScene::tri_perm): v - o in permuted
    // order is (vp - op) component by component, the same subtractions as geometry.cpp:42-56,
    // without 18 per-triangle selects (C3 at 64 spp: 134.9 -> 133.3 ms).
    const f3 op = permute(r.o, r.major);
    const float4* tpp = S.tri_perm + 4 * ((size_t)r.major * S.num_leaf_tris + first);
    // one triangle test (geometry.cpp:32-115 through the octree's rules, octree.h); true when an
    // any-hit query is answered
    auto test = [&](const float4 b, const float4 c, const float4 dd, const float4 a) -> bool {
        if (COUNT) cnt.tris++;
        f3 p0 = F3(b.x - op.x, b.y - op.y, b.z - op.z);
        f3 p1 = F3(b.w - op.x, c.x - op.y, c.y - op.z);
        f3 p2 = F3(c.z - op.x, c.w - op.y, dd.x - op.z);
        p0.x += p0.z * r.Sx;
        p0.y += p0.z * r.Sy;
        p1.x += p1.z * r.Sx;
        p1.y += p1.z * r.Sy;
        p2.x += p2.z * r.Sx;
        p2.y += p2.z * r.Sy;
        const float e0 = (p1.x * p2.y) - (p1.y * p2.x);
        const float e1 = (p2.x * p0.y) - (p2.y * p0.x);
        const float e2 = (p0.x * p1.y) - (p0.y * p1.x);
        if (!edges_accept(e0, e1, e2)) return false;
        f3 n = F3(a.x, a.y, a.z);
        const float den = dot(r.d, n);
        float tt = (a.w - dot(r.o, n)) / den;
        if (tt != tt) t.risky = true;                       // NaN passes geometry.cpp:37-39 (octree.h)
        if (!(tt > 0.f) || !(tt < t.tmax)) return false;  // geometry.cpp:37-39 with tMin = 0
        uint32_t g = __float_as_uint(dd.y);
        const uint32_t info = __float_as_uint(dd.z) & (fabsf(den) >= dd.w ? 0xFFFFFFFFu : 0x7FFFFFFFu);
        if (t.any) {
            t.bestT = tt;
            t.bestG = g;
            t.bestInfo = info;
            return true;
        }
        if (tt < t.bestT) {
            t.t2 = t.bestT;
            t.bestT = tt;
            t.bestG = g;
            t.bestInfo = info;
            t.cullT = oc_cull(S, tt);
        } else {
            if (tt == t.bestT) {
                t.risky = true;  // the octree keeps the first chunk it visits, not the lowest index
                t.bestInfo = g < t.bestG ? info : t.bestInfo;
                t.bestG = g < t.bestG ? g : t.bestG;
            }
            t.t2 = fminf(t.t2, tt);
        }
        return false;
    };
    // The plane is loaded with the vertices (same 64-B record), not after the edge test: one memory
    // round trip per record instead of two.
#if NART_TRI_PF
    // Records are loaded NART_TRI_PF at a time, all before the first of them is tested (tri_perm
    // carries padding records, so a leaf's last group may read past it): one memory round trip
    // per group of tests instead of one per test.
    constexpr uint32_t K = NART_TRI_PF;
    for (uint32_t i = 0; i < count; i += K) {
        float4 rb[K], rc[K], rd[K], ra[K];
#pragma unroll
        for (uint32_t u = 0; u < K; ++u) {
            rb[u] = tpp[4 * (i + u)];
            rc[u] = tpp[4 * (i + u) + 1];
            rd[u] = tpp[4 * (i + u) + 2];
            ra[u] = tpp[4 * (i + u) + 3];
        }
#pragma unroll
        for (uint32_t u = 0; u < K; ++u)
            if ((u == 0 || i + u < count) && test(rb[u], rc[u], rd[u], ra[u])) return true;
    }
#else
    for (uint32_t i = 0; i < count; ++i)
        if (test(tpp[4 * i], tpp[4 * i + 1], tpp[4 * i + 2], tpp[4 * i + 3])) return true;
#endif
    return !trav_pop1<SHORT>(t, sc, gs, stride, sk);
}

}  // namespace nd
#include "octree.h"
namespace nd {

template <bool COUNT>
ND bool traverse(const DScene& S, const Ray& r, float tmax, bool ANY, float& bestT, uint32_t& bestG, int* sc,
                 float* st, int stride, TraceCounters& cnt, const float4* lnodes = nullptr, int nl = 0) {
    bestT = tmax;
    bestG = NO_HIT;
    if (!S.geometry_visible) return false;
    Trav t;
    trav_begin(S, r, tmax, ANY, t);
    while (!trav_step<COUNT>(S, r, t, sc, nullptr, stride, cnt, lnodes, nl)) {
    }
    bestT = t.bestT;
    bestG = t.bestG;
    oc_resolve<COUNT>(S, r, tmax, ANY, t.risky, t.bestInfo, fminf(t.t2, oc_cull(S, t.bestT)), bestT, bestG, cnt);
    return bestG != NO_HIT;
}

// Packet traversal of a wave's coherent closest-hit queries (k_primary: the camera rays of a 16x4
// pixel block at one sample index).  The wave walks one node at a time (node index, lane mask and
// stack wave-uniform: the node and triangle records are read once per wave, not once per lane);
// each lane in the node's mask tests the node's child boxes against its own ray and cull
// distance, and a child is entered with the mask of the lanes that hit it, nearer child first by
// majority.  A lane therefore tests exactly the leaves whose boxes its own ray reaches (a
// different order than traverse(), possibly beyond its final cull distance): the closest hit
// (minimum t, ties to the lowest scene index) is the same, t2 stays a lower bound of every other
// hit and risky flags the same ties and NaNs or more -- so oc_resolve returns the reference octree's
// answer as after traverse() (path.h trav_step, octree.h).  wstk: this wave's LDS stack, 16 B per
// level.
template <bool COUNT>
ND void traverse_packet(const DScene& S, const Ray& r, float tmax, float& bestT, uint32_t& bestG, uint4* wstk,
                        TraceCounters& cnt) {
    bestT = tmax;
    bestG = NO_HIT;
    if (!S.geometry_visible) return;
    Trav t;
    trav_begin(S, r, tmax, false, t);
    const uint32_t me = __lane_id();
    int code = S.root;
    uint64_t mask = __ballot(1);
    int sp = 0;
    const f3 op = permute(r.o, r.major);
    const int maj0 = __builtin_amdgcn_readfirstlane(r.major);
    const bool umaj = __ballot(r.major != maj0) == 0;
    for (;;) {
        const bool in = (mask >> me) & 1ull;
        bool pop = false;
        if (code >= 0) {
            // code is wave-uniform: the node is read through the constant address space, i.e. as
            // one scalar load (the node array is not written while a render kernel runs)
            typedef float v4f __attribute__((ext_vector_type(4)));
            typedef const __attribute__((address_space(4))) v4f c_v4f;
            const c_v4f* np = (const c_v4f*)(uintptr_t)(S.nodes + code);
            const v4f qa = np[0], qb = np[1], qc = np[2], qk = np[3];
            const float4 a = make_float4(qa.x, qa.y, qa.z, qa.w), b = make_float4(qb.x, qb.y, qb.z, qb.w),
                         c = make_float4(qc.x, qc.y, qc.z, qc.w);
            const int4 k = make_int4(__float_as_int(qk.x), __float_as_int(qk.y), __float_as_int(qk.z), __float_as_int(qk.w));
            const f3 inv = t.inv, oi = t.oi;
            const float tx0 = fmaf(a.x, inv.x, oi.x), tx1 = fmaf(a.w, inv.x, oi.x);
            const float ty0 = fmaf(a.y, inv.y, oi.y), ty1 = fmaf(b.x, inv.y, oi.y);
            const float tz0 = fmaf(a.z, inv.z, oi.z), tz1 = fmaf(b.y, inv.z, oi.z);
            const float n0 = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1));
            const float f0 = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1));
            const float ux0 = fmaf(b.z, inv.x, oi.x), ux1 = fmaf(c.y, inv.x, oi.x);
            const float uy0 = fmaf(b.w, inv.y, oi.y), uy1 = fmaf(c.z, inv.y, oi.y);
            const float uz0 = fmaf(c.x, inv.z, oi.z), uz1 = fmaf(c.w, inv.z, oi.z);
            const float n1 = fmaxf(fmaxf(fminf(ux0, ux1), fminf(uy0, uy1)), fminf(uz0, uz1));
            const float f1 = fminf(fminf(fmaxf(ux0, ux1), fmaxf(uy0, uy1)), fmaxf(uz0, uz1));
            const bool h0 = in && (n0 <= f0) && (f0 >= 0.f) && (n0 <= t.cullT);
            const bool h1 = in && (n1 <= f1) && (f1 >= 0.f) && (n1 <= t.cullT);
            if (COUNT && in) cnt.nodes++;
            const uint64_t m0 = __ballot(h0), m1 = __ballot(h1);
            const int c0 = __builtin_amdgcn_readfirstlane(k.x), c1 = __builtin_amdgcn_readfirstlane(k.y);
            if (m0 && m1) {
                const uint64_t p1 = __ballot(h0 && h1 && n1 < n0);
                const bool one_first = 2 * __popcll(p1) > __popcll(m0 & m1);
                const int fc = one_first ? c0 : c1;
                const uint64_t fm = one_first ? m0 : m1;
                wstk[sp] = make_uint4((uint32_t)fc, (uint32_t)fm, (uint32_t)(fm >> 32), 0u);
                ++sp;
                code = one_first ? c1 : c0;
                mask = one_first ? m1 : m0;
            } else if (m0) {
                code = c0;
                mask = m0;
            } else if (m1) {
                code = c1;
                mask = m1;
            } else {
                pop = true;
            }
        } else {
            const uint32_t lc = ~(uint32_t)code;
            const uint32_t first = lc >> 5, count = (lc & 31u) + 1u;
            const float4* tpp = S.tri_perm + 4 * ((size_t)r.major * S.num_leaf_tris + first);
            if (in) {
                // trav_step's leaf loop (closest hit), operation for operation (records one at a
                // time: loading them in pairs measured no faster in k_primary, 26.4 vs 26.3 ms,
                // profiles/r05u_packet_pairs_ab.log)
                for (uint32_t i = 0; i < count; ++i) {
                    if (COUNT) cnt.tris++;
                    float4 tb, tc, dd, ta;
                    if (umaj) {  // every ray of the wave has this major axis: one scalar load
                        typedef float v4f __attribute__((ext_vector_type(4)));
                        typedef const __attribute__((address_space(4))) v4f c_v4f;
                        const c_v4f* q = (const c_v4f*)(uintptr_t)(S.tri_perm + 4 * ((size_t)maj0 * S.num_leaf_tris + first + i));
                        const v4f q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
                        tb = make_float4(q0.x, q0.y, q0.z, q0.w);
                        tc = make_float4(q1.x, q1.y, q1.z, q1.w);
                        dd = make_float4(q2.x, q2.y, q2.z, q2.w);
                        ta = make_float4(q3.x, q3.y, q3.z, q3.w);
                    } else {
                        tb = tpp[4 * i];
                        tc = tpp[4 * i + 1];
                        dd = tpp[4 * i + 2];
                        ta = tpp[4 * i + 3];
                    }
                    f3 p0 = F3(tb.x - op.x, tb.y - op.y, tb.z - op.z);
                    f3 p1 = F3(tb.w - op.x, tc.x - op.y, tc.y - op.z);
                    f3 p2 = F3(tc.z - op.x, tc.w - op.y, dd.x - op.z);
                    p0.x += p0.z * r.Sx;
                    p0.y += p0.z * r.Sy;
                    p1.x += p1.z * r.Sx;
                    p1.y += p1.z * r.Sy;
                    p2.x += p2.z * r.Sx;
                    p2.y += p2.z * r.Sy;
                    const float e0 = (p1.x * p2.y) - (p1.y * p2.x);
                    const float e1 = (p2.x * p0.y) - (p2.y * p0.x);
                    const float e2 = (p0.x * p1.y) - (p0.y * p1.x);
                    if (!edges_accept(e0, e1, e2)) continue;
                    const f3 n = F3(ta.x, ta.y, ta.z);
                    const float den = dot(r.d, n);
                    const float tt = (ta.w - dot(r.o, n)) / den;
                    if (tt != tt) t.risky = true;
                    if (!(tt > 0.f) || !(tt < t.tmax)) continue;
                    const uint32_t g = __float_as_uint(dd.y);
                    const uint32_t info = __float_as_uint(dd.z) & (fabsf(den) >= dd.w ? 0xFFFFFFFFu : 0x7FFFFFFFu);
                    if (tt < t.bestT) {
                        t.t2 = t.bestT;
                        t.bestT = tt;
                        t.bestG = g;
                        t.bestInfo = info;
                        t.cullT = oc_cull(S, tt);
                    } else {
                        if (tt == t.bestT) {
                            t.risky = true;
                            t.bestInfo = g < t.bestG ? info : t.bestInfo;
                            t.bestG = g < t.bestG ? g : t.bestG;
                        }
                        t.t2 = fminf(t.t2, tt);
                    }
                }
            }
            pop = true;
        }
        if (pop) {
            if (sp == 0) break;
            --sp;
            const uint4 e = wstk[sp];
            code = __builtin_amdgcn_readfirstlane((int)e.x);
            mask = ((uint64_t)__builtin_amdgcn_readfirstlane(e.z) << 32) | (uint64_t)__builtin_amdgcn_readfirstlane(e.y);
        }
    }
    bestT = t.bestT;
    bestG = t.bestG;
    oc_resolve<COUNT>(S, r, tmax, false, t.risky, t.bestInfo, fminf(t.t2, oc_cull(S, t.bestT)), bestT, bestG, cnt);
}

// ---------------------------------------------------------------- Intersection
struct Isect {
    f3 p, gn, sn, dpds, dpdt;
    f2 st;
    uint32_t meshID, priority, mat;
};
ND f3 load3(const float* a) { return F3(a[0], a[1], a[2]); }

// Attributes of the winning triangle (geometry.cpp:84-112) + Chunk::Intersect ids (bvh.cpp:72-75)
ND void fill_isect(const DScene& S, const Ray& r, uint32_t g, Isect& is) {
    const nart_triangle& T = S.tris[g];
    f3 v0 = load3(T.v0), v1 = load3(T.v1), v2 = load3(T.v2);
    f3 n = cross(sub(v1, v0), sub(v2, v0));
    float e0, e1, e2;
    edge_functions(r, v0, v1, v2, e0, e1, e2);
    float invDet = 1.f / (e0 + e1 + e2);
    is.p = muls(add(add(muls(v0, e0), muls(v1, e1)), muls(v2, e2)), invDet);
    float u = e0 * invDet;
    float v = e1 * invDet;
    is.gn = normalize(n);
    float w = 1 - u - v;
    is.sn = add(add(muls(load3(T.n0), u), muls(load3(T.n1), v)), muls(load3(T.n2), w));
    is.st = F2((T.uv0[0] * u + T.uv1[0] * v) + T.uv2[0] * w, (T.uv0[1] * u + T.uv1[1] * v) + T.uv2[1] * w);
    float UVDet = ((T.uv0[0] - T.uv2[0]) * (T.uv1[1] - T.uv2[1])) - ((T.uv0[1] - T.uv2[1]) * (T.uv1[0] - T.uv2[0]));
    float invUVDet = 1.f / UVDet;
    is.dpds = muls(add(muls(sub(v0, v2), T.uv1[1] - T.uv2[1]), muls(sub(v1, v2), T.uv2[1] - T.uv0[1])), invUVDet);
    is.dpdt = muls(add(muls(sub(v0, v2), T.uv2[0] - T.uv1[0]), muls(sub(v1, v2), T.uv0[0] - T.uv2[0])), invUVDet);
    uint32_t mesh = S.tri_mesh[g];
    is.meshID = mesh;
    is.priority = cst(S.meshes)[mesh].priority;
    is.mat = cst(S.meshes)[mesh].material;
}

// ---------------------------------------------------------------- patterns
ND float half_to_float(uint16_t h) {  // Imath half -> float (exact)
    uint32_t hexpmant = ((uint32_t)h << 17) >> 4;
    uint32_t v = ((uint32_t)h >> 15) << 31;
    if (hexpmant >= 0x00800000u) {
        v |= hexpmant;
        if (hexpmant >= 0x0f800000u) v |= 0x7f800000u;
        else v += 0x38000000u;
    } else if (hexpmant != 0) {
        uint32_t lc = __builtin_clz(hexpmant) - 8;
        v |= 0x38800000u;
        v |= (hexpmant << lc);
        v -= (lc << 23);
    }
    return __uint_as_float(v);
}
// (the texel's RGBA halves as one 8-B load; a non-temporal load for the volume kernel's sky lookups
// measured slower, 81.7 vs 79.4 ms, with the same fetch: profiles/r06o_sky_nt_ab.log)
ND f3 tex_fetch(const DScene& S, int tex, float su, float sv, int rough) {  // texturepattern.cpp:172-187
    const DTexture& t = cst(S.texs)[tex];
    float u = gmin(gmax(su, 0.0001f), 0.9999f);
    float v = gmin(gmax(1.f - sv, 0.0001f), 0.9999f);
    int iu = (int)((float)t.w * u);
    int iv = (int)((float)t.h * v);
    const uint16_t* px = S.tex_pool + t.offset + ((uint64_t)iv * t.w + (uint64_t)iu) * 4;
    const unsigned long long* p8 = reinterpret_cast<const unsigned long long*>(px);
    const unsigned long long q = *p8;
    float rr = half_to_float((uint16_t)(q & 0xFFFFu)), gg = half_to_float((uint16_t)((q >> 16) & 0xFFFFu)),
          bb = half_to_float((uint16_t)((q >> 32) & 0xFFFFu));
    if (rough) { rr *= rr; gg *= gg; bb *= bb; }
    return F3(rr, gg, bb);
}
template <uint32_t FM = FT_ALL>
ND f3 ptn_value(const DScene& S, const DPattern& p, f2 st) {
    if (!(FM & FT_TEX) || p.type == NART_PTN_CONSTANT) return F3(p.v[0], p.v[1], p.v[2]);
    return tex_fetch(S, p.tex, st.x, st.y, p.rough);
}

// ---------------------------------------------------------------- BxDFs
enum { B_LAMBERT, B_SPECULAR, B_SPECDIEL, B_DIEL, B_TS };
struct BxDF {
    int type;
    uint32_t flags;  // BxDF::flags member
    f3 rho, tau;
    float eta, a0, ap;
};

ND float fresnel(float eta_o, float eta_i, float cosTheta) {  // bxdf.cpp:3-22
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
ND f3 reflect(f3 w1, f3 w2) { return sub(muls(w2, 2.f * dot(w1, w2)), w1); }  // bxdf.h:14-16
ND float lambda_(float alpha, f3 w) {
    float sinT = sqrtf(1.f - (w.z * w.z));
    float tanT = (sinT / w.z);
    return (-1.f + sqrtf(1.f + (alpha * alpha * tanT * tanT))) * 0.5f;
}
ND float G_(float a, f3 wo, f3 wi) { return 1.f / (1.f + lambda_(a, wo) + lambda_(a, wi)); }
ND float G1_(float a, f3 w) { return 1.f / (1.f + lambda_(a, w)); }
ND float D_ggx(float alpha, f3 wh) {  // torrancesparrowbrdf.cpp:19-30
    float sinT = sqrtf(1.f - (wh.z * wh.z));
    float tanT = (sinT / wh.z);
    float tan2 = tanT * tanT;
    return 1.f / ((ND_PI * alpha * alpha * ((wh.z * wh.z) * (wh.z * wh.z))) * (1.f + (tan2 / (alpha * alpha))) *
                  (1.f + (tan2 / (alpha * alpha))));
}
ND float D_diel(float alpha, f3 wh) { return wh.z == 0.f ? 0.f : D_ggx(alpha, wh); }  // dielectricbrdf.cpp:19-29

// VNDF sampling (dielectricbrdf.cpp:106-139 with diel=1, torrancesparrowbrdf.cpp:68-96 with diel=0)
ND f3 sample_wh(f3 wo, float alpha, f2 sample, bool diel) {
    f3 wo_h = normalize(F3(wo.x * alpha, wo.y * alpha, wo.z));
    if (diel && wo.z < 0.f) wo_h = muls(wo_h, -1.f);
    f3 T1;
    if (diel && wo.x == 0.f && wo.y == 0.f) T1 = F3(1.f, 0.f, 0.f);
    else T1 = F3(wo_h.y, -wo_h.x, 0.f);
    T1 = normalize(T1);
    f3 T2 = normalize(cross(T1, wo_h));
    f2 vh = uniform_sample_disk(sample);
    float s = (1.f + wo_h.z) * 0.5f;
    vh.y = (s * vh.y) + ((1.f - s) * sqrtf(1.f - (vh.x * vh.x)));
    f3 wh = F3(sqrtf(1.f - (vh.x * vh.x) - (vh.y * vh.y)), vh.x, vh.y);
    wh = add(add(muls(wo_h, wh.x), muls(T1, wh.y)), muls(T2, wh.z));
    return normalize(F3(wh.x * alpha, wh.y * alpha, wh.z));
}

ND f3 bxdf_f(const BxDF& b, f3 wo, f3 wi, bool uap, float eta_outer) {
    if (b.type == B_LAMBERT) return muls(b.rho, ND_ONE_OVER_PI);  // lambertbrdf.cpp:7-11
    if (b.type == B_DIEL) {                                       // dielectricbrdf.cpp:31-80
        float alpha = uap ? b.ap : b.a0;
        float eta_o = eta_outer, eta_i = b.eta;
        if (wo.z < 0.f) { float t = eta_o; eta_o = eta_i; eta_i = t; }
        if (wo.z * wi.z >= 0.f) {
            f3 wh = normalize(add(wo, wi));
            if (wh.z < 0.f) wh = muls(wh, -1.f);
            float g = G_(alpha, wo, wi);
            float d = D_diel(alpha, wh);
            float Fr = fresnel(eta_o, eta_i, gabs(dot(wh, wo)));
            if (wo.z * wi.z == 0.f) return F3(0.f, 0.f, 0.f);
            return divs(muls(muls(muls(b.rho, g), d), Fr), (4.f * wo.z * wi.z));
        }
        f3 wh = normalize(add(muls(wo, eta_o), muls(wi, eta_i)));
        if (wh.z < 0.f) wh = muls(wh, -1.f);
        float Fr = fresnel(eta_o, eta_i, gabs(dot(wh, wo)));
        if (Fr >= 1.f) return F3(0.f, 0.f, 0.f);
        float g = G_(alpha, wo, wi);
        float d = D_diel(alpha, wh);
        float wiDotWh = dot(wi, wh);
        float woDotWh = dot(wo, wh);
        float num = g * d * (1.f - Fr) * gabs(wiDotWh) * gabs(woDotWh) * eta_o * eta_o;
        float x = ((eta_i * wiDotWh) + (eta_o * woDotWh));
        float denom = x * x * gabs(wo.z * wi.z);
        float q = num / denom;
        return mul(F3(q, q, q), b.tau);
    }
    if (b.type == B_TS) {  // torrancesparrowbrdf.cpp:32-51
        float alpha = uap ? b.ap : b.a0;
        if (wo.z < 0.f || wi.z < 0.f) return F3(0.f, 0.f, 0.f);
        f3 wh = normalize(add(wo, wi));
        float g = G_(alpha, wo, wi);
        float d = D_ggx(alpha, wh);
        float fr = fresnel(eta_outer, b.eta, dot(wh, wi));
        if (wo.z * wi.z == 0.f) return F3(0.f, 0.f, 0.f);
        return divs(muls(muls(muls(b.rho, g), d), fr), (4.f * wo.z * wi.z));
    }
    return F3(0.f, 0.f, 0.f);  // delta lobes: f == 0
}

ND float bxdf_pdf(const BxDF& b, f3 wo, f3 wi, bool uap, float eta_outer) {
    if (b.type == B_LAMBERT) return wi.z * ND_ONE_OVER_PI;
    if (b.type == B_DIEL) {  // dielectricbrdf.cpp:187-225
        float eta_o = eta_outer, eta_i = b.eta;
        if (eta_o == eta_i) return 0.f;
        float alpha = uap ? b.ap : b.a0;
        if (wo.z * wi.z >= 0.f) {
            f3 wh = normalize(add(wo, wi));
            if (wh.z < 0.f) wh = muls(wh, -1.f);
            float cosThetaH = gabs(gmin(dot(wo, wh), 1.f));
            float pdf = (D_diel(alpha, wh) * gmin(dot(wo, wh), 1.f) * G1_(alpha, wo)) / wo.z;
            return gmax(0.f, pdf / (4.f * cosThetaH));
        }
        if (wo.z < 0.f) { float t = eta_o; eta_o = eta_i; eta_i = t; }
        f3 wh = normalize(add(muls(wo, eta_o), muls(wi, eta_i)));
        if (wh.z < 0.f) wh = muls(wh, -1.f);
        float pdf = (D_diel(alpha, wh) * gmin(gabs(dot(wo, wh)), 1.f) * G1_(alpha, wo)) / gabs(wo.z);
        float dotWiWh = dot(wi, wh);
        float dotWoWh = dot(wo, wh);
        float denom = (eta_i * dotWiWh + eta_o * dotWoWh);
        float JDet = (fabsf(dotWiWh) * eta_i * eta_i) / (denom * denom);
        return pdf * JDet;
    }
    if (b.type == B_TS) {  // torrancesparrowbrdf.cpp:109-124
        float alpha = uap ? b.ap : b.a0;
        f3 wh = normalize(add(wo, wi));
        if (wh.z < 0.f) return 0.f;
        float cosThetaH = gmin(dot(wo, wh), 1.f);
        float pdf = (D_ggx(alpha, wh) * gmin(dot(wo, wh), 1.f) * G1_(alpha, wo)) / wo.z;
        return gmax(0.f, pdf / (4.f * cosThetaH));
    }
    return 0.f;
}
ND float bxdf_eta(const BxDF& b) { return b.type == B_LAMBERT ? 0.f : b.eta; }

// bxdf_f and bxdf_pdf of the same (wo, wi) in one pass: each value is computed with exactly the
// operations of those two functions, but the half vector, D and the Smith term of wo, which both
// recompute, are evaluated once (every call site of the reference pairs them: BxDF::Sample_f ends
// with Pdf and f, EstimateDirect's light strategy with Pdf and f).
template <uint32_t FM = FT_ALL>
ND f3 bxdf_f_pdf(const BxDF& b, f3 wo, f3 wi, bool uap, float eta_outer, float& pdf) {
    pdf = 0.f;
    if (ft_lambert(FM) && b.type == B_LAMBERT) {  // lambertbrdf.cpp:7-29
        pdf = wi.z * ND_ONE_OVER_PI;
        return muls(b.rho, ND_ONE_OVER_PI);
    }
    if (ft_diel(FM) && b.type == B_DIEL) {  // dielectricbrdf.cpp:31-80 (f), 187-225 (Pdf)
        // Reflection (wo.z * wi.z >= 0) and transmission evaluate the same chain -- half vector,
        // D, the Smith terms, Fresnel -- on different inputs: the reflection half vector is
        // normalize(wo + wi) = normalize(wo * 1 + wi * 1) (x * 1 is exact) and its Fresnel argument
        // |dot(wh, wo)| = |dot(wo, wh)|.  A wave whose glass lanes both reflect and transmit ran
        // the chain twice; here it runs once on per-lane selected inputs, and each division takes
        // the numerator and denominator of the lane's own branch.  Every lane computes its
        // branch's values with its branch's operations.
        const float alpha = uap ? b.ap : b.a0;
        float eta_o = eta_outer, eta_i = b.eta;
        const bool same = eta_o == eta_i;
        const float lo = lambda_(alpha, wo);
        const bool refl = wo.z * wi.z >= 0.f;
        if (wo.z < 0.f) { float t = eta_o; eta_o = eta_i; eta_i = t; }  // f swaps in both branches
        const float ea = refl ? 1.f : eta_o, eb = refl ? 1.f : eta_i;
        f3 wh = normalize(add(muls(wo, ea), muls(wi, eb)));
        if (wh.z < 0.f) wh = muls(wh, -1.f);
        const float d = D_diel(alpha, wh);
        const float wiDotWh = dot(wi, wh);
        const float woDotWh = dot(wo, wh);
        if (!same) {
            // reflection: (d * min(wo.wh, 1) * G1) / wo.z, then max(0, p / (4 |min(wo.wh, 1)|));
            // transmission: (d * min(|wo.wh|, 1) * G1) / |wo.z|, then p * (|wi.wh| eta_i^2) / denom^2
            const float p = (d * gmin(refl ? woDotWh : gabs(woDotWh), 1.f) * (1.f / (1.f + lo))) /
                            (refl ? wo.z : gabs(wo.z));
            const float cosThetaH = gabs(gmin(woDotWh, 1.f));
            const float denom = (eta_i * wiDotWh + eta_o * woDotWh);
            const float r = (refl ? p : fabsf(wiDotWh) * eta_i * eta_i) / (refl ? 4.f * cosThetaH : denom * denom);
            pdf = refl ? gmax(0.f, r) : p * r;
        }
        const float Fr = fresnel(eta_o, eta_i, gabs(woDotWh));
        const float g = 1.f / (1.f + lo + lambda_(alpha, wi));
        // f: reflection rho_c * g * d * Fr / (4 wo.z wi.z) per channel; transmission
        // (g d (1 - Fr) |wi.wh| |wo.wh| eta_o^2) / (x^2 |wo.z wi.z|) times tau_c
        const float num = g * d * (1.f - Fr) * gabs(wiDotWh) * gabs(woDotWh) * eta_o * eta_o;
        const float x = ((eta_i * wiDotWh) + (eta_o * woDotWh));
        const float den = refl ? (4.f * wo.z * wi.z) : x * x * gabs(wo.z * wi.z);
        const float qx = (refl ? ((b.rho.x * g) * d) * Fr : num) / den;
        const float qy = (refl ? ((b.rho.y * g) * d) * Fr : num) / den;
        const float qz = (refl ? ((b.rho.z * g) * d) * Fr : num) / den;
        if (refl ? wo.z * wi.z == 0.f : Fr >= 1.f) return F3(0.f, 0.f, 0.f);
        return refl ? F3(qx, qy, qz) : mul(F3(qx, qx, qx), b.tau);
    }
    if (ft_ts(FM) && b.type == B_TS) {  // torrancesparrowbrdf.cpp:32-51 (f), 109-124 (Pdf)
        const float alpha = uap ? b.ap : b.a0;
        const f3 wh = normalize(add(wo, wi));
        const float d = D_ggx(alpha, wh);
        const float lo = lambda_(alpha, wo);
        if (!(wh.z < 0.f)) {
            const float cosThetaH = gmin(dot(wo, wh), 1.f);
            const float p = (d * gmin(dot(wo, wh), 1.f) * (1.f / (1.f + lo))) / wo.z;
            pdf = gmax(0.f, p / (4.f * cosThetaH));
        }
        if (wo.z < 0.f || wi.z < 0.f) return F3(0.f, 0.f, 0.f);
        const float g = 1.f / (1.f + lo + lambda_(alpha, wi));
        const float fr = fresnel(eta_outer, b.eta, dot(wh, wi));
        if (wo.z * wi.z == 0.f) return F3(0.f, 0.f, 0.f);
        return divs(muls(muls(muls(b.rho, g), d), fr), (4.f * wo.z * wi.z));
    }
    return F3(0.f, 0.f, 0.f);  // delta lobes: f == 0, Pdf == 0
}

template <uint32_t FM = FT_ALL>
ND f3 bxdf_sample_f(const BxDF& b, f3 wo, f3& wi, float s1, f2 sample, float& pdf, uint32_t& flags, float* alpha_i,
                    bool uap, float eta_outer) {
    if (ft_lambert(FM) && b.type == B_LAMBERT) {  // lambertbrdf.cpp:13-22
        if (alpha_i) *alpha_i = 1.f;
        flags = F_DIFFUSE;
        wi = cosine_sample_hemisphere(sample, pdf);
        return muls(b.rho, ND_ONE_OVER_PI);  // bxdf_f of B_LAMBERT
    }
    if (ft_spec(FM) && b.type == B_SPECULAR) {  // specularbrdf.cpp:14-36
        if (alpha_i) *alpha_i = 0.f;
        flags = F_SPECULAR;
        wi = F3(-wo.x, -wo.y, wo.z);
        pdf = 1.f;
        if (wi.z == 0.f) return F3(1.f, 1.f, 1.f);
        return divs(muls(b.rho, fresnel(eta_outer, b.eta, wi.z)), gabs(wi.z));
    }
    if (ft_diel(FM) && b.type == B_SPECDIEL) {  // speculardielectricbrdf.cpp:15-89
        float eta_o = eta_outer, eta_i = b.eta;
        if (eta_o == eta_i) {
            wi = neg(wo);
            pdf = 0.f;
            flags |= F_TRANSMISSIVE;
            return b.tau;
        }
        if (alpha_i) *alpha_i = 0.f;
        flags = F_SPECULAR;
        if (wo.z < 0.f) { float t = eta_o; eta_o = eta_i; eta_i = t; }
        float Fr = fresnel(eta_o, eta_i, gabs(wo.z));
        if (sample.x < Fr) {
            pdf = Fr;
            wi = F3(-wo.x, -wo.y, wo.z);
            if (wi.z == 0.f) return F3(1.f, 1.f, 1.f);
            float q = Fr / gabs(wi.z);
            return mul(F3(q, q, q), b.rho);
        }
        pdf = 1.f - Fr;
        float sinT_o = sqrtf(1.f - (wo.z * wo.z));
        float sinT_i = ((eta_o / eta_i) * sinT_o);
        if (sinT_i >= 1.f) {
            wi = F3(-wo.x, -wo.y, wo.z);
            return mul(F3(1.f, 1.f, 1.f), b.rho);
        }
        flags |= F_TRANSMISSIVE;
        const f3 n = F3(0.f, 0.f, 1.f);
        f3 bb = muls(n, wo.z);
        f3 a = sub(wo, bb);
        f3 c = muls(neg(a), (eta_o / eta_i));
        f3 d = muls(neg(n), sqrtf(1.f - (sinT_i * sinT_i)));
        if (wo.z < 0.f) d = muls(d, -1.f);
        wi = normalize(add(c, d));
        float q = ((eta_o / eta_i) * (eta_o / eta_i) * (1.f - Fr)) / gabs(wi.z);
        return mul(F3(q, q, q), b.tau);
    }
    if (ft_diel(FM) && b.type == B_DIEL) {  // dielectricbrdf.cpp:82-183
        float eta_o = eta_outer, eta_i = b.eta;
        if (eta_o == eta_i) {
            wi = neg(wo);
            pdf = 0.f;
            flags |= F_TRANSMISSIVE;
            return b.tau;
        }
        float alpha = uap ? b.ap : b.a0;
        if (alpha_i) *alpha_i = alpha;
        flags = F_SPECULAR;
        if (alpha > 0.0001f) flags = F_GLOSSY;
        if (alpha >= 1.0f) flags = F_DIFFUSE;
        f3 wh = sample_wh(wo, alpha, sample, true);
        if (wo.z < 0.f) { float t = eta_o; eta_o = eta_i; eta_i = t; }
        float Fr = fresnel(eta_o, eta_i, gabs(dot(wh, wo)));
        // reflection (s1 < Fr), total internal reflection and refraction each end with
        // bxdf_f_pdf of their wi: one evaluation on the lane's wi (each lane's wi and pdf factor
        // are its branch's), not one per branch present in the wave
        const bool rf = s1 < Fr;
        float cos_o = gmin(1.f, gmax(-1.f, dot(wo, wh)));
        float sin_o = sqrtf(1.f - (cos_o * cos_o));
        float sin_i = ((eta_o / eta_i) * sin_o);
        const bool tr = !rf && !(sin_i >= 1.f);
        f3 bb = muls(wh, cos_o);
        f3 a = sub(wo, bb);
        f3 c = muls(neg(a), (eta_o / eta_i));
        f3 d = muls(neg(wh), sqrtf(1.f - (sin_i * sin_i)));
        if (dot(wo, wh) < 0.f) d = muls(d, -1.f);
        if (tr) flags |= F_TRANSMISSIVE;
        wi = normalize(tr ? add(c, d) : reflect(wo, wh));
        float pp;
        const f3 fr = bxdf_f_pdf<FM>(b, wo, wi, uap, eta_outer, pp);
        pdf = pp * (rf ? Fr : (1.f - Fr));
        return fr;
    }
    // B_TS: torrancesparrowbrdf.cpp:53-105 (a mask without it creates no other kind)
    if (!ft_ts(FM)) return F3(0.f, 0.f, 0.f);
    float alpha = uap ? b.ap : b.a0;
    if (alpha_i) *alpha_i = alpha;
    flags = F_SPECULAR;
    if (alpha > 0.001f) flags = F_GLOSSY;
    if (alpha >= 1.0f) flags = F_DIFFUSE;
    f3 wh = sample_wh(wo, alpha, sample, false);
    wi = normalize(reflect(wo, wh));
    return bxdf_f_pdf<FM>(b, wo, wi, uap, eta_outer, pdf);
}

// ---------------------------------------------------------------- BSDF (bxdf.cpp:24-115)
struct BSDF {
    f3 n_t, n_b, n;
    uint32_t num;
    BxDF b[2];
};
ND f3 to_local(const BSDF& s, f3 v) { return normalize(F3(dot(v, s.n_t), dot(v, s.n_b), dot(v, s.n))); }
ND f3 to_world(const BSDF& s, f3 v) { return normalize(add(add(muls(s.n_t, v.x), muls(s.n_b, v.y)), muls(s.n, v.z))); }
ND void build_coord_sys(BSDF& s, const Isect& is, const f3* nn) {
    s.n_t = normalize(sub(is.dpds, muls(s.n, dot(is.dpds, s.n))));
    s.n_b = normalize(cross(is.sn, s.n_t));
    if (nn) {
        s.n = normalize(to_world(s, *nn));
        s.n_t = normalize(sub(is.dpds, muls(s.n, dot(is.dpds, s.n))));
        s.n_b = normalize(cross(is.sn, s.n_t));
    }
}
ND f3 bsdf_f(const BSDF& s, f3 wo, f3 wi, bool uap, float eta_outer) {
    f3 f = F3(0.f, 0.f, 0.f);
    f = add(f, bxdf_f(s.b[0], wo, wi, uap, eta_outer));
    if (s.num > 1) f = add(f, bxdf_f(s.b[1], wo, wi, uap, eta_outer));
    return f;
}
ND float bsdf_pdf(const BSDF& s, f3 wo, f3 wi, bool uap, float eta_outer) {
    float pdf = 0.f;
    pdf += bxdf_pdf(s.b[0], wo, wi, uap, eta_outer);
    if (s.num > 1) pdf += bxdf_pdf(s.b[1], wo, wi, uap, eta_outer);
    return pdf / (float)s.num;
}
// number of lobes: two only for plastic (a mask without it knows the BSDF has one)
template <uint32_t FM>
ND uint32_t bsdf_num(const BSDF& s) { return (FM & FT_PLASTIC) ? s.num : 1u; }
// bsdf_f and bsdf_pdf together (bxdf_f_pdf per lobe; the sums in the same order)
template <uint32_t FM = FT_ALL>
ND f3 bsdf_f_pdf(const BSDF& s, f3 wo, f3 wi, bool uap, float eta_outer, float& pdf) {
    const uint32_t num = bsdf_num<FM>(s);
    float p0, p1 = 0.f;
    f3 f = F3(0.f, 0.f, 0.f);
    f = add(f, bxdf_f_pdf<FM>(s.b[0], wo, wi, uap, eta_outer, p0));
    f3 f1 = F3(0.f, 0.f, 0.f);
    if (num > 1) f1 = bxdf_f_pdf<FM>(s.b[1], wo, wi, uap, eta_outer, p1);
    if (num > 1) f = add(f, f1);
    float p = 0.f;
    p += p0;
    if (num > 1) p += p1;
    pdf = p / (float)num;
    return f;
}
// SHARE_TS: the environment-light builds of the path kernels (C4: 3,332 -> 3,259 ms); the others
// keep one evaluation per role (C3 measured 316 -> 322 ms with sharing, a register-allocation
// effect in the 256-VGPR kernel, which has no plastic lobes to share; profiles/r04y_share_ts_ab.log)
template <bool SHARE_TS = true, uint32_t FM = FT_ALL>
ND f3 bsdf_sample_f(const BSDF& s, f3 wo, f3& wi, float s1, f2 sample, float& pdf, uint32_t& flags, bool uap,
                    float eta_outer, float* alpha_i, float* eta_i) {
    const uint32_t num = bsdf_num<FM>(s);
    if (!SHARE_TS || !(FM & FT_PLASTIC)) {
        uint32_t idx = f2u8(s1 * (float)num);
        s1 = gfract(s1 * (float)num);
        const BxDF& sel = s.b[((FM & FT_PLASTIC) && idx) ? 1 : 0];
        f3 f = bxdf_sample_f<FM>(sel, wo, wi, s1, sample, pdf, flags, alpha_i, uap, eta_outer);
        if (eta_i && (flags & F_TRANSMISSIVE)) *eta_i = bxdf_eta(sel);
        if (!(flags & F_SPECULAR)) {
            if (num > 1) {
                const BxDF& o = s.b[idx ? 0 : 1];
                if (!(o.flags & F_SPECULAR)) {
                    float bp;
                    const f3 fo = bxdf_f_pdf<FM>(o, wo, wi, uap, eta_outer, bp);
                    if (bp > 0.f) {
                        pdf += bp;
                        f = add(f, fo);
                    }
                }
            }
            pdf /= (float)num;
        }
        return f;
    }
    uint32_t idx = f2u8(s1 * (float)s.num);
    s1 = gfract(s1 * (float)s.num);
    const BxDF& sel = s.b[idx ? 1 : 0];
    const BxDF& o = s.b[idx ? 0 : 1];
    // The GGX reflection lobe (B_TS) is evaluated at the sampled wi either as the sampled lobe
    // (torrancesparrowbrdf.cpp:53-105 ends with Pdf and f) or as a plastic's other lobe
    // (bxdf.cpp:87-106): a wave holding both kinds of lanes ran that evaluation twice.  Here the
    // B_TS sampling step only draws wi, and one bxdf_f_pdf serves both roles, with the lane's own
    // lobe and wi (the sums below take the same operands; + is commutative).
    const bool ts_sel = ft_ts(FM) && sel.type == B_TS;
    f3 f = F3(0.f, 0.f, 0.f);
    if (ts_sel) {  // torrancesparrowbrdf.cpp:53-105 up to the direction
        float alpha = uap ? sel.ap : sel.a0;
        if (alpha_i) *alpha_i = alpha;
        flags = F_SPECULAR;
        if (alpha > 0.001f) flags = F_GLOSSY;
        if (alpha >= 1.0f) flags = F_DIFFUSE;
        f3 wh = sample_wh(wo, alpha, sample, false);
        wi = normalize(reflect(wo, wh));
    } else {
        f = bxdf_sample_f<FM>(sel, wo, wi, s1, sample, pdf, flags, alpha_i, uap, eta_outer);
    }
    if (eta_i && (flags & F_TRANSMISSIVE)) *eta_i = bxdf_eta(sel);
    // (o is read only for two-lobe BSDFs: s.num > 1 is tested first)
    const bool other = !(flags & F_SPECULAR) && s.num > 1 && !(o.flags & F_SPECULAR);
    const bool other_ts = other && !ts_sel && o.type == B_TS;
    float tp = 0.f;
    f3 tf = F3(0.f, 0.f, 0.f);
    if (ts_sel || other_ts) tf = bxdf_f_pdf<FM>(ts_sel ? sel : o, wo, wi, uap, eta_outer, tp);
    if (ts_sel) {
        f = tf;
        pdf = tp;
    }
    if (!(flags & F_SPECULAR)) {
        if (other) {
            float bp = tp;
            f3 fo = tf;
            if (!other_ts) fo = bxdf_f_pdf<FM>(o, wo, wi, uap, eta_outer, bp);
            if (bp > 0.f) {
                pdf += bp;
                f = add(f, fo);
            }
        }
        pdf /= (float)s.num;
    }
    return f;
}
template <uint32_t FM = FT_ALL>
ND float bsdf_sample_eta(const BSDF& s, float s1) {
    return bxdf_eta(s.b[((FM & FT_PLASTIC) && f2u8(s1 * (float)s.num)) ? 1 : 0]);
}

// Material::CreateBSDF (src/materials/*.cpp).  A material kind outside FM is never tested; the
// last kind in the mask takes every remaining material (as the generic switch's default does).
template <uint32_t FM = FT_ALL>
ND void create_bsdf(const DScene& S, const Isect& is, float alphaTweak, BSDF& bs) {
    const DMaterial& m = cst(S.mats)[is.mat];
    constexpr uint32_t MM = FM & (FT_LAMBERT | FT_SPECMAT | FT_GLASS | FT_GLOSSY | FT_PLASTIC);
    constexpr uint32_t last = MM ? (1u << (31 - __builtin_clz(MM | 1u))) : FT_PLASTIC;
    const int32_t t = m.type;
    bs.n = is.sn;
    bs.num = ((FM & FT_PLASTIC) && t == NART_MAT_PLASTIC) ? 2u : 1u;
    if ((FM & FT_NMAP) && m.has_normal) {
        f3 n = ptn_value<FM>(S, m.normal, is.st);
        n = muls(n, 2.f);
        n = sub(n, F3(1.f, 1.f, 1.f));
        build_coord_sys(bs, is, &n);
    } else {
        build_coord_sys(bs, is, nullptr);
    }
    BxDF& b0 = bs.b[0];
    b0.tau = F3(0.f, 0.f, 0.f);
    b0.eta = 0.f;
    b0.a0 = 0.f;
    b0.ap = 0.f;
    if ((FM & FT_LAMBERT) && (last == FT_LAMBERT || t == NART_MAT_LAMBERT)) {  // diffusematerial.cpp:6-27
        b0.type = B_LAMBERT;
        b0.flags = F_DIFFUSE;
        b0.rho = ptn_value<FM>(S, m.rho_d, is.st);
    } else if ((FM & FT_SPECMAT) && (last == FT_SPECMAT || t == NART_MAT_SPECULAR)) {  // specularmaterial.cpp:9-43
        float alpha = 0.f;
        float ap = 1.f - ((1.f - alpha) * alphaTweak);
        b0.rho = ptn_value<FM>(S, m.rho_s, is.st);
        b0.eta = ptn_value<FM>(S, m.eta, is.st).x;
        if (ap > 0.0001f) { b0.type = B_TS; b0.flags = F_GLOSSY; b0.a0 = gmax(0.0001f, alpha); b0.ap = ap; }
        else { b0.type = B_SPECULAR; b0.flags = F_SPECULAR; }
    } else if ((FM & FT_GLASS) && (last == FT_GLASS || t == NART_MAT_GLASS)) {  // glassmaterial.cpp:11-47
        float alpha = ptn_value<FM>(S, m.alpha, is.st).x;
        float ap = 1.f - ((1.f - ptn_value<FM>(S, m.alpha, is.st).x) * alphaTweak);
        b0.rho = ptn_value<FM>(S, m.rho_s, is.st);
        b0.tau = ptn_value<FM>(S, m.tau, is.st);
        b0.eta = ptn_value<FM>(S, m.eta, is.st).x;
        if (ap > 0.0001f) { b0.type = B_DIEL; b0.flags = F_GLOSSY; b0.a0 = gmax(0.0001f, alpha); b0.ap = ap; }
        else { b0.type = B_SPECDIEL; b0.flags = F_SPECULAR; }
    } else if ((FM & FT_GLOSSY) && (last == FT_GLOSSY || t == NART_MAT_GLOSSY)) {  // glossydielectricmaterial.cpp:12-47
        float alpha = ptn_value<FM>(S, m.alpha, is.st).x;
        float ap = 1.f - ((1.f - alpha) * alphaTweak);
        b0.rho = ptn_value<FM>(S, m.rho_s, is.st);
        b0.eta = ptn_value<FM>(S, m.eta, is.st).x;
        if (ap > 0.0001f) { b0.type = B_TS; b0.flags = F_GLOSSY; b0.a0 = gmax(0.0001f, alpha); b0.ap = ap; }
        else { b0.type = B_SPECULAR; b0.flags = F_SPECULAR; }
    } else if (FM & FT_PLASTIC) {  // NART_MAT_PLASTIC: plasticmaterial.cpp:12-51
        float alpha = ptn_value<FM>(S, m.alpha, is.st).x;
        float ap = 1.f - ((1.f - alpha) * alphaTweak);
        f3 rho_d = ptn_value<FM>(S, m.rho_d, is.st);
        f3 rho_s = ptn_value<FM>(S, m.rho_s, is.st);
        float eta = ptn_value<FM>(S, m.eta, is.st).x;
        b0.type = B_LAMBERT;
        b0.flags = F_DIFFUSE;
        b0.rho = rho_d;
        BxDF& b1 = bs.b[1];
        b1.rho = rho_s;
        b1.tau = F3(0.f, 0.f, 0.f);
        b1.eta = eta;
        if (ap > 0.001f) { b1.type = B_TS; b1.flags = F_GLOSSY; b1.a0 = gmax(0.0001f, alpha); b1.ap = ap; }
        else { b1.type = B_SPECULAR; b1.flags = F_SPECULAR; b1.a0 = 0.f; b1.ap = 0.f; }
    }
}

// ---------------------------------------------------------------- lights
NHD uint32_t binary_search(float value, const float* v, uint32_t start, uint32_t end) {  // util.cpp:4-20
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
// BinarySearch through a guide table: util.cpp's loop returns ub - 1, ub = the first j in
// [start, end) with v[j] > value (end if none), whichever probes it takes; ub is monotone in value,
// so for value in guide cell c it lies in [a_c, b_c] (the bounds of the cell's end values, build_env)
// and a search of that range finds the same ub.  Two or three dependent loads instead of ~10.
NHD uint32_t guided_search(float value, const float* v, uint32_t start, uint32_t end, const uint32_t* guide) {
    if (!guide || start >= end || !(value >= 0.f)) return binary_search(value, v, start, end);
    const uint32_t c0 = f2u32(value * (float)NART_ENV_GUIDE_K);
    const uint32_t c = c0 < NART_ENV_GUIDE_K - 1u ? c0 : NART_ENV_GUIDE_K - 1u;
    const uint32_t g = guide[c];
    uint32_t lo = start + (g & 0xFFFFu), hi = start + (g >> 16);
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (v[mid] > value) hi = mid;
        else lo = mid + 1u;
    }
    return lo - 1u;
}
ND float env_pdf(const DEnvDist& d, f2 s) {  // texturepattern.cpp:104-109
    uint32_t u = f2u32(s.x * (float)d.w);
    uint32_t v = f2u32(s.y * (float)d.h);
    return d.mpdf[v] * d.cpdf[v * d.w + u];
}
ND f2 env_sample(const DEnvDist& d, f2 s, float& pdf) {  // texturepattern.cpp:72-102
    uint32_t lb = guided_search(s.y, d.mcdf, 0, d.h, d.mguide);
    float uc = 0.f;
    float vc = ((s.y - d.mcdf[lb]) / d.mpdf[lb]) + ((float)lb * d.invH);
    vc = gmin(vc, 0.9999999f);
    uint32_t v = f2u32(vc * (float)d.h);
    if (d.mpdf[v] > 0.f) {
        lb = guided_search(s.x, d.ccdf, v * (d.w + 1), v * (d.w + 1) + d.w,
                           d.cguide ? d.cguide + (size_t)v * NART_ENV_GUIDE_K : nullptr);
        lb %= (d.w + 1);
        uc = ((s.x - d.ccdf[v * (d.w + 1) + lb]) / d.cpdf[v * d.w + lb]) + ((float)lb * d.invW);
        uc = gmin(uc, 0.9999999f);
        uint32_t u = f2u32(uc * (float)d.w);
        pdf = d.mpdf[v] * d.cpdf[v * d.w + u];
    }
    return F2(uc, vc);
}

// Disk / ring Pdf (disklight.cpp:62-104, ringlight.cpp:66-112); sets st and tMax on a hit.
template <uint32_t FM = FT_ALL>
ND float area_pdf(const DLight& L, f3 p, f3 wi, f2& st, float& tMax) {
    f3 n = load3(L.n);
    if (dot(wi, n) >= 0.f) return 0.f;
    float t = (L.D - dot(p, n)) / dot(wi, n);
    if (t < 0.f) return 0.f;
    f3 pHit = add(p, muls(wi, t));
    f3 c2p = sub(pHit, load3(L.center));
    f4 c4 = F4(c2p.x, c2p.y, c2p.z, 0.f);
    float u = dot4(c4, F4(L.axu[0], L.axu[1], L.axu[2], L.axu[3])) / L.radius;
    float v = dot4(c4, F4(L.axv[0], L.axv[1], L.axv[2], L.axv[3])) / L.radius;
    u = (u + 1.f) * 0.5f;
    v = (v + 1.f) * 0.5f;
    st = F2(u, 1.f - v);
    float dist = c2p.x * c2p.x + c2p.y * c2p.y + c2p.z * c2p.z;
    if (dist > L.r2) return 0.f;
    if ((FM & FT_RING) && L.type == NART_LIGHT_RING && dist < L.ri2) return 0.f;
    float pdf = L.pdf_area;
    pdf = pdf * ((t * t) / dot(neg(wi), n));
    tMax = t;
    return pdf;
}
}  // namespace nd

#include "envlight.h"
