// Exact reproduction of the reference octree's answer (Octree::Intersect, bvh.cpp:132-176) on
// top of the device BVH2.
//
// The device BVH finds the true closest hit g* (t*) among the triangles the octree can reach.
// The octree returns the same hit iff g*'s leaf is processed, i.e.
//   (1) the leaf and every inner ancestor pass BoundingVolume::Intersect (bvh.cpp:23-60), which
//       uses unpadded boxes and divisions, so it can reject a box whose face the hit lies on;
//   (2) every inner ancestor A below the root is popped before the search stops: the search
//       stops once the best hit so far is closer than the heap top's entry distance, so A is
//       popped whenever A.key <= every hit the octree could have found before A -- any hit
//       other than g* (lower bound L2, see trav_step) or the query's initial tMax;
// and no second triangle decides the result: no exact distance tie with g* (the octree keeps the
// first chunk it visits) and no NaN plane distance (Triangle::Intersect lets NaN through,
// geometry.cpp:37-39, which changes what its chunk returns).
// oc_resolve checks (1)-(2) cheaply when the hit point is clear of its leaf box's faces,
// exactly along the leaf's ancestor chain otherwise, and replays the octree search itself
// (oc_replay: the reference's best-first search with a binary heap in a global pool) when
// neither proves the answer or a tie / NaN was seen.  Any-hit (shadow) queries are the
// reference's closest-hit search with tMax preset (pathintegrator.cpp:83-85): a proven hit
// means occluded.
#pragma once

#include "dscene.h"

namespace nd {

#define OC_INF __builtin_inff()

// glm::dot(v, axis) for the unit axes, as BoundingVolume::Intersect evaluates it (bvh.cpp:29-32)
ND void oc_axes(const Ray& r, float* oa, float* da) {
    oa[0] = (r.o.x * 1.f + r.o.y * 0.f) + r.o.z * 0.f;
    oa[1] = (r.o.x * 0.f + r.o.y * 1.f) + r.o.z * 0.f;
    oa[2] = (r.o.x * 0.f + r.o.y * 0.f) + r.o.z * 1.f;
    da[0] = (r.d.x * 1.f + r.d.y * 0.f) + r.d.z * 0.f;
    da[1] = (r.d.x * 0.f + r.d.y * 1.f) + r.d.z * 0.f;
    da[2] = (r.d.x * 0.f + r.d.y * 0.f) + r.d.z * 1.f;
}

// BoundingVolume::Intersect (bvh.cpp:23-60), IEEE divisions
ND bool oc_bv(const OcNode* N, const float* oa, const float* da, float& te) {
    float tMin = -OC_INF, tMax = OC_INF;
    for (int i = 0; i < 3; ++i) {
        float s0 = (N->bmin[i] - oa[i]) / da[i];
        float s1 = (N->bmax[i] - oa[i]) / da[i];
        if (s0 > s1) {
            const float x = s0;
            s0 = s1;
            s1 = x;
        }
        if (s0 > tMax || tMin > s1) return false;
        tMin = gmax(tMin, s0);
        tMax = gmin(tMax, s1);
    }
    te = tMin;
    return true;
}

// True when (1)-(2) hold for the hit (t, leaf L) without exact arithmetic: the hit point is
// inside L's box by a margin (64 ulps of the coordinates) on every axis where the box has
// extent, so every ancestor's slab test passes and its entry distance is below t.  On an axis
// where L is flat (a box around coplanar triangles) the slab is the single distance tf, which
// is computed exactly; the point at tf must then be clear of the other faces and tf <= bound.
ND bool oc_clear(const OcNode* L, const Ray& r, float t, float bound) {
    const float o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
    int flat = -1;
    for (int k = 0; k < 3; ++k)
        if (L->bmin[k] == L->bmax[k]) {
            if (flat >= 0) return false;
            flat = k;
        }
    float tp = t;
    if (flat >= 0) {
        const float da = flat == 0 ? (r.d.x * 1.f + r.d.y * 0.f) + r.d.z * 0.f
                                   : (flat == 1 ? (r.d.x * 0.f + r.d.y * 1.f) + r.d.z * 0.f
                                                : (r.d.x * 0.f + r.d.y * 0.f) + r.d.z * 1.f);
        const float oa = flat == 0 ? (r.o.x * 1.f + r.o.y * 0.f) + r.o.z * 0.f
                                   : (flat == 1 ? (r.o.x * 0.f + r.o.y * 1.f) + r.o.z * 0.f
                                                : (r.o.x * 0.f + r.o.y * 0.f) + r.o.z * 1.f);
        tp = (L->bmin[flat] - oa) / da;
        if (!(tp <= bound) || !(tp >= 0.f)) return false;  // also rejects NaN / inf
    }
    for (int k = 0; k < 3; ++k) {
        if (k == flat) continue;
        const float p = o[k] + tp * d[k];
        const float m = (fabsf(o[k]) + fabsf(tp * d[k])) * 0x1p-17f + 1e-30f;
        if (!(p - L->bmin[k] >= m) || !(L->bmax[k] - p >= m)) return false;
    }
    return true;
}

// (1)-(2) evaluated exactly along the leaf's ancestor chain.
ND bool oc_verify(const DScene& S, const Ray& r, int leaf, float bound) {
    float oa[3], da[3];
    oc_axes(r, oa, da);
    float key;
    if (!oc_bv(S.oc_nodes + leaf, oa, da, key)) return false;
    int a = S.oc_nodes[leaf].parent;
    while (a >= 0 && a != S.oc_root) {
        const OcNode* A = S.oc_nodes + a;
        if (!oc_bv(A, oa, da, key) || !(key <= bound)) return false;
        a = A->parent;
    }
    return true;
}

// --- replay: Octree::Intersect itself -------------------------------------------------------
// Heap entries (tEntry, node), ordered by tEntry then node creation index (the reference orders
// equal keys by node address; see oracle/nart_oracle.c qless).  The pool slots are shared by
// all lanes of the device, so entries are accessed with agent-scope atomics (coherent across
// XCDs) and a slot is owned under a lock word.
ND unsigned long long oc_pack(float key, int node) {
    return (unsigned long long)__float_as_uint(key) | ((unsigned long long)(uint32_t)node << 32);
}
ND bool oc_less(unsigned long long a, unsigned long long b) {
    const float ka = __uint_as_float((uint32_t)a), kb = __uint_as_float((uint32_t)b);
    return ka < kb || (!(kb < ka) && (int32_t)(a >> 32) < (int32_t)(b >> 32));
}
ND unsigned long long oc_ld(unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
ND void oc_st(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
ND void oc_push(unsigned long long* h, uint32_t& n, unsigned long long x) {
    uint32_t i = n++;
    while (i > 0) {
        const uint32_t p = (i - 1) / 2;
        const unsigned long long hp = oc_ld(h + p);
        if (!oc_less(x, hp)) break;
        oc_st(h + i, hp);
        i = p;
    }
    oc_st(h + i, x);
}
ND unsigned long long oc_pop(unsigned long long* h, uint32_t& n) {
    const unsigned long long top = oc_ld(h);
    const unsigned long long x = oc_ld(h + (--n));
    uint32_t i = 0;
    for (;;) {
        const uint32_t l = 2 * i + 1, rr = l + 1;
        uint32_t m = i;
        unsigned long long best = x;
        if (l < n) {
            const unsigned long long hl = oc_ld(h + l);
            if (oc_less(hl, best)) {
                m = l;
                best = hl;
            }
        }
        if (rr < n) {
            const unsigned long long hr = oc_ld(h + rr);
            if (oc_less(hr, best)) {
                m = rr;
                best = hr;
            }
        }
        if (m == i) break;
        oc_st(h + i, best);
        i = m;
    }
    if (n) oc_st(h + i, x);
    return top;
}

// Chunk::Intersect (bvh.cpp:66-79) with a fresh isect: Triangle::Intersect's distance test
// first (NaN passes), then the edge test; the last accepted triangle wins.
ND bool oc_chunk(const DScene& S, const Ray& r, uint32_t first, uint32_t count, float& tc, uint32_t& gc) {
    bool hit = false;
    tc = OC_INF;
    for (uint32_t k = 0; k < count; ++k) {
        const uint32_t g = S.oc_tris[first + k];
        const nart_triangle& T = S.tris[g];
        const f3 v0 = F3(T.v0[0], T.v0[1], T.v0[2]), v1 = F3(T.v1[0], T.v1[1], T.v1[2]),
                 v2 = F3(T.v2[0], T.v2[1], T.v2[2]);
        const f3 n = cross(sub(v1, v0), sub(v2, v0));
        const float t = (dot(v0, n) - dot(r.o, n)) / dot(r.d, n);
        if (t <= 0.f || t >= tc) continue;
        float e0, e1, e2;
        edge_functions(r, v0, v1, v2, e0, e1, e2);
        if (!edges_accept(e0, e1, e2)) continue;
        tc = t;
        gc = g;
        hit = true;
    }
    return hit;
}

ND void oc_replay(const DScene& S, const Ray& r, float tmax, float& bestT, uint32_t& bestG) {
    // The lanes of a wave that replay together share one pool entry of 64 heaps (one per lane),
    // acquired by their lowest lane alone.  A lane never spins on a lock held by a wave-mate
    // (wave-mates parked at the reconvergence point would never release it), and a holder waits
    // for nothing until it releases, so every acquisition ends however small the pool.
    const unsigned long long act = __ballot(1);
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int lane = (int)__lane_id();
    uint32_t ws = 0;
    if (lane == leader) {
        ws = (uint32_t)(((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 2654435761u) % S.oc_pool;
        for (;;) {
            uint32_t expect = 0u;
            if (__hip_atomic_compare_exchange_strong(S.oc_lock + ws, &expect, 1u, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT))
                break;
            ws = ws + 1 == S.oc_pool ? 0 : ws + 1;
        }
    }
    ws = (uint32_t)__shfl((int)ws, leader);
    // a lane only reads heap entries it wrote during this replay (push before pop), so nothing a
    // previous owner left behind is ever read
    unsigned long long* h = S.oc_heap + ((size_t)ws * 64 + (size_t)lane) * S.oc_cap;
    float oa[3], da[3];
    oc_axes(r, oa, da);
    uint32_t n = 0;
    oc_push(h, n, oc_pack(OC_INF, S.oc_root));
    float isT = tmax;
    uint32_t isG = NO_HIT;
    while (n) {
        const unsigned long long cur = oc_pop(h, n);
        const OcNode* N = S.oc_nodes + (int32_t)(cur >> 32);
        for (int c = 0; c < 8; ++c) {
            const int ch = N->children[c];
            if (ch < 0) continue;
            const OcNode* C = S.oc_nodes + ch;
            float te;
            if (!oc_bv(C, oa, da, te)) continue;
            oc_push(h, n, oc_pack(te, ch));
            if (!C->is_leaf) continue;
            for (uint32_t k = 0; k < C->chunk_count; ++k) {
                const uint32_t cf = S.oc_chunks[2 * (C->chunk_first + k)];
                const uint32_t cn = S.oc_chunks[2 * (C->chunk_first + k) + 1];
                float tc;
                uint32_t gc;
                if (oc_chunk(S, r, cf, cn, tc, gc) && tc < isT) {
                    isT = tc;
                    isG = gc;
                }
            }
        }
        if (n && isT < __uint_as_float((uint32_t)oc_ld(h))) break;
    }
    // every lane that entered has left the search loop (reconverged here)
    if (lane == leader) __hip_atomic_store(S.oc_lock + ws, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    bestT = isT;
    bestG = isG;
}

// The rare part of oc_resolve, out of line so that the path kernels' register allocation
// around their three traversal sites is not shaped by it.
ND void oc_slow(const DScene& S, const Ray& r, float tmax, bool replay, int leaf, float bound,
                                     float& bestT, uint32_t& bestG, uint32_t* cnt) {
    if (!replay) {
        cnt[0]++;
        if (oc_verify(S, r, leaf, bound)) return;
    }
    cnt[1]++;
    oc_replay(S, r, tmax, bestT, bestG);
}

// Final answer of a query the BVH traversal resolved (bestT / bestG), made equal to the
// reference octree's.  risky: a NaN distance or an exact tie was seen; t2: lower bound of every
// hit other than the winner that the octree could find (trav_step).
template <bool COUNT>
ND void oc_resolve(const DScene& S, const Ray& r, float tmax, bool any, bool risky, uint32_t info, float t2,
                   float& bestT, uint32_t& bestG, TraceCounters& cnt) {
    if (!S.oc_exact) return;
    if (S.oc_exact == 2) risky = true;  // NART_OCTREE_EXACT=2: every query replays the octree search (tests)
    int leaf = 0;
    const float bound = any ? tmax : t2;
    if (!risky) {
        if (bestG == NO_HIT) return;     // nothing reachable: the octree finds nothing either
        if (info & 0x80000000u) return;  // triangle inside its leaf box by a margin
        leaf = (int)(info & 0x7FFFFFFFu);
        if (oc_clear(S.oc_nodes + leaf, r, bestT, bound)) return;
    }
    uint32_t c[2] = {0u, 0u};
    oc_slow(S, r, tmax, risky, leaf, bound, bestT, bestG, c);
    if (COUNT) {
        cnt.oc_checks += c[0];
        cnt.oc_replays += c[1];
    }
}

}  // namespace nd
