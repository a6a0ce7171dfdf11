// Device-side BVH build (the reference builds its octree on the host,
// bvh.cpp:252-326): a linear BVH over the visible triangles, in the same node / triangle-record
// format as the host's binned-SAH build (host/bvh_build.cpp), so every traversal kernel and the
// octree emulation run unchanged.  Only the closest hit must match the reference, and the
// traversal is exact for any tree (the parity tests render with both builds), so the tree's
// shape is a performance choice: the SAH tree traces faster, this one builds in about a
// millisecond for meshes far larger than any the reference ships.
//
//   1. k_lbvh_prims     per visible triangle: bounds, centroid
//   2. k_lbvh_bounds    centroid bounds (block reduction + one block)
//   3. k_lbvh_morton    30-bit Morton code of the centroid; radix sort (hipcub) by code
//   4. leaves           runs of up to LBVH_LEAF consecutive sorted triangles
//   5. k_lbvh_karras    inner nodes over the leaves (Karras 2012, ties broken by leaf index)
//   6. k_lbvh_refit     child boxes bottom-up (the second child to arrive at a node merges)
//   7. k_lbvh_depth     node depth (walk to the root); sort by depth = breadth-first order,
//                       so any prefix of the node array is the top of the tree (LDS staging)
//   8. k_lbvh_emit      BVHNode records (padded child boxes, remapped child codes)
//   9. k_lbvh_tris      64-B triangle test records in leaf order, with the reference's float
//                       order for n = cross(v1 - v0, v2 - v0) and dot(v0, n) (geometry.cpp:33-37)
#pragma once

#include "dmath.h"
#include "dscene.h"

namespace nd {

#define LBVH_LEAF 4

struct LbvhPrim {
    float lo[3], hi[3], c[3];
    uint32_t g;
};

__global__ void k_lbvh_prims(const nart_triangle* tris, const uint32_t* vis, uint32_t m, LbvhPrim* prims) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t g = vis[i];
    const nart_triangle& T = tris[g];
    LbvhPrim p;
    for (int k = 0; k < 3; ++k) {
        p.lo[k] = fminf(fminf(T.v0[k], T.v1[k]), T.v2[k]);
        p.hi[k] = fmaxf(fmaxf(T.v0[k], T.v1[k]), T.v2[k]);
        p.c[k] = 0.5f * (p.lo[k] + p.hi[k]);
    }
    p.g = g;
    prims[i] = p;
}

// centroid bounds: partial[block] = {lo[3], hi[3]}, then one block folds the partials into out[6]
__global__ void k_lbvh_bounds(const LbvhPrim* prims, uint32_t m, float* partial) {
    __shared__ float s[6][256];
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x)
        for (int k = 0; k < 3; ++k) {
            lo[k] = fminf(lo[k], prims[i].c[k]);
            hi[k] = fmaxf(hi[k], prims[i].c[k]);
        }
    for (int k = 0; k < 3; ++k) {
        s[k][threadIdx.x] = lo[k];
        s[3 + k][threadIdx.x] = hi[k];
    }
    __syncthreads();
    for (uint32_t w = blockDim.x / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            for (int k = 0; k < 3; ++k) {
                s[k][threadIdx.x] = fminf(s[k][threadIdx.x], s[k][threadIdx.x + w]);
                s[3 + k][threadIdx.x] = fmaxf(s[3 + k][threadIdx.x], s[3 + k][threadIdx.x + w]);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) partial[blockIdx.x * 6 + threadIdx.x] = s[threadIdx.x][0];
}

__global__ void k_lbvh_bounds_final(float* partial, uint32_t nblocks) {
    if (threadIdx.x != 0) return;
    float b[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = 0; i < nblocks; ++i)
        for (int k = 0; k < 3; ++k) {
            b[k] = fminf(b[k], partial[i * 6 + k]);
            b[3 + k] = fmaxf(b[3 + k], partial[i * 6 + 3 + k]);
        }
    for (int k = 0; k < 6; ++k) partial[k] = b[k];
}

ND uint32_t lbvh_spread10(uint32_t v) {  // 10 bits -> every third bit
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__global__ void k_lbvh_morton(const LbvhPrim* prims, uint32_t m, const float* cb, uint32_t* keys, uint32_t* vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    uint32_t q[3];
    for (int k = 0; k < 3; ++k) {
        const float ext = cb[3 + k] - cb[k];
        const float u = ext > 0.f ? (prims[i].c[k] - cb[k]) / ext : 0.5f;
        q[k] = (uint32_t)fminf(fmaxf(u * 1024.f, 0.f), 1023.f);
    }
    keys[i] = (lbvh_spread10(q[0]) << 2) | (lbvh_spread10(q[1]) << 1) | lbvh_spread10(q[2]);
    vals[i] = i;
}

// Karras: common-prefix length of leaves i and j (keys = Morton code of the leaf's first
// triangle, extended by the leaf index so that every key is distinct); -1 out of range.
ND int lbvh_delta(const uint32_t* lkey, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const uint32_t a = lkey[i], b = lkey[j];
    if (a != b) return __clz(a ^ b);
    return 32 + __clz((uint32_t)i ^ (uint32_t)j);
}

// inner node i of n - 1 (n >= 2 leaves): children as (index | leaf flag), parents of both
__global__ void k_lbvh_karras(const uint32_t* lkey, int n, int2* child, int* parent_inner, int* parent_leaf) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (lbvh_delta(lkey, n, i, i + 1) - lbvh_delta(lkey, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = lbvh_delta(lkey, n, i, i - d);
    int lmax = 2;
    while (lbvh_delta(lkey, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
        if (lbvh_delta(lkey, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = lbvh_delta(lkey, n, i, j);
    int s = 0;
    for (int t = (l + 1) / 2;; t = (t + 1) / 2) {
        if (lbvh_delta(lkey, n, i, i + (s + t) * d) > dnode) s += t;
        if (t == 1) break;
    }
    const int gamma = i + s * d + min(d, 0);
    const int first = min(i, j), last = max(i, j);
    const bool lleaf = first == gamma, rleaf = last == gamma + 1;
    child[i] = make_int2(lleaf ? ~gamma : gamma, rleaf ? ~(gamma + 1) : gamma + 1);
    if (lleaf) parent_leaf[gamma] = i;
    else parent_inner[gamma] = i;
    if (rleaf) parent_leaf[gamma + 1] = i;
    else parent_inner[gamma + 1] = i;
}

struct LbvhBox {
    float lo[3], hi[3];
};

ND LbvhBox lbvh_leaf_box(const LbvhPrim* prims, uint32_t m, int leaf) {
    LbvhBox b;
    for (int k = 0; k < 3; ++k) {
        b.lo[k] = INFINITY;
        b.hi[k] = -INFINITY;
    }
    const uint32_t f = (uint32_t)leaf * LBVH_LEAF, e = min(m, f + LBVH_LEAF);
    for (uint32_t t = f; t < e; ++t)
        for (int k = 0; k < 3; ++k) {
            b.lo[k] = fminf(b.lo[k], prims[t].lo[k]);
            b.hi[k] = fmaxf(b.hi[k], prims[t].hi[k]);
        }
    return b;
}

// bottom-up boxes: one thread per leaf walks to the root; at each inner node the first arrival
// stops, the second (whose sibling's box is then complete) merges both children and goes on
__global__ void k_lbvh_refit(const LbvhPrim* sorted, uint32_t m, int n, const int2* child, const int* parent_inner,
                             const int* parent_leaf, LbvhBox* box, uint32_t* flag) {
    const int leaf = blockIdx.x * blockDim.x + threadIdx.x;
    if (leaf >= n) return;
    int node = parent_leaf[leaf];
    while (node >= 0) {
        __threadfence();
        if (atomicAdd(&flag[node], 1u) == 0u) return;
        __threadfence();
        const int2 c = child[node];
        // the sibling's box was stored by another workgroup: agent-scope loads (not through L1)
        auto inner_box = [&](int k) {
            LbvhBox r;
            for (int a = 0; a < 3; ++a) {
                r.lo[a] = __hip_atomic_load(&box[k].lo[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                r.hi[a] = __hip_atomic_load(&box[k].hi[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return r;
        };
        LbvhBox b0 = c.x < 0 ? lbvh_leaf_box(sorted, m, ~c.x) : inner_box(c.x);
        LbvhBox b1 = c.y < 0 ? lbvh_leaf_box(sorted, m, ~c.y) : inner_box(c.y);
        LbvhBox b;
        for (int k = 0; k < 3; ++k) {
            b.lo[k] = fminf(b0.lo[k], b1.lo[k]);
            b.hi[k] = fmaxf(b0.hi[k], b1.hi[k]);
        }
        // written through to L2 (agent scope) before the flag of the parent is taken
        __hip_atomic_store(&box[node].lo[0], b.lo[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&box[node].lo[1], b.lo[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&box[node].lo[2], b.lo[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&box[node].hi[0], b.hi[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&box[node].hi[1], b.hi[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&box[node].hi[2], b.hi[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        node = parent_inner[node];
    }
}

// depth of every inner node (root 0) as the sort key of the breadth-first order; max depth
__global__ void k_lbvh_depth(const int* parent_inner, int ninner, uint32_t* keys, uint32_t* vals, uint32_t* maxd) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ninner) return;
    uint32_t d = 0;
    for (int a = parent_inner[i]; a >= 0; a = parent_inner[a]) ++d;
    keys[i] = d;
    vals[i] = (uint32_t)i;
    atomicMax(maxd, d);
}

__global__ void k_lbvh_remap(const uint32_t* order, int ninner, int* remap) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < ninner) remap[order[r]] = r;
}

// BVHNode r = inner node order[r]: child boxes padded by `pad`, child codes remapped (leaf code
// ~(first << 5 | (count - 1)) over the sorted triangle records)
__global__ void k_lbvh_emit(const uint32_t* order, int ninner, const int2* child, const int* remap, const LbvhBox* box,
                            const LbvhPrim* sorted, uint32_t m, float pad, BVHNode* out) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= ninner) return;
    const int i = (int)order[r];
    const int2 c = child[i];
    BVHNode o;
    const int cc[2] = {c.x, c.y};
    for (int s = 0; s < 2; ++s) {
        LbvhBox b;
        int code;
        if (cc[s] < 0) {
            const int leaf = ~cc[s];
            b = lbvh_leaf_box(sorted, m, leaf);
            const uint32_t f = (uint32_t)leaf * LBVH_LEAF, cnt = min(m, f + LBVH_LEAF) - f;
            code = ~(int)((f << 5) | (cnt - 1));
        } else {
            b = box[cc[s]];
            code = remap[cc[s]];
        }
        float* lo = s == 0 ? o.lo0 : o.lo1;
        float* hi = s == 0 ? o.hi0 : o.hi1;
        for (int k = 0; k < 3; ++k) {
            lo[k] = b.lo[k] - pad;
            hi[k] = b.hi[k] + pad;
        }
        o.child[s] = code;
    }
    o.pad[0] = o.pad[1] = 0;
    out[r] = o;
}

__global__ void k_lbvh_gather(const LbvhPrim* prims, const uint32_t* order, uint32_t m, LbvhPrim* sorted) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) sorted[i] = prims[order[i]];
}

// leaf keys: Morton code of each leaf's first triangle
__global__ void k_lbvh_leaf_keys(const uint32_t* codes, uint32_t m, int n, uint32_t* lkey) {
    const int l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l < n) lkey[l] = codes[(uint32_t)l * LBVH_LEAF];
}

// triangle test records in leaf order (host/bvh_build.cpp build_bvh + annotate_octree_leaves:
// `info` = the octree leaf | inside bit of every scene triangle, host-computed)
__global__ void k_lbvh_tris(const nart_triangle* tris, const LbvhPrim* sorted, uint32_t m, const uint32_t* info,
                            float* rec) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t g = sorted[i].g;
    const nart_triangle& T = tris[g];
    const float e1[3] = {T.v1[0] - T.v0[0], T.v1[1] - T.v0[1], T.v1[2] - T.v0[2]};
    const float e2[3] = {T.v2[0] - T.v0[0], T.v2[1] - T.v0[1], T.v2[2] - T.v0[2]};
    const float n[3] = {e1[1] * e2[2] - e2[1] * e1[2], e1[2] * e2[0] - e2[2] * e1[0], e1[0] * e2[1] - e2[0] * e1[1]};
    const float d0 = (T.v0[0] * n[0] + T.v0[1] * n[1]) + T.v0[2] * n[2];
    float* r = rec + (size_t)i * 16;
    r[0] = n[0]; r[1] = n[1]; r[2] = n[2]; r[3] = d0;
    r[4] = T.v0[0]; r[5] = T.v0[1]; r[6] = T.v0[2]; r[7] = T.v1[0];
    r[8] = T.v1[1]; r[9] = T.v1[2]; r[10] = T.v2[0]; r[11] = T.v2[1];
    r[12] = T.v2[2];
    r[13] = __uint_as_float(g);
    r[14] = __uint_as_float(info[g]);
    r[15] = sqrtf((n[0] * n[0] + n[1] * n[1]) + n[2] * n[2]) * 0.125f;
}

// per-axis permuted vertex blocks + plane (render.hip nart_hip_create's tri_perm layout)
__global__ void k_lbvh_perm(const float* rec, uint32_t nt, float* perm) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nt) return;
    const float* r = rec + (size_t)i * 16;
    for (int m = 0; m < 3; ++m) {
        const int kx = (m + 1) % 3, ky = (m + 2) % 3, kz = m;
        float* o = perm + ((size_t)m * nt + i) * 16;
        for (int k = 0; k < 3; ++k) {
            const float* v = r + 4 + 3 * k;
            o[3 * k + 0] = v[kx];
            o[3 * k + 1] = v[ky];
            o[3 * k + 2] = v[kz];
        }
        o[9] = r[13];
        o[10] = r[14];
        o[11] = r[15];
        for (int k = 0; k < 4; ++k) o[12 + k] = r[k];
    }
}

}  // namespace nd
