// Host BVH build for the nart render path: (1) the reference octree's visibility rules,
// replayed structurally (no traversal), and (2) a binned-SAH BVH2 for the device.
#include "bvh_build.h"

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <limits>

namespace nart {
namespace {

inline float gmin(float a, float b) { return (b < a) ? b : a; }
inline float gmax(float a, float b) { return (a < b) ? b : a; }
inline uint32_t f2u32(float f) {  // static_cast<uint32_t>(float), x86-64 semantics
    if (f >= 0.f && f < 4294967296.f) return (uint32_t)f;
    if (!(f > -9.2233715e18f && f < 9.2233715e18f)) return 0u;
    return (uint32_t)(int64_t)f;
}

struct V3 { float x, y, z; };
inline V3 v3(const float* a) { return {a[0], a[1], a[2]}; }
inline V3 vmin(V3 a, V3 b) { return {gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z)}; }
inline V3 vmax(V3 a, V3 b) { return {gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z)}; }

// --- reference octree replay (bvh.cpp:178-233): only what decides visibility -------------
struct ONode {
    int children[8];
    std::vector<int> chunks;
    bool isLeaf = true;
    V3 nmin, nmax;
};
struct Octree {
    std::vector<ONode> nodes;
    std::vector<V3> cmin, cmax;  // chunk bboxes
    int add(V3 a, V3 b) {
        ONode n;
        for (int& c : n.children) c = -1;
        n.nmin = a;
        n.nmax = b;
        nodes.push_back(n);
        return (int)nodes.size() - 1;
    }
    void insert(int node, int chunk, uint8_t depth) {
        if (nodes[node].isLeaf) {
            if (nodes[node].chunks.empty() || depth >= 5) {
                nodes[node].chunks.push_back(chunk);
            } else {
                nodes[node].isLeaf = false;
                for (uint32_t i = 0; i < nodes[node].chunks.size(); ++i) {
                    int back = nodes[node].chunks.back();
                    insert(node, back, depth++);
                    nodes[node].chunks.pop_back();
                }
                insert(node, chunk, depth++);
            }
        } else {
            V3 a = cmin[chunk], b = cmax[chunk];
            V3 cc = {a.x + (b.x - a.x) * 0.5f, a.y + (b.y - a.y) * 0.5f, a.z + (b.z - a.z) * 0.5f};
            V3 nm = nodes[node].nmin, nx = nodes[node].nmax;
            V3 nc = {nm.x + (nx.x - nm.x) * 0.5f, nm.y + (nx.y - nm.y) * 0.5f, nm.z + (nx.z - nm.z) * 0.5f};
            uint8_t idx = 0;
            if (cc.x > nc.x) idx |= 1;
            if (cc.y > nc.y) idx |= 2;
            if (cc.z > nc.z) idx |= 4;
            if (nodes[node].children[idx] < 0) {
                V3 sz = {(nx.x - nm.x) * 0.5f, (nx.y - nm.y) * 0.5f, (nx.z - nm.z) * 0.5f};
                V3 lo = nc, hi = nc;
                if (idx & 1) hi.x += sz.x; else lo.x -= sz.x;
                if (idx & 2) hi.y += sz.y; else lo.y -= sz.y;
                if (idx & 4) hi.z += sz.z; else lo.z -= sz.z;
                int c = add(lo, hi);
                nodes[node].children[idx] = c;
            }
            insert(nodes[node].children[idx], chunk, depth++);
        }
    }
};

// glm::dot(v, axis) for the unit axes (bvh.cpp:95-100): (x*a.x + y*a.y) + z*a.z
inline float axdot(const V3& v, int i) {
    const float a[3] = {i == 0 ? 1.f : 0.f, i == 1 ? 1.f : 0.f, i == 2 ? 1.f : 0.f};
    return (v.x * a[0] + v.y * a[1]) + v.z * a[2];
}

// BoundingVolume of every node (Chunk::Chunk bvh.cpp:81-113, BuildBVs bvh.cpp:235-250) and the
// node / chunk / triangle tables of the device-side replay.
void export_octree(const nart_scene_blob& blob, const Octree& o, const std::vector<std::vector<uint32_t>>& chunks,
                   int root, RefOctree& out) {
    const float inf = std::numeric_limits<float>::infinity();
    std::vector<V3> cbmin(chunks.size(), V3{inf, inf, inf}), cbmax(chunks.size(), V3{-inf, -inf, -inf});
    for (size_t c = 0; c < chunks.size(); ++c)
        for (uint32_t g : chunks[c]) {
            const nart_triangle& T = blob.triangles[g];
            V3 vs[3] = {v3(T.v0), v3(T.v1), v3(T.v2)};
            float* lo = &cbmin[c].x;
            float* hi = &cbmax[c].x;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    const float d = axdot(vs[j], i);
                    lo[i] = gmin(d, lo[i]);
                    hi[i] = gmax(d, hi[i]);
                }
        }
    const size_t n = o.nodes.size();
    out.nodes.assign(n, nd::OcNode{});
    out.chunks.clear();
    out.tris.clear();
    out.tri_leaf.assign(blob.num_triangles, -1);
    out.root = root;
    for (size_t i = 0; i < n; ++i) {
        nd::OcNode& d = out.nodes[i];
        for (int k = 0; k < 3; ++k) {
            d.bmin[k] = inf;
            d.bmax[k] = -inf;
        }
        d.parent = -1;
        d.is_leaf = o.nodes[i].isLeaf ? 1 : 0;
        for (int c = 0; c < 8; ++c) d.children[c] = o.nodes[i].children[c];
    }
    for (size_t i = 0; i < n; ++i)
        for (int c = 0; c < 8; ++c)
            if (o.nodes[i].children[c] >= 0) out.nodes[o.nodes[i].children[c]].parent = (int32_t)i;
    // bottom-up extension in BuildBVs' order: leaves over their chunks, inner nodes over children 0..7
    struct Rec {
        static void go(const Octree& o, const std::vector<V3>& cbmin, const std::vector<V3>& cbmax,
                       std::vector<nd::OcNode>& nodes, int i) {
            nd::OcNode& d = nodes[i];
            auto ext = [&](const float* lo, const float* hi) {
                for (int k = 0; k < 3; ++k) {
                    d.bmin[k] = gmin(d.bmin[k], lo[k]);
                    d.bmax[k] = gmax(d.bmax[k], hi[k]);
                }
            };
            if (o.nodes[i].isLeaf) {
                for (int c : o.nodes[i].chunks) ext(&cbmin[c].x, &cbmax[c].x);
            } else {
                for (int c = 0; c < 8; ++c) {
                    const int ch = o.nodes[i].children[c];
                    if (ch < 0) continue;
                    go(o, cbmin, cbmax, nodes, ch);
                    ext(nodes[ch].bmin, nodes[ch].bmax);
                }
            }
        }
    };
    Rec::go(o, cbmin, cbmax, out.nodes, root);
    for (size_t i = 0; i < n; ++i) {
        nd::OcNode& d = out.nodes[i];
        d.chunk_first = (uint32_t)(out.chunks.size() / 2);
        d.chunk_count = 0;
        if (!o.nodes[i].isLeaf) continue;  // chunks left in a split node are orphaned (bvh.cpp:187-190)
        for (int c : o.nodes[i].chunks) {
            out.chunks.push_back((uint32_t)out.tris.size());
            out.chunks.push_back((uint32_t)chunks[c].size());
            for (uint32_t g : chunks[c]) {
                out.tris.push_back(g);
                out.tri_leaf[g] = (int32_t)i;
            }
            ++d.chunk_count;
        }
    }
}

}  // namespace

uint32_t reference_visibility(const nart_scene_blob& blob, std::vector<uint8_t>& mask, bool& root_is_leaf,
                              uint32_t& n_chunks, RefOctree* octree) {
    const float inf = std::numeric_limits<float>::infinity();
    uint32_t numTriangles = 0;
    V3 sMax = {-inf, -inf, -inf}, sMin = {inf, inf, inf};
    for (uint32_t m = 0; m < blob.num_meshes; ++m) {
        numTriangles += blob.meshes[m].num_tris;
        for (uint32_t i = 0; i < blob.meshes[m].num_tris; ++i) {
            const nart_triangle& T = blob.triangles[blob.meshes[m].first_tri + i];
            V3 vs[3] = {v3(T.v0), v3(T.v1), v3(T.v2)};
            for (const V3& v : vs) {
                sMax = vmax(v, sMax);
                sMin = vmin(v, sMin);
            }
        }
    }
    V3 size = {sMax.x - sMin.x, sMax.y - sMin.y, sMax.z - sMin.z};
    float volume = size.x * size.y * size.z;
    float nt = (float)numTriangles;
    float third = 1.f / 3.f;
    V3 q = {(nt / volume) * 3.f, (nt / volume) * 3.f, (nt / volume) * 3.f};
    V3 res = {std::floor(size.x * std::pow(q.x, third)), std::floor(size.y * std::pow(q.y, third)),
              std::floor(size.z * std::pow(q.z, third))};
    res = {gmin(gmax(res.x, 1.f), 128.f), gmin(gmax(res.y, 1.f), 128.f), gmin(gmax(res.z, 1.f), 128.f)};
    uint32_t numChunks = f2u32(res.x * res.y * res.z);
    std::vector<std::vector<uint32_t>> chunks(size_t(numChunks) + 1);
    for (uint32_t m = 0; m < blob.num_meshes; ++m)
        for (uint32_t i = 0; i < blob.meshes[m].num_tris; ++i) {
            uint32_t g = blob.meshes[m].first_tri + i;
            const nart_triangle& T = blob.triangles[g];
            V3 tm = vmin(vmin(v3(T.v0), v3(T.v1)), v3(T.v2));
            tm = {tm.x - sMin.x, tm.y - sMin.y, tm.z - sMin.z};
            V3 cc = {std::floor((tm.x / size.x) * res.x), std::floor((tm.y / size.y) * res.y),
                     std::floor((tm.z / size.z) * res.z)};
            uint32_t ci = f2u32(std::floor(cc.x * res.y * res.z + cc.y * res.z + cc.x));  // bvh.cpp:304-306
            ci = (numChunks < ci) ? numChunks : ci;
            chunks[ci].push_back(g);
        }
    Octree o;
    int root = o.add(sMin, sMax);
    o.cmin.resize(chunks.size());
    o.cmax.resize(chunks.size());
    n_chunks = 0;
    for (size_t c = 0; c < chunks.size(); ++c) {
        if (chunks[c].empty()) continue;
        ++n_chunks;
        V3 a = {inf, inf, inf}, b = {-inf, -inf, -inf};
        for (uint32_t g : chunks[c]) {
            const nart_triangle& T = blob.triangles[g];
            V3 vs[3] = {v3(T.v0), v3(T.v1), v3(T.v2)};
            for (const V3& v : vs) {
                a = vmin(a, v);
                b = vmax(b, v);
            }
        }
        o.cmin[c] = a;
        o.cmax[c] = b;
        o.insert(root, (int)c, 0);
    }
    mask.assign(blob.num_triangles, 0);
    root_is_leaf = o.nodes[root].isLeaf;
    if (octree) export_octree(blob, o, chunks, root, *octree);
    if (root_is_leaf) return 0;
    uint32_t vis = 0;
    for (const ONode& n : o.nodes)
        if (n.isLeaf)
            for (int c : n.chunks)
                for (uint32_t g : chunks[c]) {
                    mask[g] = 1;
                    ++vis;
                }
    return vis;
}

namespace {

struct BTri {
    float lo[3], hi[3], c[3];
    uint32_t g;
};
struct Box {
    float lo[3] = {std::numeric_limits<float>::infinity(), std::numeric_limits<float>::infinity(),
                   std::numeric_limits<float>::infinity()};
    float hi[3] = {-std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                   -std::numeric_limits<float>::infinity()};
    void grow(const float* a, const float* b) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], a[k]);
            hi[k] = std::max(hi[k], b[k]);
        }
    }
    void grow(const Box& o) { grow(o.lo, o.hi); }
    float area() const {
        if (!(hi[0] >= lo[0])) return 0.f;
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return 2.f * (dx * dy + dy * dz + dz * dx);
    }
};

struct Builder {
    const nart_scene_blob& blob;
    std::vector<BTri>& tris;
    float pad;
    BuiltBVH& out;
    std::vector<uint32_t> order;

    static constexpr int kMaxBins = 64;
    int kBins = 16;             // NART_BVH_BINS (<= 64)
    uint32_t kLeafTarget = 4;   // NART_BVH_LEAF: always a leaf at or below this many triangles
    uint32_t kLeafSah = 8;      // NART_BVH_LEAF_SAH: SAH may stop splitting at or below this
    float kTrav = 1.0f;         // NART_BVH_TRAV: node-visit cost relative to one triangle test
    // Depth cap.  Binned SAH can peel one bin per level off clustered or graded geometry, and
    // the traversal stack (8 B per level per lane, 256 lanes per block) lives in LDS.  From this
    // depth on, nodes split at the object median of the widest centroid axis, so the tree stays
    // below kMedianDepth + log2(triangles) <= 72 levels (stack <= 144 KiB per block).
    uint32_t kMedianDepth = 40;  // NART_BVH_MEDIAN_DEPTH

    int32_t make_leaf(uint32_t first, uint32_t count) {
        uint32_t leaf_first = (uint32_t)order.size();
        for (uint32_t i = 0; i < count; ++i) order.push_back(tris[first + i].g);
        return ~(int32_t)((leaf_first << 5) | (count - 1));
    }
    Box bounds(uint32_t first, uint32_t count) {
        Box b;
        for (uint32_t i = first; i < first + count; ++i) b.grow(tris[i].lo, tris[i].hi);
        return b;
    }
    // returns child code; depth = inner-node depth of the node being built
    int32_t build(uint32_t first, uint32_t count, uint32_t depth) {
        if (count <= kLeafTarget) return make_leaf(first, count);
        Box cb;
        for (uint32_t i = first; i < first + count; ++i) cb.grow(tris[i].c, tris[i].c);
        if (depth >= kMedianDepth) return inner(first, count, depth, median_split(first, count, cb));
        int axis = -1;
        int split_bin = -1;
        float best = std::numeric_limits<float>::infinity();
        Box total = bounds(first, count);
        for (int a = 0; a < 3; ++a) {
            float ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0.f)) continue;
            Box bb[kMaxBins];
            uint32_t bc[kMaxBins] = {0};
            for (uint32_t i = first; i < first + count; ++i) {
                int b = (int)((tris[i].c[a] - cb.lo[a]) / ext * kBins);
                b = std::min(std::max(b, 0), kBins - 1);
                bb[b].grow(tris[i].lo, tris[i].hi);
                bc[b]++;
            }
            Box lb[kMaxBins];
            uint32_t lc[kMaxBins];
            Box acc;
            uint32_t n = 0;
            for (int b = 0; b < kBins; ++b) {
                acc.grow(bb[b]);
                n += bc[b];
                lb[b] = acc;
                lc[b] = n;
            }
            Box racc;
            uint32_t rn = 0;
            for (int b = kBins - 1; b > 0; --b) {
                racc.grow(bb[b]);
                rn += bc[b];
                uint32_t ln = lc[b - 1];
                if (ln == 0 || rn == 0) continue;
                float cost = lb[b - 1].area() * ln + racc.area() * rn;
                if (cost < best) {
                    best = cost;
                    axis = a;
                    split_bin = b;
                }
            }
        }
        float leaf_cost = total.area() * count;
        bool force_split = count > NART_LEAF_MAX;
        if (axis < 0 || (!force_split && best + total.area() * kTrav >= leaf_cost && count <= kLeafSah)) {
            if (!force_split) return make_leaf(first, count);
        }
        uint32_t mid;
        if (axis >= 0) {
            float ext = cb.hi[axis] - cb.lo[axis];
            auto it = std::partition(tris.begin() + first, tris.begin() + first + count, [&](const BTri& t) {
                int b = (int)((t.c[axis] - cb.lo[axis]) / ext * kBins);
                b = std::min(std::max(b, 0), kBins - 1);
                return b < split_bin;
            });
            mid = (uint32_t)(it - tris.begin());
        } else {
            mid = first + count / 2;  // identical centroids: split by index
        }
        if (mid == first || mid == first + count) mid = first + count / 2;
        return inner(first, count, depth, mid);
    }
    // object median of the widest centroid axis (index order when every centroid coincides)
    uint32_t median_split(uint32_t first, uint32_t count, const Box& cb) {
        int axis = 0;
        for (int a = 1; a < 3; ++a)
            if (cb.hi[a] - cb.lo[a] > cb.hi[axis] - cb.lo[axis]) axis = a;
        const uint32_t mid = first + count / 2;
        if (cb.hi[axis] - cb.lo[axis] > 0.f)
            std::nth_element(tris.begin() + first, tris.begin() + mid, tris.begin() + first + count,
                             [axis](const BTri& x, const BTri& y) { return x.c[axis] < y.c[axis]; });
        return mid;
    }
    // inner node over [first, mid) and [mid, first + count)
    int32_t inner(uint32_t first, uint32_t count, uint32_t depth, uint32_t mid) {
        int32_t idx = (int32_t)out.nodes.size();
        out.nodes.emplace_back();
        out.max_stack = std::max(out.max_stack, depth + 1);
        int32_t c0 = build(first, mid - first, depth + 1);
        int32_t c1 = build(mid, first + count - mid, depth + 1);
        Box b0 = bounds(first, mid - first), b1 = bounds(mid, first + count - mid);
        nd::BVHNode& nd_ = out.nodes[idx];
        for (int k = 0; k < 3; ++k) {
            nd_.lo0[k] = b0.lo[k] - pad;
            nd_.hi0[k] = b0.hi[k] + pad;
            nd_.lo1[k] = b1.lo[k] - pad;
            nd_.hi1[k] = b1.hi[k] + pad;
        }
        nd_.child[0] = c0;
        nd_.child[1] = c1;
        nd_.pad[0] = nd_.pad[1] = 0;
        return idx;
    }
};

}  // namespace

void build_bvh(const nart_scene_blob& blob, const std::vector<uint8_t>& mask, float pad, BuiltBVH& out) {
    std::vector<BTri> tris;
    for (uint32_t g = 0; g < blob.num_triangles; ++g) {
        if (!mask[g]) continue;
        const nart_triangle& T = blob.triangles[g];
        BTri b;
        for (int k = 0; k < 3; ++k) {
            b.lo[k] = std::min(std::min(T.v0[k], T.v1[k]), T.v2[k]);
            b.hi[k] = std::max(std::max(T.v0[k], T.v1[k]), T.v2[k]);
            b.c[k] = 0.5f * (b.lo[k] + b.hi[k]);
        }
        b.g = g;
        tris.push_back(b);
    }
    out.nodes.clear();
    out.tri_isect.clear();
    out.max_stack = 1;
    out.pad = pad;
    Builder bld{blob, tris, pad, out, {}};
    if (const char* e = std::getenv("NART_BVH_BINS")) bld.kBins = std::max(2, std::min(Builder::kMaxBins, std::atoi(e)));
    if (const char* e = std::getenv("NART_BVH_LEAF")) bld.kLeafTarget = (uint32_t)std::max(1, std::min(NART_LEAF_MAX, std::atoi(e)));
    if (const char* e = std::getenv("NART_BVH_LEAF_SAH")) bld.kLeafSah = (uint32_t)std::max(1, std::min(NART_LEAF_MAX, std::atoi(e)));
    if (const char* e = std::getenv("NART_BVH_TRAV")) bld.kTrav = (float)std::atof(e);
    if (const char* e = std::getenv("NART_BVH_MEDIAN_DEPTH")) bld.kMedianDepth = (uint32_t)std::max(1, std::min(40, std::atoi(e)));
    if (tris.empty()) {
        out.root_code = -1;  // never traversed (geometry_visible = 0)
        out.num_leaf_tris = 0;
        return;
    }
    out.root_code = bld.build(0, (uint32_t)tris.size(), 0);
    out.num_leaf_tris = (uint32_t)bld.order.size();
    // Breadth-first node order: any prefix of the array is the top of the tree, which the
    // traversal kernels keep in LDS (as much as fits).
    if (out.root_code >= 0) {
        std::vector<int32_t> bfs, remap(out.nodes.size(), -1);
        bfs.push_back(out.root_code);
        for (size_t h = 0; h < bfs.size(); ++h) {
            const nd::BVHNode& n = out.nodes[bfs[h]];
            for (int c = 0; c < 2; ++c)
                if (n.child[c] >= 0) bfs.push_back(n.child[c]);
        }
        for (size_t i = 0; i < bfs.size(); ++i) remap[bfs[i]] = (int32_t)i;
        std::vector<nd::BVHNode> reordered(bfs.size());
        for (size_t i = 0; i < bfs.size(); ++i) {
            reordered[i] = out.nodes[bfs[i]];
            for (int c = 0; c < 2; ++c)
                if (reordered[i].child[c] >= 0) reordered[i].child[c] = remap[reordered[i].child[c]];
        }
        out.nodes.swap(reordered);
        out.root_code = 0;
    }
    out.tri_isect.resize(bld.order.size() * 16);
    for (size_t i = 0; i < bld.order.size(); ++i) {
        uint32_t g = bld.order[i];
        const nart_triangle& T = blob.triangles[g];
        // n = cross(v1 - v0, v2 - v0) and dot(v0, n) exactly as Triangle::Intersect computes
        // them (geometry.cpp:33-37), so the device's plane test is bit-identical
        float e1[3] = {T.v1[0] - T.v0[0], T.v1[1] - T.v0[1], T.v1[2] - T.v0[2]};
        float e2[3] = {T.v2[0] - T.v0[0], T.v2[1] - T.v0[1], T.v2[2] - T.v0[2]};
        float n[3] = {e1[1] * e2[2] - e2[1] * e1[2], e1[2] * e2[0] - e2[2] * e1[0], e1[0] * e2[1] - e2[0] * e1[1]};
        float d0 = (T.v0[0] * n[0] + T.v0[1] * n[1]) + T.v0[2] * n[2];
        float* r = &out.tri_isect[i * 16];
        r[0] = n[0]; r[1] = n[1]; r[2] = n[2]; r[3] = d0;
        r[4] = T.v0[0]; r[5] = T.v0[1]; r[6] = T.v0[2]; r[7] = T.v1[0];
        r[8] = T.v1[1]; r[9] = T.v1[2]; r[10] = T.v2[0]; r[11] = T.v2[1];
        r[12] = T.v2[2];
        std::memcpy(&r[13], &g, 4);
        r[14] = 0.f;
        r[15] = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]) * 0.125f;  // |n| cos(82.8 deg), octree.h
    }
}

// tri_isect word 14: the triangle's reference-octree leaf (bits 0-30) and bit 31 set when the
// whole triangle lies inside that leaf's box by `margin` on every axis (no flat axis).  A hit on
// it whose ray is not grazing (|dot(d, n)| >= |n| / 8, word 15; the plane distance t then places
// o + t d within ~250 ulps of the scene scale of the triangle) is clear of the leaf's faces,
// and octree.h needs no box loads for it.
void octree_leaf_info(const nart_scene_blob& blob, const RefOctree& oct, float margin, std::vector<uint32_t>& info) {
    info.assign(blob.num_triangles, 0u);
    for (uint32_t g = 0; g < blob.num_triangles; ++g) {
        const int32_t leaf = g < oct.tri_leaf.size() ? oct.tri_leaf[g] : -1;
        uint32_t v = leaf >= 0 ? (uint32_t)leaf : 0u;
        if (leaf >= 0) {
            const nd::OcNode& L = oct.nodes[leaf];
            const nart_triangle& T = blob.triangles[g];
            bool inside = true;
            for (int k = 0; k < 3 && inside; ++k) {
                const float lo = std::min(T.v0[k], std::min(T.v1[k], T.v2[k]));
                const float hi = std::max(T.v0[k], std::max(T.v1[k], T.v2[k]));
                inside = L.bmin[k] < L.bmax[k] && lo - L.bmin[k] >= margin && L.bmax[k] - hi >= margin;
            }
            if (inside) v |= 0x80000000u;
        }
        info[g] = v;
    }
}

void annotate_octree_leaves(const nart_scene_blob& blob, const RefOctree& oct, float margin, BuiltBVH& bvh) {
    std::vector<uint32_t> info;
    octree_leaf_info(blob, oct, margin, info);
    const size_t n = bvh.tri_isect.size() / 16;
    for (size_t i = 0; i < n; ++i) {
        float* r = &bvh.tri_isect[i * 16];
        uint32_t g;
        std::memcpy(&g, &r[13], 4);
        std::memcpy(&r[14], &info[g], 4);
    }
}

}  // namespace nart
