// Host-side acceleration structure build for the nart render path.
#pragma once

#include <stdint.h>

#include <vector>

#include "../../../include/nart_scene.h"
#include "../device/dscene.h"

namespace nart {

struct BuiltBVH {
    std::vector<nd::BVHNode> nodes;   // breadth-first, root = nodes[0] unless root_code < 0
    std::vector<float> tri_isect;      // 16 floats per triangle, leaf order
    int32_t root_code = 0;
    uint32_t max_stack = 1;            // deepest chain of inner nodes (traversal stack bound)
    uint32_t num_leaf_tris = 0;
    float pad = 0.f;                   // box padding applied (world units)
};

// The reference octree itself, for exact emulation of Octree::Intersect on the device.
struct RefOctree {
    std::vector<nd::OcNode> nodes;  // creation order, root first
    std::vector<uint32_t> chunks;   // (tri_first, tri_count) per leaf chunk, leaves in node order
    std::vector<uint32_t> tris;     // global triangle ids
    std::vector<int32_t> tri_leaf;  // per scene triangle: its leaf, -1 if unreachable
    int32_t root = 0;
};

// Which triangles the reference's octree can ever return (bvh.cpp:252-326): all of them
// unless the root stayed a leaf (single chunk, bvh.cpp:131 -> nothing is hit) or a leaf
// holding several chunks split and dropped all but one (bvh.cpp:187-190).
// Returns the number of visible triangles; mask[g] = 1 for visible ones.
uint32_t reference_visibility(const nart_scene_blob& blob, std::vector<uint8_t>& mask, bool& root_is_leaf,
                              uint32_t& n_chunks, RefOctree* octree = nullptr);

// Binned-SAH BVH2 over the visible triangles.  Child boxes are padded by `pad` (world units)
// so the device's fast slab test is conservative w.r.t. the exact triangle test.
void build_bvh(const nart_scene_blob& blob, const std::vector<uint8_t>& mask, float pad, BuiltBVH& out);

// Tag each BVH triangle with its octree leaf and whether it lies inside the leaf's box by
// `margin` (device/octree.h fast path).
void annotate_octree_leaves(const nart_scene_blob& blob, const RefOctree& oct, float margin, BuiltBVH& bvh);

// The same tag for every scene triangle (info[g]), for the device-side build (device/lbvh.h).
void octree_leaf_info(const nart_scene_blob& blob, const RefOctree& oct, float margin, std::vector<uint32_t>& info);

}  // namespace nart
