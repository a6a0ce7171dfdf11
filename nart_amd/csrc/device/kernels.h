// Kernels of the nart render path (gfx950):
//   k_latin    per traced pixel: RNG seed + LatinSquare            (render.cpp:81-85, sampling.cpp:72-86)
//   k_render   per traced pixel: all spp samples of Li_alpha       (render.cpp:87-107, pathintegrator.cpp)
//   k_splat    per bucket tile pixel: ordered Gaussian splat      (render.cpp:23-70)
//   k_combine  per image pixel: tiles summed in bucket raster order (render.cpp:183-203)
#pragma once

#include "path.h"

namespace nd {

// ---------------------------------------------------------------- nested-dielectric list
// IntersectionInfo list (pathintegrator.h:9-19, pathintegrator.cpp:7-36, 123-142).  The first
// ILIST_REG entries live in registers (every access an unrolled compare/select, no dynamic
// indexing); a path can only grow the list by one entry per bounce, so renders with bounces <=
// ILIST_REG never need more.  With EXT (bounces up to 32) entries ILIST_REG.. live in a per-lane
// column of global memory, entry k at x[(k - ILIST_REG) * xs] as {id, eta bits}: deep nesting is
// rare, so the kernels keep the register footprint of the short list and spill nothing (the
// former 16- and 32-entry register lists spilled 50-97 VGPRs to scratch on every access).
#define ILIST_REG 10
#define ILIST_MAX 32
// this lane's overflow column (formed at each use: no registers held across the kernel)
#define ILIST_X(A) (EXT ? (A).ilist_ext + (blockIdx.x * blockDim.x + threadIdx.x) : nullptr)
// COMPACT (scenes without textures or plastic: kernels built for such a feature mask): an entry's
// eta is not stored.  Every eta the list receives is bxdf_eta of the BSDF created at a hit on the
// entry's own mesh (the continuation's or the stepped-through interface's lobe, pathintegrator.cpp:
// 199-229), and for a one-lobe BSDF with constant patterns that is a per-mesh constant: 0 for
// Lambert, the material's eta otherwise (DScene::mesh_eta, built on the host from the same
// floats).  The list then holds 11 registers instead of 21, the same values in the same order.
template <bool EXT, bool COMPACT = false>
struct IList {
    uint32_t id[ILIST_REG];  // meshID (24 bit) | priority << 24
    float eta[COMPACT ? 1 : ILIST_REG];
    uint32_t n;

    ND bool valid(uint32_t meshID, uint32_t prio, float& eta_outer, const uint2* x, uint32_t xs,
                  const float* me = nullptr) const {
        static_assert(!(EXT && COMPACT), "the compact list has no overflow column");
        eta_outer = 1.f;
        uint32_t lastId = 0, penId = 0;
        float lastEta = 1.f, penEta = 1.f;
        bool ok = true;
#pragma unroll
        for (int k = 0; k < ILIST_REG; ++k) {
            if (k + 1 == (int)n) {
                lastId = id[k] & 0xFFFFFFu;
                if (!COMPACT) lastEta = eta[k];
            }
            if (k + 2 == (int)n) {
                if (COMPACT) penId = id[k] & 0xFFFFFFu;
                else penEta = eta[k];
            }
            if (k < (int)n && (prio & 0xFFu) < (id[k] >> 24)) ok = false;
        }
        if (EXT && n > ILIST_REG) {
            for (uint32_t k = ILIST_REG; k < n; ++k) {
                const uint2 e = x[(size_t)(k - ILIST_REG) * xs];
                if (k + 1 == n) {
                    lastId = e.x & 0xFFFFFFu;
                    lastEta = __uint_as_float(e.y);
                }
                if (k + 2 == n) penEta = __uint_as_float(e.y);
                if ((prio & 0xFFu) < (e.x >> 24)) ok = false;
            }
        }
        if (n) {
            if (lastId != meshID) eta_outer = COMPACT ? me[lastId] : lastEta;
            else if (n >= 2) eta_outer = COMPACT ? me[penId] : penEta;
        }
        return ok;
    }
    ND void update(uint32_t meshID, uint32_t prio, float eta_s, uint2* x, uint32_t xs) {
        int found = -1;
#pragma unroll
        for (int k = 0; k < ILIST_REG; ++k)
            if (k < (int)n && (id[k] & 0xFFFFFFu) == meshID) found = k;  // most recent match
        if (EXT && n > ILIST_REG)
            for (uint32_t k = ILIST_REG; k < n; ++k)
                if ((x[(size_t)(k - ILIST_REG) * xs].x & 0xFFFFFFu) == meshID) found = (int)k;
        if (found >= 0) {
            // entries (found, n) move down by one
#pragma unroll
            for (int j = 0; j + 1 < ILIST_REG; ++j) {
                if (j >= found && j + 1 < (int)n) {
                    id[j] = id[j + 1];
                    if (!COMPACT) eta[j] = eta[j + 1];
                }
            }
            if (EXT && n > ILIST_REG) {
                if (found < ILIST_REG) {
                    const uint2 e = x[0];
                    id[ILIST_REG - 1] = e.x;
                    eta[ILIST_REG - 1] = __uint_as_float(e.y);
                }
                for (uint32_t k = found > ILIST_REG ? (uint32_t)found : ILIST_REG; k + 1 < n; ++k)
                    x[(size_t)(k - ILIST_REG) * xs] = x[(size_t)(k + 1 - ILIST_REG) * xs];
            }
            --n;
        } else {
#pragma unroll
            for (int k = 0; k < ILIST_REG; ++k) {
                if (k == (int)n) {
                    id[k] = (meshID & 0xFFFFFFu) | ((prio & 0xFFu) << 24);
                    if (!COMPACT) eta[k] = eta_s;
                }
            }
            if (EXT && n >= ILIST_REG)
                x[(size_t)(n - ILIST_REG) * xs] = make_uint2((meshID & 0xFFFFFFu) | ((prio & 0xFFu) << 24), __float_as_uint(eta_s));
            ++n;
        }
    }
};

// ---------------------------------------------------------------- camera (pinholecamera.cpp:9-40)
ND Ray cast_ray(const DScene& S, f2 smp, uint32_t W, uint32_t H, uint32_t x, uint32_t y) {
    float aspect = (float)W / (float)H;
    float px = ((((float)x + smp.x) / (float)W) * 2.f - 1.f) * S.cam_tan * aspect;
    float py = ((((float)y + smp.y) / (float)H) * -2.f + 1.f) * S.cam_tan;
    f4 d = normalize4(F4(px, py, -1.f, 0.f));
    f4 o = vec_mul_mat(F4(0.f, 0.f, 0.f, 1.f), S.cam_m);
    d = vec_mul_mat(d, S.cam_m);
    return make_ray(xyz(o), xyz(d));
}

// Where a slot's samples live: sample s at first + s * stride.  64-bit, since one batch may hold
// more than 2^32 samples (e.g. 1024x1024-pixel buckets at 4096 spp: 4.3 G samples, 103 GB).
struct SlotSO {
    unsigned long long first;
    uint32_t stride, pad;
};

struct RenderArgs {
    const uint32_t* slot_xy;  // traced pixel (x | y << 16) in image coordinates
    const float2* samples;    // LatinSquare image samples, sample s of slot at slot_so (sample_index)
    const uint32_t* rng0;     // [slot] RNG state after the LatinSquare
    float4* Lout;             // Li_alpha, same indexing as samples
    // [slot] {first sample index, sample stride}.  Bucket renders lay each bucket out sample-major
    // ([bucket][s][pixel of bucket]: the splat's lanes then read neighbouring pixels' sample s
    // from one cache line); the per-sample API uses {slot * spp, 1}.
    const SlotSO* slot_so;
    uint32_t n_slots, spp, bounces, W, H, totalW, stack_depth;
    float gamma;              // roughening factor squared (pathintegrator.cpp:163)
    unsigned long long* counters;  // [5] extend rays, shadow rays, node visits, tri tests, bounces
    uint32_t lds_nodes;       // BVH nodes [0, lds_nodes) staged in LDS after the stack
    // Pixel work queue (k_render): lane g starts on slot queue[g]; with qhead set the grid is
    // persistent and a lane whose pixel is done takes queue[qbase + atomicAdd(qhead)].
    const uint32_t* queue = nullptr;
    uint32_t* qhead = nullptr;
    uint32_t qbase = 0;
    uint32_t* cost = nullptr; // cost probe: per-slot work estimate of the rendered sample(s)
    uint32_t probe_sub = 0;   // cost probe of wave groups: probe this many pixels per 64-slot
                              // group (lane gid -> group gid / probe_sub), 0: every slot
    uint32_t rq_quorum = 8;   // k_render_rq: leave a traversal phase once the wave's queue is empty
                              // and at most this many lanes still trace
    const uint32_t* prim = nullptr;  // k_render_rq: camera-ray hits from k_primary, same indexing as samples
    // k_render_rq: queue entries with bit 31 set are priority pixels (the costliest of a small
    // shard): their rays are traced first and the traversal phase ends as soon as they resolve
    uint32_t rq_prio = 0;
    // k_render_rq: issue priority (s_setprio) of waves while they hold priority pixels (0: none)
    uint32_t rq_setprio = 0;
    // k_render_rq: entries with bit 30 set too are pixels dealt to two adjacent lanes, which run
    // the pixel's sample chain with RNG speculation (see k_render_rq); the queue then holds
    // qlen entries (the first round's pixels twice), not n_slots
    uint32_t rq_pairs = 0;
    uint32_t qlen = 0;
    // k_render_rq, persistent grid without a queue: a wave whose 64 pixels are all done takes
    // the next wave-sized group of slots (64 * atomicAdd(ghead, 1)), so waves do not idle until
    // the other waves of their block end
    uint32_t* ghead = nullptr;
    // with ghead: the n-th group taken is gorder[n] (null: slot order)
    const uint32_t* gorder = nullptr;
    // k_primary: packet traversal (path.h traverse_packet) instead of one ray per lane
    uint32_t packet = 0;
    // path kernels with bounces > ILIST_REG (EXT): the dielectric list's entries beyond
    // ILIST_REG, [entry - ILIST_REG][lane], ilist_stride lanes (>= the launch's threads)
    uint2* ilist_ext = nullptr;
    uint32_t ilist_stride = 0;
    // k_render_rq lean build (WV = 3): traversal-stack entries per lane kept in LDS (the LDS layout
    // uses stack_lds, not stack_depth); entries beyond them in gstack, (stack_depth - stack_lds)
    // 8-B entries per launched thread, lane-major
    uint32_t stack_lds = 0;
    int2* gstack = nullptr;
};
#define RQ_PRIO_BIT 0x80000000u
#define RQ_PAIR_BIT 0x40000000u
#define RQ_QUAD_BIT 0x20000000u  // with RQ_PAIR_BIT: the pixel's group has four lanes, not rq_pairs

// xorshift32 state after n draws (rng.h:38-40 applied n times)
ND uint32_t rng_jump(uint32_t y, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) {
        y ^= (y << 13);
        y ^= (y >> 17);
        y ^= (y << 5);
    }
    return y;
}

ND size_t sample_index(const RenderArgs& A, uint32_t slot, uint32_t s) {
    const SlotSO so = A.slot_so[slot];
    return so.first + (size_t)s * so.stride;
}

// Stage the top BVH nodes (breadth-first prefix) into LDS; every thread of the block calls it.
// With ROT the 16-B quarter k of node i sits at quarter (k + (i >> 2)) & 3 of the node's 64 B
// (node_quarter, path.h), so that the 16-lane groups of a ds_read_b128 spread over all 16 bank
// slots of a 256-B LDS row instead of the 4 that node i mod 4 selects.
template <bool ROT = false>
ND void stage_nodes(const DScene& S, float4* dst, uint32_t n) {
    const float4* src = reinterpret_cast<const float4*>(S.nodes);
    for (uint32_t i = threadIdx.x; i < 4 * n; i += blockDim.x) dst[node_slot(i >> 2) + node_quarter<ROT>(i >> 2, i & 3u)] = src[i];
    __syncthreads();
}

// ---------------------------------------------------------------- LatinSquare per pixel
__global__ __launch_bounds__(256) void k_latin(RenderArgs A) {
    uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= A.n_slots) return;
    uint32_t xy = A.slot_xy[slot];
    uint32_t x = xy & 0xFFFFu, y = xy >> 16;
    uint32_t rng = (y * A.totalW + x) + 2463534242u;  // RNG::Seed (rng.h:10-13)
    const SlotSO so = A.slot_so[slot];
    float2* s = const_cast<float2*>(A.samples) + so.first;
    const uint32_t n = A.spp, st = so.stride;
    const float inv = 1.f / (float)n;
    for (uint32_t i = 0; i < n; ++i) {
        float a = ((float)i + rng_float(rng)) * inv;  // StratifiedSample1D, x drawn first (Q2)
        float b = ((float)i + rng_float(rng)) * inv;
        s[(size_t)i * st] = make_float2(a, b);
    }
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t c = rng_int(rng, n - 1 - i);
        float t = s[(size_t)i * st].x;
        s[(size_t)i * st].x = s[(size_t)c * st].x;
        s[(size_t)c * st].x = t;
        c = rng_int(rng, n - 1 - i);
        t = s[(size_t)i * st].y;
        s[(size_t)i * st].y = s[(size_t)c * st].y;
        s[(size_t)c * st].y = t;
    }
    const_cast<uint32_t*>(A.rng0)[slot] = rng;
}

// Same computation with the two sample arrays in LDS ([spp][64 lanes], bank = lane, so the
// random-index swaps are conflict-free); one wave per block, spp <= 256 (128 KiB of LDS).
__global__ __launch_bounds__(64) void k_latin_lds(RenderArgs A) {
    extern __shared__ __attribute__((aligned(16))) float s_lat[];
    const uint32_t lane = threadIdx.x;
    const uint32_t slot = blockIdx.x * 64 + lane;
    if (slot >= A.n_slots) return;
    const uint32_t n = A.spp;
    float* xs = s_lat + lane;
    float* ys = s_lat + (size_t)n * 64 + lane;
    uint32_t xy = A.slot_xy[slot];
    uint32_t x = xy & 0xFFFFu, y = xy >> 16;
    uint32_t rng = (y * A.totalW + x) + 2463534242u;
    const float inv = 1.f / (float)n;
    for (uint32_t i = 0; i < n; ++i) {
        xs[i * 64] = ((float)i + rng_float(rng)) * inv;
        ys[i * 64] = ((float)i + rng_float(rng)) * inv;
    }
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t c = rng_int(rng, n - 1 - i);
        float t = xs[i * 64];
        xs[i * 64] = xs[c * 64];
        xs[c * 64] = t;
        c = rng_int(rng, n - 1 - i);
        t = ys[i * 64];
        ys[i * 64] = ys[c * 64];
        ys[c * 64] = t;
    }
    const SlotSO so = A.slot_so[slot];
    float2* s = const_cast<float2*>(A.samples) + so.first;
    for (uint32_t i = 0; i < n; ++i) s[(size_t)i * so.stride] = make_float2(xs[i * 64], ys[i * 64]);
    const_cast<uint32_t*>(A.rng0)[slot] = rng;
}

// The same LatinSquare for 256 < spp <= 1024, where two float arrays per lane no longer fit in
// LDS.  The shuffles only move values, so they are replayed on 16-bit stratum indices in LDS
// ([spp][64 lanes]); the jittered stratum values are written once to a scratch area (the Lout
// buffer, which k_render fills later) laid out [block][stratum][lane], and gathered through the
// final indices.  Both index arrays share the LDS when 4*spp*64 bytes fit (spp <= 512); above
// that the x and y shuffles run as two passes over the same RNG draws.
__global__ __launch_bounds__(64) void k_latin_idx(RenderArgs A, float* scratch) {
    extern __shared__ __attribute__((aligned(16))) uint16_t s_idx[];
    const uint32_t lane = threadIdx.x;
    const uint32_t slot = blockIdx.x * 64 + lane;
    if (slot >= A.n_slots) return;
    const uint32_t n = A.spp;
    const bool both = n <= 512u;
    const uint32_t xy = A.slot_xy[slot];
    const uint32_t x = xy & 0xFFFFu, y = xy >> 16;
    uint32_t rng = (y * A.totalW + x) + 2463534242u;
    const float inv = 1.f / (float)n;
    float* vx = scratch + (size_t)blockIdx.x * 2 * n * 64 + lane;  // [stratum][lane]
    float* vy = vx + (size_t)n * 64;
    for (uint32_t i = 0; i < n; ++i) {
        vx[(size_t)i * 64] = ((float)i + rng_float(rng)) * inv;  // StratifiedSample1D, x drawn first (Q2)
        vy[(size_t)i * 64] = ((float)i + rng_float(rng)) * inv;
    }
    const uint32_t rng_gen = rng;
    const SlotSO so = A.slot_so[slot];
    float2* s = const_cast<float2*>(A.samples) + so.first;
    uint16_t* ix = s_idx + lane;
    uint16_t* iy = s_idx + (size_t)n * 64 + lane;
    for (int pass = 0; pass < (both ? 1 : 2); ++pass) {
        rng = rng_gen;
        const bool dx = both || pass == 0, dy = both || pass == 1;
        uint16_t* jy = both ? iy : ix;  // single-array passes reuse the first index array
        for (uint32_t i = 0; i < n; ++i) {
            if (dx) ix[i * 64] = (uint16_t)i;
            if (dy) jy[i * 64] = (uint16_t)i;
        }
        for (uint32_t i = 0; i < n; ++i) {
            uint32_t c = rng_int(rng, n - 1 - i);
            if (dx) {
                const uint16_t t = ix[i * 64];
                ix[i * 64] = ix[c * 64];
                ix[c * 64] = t;
            }
            c = rng_int(rng, n - 1 - i);
            if (dy) {
                const uint16_t t = jy[i * 64];
                jy[i * 64] = jy[c * 64];
                jy[c * 64] = t;
            }
        }
        // gathers in groups of NART_LATIN_G (tail below), so that one wave per CU keeps that
        // many scratch loads per array in flight instead of one
#ifndef NART_LATIN_G
#define NART_LATIN_G 64  // C5 LatinSquare 100 -> 97 ms vs 16 (32: 99)
#endif
        constexpr uint32_t G = NART_LATIN_G;
        uint32_t i = 0;
        for (; i + G <= n; i += G) {
            float gx[G], gy[G];
#pragma unroll
            for (int u = 0; u < (int)G; ++u) {
                if (dx) gx[u] = vx[(size_t)ix[(i + u) * 64] * 64];
                if (dy) gy[u] = vy[(size_t)jy[(i + u) * 64] * 64];
            }
#pragma unroll
            for (int u = 0; u < (int)G; ++u) {
                if (both) s[(size_t)(i + u) * so.stride] = make_float2(gx[u], gy[u]);
                else if (dx) s[(size_t)(i + u) * so.stride].x = gx[u];
                else s[(size_t)(i + u) * so.stride].y = gy[u];
            }
        }
        for (; i < n; ++i) {
            if (both) s[(size_t)i * so.stride] = make_float2(vx[(size_t)ix[i * 64] * 64], vy[(size_t)iy[i * 64] * 64]);
            else if (dx) s[(size_t)i * so.stride].x = vx[(size_t)ix[i * 64] * 64];
            else s[(size_t)i * so.stride].y = vy[(size_t)ix[i * 64] * 64];
        }
    }
    const_cast<uint32_t*>(A.rng0)[slot] = rng;
}

// ---------------------------------------------------------------- LatinSquare in three kernels
// The shuffle's transpositions (i, c_i) depend only on the pixel's RNG stream, never on the
// values being shuffled (sampling.cpp:80-85), and a jittered stratum value depends only on the
// stream position that drew it (sampling.cpp:64-67, 75-78).  So the serial RNG work leaves the
// LDS-bound kernel, and the values are never gathered at random from HBM:
//  k_latin_draws  lane per slot, no LDS (full occupancy): runs the pixel's 2n generation draws,
//                 recording the state after each x draw (st[k] = state after draw 2k+1), then the
//                 2n shuffle choices c_x(i), c_y(i), and writes the final state (rng0);
//  k_latin_perm   lane per slot, u16 stratum indices in LDS ([i][lane]): replays the swaps, x then
//                 y, with the choices streamed from HBM; writes the final index arrays;
//  k_latin_emit   16 slots per block, their st[] staged in LDS: sample j gets
//                 (val_x(sx[j]), val_y(sy[j])) with val_x(k) from st[k] and val_y(k) from one
//                 more xorshift step.
// Scratch (in Lout, which the path kernel overwrites later): cx, cy, sx, sy are u16 pairs in u32
// words [slot / 64][i / 2][slot % 64] (low half = even i); st is u32 [slot / 16][k][slot % 16].
struct LatinScratch {
    uint32_t *cx, *cy, *sx, *sy, *st;
    uint32_t n2;  // (spp + 1) / 2 word rows
};
#define LATIN_EMIT_SLOTS 16
#define LATIN_ST_PAD (256 * 8 * 4)  // words read past the last block's states by k_latin_emit

ND size_t latin_row(uint32_t g, uint32_t rows, uint32_t r, uint32_t lane) {
    return ((size_t)g * rows + r) * 64u + lane;
}

__global__ __launch_bounds__(256) void k_latin_draws(RenderArgs A, LatinScratch L) {
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= A.n_slots) return;
    const uint32_t g = slot >> 6, lane = slot & 63u, n = A.spp;
    const uint32_t xy = A.slot_xy[slot];
    uint32_t rng = ((xy >> 16) * A.totalW + (xy & 0xFFFFu)) + 2463534242u;  // RNG::Seed (rng.h:10-13)
    // generation: x of stratum k is draw 2k+1, y draw 2k+2 (Q2)
    uint32_t* st = L.st + (size_t)(slot / LATIN_EMIT_SLOTS) * n * LATIN_EMIT_SLOTS + slot % LATIN_EMIT_SLOTS;
    for (uint32_t k = 0; k < n; ++k) {
        rng = xorshift(rng);
        st[(size_t)k * LATIN_EMIT_SLOTS] = rng;
        rng = xorshift(rng);
    }
    for (uint32_t i2 = 0; i2 < L.n2; ++i2) {
        uint32_t wx = 0, wy = 0;
        for (uint32_t h = 0; h < 2; ++h) {
            const uint32_t i = 2 * i2 + h;
            if (i >= n) break;
            wx |= rng_int(rng, n - 1 - i) << (16 * h);  // sampling.cpp:81-84, x choice first
            wy |= rng_int(rng, n - 1 - i) << (16 * h);
        }
        L.cx[latin_row(g, L.n2, i2, lane)] = wx;
        L.cy[latin_row(g, L.n2, i2, lane)] = wy;
    }
    const_cast<uint32_t*>(A.rng0)[slot] = rng;
}

#ifndef NART_LATIN_PF
#define NART_LATIN_PF 16  // choice words (2 swaps each) loaded one batch ahead of their swaps
#endif
// BL lanes per block, each with its own u16 column of the block's [i][BL] LDS array.  BL = 80
// where one 64-lane block per CU is all the LDS holds (640 < spp <= 1024: 128 KiB of 160 per 64
// lanes): the 80-lane block fills the 160 KiB, and its second wave (16 lanes) runs its own swap
// chain on another SIMD.  The kernel is bound by one wave's instruction chain, not by lanes.
template <uint32_t BL>
__global__ __launch_bounds__(BL) void k_latin_perm(RenderArgs A, LatinScratch L) {
    extern __shared__ __attribute__((aligned(16))) uint16_t s_idx[];
    const uint32_t slot = blockIdx.x * BL + threadIdx.x;
    if (slot >= A.n_slots) return;
    const uint32_t g = slot >> 6, lane = slot & 63u;
    const uint32_t n = A.spp, n2 = L.n2;
    uint16_t* ix = s_idx + threadIdx.x;
    for (int pass = 0; pass < 2; ++pass) {
        const uint32_t* c = (pass ? L.cy : L.cx) + latin_row(g, n2, 0, lane);
        uint32_t* so = (pass ? L.sy : L.sx) + latin_row(g, n2, 0, lane);
        // rolling prefetch: the next PF choice words load while the current PF words' swaps run
        // (a batch that waits for its own loads stalls on the full HBM latency every 2*PF swaps)
        constexpr uint32_t PF = NART_LATIN_PF;
        uint32_t cur[PF], nxt[PF];
#pragma unroll
        for (uint32_t u = 0; u < PF; ++u) cur[u] = c[(size_t)u * 64];
        for (uint32_t i = 0; i < 2 * n2; ++i) ix[i * BL] = (uint16_t)i;
        // Full batches (all 2*PF swaps valid) load the next batch unconditionally (the choice
        // arrays carry PF padding rows), so that no branch sits between a load and its use: with
        // guarded loads the compiler waited for every outstanding load (vmcnt(0)) before each
        // swap, i.e. the prefetch did not hide the HBM latency.
        //
        // The second half of the shuffle needs no serial chain.  Step i swaps positions i and
        // c_i <= n-1-i, so for i >= m = ceil(n/2): c_i < m, position i is touched by no other
        // step from m on (step k touches k and c_k < m), and nothing after step i reads it.  A
        // batch of steps i >= m is then exactly (1) B_i = A[i] for the whole batch, (2) in step
        // order: r_i = A[c_i], A[c_i] = B_i, (3) A[i] = r_i: no LDS write waits for a read, where
        // a swap waits for its two reads before writing them back (the first half keeps that).
        const uint32_t m = (n + 1u) / 2u;
        uint32_t i2 = 0;
        for (; 2 * (i2 + PF) <= n; i2 += PF) {
#pragma unroll
            for (uint32_t u = 0; u < PF; ++u) nxt[u] = c[(size_t)(i2 + PF + u) * 64];
            if (2 * i2 >= m) {  // wave-uniform
                uint32_t bv[2 * PF], rv[2 * PF];
#pragma unroll
                for (uint32_t q = 0; q < 2 * PF; ++q) bv[q] = ix[(2 * i2 + q) * BL];
#pragma unroll
                for (uint32_t u = 0; u < PF; ++u) {
#pragma unroll
                    for (uint32_t h = 0; h < 2; ++h) {
                        const uint32_t ci = (cur[u] >> (16 * h)) & 0xFFFFu;
                        rv[2 * u + h] = ix[ci * BL];
                        ix[ci * BL] = (uint16_t)bv[2 * u + h];
                    }
                }
#pragma unroll
                for (uint32_t q = 0; q < 2 * PF; ++q) ix[(2 * i2 + q) * BL] = (uint16_t)rv[q];
#pragma unroll
                for (uint32_t u = 0; u < PF; ++u) cur[u] = nxt[u];
                continue;
            }
#pragma unroll
            for (uint32_t u = 0; u < PF; ++u) {
#pragma unroll
                for (uint32_t h = 0; h < 2; ++h) {
                    const uint32_t i = 2 * (i2 + u) + h;
                    const uint32_t ci = (cur[u] >> (16 * h)) & 0xFFFFu;
                    const uint16_t t = ix[i * BL];
                    ix[i * BL] = ix[ci * BL];
                    ix[ci * BL] = t;
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < PF; ++u) cur[u] = nxt[u];
        }
        for (uint32_t u = 0; u < PF; ++u) {  // the partial last batch (cur holds its words)
            for (uint32_t h = 0; h < 2; ++h) {
                const uint32_t i = 2 * (i2 + u) + h;
                if (i < n) {
                    const uint32_t ci = (cur[u] >> (16 * h)) & 0xFFFFu;
                    const uint16_t t = ix[i * BL];
                    ix[i * BL] = ix[ci * BL];
                    ix[ci * BL] = t;
                }
            }
        }
        for (uint32_t j2 = 0; j2 < n2; ++j2)
            so[(size_t)j2 * 64] = (uint32_t)ix[2 * j2 * BL] | ((uint32_t)ix[(2 * j2 + 1) * BL] << 16);
    }
}

// StratifiedSample1D (sampling.cpp:64-67) from the RNG state its UniformFloat ended in
ND float latin_value(uint32_t k, uint32_t y, float inv) {
    const float f = gmin(ND_ONE_MINUS_EPS, (float)(uint32_t)(y * 0x9E3779BBu) * 2.3283064365386963e-10f);
    return ((float)k + f) * inv;
}

// Thread t of a block: slot p = t % 16 of the block's 16, sample rows j2 = t / 16 + 16 i, so a
// wave writes 4 rows x 16 neighbouring slots (128 B each in the bucket layout).  The index words
// are loaded LATIN_EMIT_U rows ahead (the first batch before the LDS staging): with 2 blocks per
// CU the kernel is otherwise bound by waiting on them.
#ifndef LATIN_EMIT_U
#define LATIN_EMIT_U 8
#endif
__global__ __launch_bounds__(256) void k_latin_emit(RenderArgs A, LatinScratch L) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_st[];  // [k][p]
    constexpr uint32_t P = LATIN_EMIT_SLOTS, RS = 256 / P, U = LATIN_EMIT_U;
    const uint32_t n = A.spp, n2 = L.n2, t = threadIdx.x, p = t % P;
    // XCD-aware block order: the four blocks whose 16 slots share the 256-B rows of one 64-slot
    // index group are consecutive logical blocks on one XCD (blocks are dealt round robin over the
    // 8 XCDs, each with its own L2), so each row is fetched once instead of once per quarter.
    // Bijective for any grid (cdna_hip_programming.md T1).
    const uint32_t nwg = gridDim.x, q = nwg / 8u, r = nwg % 8u, x = blockIdx.x % 8u;
    const uint32_t bid = (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + blockIdx.x / 8u;
    const uint32_t slot = bid * P + p;
    const bool live = slot < A.n_slots;
    const uint32_t* sx = L.sx + latin_row(slot >> 6, n2, 0, slot & 63u);
    const uint32_t* sy = L.sy + latin_row(slot >> 6, n2, 0, slot & 63u);
    uint32_t cx[U], cy[U], nx[U], ny[U];
    const uint32_t j0 = t / P;
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
        const uint32_t j2 = j0 + u * RS;
        cx[u] = sx[(size_t)j2 * 64];  // unconditional (padded arrays): see k_latin_perm
        cy[u] = sy[(size_t)j2 * 64];
    }
    // stage the block's n*P states: 8 unconditional 16-B loads in flight per thread (the st
    // region carries LATIN_ST_PAD words of padding), guarded LDS stores
    {
        const uint4* src = reinterpret_cast<const uint4*>(L.st + (size_t)bid * n * P);
        uint4* dst = reinterpret_cast<uint4*>(s_st);
        const uint32_t cnt = n * P / 4;
        for (uint32_t b0 = 0; b0 < cnt; b0 += 256u * 8u) {
            uint4 v[8];
#pragma unroll
            for (uint32_t u = 0; u < 8; ++u) v[u] = src[b0 + u * 256u + t];
#pragma unroll
            for (uint32_t u = 0; u < 8; ++u)
                if (b0 + u * 256u + t < cnt) dst[b0 + u * 256u + t] = v[u];
        }
    }
    __syncthreads();
    if (!live) return;
    const float inv = 1.f / (float)n;
    const SlotSO so = A.slot_so[slot];
    float2* s = const_cast<float2*>(A.samples) + so.first;
    for (uint32_t jb = j0; jb < n2; jb += U * RS) {
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t j2 = jb + (U + u) * RS;
            nx[u] = sx[(size_t)j2 * 64];
            ny[u] = sy[(size_t)j2 * 64];
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                const uint32_t j = 2 * (jb + u * RS) + h;
                if (j < n) {
                    const uint32_t kx = (cx[u] >> (16 * h)) & 0xFFFFu, ky = (cy[u] >> (16 * h)) & 0xFFFFu;
                    s[(size_t)j * so.stride] = make_float2(latin_value(kx, s_st[kx * P + p], inv),
                                                           latin_value(ky, xorshift(s_st[ky * P + p]), inv));
                }
            }
            cx[u] = nx[u];
            cy[u] = ny[u];
        }
    }
}

enum { ST_EXT = 0, ST_SH1 = 1, ST_SH2 = 2 };

// ---------------------------------------------------------------- path tracing megakernel
// One lane per traced pixel; the lane walks its pixel's spp samples in order on one RNG
// stream.  Each loop iteration traces exactly one ray (extension or shadow) through the
// shared traversal loop, then advances the lane's path state machine; a lane whose path
// ends starts its next sample immediately (path regeneration), so lanes of a wave stay busy.
// Min waves per SIMD requested from the register allocator.  Without it the allocator takes
// >256 registers (VGPR + AGPR) once the environment-light code is inlined and the kernel drops
// to 1 wave/SIMD (C3 at 64 spp: 260 ms vs 151 ms at 2 waves; 3 waves spills: 178 ms).
#ifndef NART_RENDER_WAVES
#define NART_RENDER_WAVES 2
#endif
#define NART_RENDER_LB __launch_bounds__(256, NART_RENDER_WAVES)
// (Round 5: the traversal-quorum form of this kernel -- variant 2/3, C3 whole frame 517 vs 569 ms
// before the ray-queue kernel replaced it -- was retired; k_render is the cost probe and the
// fallback for BVHs too deep for the ray-queue kernel's LDS.)
template <bool EXT, bool COUNT, bool ENV>
__global__ NART_RENDER_LB void k_render(DScene S, RenderArgs A) {
    // LDS traversal stack: stack_depth entries of (node code, entry distance) per lane,
    // laid out [depth][lane] so a wave's 64 lanes hit 64 distinct banks.
    extern __shared__ __attribute__((aligned(16))) int s_dyn[];
    float* s_tn = reinterpret_cast<float*>(s_dyn + A.stack_depth * blockDim.x);
    float4* s_nodes = reinterpret_cast<float4*>(s_dyn + 2 * A.stack_depth * blockDim.x);
    stage_nodes(S, s_nodes, A.lds_nodes);
    const int nl = (int)A.lds_nodes;
    const int tid = threadIdx.x;
    const uint32_t gid = blockIdx.x * blockDim.x + tid;
    uint32_t slot = gid;
    if (A.probe_sub) {  // evenly spaced pixels of each 64-slot group
        const uint32_t q = A.probe_sub;
        slot = (gid / q) * 64u + (gid % q) * (64u / q) + (32u / q);
        if (slot >= A.n_slots) return;
    } else if (A.queue) {
        slot = gid < A.n_slots ? A.queue[gid] : 0xFFFFFFFFu;
    } else if (slot >= A.n_slots) {
        return;
    }
    uint32_t px = 0, py = 0, rng = 0, sstr = 0;
    uint64_t soff = 0;  // first sample index (64-bit: a batch may hold more than 2^32 samples)
    const float2* smp = A.samples;
    float4* out = A.Lout;
    auto take_pixel = [&](uint32_t sl) {
        slot = sl;
        const uint32_t xy = A.slot_xy[sl];
        px = xy & 0xFFFFu;
        py = xy >> 16;
        rng = A.rng0[sl];
        const SlotSO so = A.slot_so[sl];
        soff = so.first;
        sstr = so.stride;
    };
    if (slot != 0xFFFFFFFFu) take_pixel(slot);
    int* sc = reinterpret_cast<int*>(reinterpret_cast<int2*>(s_dyn) + tid);  // [depth][lane] int2
    float* stn = s_tn + tid;
    const int stride = blockDim.x;
    const float nL = (float)S.num_lights;
    TraceCounters cnt = {0u, 0u, 0u, 0u};
    uint32_t n_ext = 0, n_sh = 0, n_bounce = 0;

    uint32_t s = slot != 0xFFFFFFFFu ? 0u : A.spp;
    uint32_t iters = 0;  // outer iterations of this lane (cost probe)
    f3 L, beta, Le, c1, c2, betak, Led;
    float alpha = 0.f, eta_sampled = 1.f, eta_outer = 1.f, alphaTweak = 1.f;
    uint32_t flags = 0, bounce = 0;
    IList<EXT> list;
    list.n = 0;
    Ray ray, cur, nxt, sh2;
    float tmax = 0.f, sh2max = 0.f;
    int stage = ST_EXT;
    bool lightHit = false, use1 = false, use2 = false, cont = false, have_ed = false;
    bool new_sample = true, new_bounce = false;

    for (;;) {
        if (A.qhead) {
            // refill lanes whose pixel is done: one queue atomic per wave
            const bool need = new_sample && s >= A.spp;
            const uint64_t m = __ballot(need);
            if (m) {
                const int leader = __builtin_ctzll(m);
                uint32_t base = 0;
                if ((int)__lane_id() == leader) base = atomicAdd(A.qhead, (uint32_t)__popcll(m));
                base = __builtin_amdgcn_readlane(base, leader);
                if (need) {
                    const uint32_t idx = A.qbase + base +
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    if (idx < A.n_slots) {
                        take_pixel(A.queue[idx]);
                        s = 0;
                    }
                }
            }
        }
        ++iters;
        if (new_sample) {
            if (s >= A.spp) break;
            float2 sm = smp[soff + (uint64_t)s * sstr];
            ray = cast_ray(S, F2(sm.x, sm.y), A.W, A.H, px, py);
            L = F3(0.f, 0.f, 0.f);
            alpha = 0.f;
            eta_sampled = 1.f;
            eta_outer = 1.f;
            beta = F3(1.f, 1.f, 1.f);
            flags = 0;
            alphaTweak = 1.f;
            bounce = 0;
            list.n = 0;
            new_sample = false;
            new_bounce = true;
        }
        if (new_bounce) {
            new_bounce = false;
            if (bounce >= A.bounces) {
                out[soff + (uint64_t)s * sstr] = make_float4(L.x, L.y, L.z, alpha);
                ++s;
                new_sample = true;
                continue;
            }
            // light intersections (pathintegrator.cpp:167-182)
            float lightTMax = __builtin_inff();
            lightHit = false;
            Le = F3(0.f, 0.f, 0.f);
            uint32_t lwin = 0;
            for (uint32_t j = 0; j < S.num_lights; ++j) {
                float lt = __builtin_inff();
                light_bound<ENV>(uniform_light(S, j), ray.o, ray.d, lt);
                if (lt < lightTMax) {
                    lightTMax = lt;
                    lightHit = true;
                    alpha = 1.f;
                    lwin = j;
                }
            }
            // Le (the radiance of the light that set the bound) only matters for the camera ray
            if (bounce == 0 && lightHit) {
                float lt = __builtin_inff();
                Le = light_li<ENV>(S, cst(S.lights)[lwin], ray.o, ray.d, nullptr, lt);
            }
            cur = ray;
            tmax = lightTMax;
            stage = ST_EXT;
            if (COUNT) ++n_ext;
        }

        float bt;
        uint32_t bg;
        bool hit;
        {
        hit = traverse<COUNT>(S, cur, tmax, stage != ST_EXT, bt, bg, sc, stn, stride, cnt, s_nodes, nl);
        }
        bool resolve = false;
        if (stage == ST_EXT) {
            if (!hit) {
                // escaped: at bounce 0 the light seen directly is the result; at bounce > 0 the
                // reference repeats the same miss until the loop ends (no RNG, no state change)
                if (bounce == 0 && lightHit) L = Le;
                out[soff + (uint64_t)s * sstr] = make_float4(L.x, L.y, L.z, alpha);
                ++s;
                new_sample = true;
                continue;
            }
            if (COUNT) ++n_bounce;  // shaded hit
            Isect is;
            fill_isect(S, cur, bg, is);
            BSDF bsdf;
            create_bsdf(S, is, alphaTweak, bsdf);
            use1 = use2 = false;
            if (list.valid(is.meshID, is.priority, eta_outer, ILIST_X(A), A.ilist_stride)) {
                if (bounce == 0) alpha = 1.f;
                const f3 wo = to_local(bsdf, neg(cur.d));
                // ---- EstimateDirect (pathintegrator.cpp:38-121)
                const DLight& Lg = cst(S.lights)[f2u8(gmin(rng_float(rng), ND_ONE_MINUS_EPS) * nL)];
                float sPdf = 0.f, lPdf = 0.f;
                float sx = rng_float(rng);
                float sy = rng_float(rng);
                float bsmp = rng_float(rng);
                uint32_t dflags = 0;
                f3 wi;
                f3 f = bsdf_sample_f<ENV>(bsdf, wo, wi, bsmp, F2(sx, sy), sPdf, dflags, true, eta_outer, nullptr, nullptr);
                if (sPdf > 0.f) {
                    float flip = wi.z > 0.f ? 1.f : -1.f;
                    f3 wW = to_world(bsdf, wi);
                    float lt = __builtin_inff();
                    f3 Li = light_li<ENV>(S, Lg, is.p, wW, &lPdf, lt);
                    float weight = 1.f;
                    bool add1 = true;
                    if (!(dflags & F_SPECULAR)) {
                        weight = (sPdf * sPdf) / (sPdf * sPdf + lPdf * lPdf);
                        add1 = lPdf > 0.f;
                    }
                    if (add1) {
                        c1 = divs(muls(muls(mul(f, Li), gabs(wi.z)), weight), sPdf);
                        // an all-zero term cannot change the sum: skip its shadow ray
                        use1 = !(c1.x == 0.f && c1.y == 0.f && c1.z == 0.f);
                        if (use1) {
                            cur = make_ray(add(is.p, muls(muls(is.gn, SHADOW_BIAS), flip)), wW);
                            tmax = lt;
                        }
                    }
                }
                lPdf = 0.f;
                float lx = rng_float(rng);
                float ly = rng_float(rng);
                f3 wiW;
                float lt2 = __builtin_inff();
                f3 Li2 = light_sample_li<ENV>(S, Lg, is.p, wiW, F2(lx, ly), lPdf, lt2);
                f3 wi2 = to_local(bsdf, wiW);
                if (lPdf > 0.f) {
                    float sp2;
                    const f3 fv = bsdf_f_pdf(bsdf, wo, wi2, true, eta_outer, sp2);
                    if (sp2 > 0.f) {
                        float weight = (lPdf * lPdf) / (sp2 * sp2 + lPdf * lPdf);
                        c2 = divs(muls(muls(mul(fv, Li2), gabs(wi2.z)), weight), lPdf);
                        use2 = !(c2.x == 0.f && c2.y == 0.f && c2.z == 0.f);
                        if (use2) {
                            float flip2 = wi2.z > 0.f ? 1.f : -1.f;
                            sh2 = make_ray(add(is.p, muls(muls(is.gn, SHADOW_BIAS), flip2)), wiW);
                            sh2max = lt2;
                        }
                    }
                }
                betak = beta;
                have_ed = true;
                // ---- continuation (pathintegrator.cpp:199-220)
                float a = rng_float(rng);
                float b = rng_float(rng);
                float bs2 = rng_float(rng);
                float cpdf = 0.f, alpha_i = 0.f;
                f3 wic;
                f3 fc = bsdf_sample_f<ENV>(bsdf, wo, wic, bs2, F2(a, b), cpdf, flags, false, eta_outer, &alpha_i,
                                      &eta_sampled);
                if (cpdf <= 0.f) {
                    cont = false;
                } else {
                    alphaTweak = (1.f - (A.gamma * alpha_i)) * alphaTweak;
                    beta = mul(beta, muls(divs(fc, cpdf), gabs(wic.z)));
                    float flip = wic.z > 0.f ? 1.f : -1.f;
                    nxt = make_ray(add(is.p, muls(muls(is.gn, SHADOW_BIAS), flip)), to_world(bsdf, wic));
                    cont = true;
                }
            } else {
                // lower-priority interface: step through (pathintegrator.cpp:223-229)
                nxt = make_ray(add(is.p, muls(cur.d, SHADOW_BIAS)), cur.d);
                flags = F_TRANSMISSIVE;
                float bs2 = rng_float(rng);
                eta_sampled = bsdf_sample_eta(bsdf, bs2);
                cont = true;
                have_ed = false;
            }
            if (cont) {
                if (flags & F_TRANSMISSIVE) list.update(is.meshID, is.priority, eta_sampled, ILIST_X(A), A.ilist_stride);
                // Russian roulette (pathintegrator.cpp:236-246)
                float q = gmax((beta.x + beta.y + beta.z) * 0.33333f, 0.f);
                if (bounce > 3) {
                    if (q >= rng_float(rng)) beta = divs(beta, q);
                    else cont = false;
                }
            }
            ++bounce;
            Led = F3(0.f, 0.f, 0.f);
            if (use1) {
                stage = ST_SH1;
                if (COUNT) ++n_sh;
            } else if (use2) {
                stage = ST_SH2;
                cur = sh2;
                tmax = sh2max;
                if (COUNT) ++n_sh;
            } else {
                resolve = true;
            }
        } else if (stage == ST_SH1) {
            if (!hit) Led = add(Led, c1);
            if (use2) {
                stage = ST_SH2;
                cur = sh2;
                tmax = sh2max;
                if (COUNT) ++n_sh;
            } else {
                resolve = true;
            }
        } else {
            if (!hit) Led = add(Led, c2);
            resolve = true;
        }

        if (resolve) {
            // L += EstimateDirect(...) * beta, with EstimateDirect = ((0 + c1) + c2) * numLights
            if (have_ed) L = add(L, mul(muls(Led, nL), betak));
            if (cont) {
                ray = nxt;
                new_bounce = true;
            } else {
                out[soff + (uint64_t)s * sstr] = make_float4(L.x, L.y, L.z, alpha);
                ++s;
                new_sample = true;
            }
        }
    }
    if (A.cost) {  // cost probe (one pixel per lane, no queue): node/triangle/iteration weights
        A.cost[gid] = cnt.nodes + 2u * cnt.tris + 30u * iters;
        return;
    }
    if (COUNT) {
        atomicAdd(&A.counters[0], (unsigned long long)n_ext);
        atomicAdd(&A.counters[1], (unsigned long long)n_sh);
        atomicAdd(&A.counters[2], (unsigned long long)cnt.nodes);
        atomicAdd(&A.counters[3], (unsigned long long)cnt.tris);
        atomicAdd(&A.counters[4], (unsigned long long)n_bounce);
        atomicAdd(&A.counters[5], (unsigned long long)cnt.oc_checks);
        atomicAdd(&A.counters[6], (unsigned long long)cnt.oc_replays);
    }
}

// ---------------------------------------------------------------- camera rays, traced coherently
// The closest hit of every sample's camera ray depends only on its LatinSquare sample, not on the
// RNG stream, so all of a batch's camera rays are traced here before the path kernel runs: lane =
// traced pixel, all lanes of a wave (a 16x4 block of a bucket) on the same sample index at once,
// so their rays run nearly the same traversal (the path kernel's lanes are at unrelated path
// stages).  Light loop bound (pathintegrator.cpp:167-182) and octree answer as in k_render_rq;
// hit[sample] = closest triangle or NO_HIT.
template <bool COUNT, bool ENV, uint32_t FM = FT_ALL>
#ifndef NART_PRIMARY_WAVES
// minimum waves per SIMD requested for k_primary: 4 (36 VGPRs spilled, latency hidden by the fourth
// wave) vs the allocator's 3: C3 23.05 -> 21.1 ms, C4 1080p/32 3.31 -> 3.21 ms (profiles/r05ao_primary_waves_ab.txt)
#define NART_PRIMARY_WAVES 4
#endif
__global__ __launch_bounds__(256, NART_PRIMARY_WAVES) void k_primary(DScene S, RenderArgs A, uint32_t* hit) {
    extern __shared__ __attribute__((aligned(16))) int s_dyn[];
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot >= A.n_slots) return;
    int* sc = reinterpret_cast<int*>(reinterpret_cast<int2*>(s_dyn) + threadIdx.x);
    const uint32_t xy = A.slot_xy[slot];
    const uint32_t px = xy & 0xFFFFu, py = xy >> 16;
    const SlotSO so = A.slot_so[slot];
    TraceCounters cnt = {0u, 0u, 0u, 0u};
    auto camera_hit = [&](float2 sm) {
        const Ray ray = cast_ray(S, F2(sm.x, sm.y), A.W, A.H, px, py);
        float lightTMax = __builtin_inff();
        for (uint32_t j = 0; j < S.num_lights; ++j) {
            float lt = __builtin_inff();
            light_bound<ENV, FM>(uniform_light(S, j), ray.o, ray.d, lt);  // only the bound: no radiance
            if (lt < lightTMax) lightTMax = lt;
        }
        float bt;
        uint32_t bg;
        if (A.packet)
            traverse_packet<COUNT>(S, ray, lightTMax, bt, bg, reinterpret_cast<uint4*>(s_dyn) + (threadIdx.x >> 6) * A.stack_depth,
                                   cnt);
        else
            traverse<COUNT>(S, ray, lightTMax, false, bt, bg, sc, nullptr, blockDim.x, cnt, nullptr, 0);
        return bg;
    };
    if (so.stride == 1u && (A.spp & 7u) == 0u && (so.first & 7u) == 0u) {
        // pixel-major rows (the default whole-frame layout): a lane's samples are contiguous, so
        // it reads 8 samples (64 B) and writes 8 hits (32 B) per access instead of one 8-B / 4-B
        // access per sample, each to a line the lock-step lanes of the wave do not share.  The
        // one-sample accesses made k_primary move ~10x its streaming bytes through HBM (the
        // lines were evicted between a lane's consecutive samples: VERDICT r03 weak #4)
        const float4* sp = reinterpret_cast<const float4*>(A.samples + so.first);
        uint4* hp = reinterpret_cast<uint4*>(hit + so.first);
        for (uint32_t c = 0; c < A.spp / 8u; ++c) {
            const float4 q0 = sp[4 * c], q1 = sp[4 * c + 1], q2 = sp[4 * c + 2], q3 = sp[4 * c + 3];
            uint4 h0 = make_uint4(0u, 0u, 0u, 0u), h1 = h0;
            // one traversal call site (selects pick the k-th sample and hit slot): the body is
            // not duplicated 8 times in the instruction cache
#pragma unroll 1
            for (uint32_t k = 0; k < 8u; ++k) {
                const float4 q = k < 2u ? q0 : (k < 4u ? q1 : (k < 6u ? q2 : q3));
                const uint32_t bg = camera_hit((k & 1u) ? make_float2(q.z, q.w) : make_float2(q.x, q.y));
                h0.x = k == 0u ? bg : h0.x;
                h0.y = k == 1u ? bg : h0.y;
                h0.z = k == 2u ? bg : h0.z;
                h0.w = k == 3u ? bg : h0.w;
                h1.x = k == 4u ? bg : h1.x;
                h1.y = k == 5u ? bg : h1.y;
                h1.z = k == 6u ? bg : h1.z;
                h1.w = k == 7u ? bg : h1.w;
            }
            hp[2 * c] = h0;
            hp[2 * c + 1] = h1;
        }
    } else {
        for (uint32_t s = 0; s < A.spp; ++s) {
            const uint64_t idx = so.first + (uint64_t)s * so.stride;
            hit[idx] = camera_hit(A.samples[idx]);
        }
    }
    if (COUNT) {
        atomicAdd(&A.counters[0], (unsigned long long)A.spp);
        atomicAdd(&A.counters[2], (unsigned long long)cnt.nodes);
        atomicAdd(&A.counters[3], (unsigned long long)cnt.tris);
        atomicAdd(&A.counters[5], (unsigned long long)cnt.oc_checks);
        atomicAdd(&A.counters[6], (unsigned long long)cnt.oc_replays);
    }
}

// ---------------------------------------------------------------- path tracing with a wave ray queue
// k_render_rq: the same per-lane path state machine as k_render (one lane per traced pixel,
// its samples in order on one RNG stream), but the lanes of a wave share their rays.  Shading
// a hit yields up to three independent queries -- EstimateDirect's two shadow rays and the
// continuation (whose light-loop bound is known at once) -- because none of their results feeds
// back into the RNG draws or the continuation.  They go into the wave's LDS outbox; in the
// traversal phase every lane takes the next queued ray of any lane as soon as its current one
// resolves, so lanes stay busy until the wave's queue drains instead of idling behind the
// slowest query of each round.  A path whose results are all in then accumulates the
// EstimateDirect term in the reference's order ((0 + c1) + c2) * nL * beta, and shades its
// next hit.  Each lane's operations and their order are those of k_render (bit-identical).
//
// LDS per wave: outbox [kind][lane] 32 B {o, tmax}, {d, -} (kind 0 continuation / camera
// ray, 1 and 2 the shadow rays), results [lane] {ext hit, shadow 1, shadow 2}, and two rings
// of queued (lane, kind) ids: priority lanes' rays and the others.  A wave has at most 192 rays
// outstanding (three per lane), so 256-entry rings with 8-bit wrap never overflow.
//
// Priority lanes (small shards, RenderArgs::rq_prio): the costliest pixels' serial sample
// chains set a small shard's time, and in a full wave each of their bounces waited for every
// queued ray of the wave (~3 traversals per lane) before the next path phase.  Their rays are
// taken first, and the traversal phase ends once no priority ray is queued or in flight while a
// priority lane waits for its results; the other lanes' rays stay queued or keep their
// traversal state for the next phase.  Only the order of work changes (bit-identical).
//
// Speculative pairs (RenderArgs::rq_pairs, small shards): a pixel's samples form one chain only
// through its RNG stream -- sample k+1 starts from the xorshift state sample k ends with -- and the
// number of draws a sample takes is highly predictable (glassSphere: 76-91 % of a costly pixel's
// samples take exactly 46 draws, 5 bounces).  A costly pixel therefore gets two lanes: one runs
// the chain's frontier sample F from its true start state, the other runs sample F+1 from the
// state F would end with if it took the predicted number of draws (Boyer-Moore majority of the
// pixel's counts so far).  When F ends, its end state is F+1's true start: if it equals the
// speculative start, F+1's work is kept (a sample's result depends only on the pixel, the sample
// index and the start state, so it is exactly the chain's result); otherwise it is dropped and
// F+1 runs again from the true state.  Results are written only once verified.  Up to two
// samples per chain step instead of one for the costliest pixels, whose chains bound a small
// shard; the frame is unchanged (bit-identical).
#define RQ_PENDING 0xFFFFFFFEu
#define RQ_RING 256u
NHD size_t rq_lds_bytes(uint32_t stack_depth, uint32_t block) {
    const uint32_t waves = block / 64;
    return (size_t)stack_depth * block * 8 + (size_t)waves * 3 * 64 * 32 + (size_t)block * 16 +
           (size_t)waves * 2 * RQ_RING;
}

// 512-thread blocks: one block of 8 waves per CU shares one copy of the staged BVH nodes (twice
// as many nodes in LDS).  With the wave-group refill (no wave waits for its block) C3 392 vs
// 407 ms per frame (profiles/r02m_rq_block_ab.log); before it, blocks retiring as a whole made
// 256 faster (132.6 vs 121.5 ms at 64 spp)
#ifndef NART_RQ_BLOCK
#define NART_RQ_BLOCK 512
#endif
// The counter pass (COUNT: untimed, its counts are per ray and do not depend on the schedule) runs
// 256-lane blocks at one wave per SIMD, so its counters do not push the kernel past 256 VGPRs.
//
// WV = 3: the lean throughput build for launches of >= 3 rounds of resident waves (whole frames),
// which never use priority lanes or speculative pairs: that code and its state compiled out, 768-lane
// blocks (12 waves per CU) at three waves per SIMD; only for scenes whose specialised build fits
// 168 VGPRs and whose traversal stack fits the block's LDS (render.hip lean_fits).
#define RQ_BLOCK_OF(COUNT, WV) ((COUNT) ? 256 : ((WV) == 3 ? 768 : NART_RQ_BLOCK))
//
// PR = false (with WV = 3): the lean build proper.  PR = true keeps the small-shard schedule's code
// (priority lanes, speculative pairs, raised issue priority) at three waves per SIMD.
template <bool EXT, bool COUNT, bool ENV, uint32_t FM = FT_ALL, int WV = 2, bool PR = true>
__global__ __launch_bounds__(RQ_BLOCK_OF(COUNT, WV), COUNT ? 1 : (WV == 3 ? 3 : NART_RENDER_WAVES)) void k_render_rq(DScene S, RenderArgs A) {
    // priority lanes, speculative groups and raised issue priority: small-shard schedules only
    const uint32_t rq_prio = PR ? A.rq_prio : 0u, rq_pairs = PR ? A.rq_pairs : 0u;
    // a lean build whose shading needs more than Lambert lobes and area lights fits 168 VGPRs only
    // without the paired sample reads and with the traced ray re-formed per phase (below); the
    // Lambert-only build keeps both (132 -> 164 VGPRs, still three waves)
    constexpr bool TIGHT = WV == 3 && (FM & ~(FT_LAMBERT | FT_DISK | FT_RING)) != 0u;
    const uint32_t rq_setprio = PR ? A.rq_setprio : 0u;
    extern __shared__ __attribute__((aligned(16))) int s_dyn[];
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const int stride = blockDim.x;
    const uint32_t nwave = blockDim.x / 64;
    int2* s_stack = reinterpret_cast<int2*>(s_dyn);
    constexpr bool SHORT = WV == 3;  // short LDS stack (RenderArgs::stack_lds)
    const uint32_t sk = SHORT ? A.stack_lds : A.stack_depth;
    float4* s_out = reinterpret_cast<float4*>(s_stack + sk * blockDim.x);  // [wave][kind][lane][2]
    uint4* s_res = reinterpret_cast<uint4*>(s_out + nwave * 3 * 64 * 2);             // [wave*64 + lane]
    uint8_t* s_nring = reinterpret_cast<uint8_t*>(s_res + blockDim.x) + wv * 2 * RQ_RING;  // this wave's id rings
    uint8_t* s_pring = s_nring + RQ_RING;
    float4* s_nodes = reinterpret_cast<float4*>(reinterpret_cast<uint8_t*>(s_res + blockDim.x) + nwave * 2 * RQ_RING);
    stage_nodes<ENV>(S, s_nodes, A.lds_nodes);
    const int nl = (int)A.lds_nodes;
    float4* my_out = s_out + (size_t)wv * 3 * 64 * 2;  // kind k, lane l: my_out[(k * 64 + l) * 2]
    uint4* my_res = s_res + tid;
    int* sc = reinterpret_cast<int*>(s_stack + tid);
    const float nL = (float)S.num_lights;
    const uint32_t gid = blockIdx.x * blockDim.x + tid;
    int2* gstk = SHORT ? A.gstack + (size_t)gid * (A.stack_depth - sk) : nullptr;

    uint32_t slot = gid;
    bool gdone = false;  // ghead: no slot group left
    if (A.ghead) {
        uint32_t g = 0;
        if (lane == 0) g = atomicAdd(A.ghead, 1u);
        g = __builtin_amdgcn_readfirstlane(g);
        gdone = 64u * g >= A.n_slots;
        if (A.gorder && !gdone) g = A.gorder[g];
        slot = 64u * g + (uint32_t)lane;
        if (gdone || slot >= A.n_slots) slot = 0xFFFFFFFFu;
    } else if (A.queue) {
        slot = gid < (A.qlen ? A.qlen : A.n_slots) ? A.queue[gid] : 0xFFFFFFFFu;
    } else if (slot >= A.n_slots) {
        slot = 0xFFFFFFFFu;  // the lane still serves its wave's queue
    }
    uint32_t px = 0, py = 0, rng = 0, sstr = 0;
    uint64_t soff = 0;
    bool prio = false;  // this lane's pixel is a priority pixel (queue entry bit 31)
    // speculative pair state (rq_pairs): pm = the lane is one of its pixel's two lanes; the job is
    // sample s (A.spp: none) from start state jst, verified (start known true) or speculative,
    // finished (result jres held until verified, end state jend, nd draws) or doomed (dropped
    // while its rays are still in flight).  pF / pR: the chain frontier (first sample not yet
    // written) and its true start state; bm: majority vote over the draw counts (val | cnt << 16).
    bool pm = false;
    uint32_t pQ = 1;  // lanes of this pixel's speculative group (rq_pairs, or 4 with RQ_QUAD_BIT)
    uint32_t jfl = 0, jst = 0, jend = 0, nd = 0, pF = 0, pR = 0, bm = 0;
    float4 jres = make_float4(0.f, 0.f, 0.f, 0.f);
    enum { J_VER = 1, J_FIN = 2, J_DOOM = 4 };
    // the lane's next sample and camera hit, read with the current one (c_s: its index, or none)
    uint32_t c_s = 0xFFFFFFFFu, c_prim = NO_HIT;
    float2 c_sm = make_float2(0.f, 0.f);
    auto take_pixel = [&](uint32_t sl) {
        c_s = 0xFFFFFFFFu;
        prio = rq_prio && (sl & RQ_PRIO_BIT);
        pm = rq_pairs && (sl & RQ_PAIR_BIT);
        pQ = (rq_pairs && (sl & RQ_QUAD_BIT)) ? 4u : (rq_pairs ? rq_pairs : 1u);
        if (rq_prio) sl &= ~(RQ_PRIO_BIT | RQ_PAIR_BIT | RQ_QUAD_BIT);
        slot = sl;
        const uint32_t xy = A.slot_xy[sl];
        px = xy & 0xFFFFu;
        py = xy >> 16;
        rng = A.rng0[sl];
        const SlotSO so = A.slot_so[sl];
        soff = so.first;
        sstr = so.stride;
    };
    if (slot != 0xFFFFFFFFu) take_pixel(slot);
    uint32_t s = slot != 0xFFFFFFFFu ? 0u : A.spp;
    if (pm) {
        // the even lane starts the chain (verified); the odd lane joins once a draw count is known
        pF = 0;
        pR = rng;
        bm = 0;
        jst = rng;
        jfl = J_VER;
        if (lane & (pQ - 1u)) {
            s = A.spp;
            jfl = 0;
        }
    }

    TraceCounters cnt = {0u, 0u, 0u, 0u};
    uint32_t n_ext = 0, n_sh = 0, n_bounce = 0;
    f3 L = F3(0.f, 0.f, 0.f), beta = F3(0.f, 0.f, 0.f);
    f3 c1 = F3(0.f, 0.f, 0.f), c2 = F3(0.f, 0.f, 0.f), betak = F3(0.f, 0.f, 0.f);
    float alpha = 0.f, eta_sampled = 1.f, eta_outer = 1.f, alphaTweak = 1.f;
    uint32_t flags = 0, bounce = 0;
    // the compact list (no eta registers) where the feature mask allows it
    constexpr bool CL = !EXT && !(FM & (FT_TEX | FT_PLASTIC));
    IList<EXT, CL> list;
    list.n = 0;
    bool lightHit = false, use1 = false, use2 = false, have_ed = false, ext_pending = false;
    bool waiting = false;  // rays of this lane's path are queued or in flight
    uint32_t newk = 0;     // rays this lane queued in the current path phase (bit per kind)

    // traversal state of the ray this lane is tracing (any lane's)
    Trav tq;
    Ray tr;
    uint32_t tid8 = 0;  // queued id: owner lane | kind << 6
    bool tracing = false;
    bool tr_prio = false;  // the ray being traced is a priority lane's
    // wave-uniform ring positions (ids at [pos & (RQ_RING - 1)]): other / priority rays
    uint32_t nh = 0, nt = 0, ph = 0, pt = 0;

    auto put_ray = [&](int kind, f3 o, f3 d, float tmax) {
        float4* e = my_out + (kind * 64 + lane) * 2;
        e[0] = make_float4(o.x, o.y, o.z, tmax);
        e[1] = make_float4(d.x, d.y, d.z, 0.f);
        newk |= 1u << kind;
    };
    // light intersections of a new extension ray (pathintegrator.cpp:167-182): Le, lightHit,
    // alpha; returns the query bound
    // The loop keeps only the bound and the index of the light that set it (lwin): the radiance Le
    // of that light reaches L only when the camera ray escapes (pathintegrator.cpp:252-256, Q7),
    // and light_le evaluates it then -- the same light_li of the same ray, so the same Le -- instead
    // of evaluating every light's radiance on every ray (the environment light: acosf + atan2f +
    // a texture fetch).
    uint32_t lwin = 0;
    auto light_loop = [&](f3 o, f3 d) {
        float lightTMax = __builtin_inff();
        lightHit = false;
        for (uint32_t j = 0; j < S.num_lights; ++j) {
            float lt = __builtin_inff();
            light_bound<ENV, FM>(uniform_light(S, j), o, d, lt);
            if (lt < lightTMax) {
                lightTMax = lt;
                lightHit = true;
                alpha = 1.f;
                lwin = j;
            }
        }
        return lightTMax;
    };
    auto light_le = [&](f3 o, f3 d) {
        float lt = __builtin_inff();
        return light_li<ENV, FM>(S, cst(S.lights)[lwin], o, d, nullptr, lt);
    };
    auto draw = [&]() {
        ++nd;
        return rng_float(rng);
    };
    // a sample's result: written at once, or held by a pair lane until verified.  (Pairing an even
    // sample's result with the odd one after it as one 32-B store cut the writes 26.6 -> 11.1 GB
    // per C3 launch but ran 2.3 % slower, profiles/r05j_pair_writes_ab.log; retired in round 6.)
    auto end_sample = [&](float4 v) {
        if (pm) {
            jres = v;
            jend = rng;
            jfl |= J_FIN;
        } else {
            A.Lout[soff + (uint64_t)s * sstr] = v;
            ++s;
        }
    };
    auto queue_ext = [&](f3 o, f3 d) {
        put_ray(0, o, d, light_loop(o, d));
        ext_pending = true;
        if (COUNT) ++n_ext;
    };

    bool raised = false;  // this wave runs at a raised issue priority (A.rq_setprio)
    for (;;) {
        // ---------------- path phase
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        newk = 0;
        if (rq_setprio) {
            const bool want = __ballot(prio && (pm || waiting || s < A.spp)) != 0;
            if (want != raised) {
                if (want) __builtin_amdgcn_s_setprio(2);
                else __builtin_amdgcn_s_setprio(0);
                raised = want;
            }
        }
        // 1. results of lanes whose queries are all in: EstimateDirect term, then the hit to
        //    shade or the end of the sample
        bool need_shade = false;
        uint32_t hitg = NO_HIT;
        if (waiting) {
            const uint4 r = *my_res;
            if ((!ext_pending || r.x != RQ_PENDING) && (!use1 || r.y != 2u) && (!use2 || r.z != 2u)) {
                waiting = false;
                if (jfl & J_DOOM) {
                    jfl = 0;  // a dropped speculative job: its rays are back, nothing to keep
                } else {
                // L += EstimateDirect(...) * beta, EstimateDirect = ((0 + c1) + c2) * numLights
                if (have_ed) {
                    f3 Led = F3(0.f, 0.f, 0.f);
                    if (use1 && r.y == 0u) Led = add(Led, c1);
                    if (use2 && r.z == 0u) Led = add(Led, c2);
                    L = add(L, mul(muls(Led, nL), betak));
                }
                if (ext_pending && r.x != NO_HIT) {
                    need_shade = true;
                    hitg = r.x;
                } else {
                    // escaped (at bounce 0 the light seen directly is the result, Q6, Q7) or ended
                    if (ext_pending && bounce == 0 && lightHit) {
                        // the camera ray, still in this lane's outbox entry of kind 0
                        const float4 ro = my_out[lane * 2], rd = my_out[lane * 2 + 1];
                        L = light_le(F3(ro.x, ro.y, ro.z), F3(rd.x, rd.y, rd.z));
                    }
                    end_sample(make_float4(L.x, L.y, L.z, alpha));
                }
                }
            }
        }
        // speculative lane groups (A.rq_pairs = Q lanes per costly pixel, 2 or 4): commit verified
        // results in sample order, check speculative starts, hand out the next jobs.  Every lane of
        // a group evaluates the same function of the group's Q job records (exchanged with
        // shuffles inside the group) and keeps its own record.  Jobs in flight always cover a
        // contiguous run of samples [pF, hs]; a job becomes verified when it reaches the frontier
        // with the frontier's true start state, otherwise every job of the run is dropped.
        if (rq_pairs) {
            const uint32_t Q = pQ, gb = (uint32_t)lane & ~(Q - 1u), mi = (uint32_t)lane & (Q - 1u);
            const uint32_t NONE = A.spp;
            uint32_t gs[4], gst[4], gfl[4], gend[4], gnd[4];
            bool gw[4], gchg[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const int src = (int)(gb + (k < Q ? k : 0u));
                gs[k] = __shfl(s, src);
                gst[k] = __shfl(jst, src);
                gfl[k] = __shfl(jfl, src);
                gend[k] = __shfl(jend, src);
                gnd[k] = __shfl(nd, src);
                gw[k] = __shfl(waiting ? 1u : 0u, src) != 0u;
                gchg[k] = false;
                if (k >= Q) {
                    gs[k] = NONE;
                    gfl[k] = 0u;
                }
            }
            if (pm) {
#pragma unroll
                for (uint32_t it = 0; it < 4; ++it) {
                    uint32_t kc = 4u;
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k)
                        if (gs[k] == pF && (gfl[k] & J_VER) && (gfl[k] & J_FIN)) kc = k;
                    if (kc == 4u) break;
                    if (kc == mi) A.Lout[soff + (uint64_t)pF * sstr] = jres;
                    // majority vote over the committed samples' draw counts
                    uint32_t n = 0u, e = 0u;
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k)
                        if (k == kc) {
                            n = gnd[k];
                            e = gend[k];
                        }
                    const uint32_t bv = bm & 0xFFFFu, bc = bm >> 16;
                    bm = (n == bv) ? (bv | ((bc + 1u) << 16)) : (bc == 0u ? (n | (1u << 16)) : (bv | ((bc - 1u) << 16)));
                    pR = e;
                    ++pF;
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k)
                        if (k == kc) {
                            gs[k] = NONE;
                            gfl[k] = 0u;
                        }
                    // the new frontier's job: keep it iff it started from the true state, else
                    // drop every job of the run (their starts were predicted from it)
                    bool bad = false;
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k)
                        if (gs[k] == pF && !(gfl[k] & J_VER)) {
                            if (gst[k] == pR) gfl[k] |= J_VER;
                            else bad = true;
                        }
                    if (bad) {
#pragma unroll
                        for (uint32_t k = 0; k < 4; ++k)
                            if (gs[k] != NONE) {
                                gfl[k] = gw[k] ? J_DOOM : 0u;
                                gs[k] = NONE;
                                gchg[k] = true;
                            }
                    }
                }
                // next jobs, in lane order: the frontier from its true state when no job holds it,
                // else the sample after the run from the last job's end state (if finished) or
                // its start advanced by the predicted number of draws
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k) {
                    if (gs[k] != NONE || (gfl[k] & J_DOOM) || k >= Q) continue;
                    uint32_t hs = NONE, hst = 0u, hfl = 0u, hend = 0u;
#pragma unroll
                    for (uint32_t j = 0; j < 4; ++j)
                        if (gs[j] != NONE && (hs == NONE || gs[j] > hs)) {
                            hs = gs[j];
                            hst = gst[j];
                            hfl = gfl[j];
                            hend = gend[j];
                        }
                    if (hs == NONE) {
                        if (pF < A.spp) {
                            gs[k] = pF;
                            gst[k] = pR;
                            gfl[k] = J_VER;
                            gchg[k] = true;
                        }
                    } else if (hs + 1u < A.spp && (bm >> 16) != 0u) {
                        gs[k] = hs + 1u;
                        gst[k] = (hfl & J_FIN) ? hend : rng_jump(hst, bm & 0xFFFFu);
                        gfl[k] = 0u;
                        gchg[k] = true;
                    }
                }
                uint32_t ms = NONE, mst = 0u, mfl = 0u;
                bool mchg = false, any_doom = false, all_none = true;
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k) {
                    if (k == mi) {
                        ms = gs[k];
                        mst = gst[k];
                        mfl = gfl[k];
                        mchg = gchg[k];
                    }
                    any_doom = any_doom || (gfl[k] & J_DOOM);
                    all_none = all_none && gs[k] == NONE;
                }
                if (mchg) {
                    need_shade = false;  // a dropped job's pending hit, or a job that starts afresh
                    rng = mst;
                }
                s = ms;
                jst = mst;
                jfl = mfl;
                if (pF >= A.spp && all_none && !any_doom) pm = false;
            }
        }
        // pixel refill (persistent grid): one queue atomic per wave
        if (A.qhead) {
            const bool need = !pm && !waiting && s >= A.spp && slot != 0xFFFFFFFEu;
            const uint64_t m = __ballot(need);
            if (m) {
                const int leader = __builtin_ctzll(m);
                uint32_t base = 0;
                if ((int)__lane_id() == leader) base = atomicAdd(A.qhead, (uint32_t)__popcll(m));
                base = __builtin_amdgcn_readlane(base, leader);
                if (need) {
                    const uint32_t idx = A.qbase + base +
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    if (idx < (A.qlen ? A.qlen : A.n_slots)) {
                        take_pixel(A.queue[idx]);
                        s = 0;
                    } else {
                        slot = 0xFFFFFFFEu;  // queue exhausted: no further refill attempts
                    }
                }
            }
        }
        if (A.ghead && !gdone && __ballot(waiting || need_shade || tracing || s < A.spp) == 0) {
            // every pixel of the wave is done: the next group of 64 slots (one atomic per wave)
            uint32_t g = 0;
            if (lane == 0) g = atomicAdd(A.ghead, 1u);
            g = __builtin_amdgcn_readfirstlane(g);
            gdone = 64u * g >= A.n_slots;
            if (A.gorder && !gdone) g = A.gorder[g];
            const uint32_t sl = 64u * g + (uint32_t)lane;
            if (!gdone && sl < A.n_slots) {
                take_pixel(sl);
                s = 0;
            }
        }
        bool active = !waiting && !need_shade && s < A.spp && !(jfl & J_FIN);
        // 2. new samples (pathintegrator.cpp:144-166; render.cpp:87-95).  A camera ray that
        //    k_primary found to escape, or a zero bounce limit, ends its sample here, so loop until
        //    a hit is to be shaded, a ray is queued or the pixel is done.
        while (active) {
            nd = 0;
            // pixel-major rows (stride 1): samples and camera hits are read in pairs, the odd one
            // kept for the lane's next sample -- each read of a line the lane's neighbours do not
            // share then serves two samples
            float2 sm;
            uint32_t gprim = NO_HIT;
            {
                const uint64_t si = soff + (uint64_t)s * sstr;
                // (not in the environment-light, deep-list, counter-pass or lean builds, whose registers
                // would spill)
                constexpr bool PF = !ENV && !EXT && !COUNT && !TIGHT;
                if (PF && s == c_s) {
                    sm = c_sm;
                    gprim = c_prim;
                } else if (PF && sstr == 1u && (si & 1u) == 0u && s + 1u < A.spp) {
                    const float4 q = reinterpret_cast<const float4*>(A.samples)[si >> 1];
                    sm = make_float2(q.x, q.y);
                    c_sm = make_float2(q.z, q.w);
                    if (A.prim) {
                        const uint2 h = reinterpret_cast<const uint2*>(A.prim)[si >> 1];
                        gprim = h.x;
                        c_prim = h.y;
                    }
                    c_s = s + 1u;
                } else {
                    sm = A.samples[si];
                    if (A.prim) gprim = A.prim[si];
                }
            }
            const Ray ray = cast_ray(S, F2(sm.x, sm.y), A.W, A.H, px, py);
            L = F3(0.f, 0.f, 0.f);
            alpha = 0.f;
            eta_sampled = 1.f;
            eta_outer = 1.f;
            beta = F3(1.f, 1.f, 1.f);
            flags = 0;
            alphaTweak = 1.f;
            bounce = 0;
            list.n = 0;
            use1 = use2 = have_ed = false;
            ext_pending = false;
            if (A.bounces == 0) {
                end_sample(make_float4(0.f, 0.f, 0.f, 0.f));
                active = !pm && s < A.spp;
                continue;
            }
            if (A.prim) {
                // camera ray traced by k_primary: shade its hit in this phase
                const uint32_t g = gprim;
                const float t = light_loop(ray.o, ray.d);
                if (g == NO_HIT) {
                    if (lightHit) L = light_le(ray.o, ray.d);
                    end_sample(make_float4(L.x, L.y, L.z, alpha));
                    active = !pm && s < A.spp;
                    continue;
                }
                float4* e = my_out + lane * 2;
                e[0] = make_float4(ray.o.x, ray.o.y, ray.o.z, t);
                e[1] = make_float4(ray.d.x, ray.d.y, ray.d.z, 0.f);
                need_shade = true;
                hitg = g;
            } else {
                queue_ext(ray.o, ray.d);
                waiting = true;
            }
            active = false;
        }
        // 3. shade the hits (pathintegrator.cpp:185-246)
        if (need_shade) {
            if (COUNT) ++n_bounce;
            const float4 ro = my_out[lane * 2], rd = my_out[lane * 2 + 1];
            const Ray cur = make_ray(F3(ro.x, ro.y, ro.z), F3(rd.x, rd.y, rd.z));
            Isect is;
            fill_isect(S, cur, hitg, is);
            BSDF bsdf;
            create_bsdf<FM>(S, is, alphaTweak, bsdf);
            use1 = use2 = false;
            bool cont;
            f3 no, nd;
            if (list.valid(is.meshID, is.priority, eta_outer, ILIST_X(A), A.ilist_stride, S.mesh_eta)) {
                if (bounce == 0) alpha = 1.f;
                const f3 wo = to_local(bsdf, neg(cur.d));
                // ---- EstimateDirect (pathintegrator.cpp:38-121)
                const uint32_t lsel = f2u8(gmin(draw(), ND_ONE_MINUS_EPS) * nL);
                const DLight& Lg = cst(S.lights)[lsel];
                // One light (every BASELINE scene): the pick is 0 on every lane, so the light is
                // read through a wave-uniform index (scalar loads of the light record and, for an
                // environment light, its sampling tables): C3 / C2 frames -1.3 %, C4 -0.9 %
                // (profiles/r05am_one_light_all.log, r05al_c4_one_light_ab.log)
                const bool one_light = S.num_lights == 1u;
                float sPdf = 0.f, lPdf = 0.f;
                float sx = draw();
                float sy = draw();
                float bsmp = draw();
                uint32_t dflags = 0;
                f3 wi;
                f3 f = bsdf_sample_f<ENV, FM>(bsdf, wo, wi, bsmp, F2(sx, sy), sPdf, dflags, true, eta_outer, nullptr,
                                     nullptr);
                if (sPdf > 0.f) {
                    float flip = wi.z > 0.f ? 1.f : -1.f;
                    f3 wW = to_world(bsdf, wi);
                    float lt = __builtin_inff();
                    f3 Li = one_light ? light_li<ENV, FM>(S, uniform_light(S, 0u), is.p, wW, &lPdf, lt)
                                      : light_li<ENV, FM>(S, Lg, is.p, wW, &lPdf, lt);
                    float weight = 1.f;
                    bool add1 = true;
                    if (!(dflags & F_SPECULAR)) {
                        weight = (sPdf * sPdf) / (sPdf * sPdf + lPdf * lPdf);
                        add1 = lPdf > 0.f;
                    }
                    if (add1) {
                        c1 = divs(muls(muls(mul(f, Li), gabs(wi.z)), weight), sPdf);
                        // an all-zero term cannot change the sum: skip its shadow ray
                        use1 = !(c1.x == 0.f && c1.y == 0.f && c1.z == 0.f);
                        if (use1) put_ray(1, add(is.p, muls(muls(is.gn, SHADOW_BIAS), flip)), wW, lt);
                    }
                }
                lPdf = 0.f;
                float lx = draw();
                float ly = draw();
                f3 wiW;
                float lt2 = __builtin_inff();
                f3 Li2 = one_light ? light_sample_li<ENV, FM>(S, uniform_light(S, 0u), is.p, wiW, F2(lx, ly), lPdf, lt2)
                                   : light_sample_li<ENV, FM>(S, Lg, is.p, wiW, F2(lx, ly), lPdf, lt2);
                f3 wi2 = to_local(bsdf, wiW);
                if (lPdf > 0.f) {
                    float sp2;
                    const f3 fv = bsdf_f_pdf<FM>(bsdf, wo, wi2, true, eta_outer, sp2);
                    if (sp2 > 0.f) {
                        float weight = (lPdf * lPdf) / (sp2 * sp2 + lPdf * lPdf);
                        c2 = divs(muls(muls(mul(fv, Li2), gabs(wi2.z)), weight), lPdf);
                        use2 = !(c2.x == 0.f && c2.y == 0.f && c2.z == 0.f);
                        if (use2) {
                            float flip2 = wi2.z > 0.f ? 1.f : -1.f;
                            put_ray(2, add(is.p, muls(muls(is.gn, SHADOW_BIAS), flip2)), wiW, lt2);
                        }
                    }
                }
                betak = beta;
                have_ed = true;
                // ---- continuation (pathintegrator.cpp:199-220)
                float a = draw();
                float b = draw();
                float bs2 = draw();
                float cpdf = 0.f, alpha_i = 0.f;
                f3 wic;
                f3 fc = bsdf_sample_f<ENV, FM>(bsdf, wo, wic, bs2, F2(a, b), cpdf, flags, false, eta_outer, &alpha_i,
                                      &eta_sampled);
                if (cpdf <= 0.f) {
                    cont = false;
                } else {
                    alphaTweak = (1.f - (A.gamma * alpha_i)) * alphaTweak;
                    beta = mul(beta, muls(divs(fc, cpdf), gabs(wic.z)));
                    float flip = wic.z > 0.f ? 1.f : -1.f;
                    no = add(is.p, muls(muls(is.gn, SHADOW_BIAS), flip));
                    nd = to_world(bsdf, wic);
                    cont = true;
                }
            } else {
                // lower-priority interface: step through (pathintegrator.cpp:223-229)
                no = add(is.p, muls(cur.d, SHADOW_BIAS));
                nd = cur.d;
                flags = F_TRANSMISSIVE;
                float bs2 = draw();
                eta_sampled = bsdf_sample_eta<FM>(bsdf, bs2);
                cont = true;
                have_ed = false;
            }
            if (cont) {
                if (flags & F_TRANSMISSIVE) list.update(is.meshID, is.priority, eta_sampled, ILIST_X(A), A.ilist_stride);
                // Russian roulette (pathintegrator.cpp:236-246)
                float q = gmax((beta.x + beta.y + beta.z) * 0.33333f, 0.f);
                if (bounce > 3) {
                    if (q >= draw()) beta = divs(beta, q);
                    else cont = false;
                }
            }
            ++bounce;
            if (COUNT) n_sh += (use1 ? 1u : 0u) + (use2 ? 1u : 0u);
            ext_pending = false;
            if (cont && bounce < A.bounces) queue_ext(no, nd);
            if (newk) {
                waiting = true;
            } else {
                // no query left (path ended, or ended at the bounce limit): the EstimateDirect
                // term of this bounce, if any, is still owed
                if (have_ed) L = add(L, mul(muls(F3(0.f, 0.f, 0.f), nL), betak));
                end_sample(make_float4(L.x, L.y, L.z, alpha));
            }
        }
        // queued rays: init the result words, then list the (lane, kind) ids in kind order
        if (newk) {
            uint4 r0 = *my_res;
            if (newk & 1u) r0.x = RQ_PENDING;
            if (newk & 2u) r0.y = 2u;
            if (newk & 4u) r0.z = 2u;
            *my_res = r0;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const bool want = (newk >> k) & 1u;
            const bool wp = want && prio, wn = want && !prio;
            const uint64_t m = __ballot(wn);
            if (wn) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                s_nring[(nt + rank) & (RQ_RING - 1u)] = (uint8_t)(lane | (k << 6));
            }
            nt += (uint32_t)__popcll(m);
            if (rq_prio) {
                const uint64_t mp = __ballot(wp);
                if (wp) {
                    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mp >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)mp, 0u));
                    s_pring[(pt + rank) & (RQ_RING - 1u)] = (uint8_t)(lane | (k << 6));
                }
                pt += (uint32_t)__popcll(mp);
            }
        }
        // a lane whose sample ended while shading starts its next sample in the next phase; one
        // whose pixel is done may still get a pixel from the queue
        const bool more = !waiting && (s < A.spp || pm || (A.qhead && slot != 0xFFFFFFFEu) || (A.ghead && !gdone));
        if (__ballot(waiting || tracing || more) == 0) break;  // every path of the wave is done
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");

        // ---------------- traversal phase: lanes take the wave's queued rays in turn
        if (TIGHT) {
            // lean build: the traced ray and its slab-test constants are formed again from the ray's
            // outbox entry (it stays there until the ray resolves) with trav_begin's operations, so
            // they are not held in registers through the path phase (the old values are dead: the
            // same bits, 16 fewer registers at the shading peak)
            if (tracing) {
                const uint32_t owner = tid8 & 63u, kind = tid8 >> 6;
                const float4 a = my_out[(kind * 64 + owner) * 2], b = my_out[(kind * 64 + owner) * 2 + 1];
                tr = make_ray(F3(a.x, a.y, a.z), F3(b.x, b.y, b.z));
                trav_slab(tr, tq);
            } else {
                tr = Ray{};
                tq.inv = tq.oi = F3(0.f, 0.f, 0.f);
            }
        }
        for (;;) {
            const bool need = !tracing;
            const uint64_t mn = __ballot(need);
            const uint32_t avp = pt - ph, avn = nt - nh;
            if (mn && avp + avn > 0u) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mn >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)mn, 0u));
                if (need && rank < avp + avn) {
                    tr_prio = rank < avp;
                    tid8 = tr_prio ? s_pring[(ph + rank) & (RQ_RING - 1u)] : s_nring[(nh + rank - avp) & (RQ_RING - 1u)];
                    const uint32_t owner = tid8 & 63u, kind = tid8 >> 6;
                    const float4 a = my_out[(kind * 64 + owner) * 2], b = my_out[(kind * 64 + owner) * 2 + 1];
                    tr = make_ray(F3(a.x, a.y, a.z), F3(b.x, b.y, b.z));
                    trav_begin(S, tr, a.w, kind != 0u, tq);
                    tracing = true;
                }
                const uint32_t took = min((uint32_t)__popcll(mn), avp + avn);
                const uint32_t tp = min(took, avp);
                ph += tp;
                nh += took - tp;
            }
            bool fin = false;
            if (tracing) {
                fin = !S.geometry_visible;  // one-chunk scenes render no geometry (Q14)
                if (!fin) fin = trav_step<COUNT, ENV, SHORT>(S, tr, tq, sc, gstk, stride, cnt, s_nodes, nl, (int)sk);
            }
            if (fin) {
                tracing = false;
                float bt = tq.bestT;
                uint32_t bg = tq.bestG;
                if (S.geometry_visible)
                    oc_resolve<COUNT>(S, tr, tq.tmax, tq.any, tq.risky, tq.bestInfo, fminf(tq.t2, oc_cull(S, tq.bestT)),
                                      bt, bg, cnt);
                uint32_t* rw = reinterpret_cast<uint32_t*>(s_res + wv * 64 + (tid8 & 63u));
                const uint32_t kind = tid8 >> 6;
                rw[kind] = kind == 0u ? bg : (bg != NO_HIT ? 1u : 0u);
            }
            // priority rays all resolved and a priority lane waits on its results: shade it now (ending
            // the phase as soon as 1/2/4/8 priority lanes were ready, with other priority rays still in
            // flight, measured slower: C3 1/8 shard 121/114/102/94 vs 90 ms, profiles/r05d_rq_early_ab.log
            // -- more path phases, each costing the union of the wave's shading branches; and letting
            // the other lanes sit out the path phases the priority rule starts unless 8 / 24 / 64 of
            // them are ready: 89.9 / 91.0 / 94.4 vs 88.9 ms)
            if (rq_prio && ph == pt && __ballot(tracing && tr_prio) == 0 && __ballot(waiting && prio) != 0) break;

            if (ph == pt && nh == nt && (uint32_t)__popcll(__ballot(tracing)) <= A.rq_quorum) break;
        }
    }
    if (COUNT) {
        atomicAdd(&A.counters[0], (unsigned long long)n_ext);
        atomicAdd(&A.counters[1], (unsigned long long)n_sh);
        atomicAdd(&A.counters[2], (unsigned long long)cnt.nodes);
        atomicAdd(&A.counters[3], (unsigned long long)cnt.tris);
        atomicAdd(&A.counters[4], (unsigned long long)n_bounce);
        atomicAdd(&A.counters[5], (unsigned long long)cnt.oc_checks);
        atomicAdd(&A.counters[6], (unsigned long long)cnt.oc_replays);
    }
}

// ---------------------------------------------------------------- splat (gather form)
struct SplatArgs {
    const uint32_t* bucket_ids;   // [n_buckets] bucket id = by * nbx + bx
    const uint32_t* bucket_base;  // [n_buckets] first slot of each bucket
    const float2* samples;        // sample-major per bucket (RenderArgs::slot_so)
    const float4* Lout;           // same layout
    float* tiles;                 // [n_buckets][tile*tile][5] (nart_pixel AoS)
    const float* table;           // [64] Gaussian filter table
    const float* thr;             // [65] filter-index thresholds on d2 (splat_thresholds), or null
    float idx_scale;              // 64 / fw: the estimate of the filter index that thr corrects
    uint32_t n_buckets, spp, B, fb, tile, nbx, totalW, totalH;
    float fw;
    float invB, invFw;            // exact reciprocals when B / fw are powers of two, else 0
    // filter weight by d2 cell (splat_lut): cell = clamp((bits(d2) >> 16) - lut_b0, 0, lut_n - 1),
    // {threshold, weight below, weight at or above, -}; null when the table does not apply
    const float4* lut = nullptr;
    uint32_t lut_b0 = 0, lut_n = 0;
};
#define SPLAT_LUT_MAX 2048

// a / b, or a * (1/b) when 1/b is an exact power of two (bit-identical, avoids the
// correctly-rounded division sequence)
ND float div_exact(float a, float b, float inv) { return inv != 0.f ? a * inv : a / b; }

// Exact AddSample test: does this sample's splat loop (render.cpp:27-68) visit tile pixel
// (tx, ty)?  If so, return the filter weight it adds there.
//
// With mx = glm::mod(sc - fb, B) = a - B*k, k = floor(a / B) (a = sc - fb), every term of
// tileX(x) = floor(((x + 0.5) - sc) + mx + fb) is exact for coordinates < 2^22 (Sterbenz
// subtraction, an integer multiple of B, a half-integer sum), so tileX(x) = x - B*k exactly and
// the splat column that lands on tile column tx is x = tx + B*k.  k is the bucket column of the
// sample, or the next one when x + u rounds up to the bucket edge (the reference then writes the
// contribution near the tile's origin; so does this).
ND bool splat_hits(const SplatArgs& A, const float* table, float scx, float scy, uint32_t tx, uint32_t ty, float& w) {
    const float fw = A.fw, fb = (float)A.fb, Bf = (float)A.B;
    const uint32_t x0 = (uint32_t)floorf(scx - fw), x1 = (uint32_t)ceilf(scx + fw);
    const uint32_t y0 = (uint32_t)floorf(scy - fw), y1 = (uint32_t)ceilf(scy + fw);
    const uint32_t kx = (uint32_t)floorf(div_exact(scx - fb, Bf, A.invB));
    const uint32_t ky = (uint32_t)floorf(div_exact(scy - fb, Bf, A.invB));
    const uint32_t xs = tx + A.B * kx, ys = ty + A.B * ky;
    const bool hit = xs >= x0 && xs < x1 && ys >= y0 && ys < y1;
    const float distX = ((float)xs + 0.5f) - scx;
    const float distY = ((float)ys + 0.5f) - scy;
    const float dist = sqrtf(distX * distX + distY * distY);
    // static_cast<uint8_t>(float) on x86-64: truncate to int, keep the low byte
    uint32_t fi = (uint32_t)(int32_t)(div_exact(dist, fw, A.invFw) * 64) & 0xFFu;
    fi = (63u < fi) ? 63u : fi;
    w = table[fi];
    return hit;
}

// splat_hits with the filter index taken from the d2 thresholds: a hardware sqrt estimates the
// index within one step and two threshold compares make it exact (no correctly rounded sqrt and
// division per pair).
ND bool splat_hits_thr(const SplatArgs& A, const float* table, const float* thr, float scx, float scy, uint32_t tx,
                       uint32_t ty, float& w) {
    const float fw = A.fw, fb = (float)A.fb, Bf = (float)A.B;
    const uint32_t x0 = (uint32_t)floorf(scx - fw), x1 = (uint32_t)ceilf(scx + fw);
    const uint32_t y0 = (uint32_t)floorf(scy - fw), y1 = (uint32_t)ceilf(scy + fw);
    const uint32_t kx = (uint32_t)floorf(div_exact(scx - fb, Bf, A.invB));
    const uint32_t ky = (uint32_t)floorf(div_exact(scy - fb, Bf, A.invB));
    const uint32_t xs = tx + A.B * kx, ys = ty + A.B * ky;
    const bool hit = xs >= x0 && xs < x1 && ys >= y0 && ys < y1;
    const float distX = ((float)xs + 0.5f) - scx;
    const float distY = ((float)ys + 0.5f) - scy;
    const float d2 = distX * distX + distY * distY;
    int g = (int)(__builtin_amdgcn_sqrtf(d2) * A.idx_scale);
    g = g < 0 ? 0 : (g > 63 ? 63 : g);
    const float t0 = thr[g], t1 = thr[g + 1];
    const int fi = g - (d2 < t0 ? 1 : 0) + (d2 >= t1 ? 1 : 0);
    w = table[fi];
    return hit;
}

// splat_hits_fast: the compare-only form of splat_hits_thr for a power-of-two bucket size, which
// k_splat_col4 and k_splat_skew inline (the one-pixel-per-lane kernel that used it alone, splat
// mode 2, was retired in round 5):
//  * k = floor((sc - fb) / B): sc - fb is exact (both are multiples of ulp(sc)) and lies in
//    [origin + S, origin + S + 1] for bucket-local column S, and / B is exact, so k is the bucket
//    column, plus one exactly when sc - fb >= origin + B, i.e. sc >= edge (= bucket origin + B + fb);
//  * floor(a) <= xs  <=>  a < xs + 1  and  xs < ceil(b)  <=>  xs < b  for an integer xs, with
//    a = RN(sc - fw) and b = RN(sc + fw) as the reference rounds them;
//  * dist and the filter index as in splat_hits_thr.

// MODE 0: direct AddSample arithmetic (splat_hits); 1: filter index from thresholds
// (splat_hits_thr).  The fallbacks of the splat: any bucket size and filter width.
template <int MODE>
__global__ __launch_bounds__(256) void k_splat(SplatArgs A) {
    __shared__ float s_table[64];
    __shared__ float s_thr[65];
    if (threadIdx.x < 64) s_table[threadIdx.x] = A.table[threadIdx.x];
    if (MODE > 0 && threadIdx.x < 65) s_thr[threadIdx.x] = A.thr[threadIdx.x];
    __syncthreads();
#define NART_SPLAT_HITS(scx, scy, w)                                                                        \
    (MODE == 1 ? splat_hits_thr(A, s_table, s_thr, scx, scy, tx, ty, w) : splat_hits(A, s_table, scx, scy, tx, ty, w))
    const uint32_t tpx = A.tile * A.tile;
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (uint64_t)A.n_buckets * tpx) return;
    const uint32_t bi = (uint32_t)(gid / tpx), tp = (uint32_t)(gid % tpx);
    const uint32_t tx = tp % A.tile, ty = tp / A.tile;
    const uint32_t bid = A.bucket_ids[bi];
    const uint32_t bx = bid % A.nbx, by = bid / A.nbx;
    const uint32_t x0 = A.B * bx, y0 = A.B * by;
    const uint32_t x1 = min(A.B * (bx + 1), A.totalW), y1 = min(A.B * (by + 1), A.totalH);
    const int bw = (int)(x1 - x0), bh = (int)(y1 - y0);
    const uint32_t npx = (uint32_t)(bw * bh);
    const uint32_t base = A.bucket_base[bi];
    // Candidate source pixels.  A sample of bucket-local column S has sc - x0 in [S+fb, S+fb+1],
    // so its splat columns span [S+fb-ceil(fw), S+fb+1+fw): tile column tx can only be reached
    // from S in [tx-fb-ceil(fw), tx-fb+ceil(fw)].  Samples of the last column can also wrap to
    // the next bucket origin (splat_hits) and then reach tx <= fb+ceil(fw).  Same for rows.
    const int r = (int)ceilf(A.fw);
    const int sxlo = max(0, (int)tx - (int)A.fb - r), sxhi = min(bw - 1, (int)tx - (int)A.fb + r);
    const int sylo = max(0, (int)ty - (int)A.fb - r), syhi = min(bh - 1, (int)ty - (int)A.fb + r);
    float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f, ws = 0.f;
    const bool wrapx = bw == (int)A.B && (int)tx <= (int)A.fb + r + 1 && bw - 1 > sxhi;
    const bool wrapy = bh == (int)A.B && (int)ty <= (int)A.fb + r + 1 && bh - 1 > syhi;
    const int nrow = (syhi >= sylo ? syhi - sylo + 1 : 0) + (wrapy ? 1 : 0);
    const int ncol = (sxhi >= sxlo ? sxhi - sxlo + 1 : 0) + (wrapx ? 1 : 0);
    for (int ri = 0; ri < nrow; ++ri) {
        const int sy = (sylo + ri <= syhi) ? sylo + ri : bh - 1;
        const float fy = (float)(y0 + (uint32_t)sy + A.fb);
        for (int ci = 0; ci < ncol; ++ci) {
            const int sx = (sxlo + ci <= sxhi) ? sxlo + ci : bw - 1;
            const float fx = (float)(x0 + (uint32_t)sx + A.fb);
            // sample-major bucket layout (RenderArgs::slot_so): sample i of local pixel q at
            // base*spp + i*npx + q, so lanes on neighbouring source pixels share cache lines
            const uint64_t first = (uint64_t)base * A.spp + (uint32_t)(sy * bw + sx);
            const float2* sp = A.samples + first;
            const float4* lp = A.Lout + first;
            uint32_t i = 0;
            // 4 samples per step: all loads issued up front, adds applied in sample order
#ifndef NART_SPLAT_PF
#define NART_SPLAT_PF 1
#endif
#if NART_SPLAT_PF
            // software pipelined: the next 4 samples are in flight while these 4 are splatted
            float2 nu0, nu1, nu2, nu3;
            float4 nL0, nL1, nL2, nL3;
            if (A.spp >= 4) {
                nu0 = sp[0], nu1 = sp[npx], nu2 = sp[(size_t)2 * npx], nu3 = sp[(size_t)3 * npx];
                nL0 = lp[0], nL1 = lp[npx], nL2 = lp[(size_t)2 * npx], nL3 = lp[(size_t)3 * npx];
            }
            for (; i + 4 <= A.spp; i += 4) {
                const float2 uv0 = nu0, uv1 = nu1, uv2 = nu2, uv3 = nu3;
                const float4 L0 = nL0, L1 = nL1, L2 = nL2, L3 = nL3;
                if (i + 8 <= A.spp) {
                    const size_t k0 = (size_t)(i + 4) * npx;
                    nu0 = sp[k0], nu1 = sp[k0 + npx], nu2 = sp[k0 + (size_t)2 * npx], nu3 = sp[k0 + (size_t)3 * npx];
                    nL0 = lp[k0], nL1 = lp[k0 + npx], nL2 = lp[k0 + (size_t)2 * npx], nL3 = lp[k0 + (size_t)3 * npx];
                }
#else
            for (; i + 4 <= A.spp; i += 4) {
                const size_t k0 = (size_t)i * npx;
                float2 uv0 = sp[k0], uv1 = sp[k0 + npx], uv2 = sp[k0 + (size_t)2 * npx], uv3 = sp[k0 + (size_t)3 * npx];
                float4 L0 = lp[k0], L1 = lp[k0 + npx], L2 = lp[k0 + (size_t)2 * npx], L3 = lp[k0 + (size_t)3 * npx];
#endif
                float w0, w1, w2, w3;
                bool h0 = NART_SPLAT_HITS(fx + uv0.x, fy + uv0.y, w0);
                bool h1 = NART_SPLAT_HITS(fx + uv1.x, fy + uv1.y, w1);
                bool h2 = NART_SPLAT_HITS(fx + uv2.x, fy + uv2.y, w2);
                bool h3 = NART_SPLAT_HITS(fx + uv3.x, fy + uv3.y, w3);
                if (h0) { c0 += L0.x * w0; c1 += L0.y * w0; c2 += L0.z * w0; c3 += L0.w * w0; ws += w0; }
                if (h1) { c0 += L1.x * w1; c1 += L1.y * w1; c2 += L1.z * w1; c3 += L1.w * w1; ws += w1; }
                if (h2) { c0 += L2.x * w2; c1 += L2.y * w2; c2 += L2.z * w2; c3 += L2.w * w2; ws += w2; }
                if (h3) { c0 += L3.x * w3; c1 += L3.y * w3; c2 += L3.z * w3; c3 += L3.w * w3; ws += w3; }
            }
            for (; i < A.spp; ++i) {
                float2 uv = sp[(size_t)i * npx];
                float w;
                if (NART_SPLAT_HITS(fx + uv.x, fy + uv.y, w)) {
                    float4 Lv = lp[(size_t)i * npx];
                    c0 += Lv.x * w;
                    c1 += Lv.y * w;
                    c2 += Lv.z * w;
                    c3 += Lv.w * w;
                    ws += w;
                }
            }
        }
    }
#undef NART_SPLAT_HITS
    float* o = A.tiles + ((uint64_t)bi * tpx + tp) * 5;
    o[0] = c0;
    o[1] = c1;
    o[2] = c2;
    o[3] = c3;
    o[4] = ws;
}

// NP (4) vertically adjacent tile pixels per lane (power-of-two buckets, threshold filter index:
// the splat_hits_fast arithmetic).  Consecutive lanes take consecutive tile columns, so a wave's
// loads of sample i cover contiguous source pixels as in k_splat, and each loaded sample serves
// up to four pixels (8 source rows x 5 columns per 4 pixels instead of 4 x 25: the splat is
// bound by re-fetching samples through a 4 %-hit L2).  The four pixels share their candidate
// columns; their candidate rows are windows of one union range (plus the bucket-edge wrap row),
// visited in ascending order, so each pixel still receives its samples in the reference's
// (source pixel raster, sample) order.  Per-sample work (position, bucket-edge tests, the
// column test and x distance) is shared.  (Four horizontal pixels per lane measured slower:
// lanes then read source pixels four apart and the L1 misses rose by a third.)
// splat_lut cell of d2: clamp((bits(d2) >> 16) - b0, 0, last), the clamp as one v_med3_i32
// (the compiler forms it only for constant bounds)
ND int lut_cell(float d2, int b0, int last) {
    const int c = (int)(__float_as_uint(d2) >> 16) - b0;
    int r;
    asm("v_med3_i32 %0, %1, 0, %2" : "=v"(r) : "v"(c), "s"(last));
    return r;
}
typedef float nd_f2v __attribute__((ext_vector_type(2)));  // packed-math pairs (v_pk_mul/add_f32)
template <int NP, bool LUT>
__global__ __launch_bounds__(256) void k_splat_col4(SplatArgs A) {
    __shared__ float s_table[64];
    __shared__ float s_thr[65];
    __shared__ float4 s_lut[LUT ? SPLAT_LUT_MAX : 1];
    if (threadIdx.x < 64) s_table[threadIdx.x] = A.table[threadIdx.x];
    if (threadIdx.x < 65) s_thr[threadIdx.x] = A.thr[threadIdx.x];
    if (LUT)
        for (uint32_t i = threadIdx.x; i < A.lut_n; i += blockDim.x) s_lut[i] = A.lut[i];
    __syncthreads();
    const uint32_t gpc = (A.tile + NP - 1) / NP, lpb = A.tile * gpc;  // lane groups per tile column / bucket
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (uint64_t)A.n_buckets * lpb) return;
    const uint32_t bi = (uint32_t)(gid / lpb), rem = (uint32_t)(gid % lpb);
    const uint32_t tx = rem % A.tile, ty0 = (rem / A.tile) * NP;
    const uint32_t bid = A.bucket_ids[bi];
    const uint32_t bx = bid % A.nbx, by = bid / A.nbx;
    const uint32_t x0 = A.B * bx, y0 = A.B * by;
    const uint32_t x1 = min(A.B * (bx + 1), A.totalW), y1 = min(A.B * (by + 1), A.totalH);
    const int bw = (int)(x1 - x0), bh = (int)(y1 - y0);
    const uint32_t npx = (uint32_t)(bw * bh);
    const uint32_t base = A.bucket_base[bi];
    const int r = (int)ceilf(A.fw), fb = (int)A.fb;
    const int sxlo = max(0, (int)tx - fb - r), sxhi = min(bw - 1, (int)tx - fb + r);
    const bool wrapx = bw == (int)A.B && (int)tx <= fb + r + 1 && bw - 1 > sxhi;
    const int ncol = (sxhi >= sxlo ? sxhi - sxlo + 1 : 0) + (wrapx ? 1 : 0);
    int lo[NP], hi[NP];
    bool val[NP], wr[NP];
    int ulo = 1 << 30, uhi = -1;
    bool anywrap = false;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const int ty = (int)ty0 + j;
        val[j] = ty < (int)A.tile;
        lo[j] = max(0, ty - fb - r);
        hi[j] = min(bh - 1, ty - fb + r);
        wr[j] = val[j] && bh == (int)A.B && ty <= fb + r + 1 && bh - 1 > hi[j];
        if (val[j] && hi[j] >= lo[j]) {
            ulo = min(ulo, lo[j]);
            uhi = max(uhi, hi[j]);
        }
        anywrap = anywrap || wr[j];
    }
    const bool extra = anywrap && bh - 1 > uhi;
    const int nrow = (uhi >= ulo ? uhi - ulo + 1 : 0) + (extra ? 1 : 0);
    const float fw = A.fw;
    const float xsA = (float)(tx + x0), xsB = (float)(tx + x0 + A.B);
    const float ysA0 = (float)(ty0 + y0), ysB0 = (float)(ty0 + y0 + A.B);
    const float edgeX = (float)(x0 + A.B + A.fb), edgeY = (float)(y0 + A.B + A.fb);
    // accumulators: {contribution.xy}, {contribution.zw} as packed pairs, and the weight sum (the
    // same IEEE products and sums per channel as five scalar ones: bit-identical)
    nd_f2v cxy[NP], czw[NP];
    float cws[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        cxy[j] = nd_f2v{0.f, 0.f};
        czw[j] = nd_f2v{0.f, 0.f};
        cws[j] = 0.f;
    }
    const int lut_b0 = (int)A.lut_b0, lut_last = (int)A.lut_n - 1;
    for (int ri = 0; ri < nrow; ++ri) {
        const int sy = (ulo + ri <= uhi) ? ulo + ri : bh - 1;
        bool act[NP];
#pragma unroll
        for (int j = 0; j < NP; ++j) act[j] = val[j] && ((sy >= lo[j] && sy <= hi[j]) || (wr[j] && sy == bh - 1));
        const float fy = (float)(y0 + (uint32_t)sy + A.fb);
        for (int ci = 0; ci < ncol; ++ci) {
            const int sx = (sxlo + ci <= sxhi) ? sxlo + ci : bw - 1;
            const float fx = (float)(x0 + (uint32_t)sx + A.fb);
            const uint64_t first = (uint64_t)base * A.spp + (uint32_t)(sy * bw + sx);
            const float2* sp = A.samples + first;
            const float4* lp = A.Lout + first;
            auto splat1 = [&](float2 uv, float4 L) {
                const float scx = fx + uv.x, scy = fy + uv.y;
                const float xs = scx >= edgeX ? xsB : xsA;
                const bool xhit = (scx - fw) < xs + 1.f && xs < (scx + fw);
                const float distX = (xs + 0.5f) - scx;
                const float dx2 = distX * distX;
                const float yb = scy >= edgeY ? ysB0 : ysA0;
                const float loy = scy - fw, hiy = scy + fw;
#pragma unroll
                for (int j = 0; j < NP; ++j) {
                    if (!act[j]) continue;
                    const float ys = yb + (float)j;
                    const bool hit = xhit && loy < ys + 1.f && ys < hiy;
                    const float distY = (ys + 0.5f) - scy;
                    const float d2 = dx2 + distY * distY;  // = distX^2 + distY^2 (IEEE + commutes)
                    float w;
                    if (LUT) {  // one LDS read: the d2 cell's threshold and the weights on either side
                        int cell = (int)(__float_as_uint(d2) >> 16) - lut_b0;
                        cell = cell < 0 ? 0 : (cell > lut_last ? lut_last : cell);
                        const float4 e = s_lut[cell];
                        w = d2 >= e.x ? e.z : e.y;
                    } else {
                        int g = (int)(__builtin_amdgcn_sqrtf(d2) * A.idx_scale);
                        g = g < 0 ? 0 : (g > 63 ? 63 : g);
                        const float t0 = s_thr[g], t1 = s_thr[g + 1];
                        const int fi = g - (d2 < t0 ? 1 : 0) + (d2 >= t1 ? 1 : 0);
                        w = s_table[fi];
                    }
                    if (hit) {
                        const nd_f2v w2 = nd_f2v{w, w};
                        cxy[j] += nd_f2v{L.x, L.y} * w2;
                        czw[j] += nd_f2v{L.z, L.w} * w2;
                        cws[j] += w;
                    }
                }
            };
#ifndef NART_COL4_PF
#define NART_COL4_PF 4
#endif
            constexpr uint32_t PF = NART_COL4_PF;  // samples per group; the next group is in flight
            uint32_t i = 0;
            float2 nu[PF];
            float4 nL[PF];
            if (A.spp >= PF) {
#pragma unroll
                for (uint32_t u = 0; u < PF; ++u) {
                    nu[u] = sp[(size_t)u * npx];
                    nL[u] = lp[(size_t)u * npx];
                }
            }
            for (; i + PF <= A.spp; i += PF) {
                float2 uv[PF];
                float4 Lv[PF];
#pragma unroll
                for (uint32_t u = 0; u < PF; ++u) {
                    uv[u] = nu[u];
                    Lv[u] = nL[u];
                }
                if (i + 2 * PF <= A.spp) {
                    const size_t k0 = (size_t)(i + PF) * npx;
#pragma unroll
                    for (uint32_t u = 0; u < PF; ++u) {
                        nu[u] = sp[k0 + (size_t)u * npx];
                        nL[u] = lp[k0 + (size_t)u * npx];
                    }
                }
#pragma unroll
                for (uint32_t u = 0; u < PF; ++u) splat1(uv[u], Lv[u]);
            }
            for (; i < A.spp; ++i) splat1(sp[(size_t)i * npx], lp[(size_t)i * npx]);
        }
    }
    const uint32_t tpx = A.tile * A.tile;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        if (!val[j]) continue;
        float* o = A.tiles + ((uint64_t)bi * tpx + (ty0 + j) * A.tile + tx) * 5;
        o[0] = cxy[j].x;
        o[1] = cxy[j].y;
        o[2] = czw[j].x;
        o[3] = czw[j].y;
        o[4] = cws[j];
    }
}

// k_splat_skew's per-sample steps.  skew_prep forms the W window rows' image coordinates
// ys_k = yb + k (exact small integers) and distance terms two rows per packed instruction
// ((ys_k + 0.5) - scy and d2 = dx2 + distY^2 are the same IEEE operations per row; ys_k + 1 is
// ys_{k+1}) and issues the W weight-cell reads together (a read inside each row's branch waited
// for its own LDS round trip; a row that is not hit reads a clamped, valid cell and discards it).
template <int W>
struct SkewPrep {
    float ys[2 * ((W + 2) / 2)], d2[2 * ((W + 2) / 2)];
    float4 ev[W];
    float loy, hiy;
    bool xhit;
};
template <int W>
ND void skew_prep(SkewPrep<W>& p, float2 uv, float fx, float fy, float edgeX, float edgeY, float xsA, float xsB,
                  float ybA, float ybB, float fw, const float4* s_lut, int lut_b0, int lut_last) {
    constexpr int WP = (W + 2) / 2;  // row pairs covering ys_0 .. ys_W
    const float scx = fx + uv.x, scy = fy + uv.y;
    const float xs = scx >= edgeX ? xsB : xsA;
    p.xhit = (scx - fw) < xs + 1.f && xs < (scx + fw);
    const float distX = (xs + 0.5f) - scx;
    const float dx2 = distX * distX;
    const float yb = scy >= edgeY ? ybB : ybA;
    p.loy = scy - fw;
    p.hiy = scy + fw;
#pragma unroll
    for (int k = 0; k < WP; ++k) {
        const nd_f2v y2 = nd_f2v{yb, yb} + nd_f2v{(float)(2 * k), (float)(2 * k + 1)};
        const nd_f2v dy = (y2 + nd_f2v{0.5f, 0.5f}) - nd_f2v{scy, scy};
        const nd_f2v dd = nd_f2v{dx2, dx2} + dy * dy;
        p.ys[2 * k] = y2.x;
        p.ys[2 * k + 1] = y2.y;
        p.d2[2 * k] = dd.x;
        p.d2[2 * k + 1] = dd.y;
    }
#pragma unroll
    for (int k = 0; k < W; ++k) p.ev[k] = s_lut[lut_cell(p.d2[k], lut_b0, lut_last)];
}
// Row k is hit iff xhit && loy < ys_{k+1} && ys_k < hiy.  Both row tests are monotone in k
// (ys_k = yb + k exactly), so every row is hit iff row 0 passes the first and row W-1 the
// second -- all but never fails (a sample exactly on a pixel edge): the rows then accumulate
// without per-row branches (4-5 scalar exec-mask instructions and two compares per row).
// (A wave-uniform form of this test -- a ballot, the per-row path for the whole wave when any
// lane misses a row -- measured slower: C5 splat 69.4-70.5 vs 68.2-68.8 ms,
// profiles/r05r_skew_uniform_ab.log.)
template <int W>
ND bool skew_all_rows(const SkewPrep<W>& p) {
    return p.xhit && p.loy < p.ys[1] && p.ys[W - 1] < p.hiy;
}
template <int W>
ND void skew_add_all(const SkewPrep<W>& p, float4 L, nd_f2v (&cxy)[W], nd_f2v (&czw)[W], float (&cws)[W]) {
#pragma unroll
    for (int k = 0; k < W; ++k) {
        const float w = p.d2[k] >= p.ev[k].x ? p.ev[k].z : p.ev[k].y;
        const nd_f2v w2 = nd_f2v{w, w};
        cxy[k] += nd_f2v{L.x, L.y} * w2;
        czw[k] += nd_f2v{L.z, L.w} * w2;
        cws[k] += w;
    }
}
template <int W>
ND void skew_add_rows(const SkewPrep<W>& p, float4 L, nd_f2v (&cxy)[W], nd_f2v (&czw)[W], float (&cws)[W]) {
    if (skew_all_rows(p)) {
        skew_add_all(p, L, cxy, czw, cws);
        return;
    }
#pragma unroll
    for (int k = 0; k < W; ++k) {
        if (p.xhit && p.loy < p.ys[k + 1] && p.ys[k] < p.hiy) {
            const float w = p.d2[k] >= p.ev[k].x ? p.ev[k].z : p.ev[k].y;
            const nd_f2v w2 = nd_f2v{w, w};
            cxy[k] += nd_f2v{L.x, L.y} * w2;
            czw[k] += nd_f2v{L.z, L.w} * w2;
            cws[k] += w;
        }
    }
}

// Skewed-time splat over the pixel-major sample layout (sample i of bucket-local pixel q at
// (base + q) * spp + i), one lane per tile column, LUT filter weights (power-of-two buckets).
// AddSample (render.cpp:23-70) adds a bucket's sources to the tile in raster order; a tile pixel
// (tx, ty) receives sources (sy, sx) with sy in [ty-2R, ty], sx in [tx-2R, tx] (R = filterBounds),
// i.e. in increasing step t = W sy + sx (W = 2R + 1 > the window's column span).  Processing
// source s at step t(s) for all its consumers at once therefore keeps every tile pixel's order,
// and at step t lane tx has exactly one candidate source: the sx in [tx-2R, tx] with
// sx = t (mod W), sy = (t - sx) / W, which it adds to its W window rows [sy, sy+2R] (registers;
// a row is written out once its last source row is done).  The W lanes tx in [sx, sx+2R] read
// source s at the same step, so each sample is fetched once per bucket (k_splat_col4 fetches it
// ~12 times through L2), and each loaded sample serves W tile pixels of the lane.
// Bucket-edge wraps (a last-column / last-row sample whose coordinate rounds onto the next
// bucket's origin: splat_hits) go to tile columns / rows 0..2R+1 at their raster position: a
// pre-pass flags the edge sources that have such samples, and only flagged sources get the
// extra passes (the x wrap: source (sy, B-1) after the lane's last source of row sy, as the
// gather kernels' extra column; the y wrap: the already written rows 0..2R+1, read back and
// updated at source row B-1).  Per pair the arithmetic is splat_hits_fast + the LUT weight, as
// in k_splat_col4: bit-identical.
#ifndef NART_SKEW_PF
#define NART_SKEW_PF 4  // samples per group; the next group is in flight
#endif
// NB bands: a bucket's tile rows split into NB bands of ceil(T/NB) rows, each band a unit of T
// lanes with its own source rows [band start - 2R, band end - 1] (the 2R rows before a band are
// read by both neighbours): NB times the waves for ~1/NB of the steps each, for launches whose
// time is otherwise the waves' latency (VALU ~30 % busy at 2.7 waves per SIMD).
template <int R, int NB>
__global__ __launch_bounds__(256, 2) void k_splat_skew(SplatArgs A) {
    constexpr int W = 2 * R + 1, NWR = 2 * R + 2;
    extern __shared__ __attribute__((aligned(16))) float4 s_dyn4[];
    float4* s_lut = s_dyn4;
    uint32_t* s_flag = reinterpret_cast<uint32_t*>(s_dyn4 + A.lut_n);  // [bucket of block][x, y]
    const uint32_t T = A.tile, PB = 64u / T, wv = threadIdx.x >> 6, l = threadIdx.x & 63u;
    for (uint32_t i = threadIdx.x; i < A.lut_n; i += blockDim.x) s_lut[i] = A.lut[i];
    if (threadIdx.x < 8u * PB) s_flag[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t lb = l / T, tx = l % T;
    const uint32_t unit = (blockIdx.x * 4u + wv) * PB + lb, bi = unit / NB, band = unit % NB;
    const bool live = lb < PB && bi < A.n_buckets;
    const int rpb = ((int)T + NB - 1) / NB, tr0 = (int)band * rpb, tr1 = min((int)T, tr0 + rpb);  // tile rows
    uint32_t* flag = s_flag + 2u * (wv * PB + (lb < PB ? lb : 0u));
    uint32_t bid = 0, x0 = 0, y0 = 0, base = 0;
    int bw = 0, bh = 0;
    const int B = (int)A.B;
    if (live) {
        bid = A.bucket_ids[bi];
        x0 = A.B * (bid % A.nbx);
        y0 = A.B * (bid / A.nbx);
        bw = (int)(min(x0 + A.B, A.totalW) - x0);
        bh = (int)(min(y0 + A.B, A.totalH) - y0);
        base = A.bucket_base[bi];
    }
    const float fw = A.fw;
    const float edgeX = (float)(x0 + A.B + A.fb), edgeY = (float)(y0 + A.B + A.fb);
    // pre-pass: which last-column sources (bit sy) / last-row sources (bit sx) have wrapping samples
    if (live) {
        for (int k = (int)tx; k < 2 * B; k += (int)T) {
            const bool colsrc = k < B;
            const int sy = colsrc ? k : B - 1, sx = colsrc ? B - 1 : k - B;
            if ((colsrc && bw != B) || (!colsrc && bh != B) || sy >= bh || sx >= bw) continue;
            const float2* sp = A.samples + (size_t)(base + (uint32_t)(sy * bw + sx)) * A.spp;
            const float f = colsrc ? (float)(x0 + (uint32_t)sx + A.fb) : (float)(y0 + (uint32_t)sy + A.fb);
            const float edge = colsrc ? edgeX : edgeY;
            bool any = false;
            for (uint32_t i = 0; i < A.spp && !any; ++i) {
                const float2 u = sp[i];
                any = (f + (colsrc ? u.x : u.y)) >= edge;
            }
            if (any) atomicOr(flag + (colsrc ? 0 : 1), 1u << (colsrc ? sy : sx));
        }
    }
    __syncthreads();
    if (!live) return;
    const uint32_t flagX = flag[0], flagY = flag[1];
    const float xsA = (float)(tx + x0), xsB = (float)(tx + x0 + A.B);
    const int lut_b0 = (int)A.lut_b0, lut_last = (int)A.lut_n - 1;
    nd_f2v cxy[W], czw[W];
    float cws[W];
#pragma unroll
    for (int k = 0; k < W; ++k) {
        cxy[k] = nd_f2v{0.f, 0.f};
        czw[k] = nd_f2v{0.f, 0.f};
        cws[k] = 0.f;
    }
    const int sr0 = max(0, tr0 - 2 * R);  // first source row of the band
    int wb = sr0;                          // tile row of cxy[0]
    const uint32_t tpx = T * T;
    float* out = A.tiles + ((uint64_t)bi * tpx + tx) * 5;  // + ty * T * 5
    auto retire = [&]() {  // rows outside the band belong to a neighbour unit
        if (wb >= tr0 && wb < tr1) {
            float* o = out + (size_t)wb * T * 5;
            o[0] = cxy[0].x;
            o[1] = cxy[0].y;
            o[2] = czw[0].x;
            o[3] = czw[0].y;
            o[4] = cws[0];
        }
#pragma unroll
        for (int k = 0; k + 1 < W; ++k) {
            cxy[k] = cxy[k + 1];
            czw[k] = czw[k + 1];
            cws[k] = cws[k + 1];
        }
        cxy[W - 1] = nd_f2v{0.f, 0.f};
        czw[W - 1] = nd_f2v{0.f, 0.f};
        cws[W - 1] = 0.f;
        ++wb;
    };
    float fy = 0.f, ybA = 0.f, ybB = 0.f;  // per source row: fy, and the window's first image row
                                           // without / with the y wrap (splat_hits_fast)
    float fx = 0.f;
    // one sample into the window rows wb .. wb+2R: skew_prep + skew_add_all / skew_add_rows
    auto splat_w = [&](float2 uv, float4 L) {
        SkewPrep<W> p;
        skew_prep(p, uv, fx, fy, edgeX, edgeY, xsA, xsB, ybA, ybB, fw, s_lut, lut_b0, lut_last);
        skew_add_rows(p, L, cxy, czw, cws);
    };
    // a group of PF samples: every sample's distance terms and cell reads first (one basic block,
    // so one sample's LDS round trip overlaps the next one's arithmetic; per-sample branches had
    // kept the scheduler to one sample at a time), then the accumulation in sample order,
    // branch-free when every row of every sample is hit -- each accumulator receives the same
    // products in the same order as from splat_w
    constexpr uint32_t PF = NART_SKEW_PF;
    constexpr uint32_t G = R >= 3 ? 2u : PF;  // samples per group (R = 3: 7 rows each, 2 waves/SIMD)
    static_assert(PF % G == 0, "prefetch group = whole sample groups");
    auto splat_grp = [&](const float2* uv, const float4* L) {
        SkewPrep<W> p[G];
        bool all = true;
#pragma unroll
        for (uint32_t u = 0; u < G; ++u) {
            skew_prep(p[u], uv[u], fx, fy, edgeX, edgeY, xsA, xsB, ybA, ybB, fw, s_lut, lut_b0, lut_last);
            all = all && skew_all_rows(p[u]);
        }
        if (all) {
#pragma unroll
            for (uint32_t u = 0; u < G; ++u) skew_add_all(p[u], L[u], cxy, czw, cws);
        } else {
#pragma unroll
            for (uint32_t u = 0; u < G; ++u) skew_add_rows(p[u], L[u], cxy, czw, cws);
        }
    };
    auto source_pass = [&](int sy, int sx) {  // every sample of bucket-local pixel (sx, sy)
        const size_t first = (size_t)(base + (uint32_t)(sy * bw + sx)) * A.spp;
        const float2* sp = A.samples + first;
        const float4* lp = A.Lout + first;
        fx = (float)(x0 + (uint32_t)sx + A.fb);
        uint32_t i = 0;
        float2 nu[PF];
        float4 nL[PF];
        if (A.spp >= PF) {
#pragma unroll
            for (uint32_t u = 0; u < PF; ++u) {
                nu[u] = sp[u];
                nL[u] = lp[u];
            }
        }
        for (; i + PF <= A.spp; i += PF) {
            float2 uv[PF];
            float4 Lv[PF];
#pragma unroll
            for (uint32_t u = 0; u < PF; ++u) {
                uv[u] = nu[u];
                Lv[u] = nL[u];
            }
            if (i + 2 * PF <= A.spp) {
#pragma unroll
                for (uint32_t u = 0; u < PF; ++u) {
                    nu[u] = sp[i + PF + u];
                    nL[u] = lp[i + PF + u];
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < PF; u += G) splat_grp(uv + u, Lv + u);
        }
        for (; i < A.spp; ++i) splat_w(sp[i], lp[i]);
    };
    // y wrap (rare): samples of last-row source (B-1, sx) at or past edgeY into the written
    // tile rows 0 .. min(2R+1, B-2) of this lane's column, read back from the tile output
    auto ywrap_pass = [&](int sx) {
        const int sy = B - 1;
        const size_t first = (size_t)(base + (uint32_t)(sy * bw + sx)) * A.spp;
        const float2* sp = A.samples + first;
        const float4* lp = A.Lout + first;
        const float fxw = (float)(x0 + (uint32_t)sx + A.fb), fyw = (float)(y0 + (uint32_t)sy + A.fb);
        const int nr = min(NWR, B - 1);
        float acc[NWR][5];
#pragma unroll
        for (int k = 0; k < NWR; ++k)
#pragma unroll
            for (int c = 0; c < 5; ++c) acc[k][c] = k < nr ? out[(size_t)k * T * 5 + c] : 0.f;
        const float ysB0 = (float)(y0 + A.B);
        for (uint32_t i = 0; i < A.spp; ++i) {
            const float2 uv = sp[i];
            const float scx = fxw + uv.x, scy = fyw + uv.y;
            if (!(scy >= edgeY)) continue;
            const float4 L = lp[i];
            const float xs = scx >= edgeX ? xsB : xsA;
            const bool xhit = (scx - fw) < xs + 1.f && xs < (scx + fw);
            const float distX = (xs + 0.5f) - scx;
            const float dx2 = distX * distX;
            const float loy = scy - fw, hiy = scy + fw;
#pragma unroll
            for (int k = 0; k < NWR; ++k) {
                const float ys = ysB0 + (float)k;
                const bool hit = k < nr && xhit && loy < ys + 1.f && ys < hiy;
                const float distY = (ys + 0.5f) - scy;
                const float d2 = dx2 + distY * distY;
                int cell = (int)(__float_as_uint(d2) >> 16) - lut_b0;
                cell = cell < 0 ? 0 : (cell > lut_last ? lut_last : cell);
                const float4 e = s_lut[cell];
                const float w = d2 >= e.x ? e.z : e.y;
                if (hit) {
                    acc[k][0] += L.x * w;
                    acc[k][1] += L.y * w;
                    acc[k][2] += L.z * w;
                    acc[k][3] += L.w * w;
                    acc[k][4] += w;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < NWR; ++k)
            if (k < nr)
#pragma unroll
                for (int c = 0; c < 5; ++c) out[(size_t)k * T * 5 + c] = acc[k][c];
    };
    const bool xwrap_lane = bw == B && (int)tx <= 2 * R + 1 && bw - 1 > (int)tx;
    const int sr1 = min(bh - 1, tr1 - 1);  // last source row of the band
    const int tmax = W * (min(B, rpb + 2 * R) - 1) + (B - 1);  // wave-uniform step count
    for (int t0 = 0; t0 <= tmax; ++t0) {
        const int t = t0 + W * sr0;
        const int d = (((int)tx - t) % W + W) % W;
        const int sx = (int)tx - d, sy = (t - sx) / W;
        if (sx < 0 || sx >= bw || sy < sr0 || sy > sr1) continue;
        while (wb < sy) retire();
        fy = (float)(y0 + (uint32_t)sy + A.fb);
        ybA = (float)(y0 + (uint32_t)sy);
        ybB = (float)(y0 + A.B + (uint32_t)sy);
        source_pass(sy, sx);
        if (xwrap_lane && sx == (int)tx && ((flagX >> sy) & 1u)) source_pass(sy, bw - 1);  // the gather kernels' extra column
    }
    while (wb < tr1) retire();
    // y wrap: last-row samples into tile rows 0 .. 2R+1 (the first band's), after all their other
    // sources, in the raster order of their source columns, the extra column last
    if (tr0 == 0 && bh == B) {
        for (int sx = max(0, (int)tx - 2 * R); sx <= min(bw - 1, (int)tx); ++sx)
            if ((flagY >> sx) & 1u) ywrap_pass(sx);
        if (xwrap_lane && ((flagY >> (bw - 1)) & 1u)) ywrap_pass(bw - 1);
    }
}

// The skewed-time splat with the W = 2R+1 window rows of a tile column on W lanes instead of one
// (k_splat_rows, launches too small to fill the GPU with k_splat_skew's one lane per column).
// Lane (k, tx) of a bucket owns the tile rows r = k (mod W) of column tx, one at a time: at step t
// it takes the same source (sy, sx) as k_splat_skew's lane tx and adds each sample to the one row
// r in [sy, sy + 2R] with r = k (mod W), r = sy + ((k - sy) mod W), with k_splat_skew's operations
// for that row (ys = yb + (r - sy), the same hit test, d2, LUT cell and packed products).  A row's
// sources still arrive in raster order (t = W sy + sx), and a class's rows in increasing order, so
// a lane writes row r once the next source needs row r + W (rows without sources are written as
// zeros).  Five times the lanes of k_splat_skew, each doing the work of one row per sample
// (one accumulator, few registers); the W lanes of a column load the same sample (one L1 line).
// Bucket-edge wraps as in k_splat_skew: the extra column source (sy, B-1) after the lane's last
// source of row sy; y wraps into the written rows 0..2R+1 read back after all regular steps.
#ifndef NART_ROWS_PF
#define NART_ROWS_PF 4  // samples per group; the next group is in flight (few waves: latency-bound)
#endif
template <int R>
__global__ __launch_bounds__(512) void k_splat_rows(SplatArgs A) {
    constexpr int W = 2 * R + 1, NWR = 2 * R + 2;
    extern __shared__ __attribute__((aligned(16))) float4 s_dyn4[];
    float4* s_lut = s_dyn4;
    const uint32_t T = A.tile, U = T * (uint32_t)W, UB = blockDim.x / U;  // lanes per bucket, buckets per block
    uint32_t* s_flag = reinterpret_cast<uint32_t*>(s_dyn4 + A.lut_n);    // [bucket of block][x, y]
    for (uint32_t i = threadIdx.x; i < A.lut_n; i += blockDim.x) s_lut[i] = A.lut[i];
    if (threadIdx.x < 2u * UB) s_flag[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t lb = threadIdx.x / U, j = threadIdx.x % U;
    const uint32_t k = j / T, tx = j % T;
    const uint32_t bi = blockIdx.x * UB + lb;
    const bool live = lb < UB && bi < A.n_buckets;
    uint32_t* flag = s_flag + 2u * (lb < UB ? lb : 0u);
    uint32_t bid = 0, x0 = 0, y0 = 0, base = 0;
    int bw = 0, bh = 0;
    const int B = (int)A.B;
    if (live) {
        bid = A.bucket_ids[bi];
        x0 = A.B * (bid % A.nbx);
        y0 = A.B * (bid / A.nbx);
        bw = (int)(min(x0 + A.B, A.totalW) - x0);
        bh = (int)(min(y0 + A.B, A.totalH) - y0);
        base = A.bucket_base[bi];
    }
    const float fw = A.fw;
    const float edgeX = (float)(x0 + A.B + A.fb), edgeY = (float)(y0 + A.B + A.fb);
    // pre-pass: which last-column sources (bit sy) / last-row sources (bit sx) have wrapping samples
    if (live) {
        for (int q = (int)j; q < 2 * B; q += (int)U) {
            const bool colsrc = q < B;
            const int sy = colsrc ? q : B - 1, sx = colsrc ? B - 1 : q - B;
            if ((colsrc && bw != B) || (!colsrc && bh != B) || sy >= bh || sx >= bw) continue;
            const float2* sp = A.samples + (size_t)(base + (uint32_t)(sy * bw + sx)) * A.spp;
            const float f = colsrc ? (float)(x0 + (uint32_t)sx + A.fb) : (float)(y0 + (uint32_t)sy + A.fb);
            const float edge = colsrc ? edgeX : edgeY;
            bool any = false;
            for (uint32_t i = 0; i < A.spp && !any; ++i) {
                const float2 u = sp[i];
                any = (f + (colsrc ? u.x : u.y)) >= edge;
            }
            if (any) atomicOr(flag + (colsrc ? 0 : 1), 1u << (colsrc ? sy : sx));
        }
    }
    __syncthreads();
    if (!live) return;
    const uint32_t flagX = flag[0], flagY = flag[1];
    const float xsA = (float)(tx + x0), xsB = (float)(tx + x0 + A.B);
    const int lut_b0 = (int)A.lut_b0, lut_last = (int)A.lut_n - 1;
    const uint32_t tpx = T * T;
    float* out = A.tiles + ((uint64_t)bi * tpx + tx) * 5;  // + row * T * 5
    nd_f2v cxy = nd_f2v{0.f, 0.f}, czw = nd_f2v{0.f, 0.f};
    float cws = 0.f;
    int wr = (int)k;  // the open row of this lane's class
    auto write_row = [&]() {
        float* o = out + (size_t)wr * T * 5;
        o[0] = cxy.x;
        o[1] = cxy.y;
        o[2] = czw.x;
        o[3] = czw.y;
        o[4] = cws;
        cxy = nd_f2v{0.f, 0.f};
        czw = nd_f2v{0.f, 0.f};
        cws = 0.f;
        wr += W;
    };
    // one sample into row r (the lane's open row): k_splat_skew's operations for that row.  (Issuing
    // a sample group's LUT reads together with select accumulation measured no faster here: C3 1/2,
    // 1/4 shards 15.4 / 8.6 vs 14.6 / 7.9 ms, profiles/r05e_splat_rows_ab.log)
    float fx = 0.f, ybA = 0.f, ybB = 0.f, fy = 0.f, dk = 0.f;  // dk = r - sy
    auto splat_r = [&](float2 uv, float4 L) {
        const float scx = fx + uv.x, scy = fy + uv.y;
        const float xs = scx >= edgeX ? xsB : xsA;
        const bool xhit = (scx - fw) < xs + 1.f && xs < (scx + fw);
        const float distX = (xs + 0.5f) - scx;
        const float dx2 = distX * distX;
        const float yb = scy >= edgeY ? ybB : ybA;
        const float ys = yb + dk;
        const float dy = (ys + 0.5f) - scy;
        const float d2 = dx2 + dy * dy;
        const float4 e = s_lut[lut_cell(d2, lut_b0, lut_last)];
        const float w = d2 >= e.x ? e.z : e.y;
        if (xhit && (scy - fw) < ys + 1.f && ys < (scy + fw)) {
            const nd_f2v w2 = nd_f2v{w, w};
            cxy += nd_f2v{L.x, L.y} * w2;
            czw += nd_f2v{L.z, L.w} * w2;
            cws += w;
        }
    };
    auto source_pass = [&](int sy, int sx) {  // every sample of bucket-local pixel (sx, sy)
        const size_t first = (size_t)(base + (uint32_t)(sy * bw + sx)) * A.spp;
        const float2* sp = A.samples + first;
        const float4* lp = A.Lout + first;
        fx = (float)(x0 + (uint32_t)sx + A.fb);
        constexpr uint32_t PF = NART_ROWS_PF;
        uint32_t i = 0;
        float2 nu[PF];
        float4 nL[PF];
        if (A.spp >= PF) {
#pragma unroll
            for (uint32_t u = 0; u < PF; ++u) {
                nu[u] = sp[u];
                nL[u] = lp[u];
            }
        }
        for (; i + PF <= A.spp; i += PF) {
            float2 uv[PF];
            float4 Lv[PF];
#pragma unroll
            for (uint32_t u = 0; u < PF; ++u) {
                uv[u] = nu[u];
                Lv[u] = nL[u];
            }
            if (i + 2 * PF <= A.spp) {
#pragma unroll
                for (uint32_t u = 0; u < PF; ++u) {
                    nu[u] = sp[i + PF + u];
                    nL[u] = lp[i + PF + u];
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < PF; ++u) splat_r(uv[u], Lv[u]);
        }
        for (; i < A.spp; ++i) splat_r(sp[i], lp[i]);
    };
    const bool xwrap_lane = bw == B && (int)tx <= 2 * R + 1 && bw - 1 > (int)tx;
    const int tmax = W * (B - 1) + (B - 1);  // wave-uniform step count (k_splat_skew's, one band)
    for (int t = 0; t <= tmax; ++t) {
        const int d = (((int)tx - t) % W + W) % W;
        const int sx = (int)tx - d, sy = (t - sx) / W;
        if (sx < 0 || sx >= bw || sy < 0 || sy >= bh) continue;
        const int r = sy + (((int)k - sy) % W + W) % W;  // this class's row in [sy, sy + 2R]
        while (wr < r) write_row();
        fy = (float)(y0 + (uint32_t)sy + A.fb);
        ybA = (float)(y0 + (uint32_t)sy);
        ybB = (float)(y0 + A.B + (uint32_t)sy);
        dk = (float)(r - sy);
        source_pass(sy, sx);
        if (xwrap_lane && sx == (int)tx && ((flagX >> sy) & 1u)) source_pass(sy, bw - 1);  // the extra column
    }
    while (wr < (int)T) write_row();
    // y wrap: last-row samples into tile rows 0 .. 2R+1 of this class, after all their other
    // sources, in the raster order of their source columns, the extra column last
    if (bh == B) {
        const int nr = min(NWR, B - 1);
        const float ysB0 = (float)(y0 + A.B);
        auto ywrap_pass = [&](int sx) {
            const int sy = B - 1;
            const size_t first = (size_t)(base + (uint32_t)(sy * bw + sx)) * A.spp;
            const float2* sp = A.samples + first;
            const float4* lp = A.Lout + first;
            const float fxw = (float)(x0 + (uint32_t)sx + A.fb), fyw = (float)(y0 + (uint32_t)sy + A.fb);
            for (int rr = (int)k; rr < nr; rr += W) {
                float acc[5];
#pragma unroll
                for (int c = 0; c < 5; ++c) acc[c] = out[(size_t)rr * T * 5 + c];
                const float ys = ysB0 + (float)rr;
                for (uint32_t i = 0; i < A.spp; ++i) {
                    const float2 uv = sp[i];
                    const float scx = fxw + uv.x, scy = fyw + uv.y;
                    if (!(scy >= edgeY)) continue;
                    const float4 L = lp[i];
                    const float xs = scx >= edgeX ? xsB : xsA;
                    const bool xhit = (scx - fw) < xs + 1.f && xs < (scx + fw);
                    const float distX = (xs + 0.5f) - scx;
                    const float dx2 = distX * distX;
                    const bool hit = xhit && (scy - fw) < ys + 1.f && ys < (scy + fw);
                    const float distY = (ys + 0.5f) - scy;
                    const float d2 = dx2 + distY * distY;
                    int cell = (int)(__float_as_uint(d2) >> 16) - lut_b0;
                    cell = cell < 0 ? 0 : (cell > lut_last ? lut_last : cell);
                    const float4 e = s_lut[cell];
                    const float w = d2 >= e.x ? e.z : e.y;
                    if (hit) {
                        acc[0] += L.x * w;
                        acc[1] += L.y * w;
                        acc[2] += L.z * w;
                        acc[3] += L.w * w;
                        acc[4] += w;
                    }
                }
#pragma unroll
                for (int c = 0; c < 5; ++c) out[(size_t)rr * T * 5 + c] = acc[c];
            }
        };
        for (int sx = max(0, (int)tx - 2 * R); sx <= min(bw - 1, (int)tx); ++sx)
            if ((flagY >> sx) & 1u) ywrap_pass(sx);
        if (xwrap_lane && ((flagY >> (bw - 1)) & 1u)) ywrap_pass(bw - 1);
    }
}

// ---------------------------------------------------------------- combine
struct CombineArgs {
    const float* tiles;  // [bucket id][tile*tile][5]
    float* image;        // [totalH][totalW][5]
    uint32_t W, H, B, fb, tile, nbx, nby, totalW, totalH;
};
__global__ __launch_bounds__(256) void k_combine(CombineArgs A) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (uint64_t)A.totalW * A.totalH) return;
    const uint32_t pX = (uint32_t)(gid % A.totalW), pY = (uint32_t)(gid / A.totalW);
    float c[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    if (pX < A.W + A.fb && pY < A.H + A.fb) {
        const uint32_t ilo = pX + 1 > A.tile ? (pX + 1 - A.tile + A.B - 1) / A.B : 0;
        const uint32_t ihi = min(pX / A.B, A.nbx - 1);
        const uint32_t jlo = pY + 1 > A.tile ? (pY + 1 - A.tile + A.B - 1) / A.B : 0;
        const uint32_t jhi = min(pY / A.B, A.nby - 1);
        for (uint32_t j = jlo; j <= jhi; ++j)
            for (uint32_t i = ilo; i <= ihi; ++i) {
                const float* t = A.tiles + ((uint64_t)(j * A.nbx + i) * A.tile * A.tile +
                                            (uint64_t)(pY - j * A.B) * A.tile + (pX - i * A.B)) * 5;
#pragma unroll
                for (int k = 0; k < 5; ++k) c[k] += t[k];
            }
    }
    float* o = A.image + gid * 5;
#pragma unroll
    for (int k = 0; k < 5; ++k) o[k] = c[k];
}

// ---------------------------------------------------------------- libm self-test
__global__ void k_sincos(const float* x, uint32_t n, float* s, float* c) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    s[i] = glibc_sinf(x[i]);
    c[i] = glibc_cosf(x[i]);
}

}  // namespace nd
