/*
 * nart_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of shanesimmsart/nart's render path (RenderSession::Render and everything
 * below it), written in plain C from the reference sources.  It is the checker for the HIP
 * path and the timed CPU baseline ("kind": "port").  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product never links or calls it.
 *
 * PARITY UNPINNED: the reference ships no tests, golden vectors or fixture images, and it
 * cannot be built in this image (it needs GLM, OpenEXR/Imath, oneTBB and nlohmann 3.11 via
 * CMake FetchContent; building it against stand-in headers is not allowed).  The restatement
 * is pinned only where a third-party dependency's arithmetic can be checked here: glibc 2.35
 * sinf/cosf (used through glm::sin/cos) are called directly, and the device port of them is
 * checked exhaustively against this libm (tests/test_libm_parity.py).  GLM 0.9.9.8 operation
 * order is restated from its published scalar code paths (DESIGN.md lists the assumptions).
 */
#ifndef NART_ORACLE_H
#define NART_ORACLE_H

#include "../include/nart_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_scene oracle_scene;

/* Builds the reference octree BVH (bvh.cpp:252-326) and light/material views of the blob.
   The blob must stay alive while the oracle scene is used. */
int oracle_create(const nart_scene_blob* blob, oracle_scene** out);
void oracle_destroy(oracle_scene* s);

/* RenderSession::Render (render.cpp:114-206) with `threads` workers on a dynamic bucket
   queue (tbb::task_group stand-in).  image: totalW*totalH Pixels. */
int oracle_render(oracle_scene* s, const nart_render_params* p, nart_pixel* image, int threads);

/* RenderTile for a list of bucket ids into tiles[i] (tile_size^2 Pixels each). */
int oracle_render_buckets(oracle_scene* s, const nart_render_params* p, const uint32_t* ids,
                          uint32_t n, nart_pixel* tiles, int threads);

/* Per-sample Li_alpha for pixels [x0,x0+w) x [y0,y0+h): out[((y-y0)*w+(x-x0))*spp+i][4];
   uv (optional) receives the Latin-square image samples [..][2]. */
int oracle_render_samples(oracle_scene* s, const nart_render_params* p, uint32_t x0, uint32_t y0,
                          uint32_t w, uint32_t h, float* out, float* uv);

/* Stats of the reference octree build (for tests of Q14 and the chunk-index quirk).
   grid_res[0..2] = grid resolution, grid_res[3] = triangles reachable by traversal. */
int oracle_bvh_stats(const oracle_scene* s, uint32_t* n_chunks, uint32_t* max_chunk_tris,
                     uint32_t* root_is_leaf, uint32_t* grid_res);

/* Individual primitives for known-answer tests. */
void oracle_rng_stream(uint32_t seed, uint32_t n, float* out);
void oracle_latin_square(uint32_t seed, uint32_t spp, float* out_xy, uint32_t* rng_state_after);
float oracle_fresnel(float eta_o, float eta_i, float cos_theta);
/* BinarySearch (util.cpp:4-20) as the environment light's CDF inversion uses it. */
uint32_t oracle_binary_search(float value, const float* v, uint32_t start, uint32_t end);
/* Test statistic: the longest nested-dielectric list a path of this process reached (reset: zero it). */
uint32_t oracle_max_list(int reset);

#ifdef __cplusplus
}
#endif
#endif
