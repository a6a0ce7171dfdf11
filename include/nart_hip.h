/*
 * nart_hip.h — MI355X (gfx950) render path, C ABI.
 *
 * Replaces the reference's per-session hot path
 *     std::vector<Pixel> RenderSession::Render() const      src/core/render.cpp:114-206
 * (bucket loop + per-pixel RNG seed + Latin square + Camera::CastRay + Integrator::Li_alpha +
 *  AddSample Gaussian splat + bucket-raster tile combine) with HIP kernels on one device.
 * Li_alpha (src/integrators/pathintegrator.cpp:144-259) with its BVH traversal
 * (src/core/bvh.cpp:132-176), BSDFs (src/core/bxdf.cpp, src/bxdfs/<name>.cpp), materials
 * (src/materials/<type>material.cpp) and lights (src/lights/<type>light.cpp) run on the device.
 *
 * All entry points return NART_OK (0) or a negative NART_E_* code (nart_scene.h); no C++
 * exception crosses the ABI and nothing aborts.  A context owns all device memory of its
 * device(s) (and, multi-device, its streams and RCCL communicator) and is not thread-safe (one
 * caller thread, like the reference's main thread).
 */
#ifndef NART_HIP_H
#define NART_HIP_H

#include <stddef.h>
#include <stdint.h>

#include "nart_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nart_ctx nart_ctx;

typedef struct nart_render_stats {
    double render_ms;       /* wall time of the render call (host clock)               */
    double kernel_ms;       /* device time of the path-tracing kernels (HIP events)     */
    double splat_ms;        /* device time of the splat + combine kernels               */
    uint32_t kernel_launches; /* number of path-tracing kernel launches timed in kernel_ms */
    uint32_t schedule;      /* NART_SCHED_* bits: the scheduling paths the render took (OR over
                               its launches; observability for tests and benches)         */
    uint64_t samples;       /* camera samples counted in the metric (W*H*spp share)     */
    uint64_t traced_samples;/* samples actually traced (incl. extra rows, render.cpp:164) */
    /* Counter pass only (nart_hip_set_counters(ctx,1)); zero otherwise.  bounces = extension
     * hits shaded (BSDF + EstimateDirect + continuation). */
    uint64_t rays_extend, rays_shadow, node_visits, tri_tests, bounces;
    double latin_ms;        /* device time of the LatinSquare kernel                    */
    /* Counter pass only: hits whose octree reachability needed the exact ancestor-chain check,
     * and queries answered by replaying the reference octree search (device/octree.h). */
    uint64_t octree_checks, octree_replays;
    double primary_ms;      /* part of kernel_ms: the camera-ray kernel that runs before the path
                               kernel (k_primary, default variant only)                  */
} nart_render_stats;

/* nart_render_stats.schedule bits */
#define NART_SCHED_PROBE_QUEUE 0x1u  /* cost probe + pixel queue, persistent refill lanes          */
#define NART_SCHED_PRIORITY    0x2u  /* priority lanes for the costliest pixels (ray-queue kernel) */
#define NART_SCHED_SPEC_PAIRS  0x4u  /* speculative lane groups on the costliest pixels            */
#define NART_SCHED_WAVE_GROUPS 0x8u  /* wave-group refill in probe order (ray-queue kernel)        */
#define NART_SCHED_VOL_QUEUE   0x10u /* volume kernel: cost probe, costliest groups first          */
#define NART_SCHED_VOL_SPARSE  0x20u /* volume kernel: sparse waves for the costliest groups       */
#define NART_SCHED_SPLAT_SKEW  0x40u /* skewed-time splat (k_splat_skew)                           */
#define NART_SCHED_PRIMARY     0x80u /* camera rays traced first (k_primary)                       */
#define NART_SCHED_SPLAT_ROWS  0x100u /* skewed-time splat, W lanes per tile column (k_splat_rows)  */
#define NART_SCHED_HALF_WAVES  0x200u /* costliest pixels on one wave per SIMD, raised priority     */
#define NART_SCHED_SPECIALIZED 0x400u /* a scene-specialised path-kernel build ran (nart_hip_set_specialize) */
#define NART_SCHED_LEAN        0x800u /* the lean three-waves-per-SIMD build of a throughput-bound launch */

/* Upload the scene, build the device BVH.  device_id: HIP ordinal. */
int nart_hip_create(const nart_scene_blob* scene, int device_id, nart_ctx** out);
void nart_hip_destroy(nart_ctx* ctx);
const char* nart_hip_last_error(const nart_ctx* ctx);

/* Multi-GPU context over device_ids[0..n_devices) of this node, replacing the reference's
   tbb::task_group over host cores (render.cpp:152-177): the scene is uploaded to every device;
   nart_hip_render shards the buckets (dealt in a low-discrepancy order, nart_hip_shard_buckets), renders
   the shares concurrently (one host thread per device), gathers the tiles to device_ids[0] with
   the library's own RCCL communicator (ncclCommInitAll over the list; ncclSend/ncclRecv over
   xGMI) and combines them there in bucket raster order (render.cpp:183-203), so the image is
   bit-identical for any n.  n_devices == 1 is exactly nart_hip_create.  Repeated ordinals (a
   rehearsal of n devices on fewer GPUs) gather with device copies, since RCCL needs distinct
   GPUs; NART_GATHER=rccl|copy overrides (read at creation).  If librccl cannot be loaded or
   ncclCommInitAll fails, the context falls back to the device-copy gather (same image;
   nart_hip_context_devices reports it); only NART_GATHER=rccl then fails with NART_E_RCCL.
   A gather that fails inside the RCCL group still closes the group (ncclGroupEnd), returns
   NART_E_RCCL and marks the context unusable: every later render returns NART_E_RCCL, and the
   caller destroys the context and creates a new one. */
int nart_hip_create_multi(const nart_scene_blob* scene, const int* device_ids, int n_devices, nart_ctx** out);

/* Devices of a context (1 for nart_hip_create) and its gather: uses_rccl = 1 RCCL, 0 device
   copies, 2 device copies because RCCL was unavailable (the fallback above). */
int nart_hip_context_devices(const nart_ctx* ctx, int* n_devices, int* uses_rccl);

/* Test hook (no reference counterpart): fault 1 makes the next RCCL gather of a multi-device
   context post a send to a rank that does not exist, exercising the failure path above; 0 clears.
   No effect on device-copy gathers. */
int nart_hip_debug_fault(nart_ctx* ctx, int fault);

/* HIP devices visible to this process. */
int nart_hip_device_count(int* count);

/* Host only: the buckets device device_index of n_devices renders, ascending, into ids (may be
   null to query the count).  A diagonal lattice: bucket id b = by*n_buckets_x + bx goes to device
   (bx + s*by) % n_devices, s the step in [1, n) coprime to n closest to 0.382 n (3 for 8 devices),
   so every region of the frame splits evenly over the devices (nart_amd/dist.py bucket_owners). */
int nart_hip_shard_buckets(uint32_t n_buckets_x, uint32_t n_buckets, uint32_t n_devices, uint32_t device_index,
                           uint32_t* ids, uint32_t* count);

/* Whole-session render into device memory: as nart_hip_render, but the combined image stays on
   the (first) device, in a buffer the context owns (valid until the next render or destroy), and
   *d_image points at it -- no PCIe copy.  Multi-device contexts gather the tiles to device 0 with
   their RCCL send/receive group (or device copies) first.  Synchronous. */
int nart_hip_render_device(nart_ctx* ctx, const nart_render_params* p, const nart_pixel** d_image,
                           nart_render_stats* stats);

/* Whole-session render, Render()-equivalent: fills a caller-owned host buffer of
   totalW*totalH nart_pixel (render.cpp:114-206 contract, render.h:18-21 layout). */
int nart_hip_render(nart_ctx* ctx, const nart_render_params* p, nart_pixel* image,
                    nart_render_stats* stats);

/* Multi-GPU building block: render the listed buckets (bucket id = by*nBucketsX + bx) into
   device-resident tiles d_tiles[i] (tile_size^2 nart_pixel each, same order as the list) on
   `stream` (a hipStream_t, may be 0).  bucket_ids is a host array.  Asynchronous w.r.t. the
   host except for small scratch uploads; synchronise the stream before reading d_tiles. */
int nart_hip_render_buckets_async(nart_ctx* ctx, const nart_render_params* p,
                                  const uint32_t* bucket_ids, uint32_t n_buckets,
                                  nart_pixel* d_tiles, void* stream, nart_render_stats* stats);

/* Device combine: d_tiles indexed by bucket id (all nBucketsX*nBucketsY tiles) into the
   totalW*totalH device image, bucket raster order (render.cpp:183-203). */
int nart_hip_combine_async(nart_ctx* ctx, const nart_render_params* p, const nart_pixel* d_tiles,
                           nart_pixel* d_image, void* stream);

/* Debug / parity: per-sample Li_alpha (float4) for pixels [x0,x0+w) x [y0,y0+h) in image
   coordinates, all spp samples, into host out[((y-y0)*w + (x-x0))*spp + s][4]. */
int nart_hip_render_samples(nart_ctx* ctx, const nart_render_params* p, uint32_t x0, uint32_t y0,
                            uint32_t w, uint32_t h, float* out);

/* Enable the deterministic counter pass (node visits, triangle tests, rays) for the next
   renders.  Slower; used to compute algorithmic bytes per sample. */
int nart_hip_set_counters(nart_ctx* ctx, int enable);

/* Device self-test: glibc-equivalent sinf/cosf over n inputs (parity of the device libm). */
int nart_hip_eval_sincos(nart_ctx* ctx, const float* x, uint32_t n, float* sin_out, float* cos_out);

/* Splat filter-index thresholds (host only, no device): thr65[k] = the least d2 whose AddSample
   filter index (render.cpp:43-49) is >= k.  NART_E_INVALID when filter_width is too small for
   them (the splat then evaluates sqrt and division per pair). */
int nart_hip_splat_thresholds(float filter_width, float* thr65);

/* Splat filter weight by d2 cell (host only): cell c holds the floats whose bits >> 16 equal
   b0 + c, as {threshold t, weight below t, weight at or above t, 0} (at most one threshold per
   cell), cells4 with room for 2048 cells.  NART_E_INVALID where the thresholds do not apply. */
int nart_hip_splat_lut(float filter_width, float* cells4, uint32_t* n_cells, uint32_t* b0);

/* Environment-map CDF search (host only, no device; test hook for the guide tables of
   path.h guided_search): for each of values[0, m), the reference's BinarySearch over v[0, n)
   (util.cpp:4-20) into full[] and the guided search into guided[].  Returns 1 if a guide table
   was built for v (non-decreasing, NaN-free, n < 2^16), 0 if not (the guided search is then the
   full search), NART_E_INVALID on bad arguments. */
int nart_hip_env_search(const float* v, uint32_t n, const float* values, uint32_t m, uint32_t* full,
                        uint32_t* guided);

/* Acceleration structure the context would build for a scene (host only, no device): BVH2 node
   count, traversal stack depth (levels; the device keeps 8 B per level per lane in LDS) and the
   triangles in leaves.  Deep trees are capped (median splits past 40 levels), so stack_depth
   stays <= 72; nart_hip_create returns NART_E_UNSUPPORTED if the stack would not fit in LDS. */
typedef struct nart_bvh_info {
    uint32_t num_nodes;
    uint32_t stack_depth;
    uint32_t num_leaf_tris;
    uint32_t reserved;
} nart_bvh_info;
int nart_hip_bvh_info(const nart_scene_blob* scene, nart_bvh_info* out);

/* The acceleration structure a context built: nodes, stack depth, leaf triangles; reserved = 1
   when it was built on the device (NART_BVH_BUILD=device: a linear BVH, device/lbvh.h; default
   the host's binned SAH), and the build time in ms (host wall clock, uploads included). */
int nart_hip_context_bvh(const nart_ctx* ctx, nart_bvh_info* out, double* build_ms);

/* Kernel variant (all render bit-identical images):
   0 = megakernel with a wave ray queue (default; scenes whose BVH is too deep for its 512-lane
       LDS layout run variant 3's kernel),
   3 = megakernel, one lane per pixel, each query traced to completion.
   1 (the wavefront variant, 2x slower) and 2 (variant 3 with a traversal quorum) were retired:
   NART_E_UNSUPPORTED. */
int nart_hip_set_variant(nart_ctx* ctx, int variant);

/* Scene-specialised path kernels (no reference counterpart; all builds render the same image).
   The context derives a feature mask from the scene (material kinds, light kinds, textured
   patterns, normal maps: NART_FT_* bits, device/path.h FT_*) and runs the ray-queue kernel built
   for the first mask that covers it -- glassSphere's, the Cornell box's, C4's -- so that code for
   kinds the scene lacks is not compiled into the kernel; throughput-bound launches (whole frames)
   of scenes whose traversal stack fits take the lean build of that mask (no priority lanes or
   speculative pairs, three waves per SIMD: NART_SCHED_LEAN).  mode 0 forces the generic build, 1
   the specialised builds without the lean one, 2 (default) all of them.  nart_hip_scene_features
   reports the scene's mask and the mask of the build the last render launched (0x3FF = generic). */
int nart_hip_set_specialize(nart_ctx* ctx, int mode);
int nart_hip_scene_features(const nart_ctx* ctx, uint32_t* features, uint32_t* build);
/* Host only (no device): the feature mask a context would derive for a scene. */
int nart_hip_scene_features_of(const nart_scene_blob* scene, uint32_t* features);
#define NART_FT_LAMBERT 0x1u
#define NART_FT_SPECULAR 0x2u
#define NART_FT_GLASS 0x4u
#define NART_FT_GLOSSY 0x8u
#define NART_FT_PLASTIC 0x10u
#define NART_FT_DISK 0x20u
#define NART_FT_RING 0x40u
#define NART_FT_ENVIRONMENT 0x80u
#define NART_FT_TEXTURE 0x100u
#define NART_FT_NORMAL_MAP 0x200u
#define NART_FT_ALL 0x3FFu

/* Splat kernel (all bit-identical): -1 = automatic (the default: 4 when the launch fills >= 1
   wave per SIMD, else 5), 4 = skewed-time tile columns over the pixel-major sample layout (each
   sample fetched once per bucket), 5 = the same with one lane per (tile column, row class), for
   small launches, 3 = four tile pixels per lane over the sample-major layout;
   1, 0 = one tile pixel per lane with the threshold / direct filter-index arithmetic (2 = 1).
   Modes fall back to a lower one where their preconditions (power-of-two buckets <= 32, filter
   bounds 1-3, threshold table and weight LUT) do not hold.  (An LDS-staged mode, an unskewed
   tile-column sweep and a compare-only one-pixel mode measured slower and were retired.) */
int nart_hip_set_splat_mode(nart_ctx* ctx, int mode);

#ifdef __cplusplus
}
#endif
#endif
