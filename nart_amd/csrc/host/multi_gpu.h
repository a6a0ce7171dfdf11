// Multi-GPU render context (nart_hip_create_multi), included by render.hip.
//
// The reference renders a session's buckets with a tbb::task_group over every host core and sums
// their tiles into the image in bucket raster order (render.cpp:152-203).  Here one process drives
// N GPUs of the node:
//   * the scene lives on every device (one single-device sub-context each, nart_hip_create);
//   * buckets are dealt over the devices on a diagonal lattice (shard_ids: every region of a frame
//     spreads evenly over all devices; nart_hip_shard_buckets);
//   * one host thread per device renders its share into device-resident tiles (render_buckets);
//   * the tiles are gathered to device 0 with one RCCL group of ncclSend / ncclRecv over xGMI
//     (library-owned communicator, ncclCommInitAll over the device list), permuted into bucket-id
//     order and combined in bucket raster order on device 0 (k_combine) -- so the image is
//     bit-identical for any N.
// RCCL is loaded at run time (dlopen), so single-device use never needs it.  A device list with
// repeated ordinals (a rehearsal of N ranks on fewer GPUs) gathers with device copies instead,
// since an RCCL communicator needs distinct GPUs.  NART_GATHER=rccl|copy overrides the choice
// (rccl on one device runs a self send/receive through RCCL).
#pragma once

#include <dlfcn.h>

#include <mutex>
#include <thread>

namespace {

struct RcclApi {
    bool ok = false;
    std::string err;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*ErrStr)(ncclResult_t) = nullptr;
};

const RcclApi& rccl_api() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) {
            api.err = std::string("cannot load librccl: ") + dlerror();
            return;
        }
        bool all = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            all = all && fn;
        };
        sym(api.CommInitAll, "ncclCommInitAll");
        sym(api.CommDestroy, "ncclCommDestroy");
        sym(api.GroupStart, "ncclGroupStart");
        sym(api.GroupEnd, "ncclGroupEnd");
        sym(api.Send, "ncclSend");
        sym(api.Recv, "ncclRecv");
        sym(api.ErrStr, "ncclGetErrorString");
        api.ok = all;
        if (!all) api.err = "librccl lacks ncclCommInitAll/ncclSend/ncclRecv";
    });
    return api;
}

// Bucket ids of device d out of n, in ascending order: a diagonal lattice, bucket (bx, by) on
// device (bx + s*by) % n with s = lattice_step(n), the s in [1, n) coprime to n closest to 0.382 n.
// Every run of n buckets along a row or a column holds each device once, so every region of the
// frame -- the costly glass of C3 -- splits evenly over the devices.  (b % n gave whole vertical
// stripes when n divides the bucket-column count: C3 1/8 shards 86-101 ms.)  Must match
// nart_amd/dist.py bucket_owners.
uint32_t lattice_step(uint32_t n) {
    uint32_t best = 0;
    double bd = 1e30;
    for (uint32_t s = 1; s < n; ++s) {
        uint32_t a = s, b = n;
        while (b) {
            const uint32_t t = a % b;
            a = b;
            b = t;
        }
        const double dd = std::fabs((double)s - 0.382 * (double)n);
        if (a == 1 && dd < bd) {
            bd = dd;
            best = s;
        }
    }
    return best;
}

std::vector<uint32_t> shard_ids(uint32_t nbx, uint32_t n_buckets, uint32_t n, uint32_t d) {
    std::vector<uint32_t> ids;
    const uint32_t s = lattice_step(n);
    for (uint32_t b = 0; b < n_buckets; ++b)
        if ((uint32_t)(((uint64_t)(b % nbx) + (uint64_t)s * (b / nbx)) % n) == d) ids.push_back(b);
    return ids;
}

// Gathered slabs (device after device, each in its ascending id order) -> tiles in bucket-id
// order: slab tile i is bucket map[i].  One block per bucket.
__global__ void k_unshard(const float* slabs, float* by_id, const uint32_t* map, uint32_t n_buckets, uint32_t tile_floats) {
    const uint32_t i = blockIdx.x;
    if (i >= n_buckets) return;
    const float* src = slabs + (size_t)i * tile_floats;
    float* dst = by_id + (size_t)map[i] * tile_floats;
    for (uint32_t k = threadIdx.x; k < tile_floats; k += blockDim.x) dst[k] = src[k];
}

// One render's device statistics: device times of the slowest device (the devices run
// concurrently), work counts summed.  The caller adds the result to its own stats, as the
// single-device path does (a stats struct reused over renders keeps accumulating).
void merge_stats(nart_render_stats& out, const nart_render_stats& s) {
    out.kernel_ms = std::max(out.kernel_ms, s.kernel_ms);
    out.splat_ms = std::max(out.splat_ms, s.splat_ms);
    out.latin_ms = std::max(out.latin_ms, s.latin_ms);
    out.primary_ms = std::max(out.primary_ms, s.primary_ms);
    out.kernel_launches = std::max(out.kernel_launches, s.kernel_launches);
    out.schedule |= s.schedule;
    out.samples += s.samples;
    out.traced_samples += s.traced_samples;
    out.rays_extend += s.rays_extend;
    out.rays_shadow += s.rays_shadow;
    out.node_visits += s.node_visits;
    out.tri_tests += s.tri_tests;
    out.bounces += s.bounces;
    out.octree_checks += s.octree_checks;
    out.octree_replays += s.octree_replays;
}

int ensure_dev(nart_ctx* ctx, int dev, void*& buf, size_t& cap, size_t bytes, const char* what) {
    if (bytes <= cap) return NART_OK;
    HIPCHK(hipSetDevice(dev));
    if (buf) hipFree(buf);
    buf = nullptr;
    cap = 0;
    if (int rc = dmalloc(ctx, &buf, bytes, what)) return rc;
    cap = bytes;
    return NART_OK;
}

// Render(), multi-device: shard, render concurrently, gather to device 0, combine, copy out (image
// null: the combined image stays in ctx->d_image on device 0, nart_hip_render_device).
int render_multi(nart_ctx* ctx, const nart_render_params* p, nart_pixel* image, nart_render_stats* stats) {
    const uint32_t n = (uint32_t)ctx->subs.size();
    if (ctx->rccl_broken)
        return fail(ctx, NART_E_RCCL, "an earlier RCCL gather of this context failed; destroy it and create a new one");
    int rc = check_params(ctx->subs[0], p);
    if (rc) return fail(ctx, rc, ctx->subs[0]->err);
    nart_session_geometry g;
    nart_session_geometry_of(p, &g);
    const uint32_t nb = g.n_buckets_x * g.n_buckets_y;
    const size_t tile_floats = (size_t)g.tile_size * g.tile_size * 5;
    std::vector<std::vector<uint32_t>> ids(n);
    for (uint32_t d = 0; d < n; ++d) {
        ids[d] = shard_ids(g.n_buckets_x, nb, n, d);
        const size_t bytes = std::max<size_t>(1, ids[d].size()) * tile_floats * 4;
        if ((rc = ensure_dev(ctx, ctx->devs[d], ctx->sub_tiles[d], ctx->sub_cap[d], bytes, "device tiles"))) return rc;
    }
    const int dev0 = ctx->devs[0];
    const size_t all_bytes = (size_t)nb * tile_floats * 4;
    const size_t img_bytes = (size_t)g.total_width * g.total_height * sizeof(nart_pixel);
    if ((rc = ensure_dev(ctx, dev0, ctx->d_gather, ctx->cap_gather, all_bytes, "gathered tiles")) ||
        (rc = ensure_dev(ctx, dev0, ctx->d_byid, ctx->cap_byid, all_bytes, "tiles by bucket id")) ||
        (rc = ensure_dev(ctx, dev0, ctx->d_image, ctx->cap_image, img_bytes, "image")))
        return rc;

    // 1. every device renders its buckets (one host thread each, like the TBB task group)
    std::vector<int> rcs(n, NART_OK);
    std::vector<nart_render_stats> st(n);
    std::vector<std::thread> th;
    auto work = [&](uint32_t d) {
        if (ids[d].empty()) return;
        if (hipSetDevice(ctx->devs[d]) != hipSuccess) {
            rcs[d] = NART_E_HIP;
            return;
        }
        rcs[d] = render_buckets(ctx->subs[d], p, ids[d].data(), (uint32_t)ids[d].size(),
                                static_cast<float*>(ctx->sub_tiles[d]), ctx->streams[d], &st[d]);
        if (rcs[d] == NART_OK && hipStreamSynchronize(ctx->streams[d]) != hipSuccess) rcs[d] = NART_E_HIP;
    };
    for (uint32_t d = 0; d < n; ++d) std::memset(&st[d], 0, sizeof(st[d]));
    try {
        th.reserve(n);
        for (uint32_t d = 0; d < n; ++d) th.emplace_back(work, d);
    } catch (...) {
        // no thread (or no room for one): join the ones started, report; nothing escapes the ABI
        for (auto& t : th) t.join();
        return fail(ctx, NART_E_OOM, "cannot start the per-device render threads");
    }
    for (auto& t : th) t.join();
    for (uint32_t d = 0; d < n; ++d)
        if (rcs[d] != NART_OK)
            return fail(ctx, rcs[d], "device " + std::to_string(ctx->devs[d]) + ": " + ctx->subs[d]->err);

    // 2. gather the slabs to device 0 (rank order), RCCL over xGMI or device copies
    std::vector<size_t> first_b(n, 0);
    for (uint32_t d = 1; d < n; ++d) first_b[d] = first_b[d - 1] + ids[d - 1].size();
    float* slabs = static_cast<float*>(ctx->d_gather);
    hipStream_t s0 = ctx->streams[0];
    if (ctx->gather_rccl) {
        // every error inside the group is recorded and the group is always closed (an open group
        // would capture the next render's calls); a failed gather leaves the communicator in an
        // unknown state, so the context refuses further renders (rccl_broken)
        const RcclApi& R = rccl_api();
        ncclResult_t first = ncclSuccess;
        std::string where;
        auto note = [&](ncclResult_t r, const char* what) {
            if (r != ncclSuccess && first == ncclSuccess) {
                first = r;
                where = what;
            }
        };
        note(R.GroupStart(), "ncclGroupStart");
        if (first == ncclSuccess) {
            // test hook (nart_hip_debug_fault 1): the last device that owns buckets sends to a rank
            // that does not exist, after the receives of the devices before it are posted
            uint32_t last = n;
            for (uint32_t d = 0; d < n; ++d)
                if (!ids[d].empty()) last = d;
            const int bad_peer = ctx->debug_fault == 1 ? (int)n : 0;
            for (uint32_t d = 0; d < n; ++d) {
                if (ids[d].empty()) continue;
                const size_t cnt = ids[d].size() * tile_floats;
                note(R.Send(ctx->sub_tiles[d], cnt, ncclFloat32, d == last ? bad_peer : 0, ctx->comms[d], ctx->streams[d]),
                     "ncclSend");
                note(R.Recv(slabs + first_b[d] * tile_floats, cnt, ncclFloat32, (int)d, ctx->comms[0], s0), "ncclRecv");
            }
            note(R.GroupEnd(), "ncclGroupEnd");
        }
        ctx->debug_fault = 0;
        if (first != ncclSuccess) {
            ctx->rccl_broken = true;
            for (uint32_t d = 0; d < n; ++d) {
                hipSetDevice(ctx->devs[d]);
                hipStreamSynchronize(ctx->streams[d]);
            }
            (void)hipGetLastError();
            return fail(ctx, NART_E_RCCL, where + ": " + R.ErrStr(first) +
                                              " (context unusable: destroy it and create a new one)");
        }
        for (uint32_t d = 1; d < n; ++d) {
            HIPCHK(hipSetDevice(ctx->devs[d]));
            HIPCHK(hipStreamSynchronize(ctx->streams[d]));
        }
        HIPCHK(hipSetDevice(dev0));
    } else {
        HIPCHK(hipSetDevice(dev0));
        for (uint32_t d = 0; d < n; ++d)
            if (!ids[d].empty())
                HIPCHK(hipMemcpyPeerAsync(slabs + first_b[d] * tile_floats, dev0, ctx->sub_tiles[d], ctx->devs[d],
                                          ids[d].size() * tile_floats * 4, s0));
    }

    // 3. bucket-id order, raster-order combine on device 0, image to the host
    std::vector<uint32_t> map;
    map.reserve(nb);
    for (uint32_t d = 0; d < n; ++d) map.insert(map.end(), ids[d].begin(), ids[d].end());
    if ((rc = ensure_dev(ctx, dev0, ctx->d_slab_map, ctx->cap_slab_map, (size_t)nb * 4, "slab map"))) return rc;
    HIPCHK(hipMemcpyAsync(ctx->d_slab_map, map.data(), (size_t)nb * 4, hipMemcpyHostToDevice, s0));
    hipLaunchKernelGGL(k_unshard, dim3(nb), dim3(256), 0, s0, slabs, static_cast<float*>(ctx->d_byid),
                       static_cast<const uint32_t*>(ctx->d_slab_map), nb, (uint32_t)tile_floats);
    HIPCHK(hipGetLastError());
    if ((rc = nart_hip_combine_async(ctx->subs[0], p, static_cast<const nart_pixel*>(ctx->d_byid),
                                     static_cast<nart_pixel*>(ctx->d_image), s0)))
        return fail(ctx, rc, ctx->subs[0]->err);
    if (image) HIPCHK(hipMemcpyAsync(image, ctx->d_image, img_bytes, hipMemcpyDeviceToHost, s0));
    HIPCHK(hipStreamSynchronize(s0));
    if (stats) {
        nart_render_stats m;
        std::memset(&m, 0, sizeof(m));
        for (uint32_t d = 0; d < n; ++d) merge_stats(m, st[d]);
        stats->kernel_ms += m.kernel_ms;
        stats->splat_ms += m.splat_ms;
        stats->latin_ms += m.latin_ms;
        stats->primary_ms += m.primary_ms;
        stats->kernel_launches += m.kernel_launches;
        stats->schedule |= m.schedule;
        stats->samples += m.samples;
        stats->traced_samples += m.traced_samples;
        stats->rays_extend += m.rays_extend;
        stats->rays_shadow += m.rays_shadow;
        stats->node_visits += m.node_visits;
        stats->tri_tests += m.tri_tests;
        stats->bounces += m.bounces;
        stats->octree_checks += m.octree_checks;
        stats->octree_replays += m.octree_replays;
    }
    return NART_OK;
}

}  // namespace
