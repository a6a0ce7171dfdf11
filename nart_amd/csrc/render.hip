// C-ABI of the MI355X render path (include/nart_hip.h): context creation (scene upload, BVH
// build, light precomputation) and the Render()-equivalent launch sequence.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>  // types only: RCCL is loaded at run time by the multi-device context

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/nart_hip.h"
#include "device/lbvh.h"
#include "device/volume.h"
#include "host/bvh_build.h"

using namespace nd;

struct nart_ctx {
    int device = 0;
    std::string err;
    DScene scene;
    uint32_t stack_depth = 1;
    uint32_t num_nodes = 0;
    int variant = 0;
    // 3 four pixels per lane (default), 2/1/0 one pixel per lane
    int splat_mode = -1;  // -1: automatic (render_buckets)
    bool counters = false;
    bool has_env = false;  // scene has an environment light (selects the k_render build)
    uint32_t features = FT_ALL;  // scene feature mask (scene_features): selects the k_render_rq build
    bool specialize = true;      // nart_hip_set_specialize: scene-specialised path kernels
    uint32_t fm_used = FT_ALL;   // the feature mask of the last path-kernel build launched
    bool lean = true;            // the three-waves-per-SIMD build where it fits (lean_fits)
    // scene buffers
    void* d_nodes = nullptr;
    void* d_tri_isect = nullptr;
    void* d_tri_perm = nullptr;
    void* d_tris = nullptr;
    void* d_tri_mesh = nullptr;
    void* d_meshes = nullptr;
    void* d_mesh_eta = nullptr;  // DScene::mesh_eta
    void* d_mats = nullptr;
    void* d_lights = nullptr;
    void* d_texs = nullptr;
    void* d_tex_pool = nullptr;
    void* d_envs = nullptr;
    void* d_density = nullptr;
    void* d_oc_nodes = nullptr;   // reference octree (octree.h)
    void* d_oc_chunks = nullptr;
    void* d_oc_tris = nullptr;
    void* d_tri_leaf = nullptr;
    void* d_oc_lock = nullptr;    // replay heap pool
    void* d_oc_heap = nullptr;
    std::vector<void*> env_bufs;  // Piecewise2DDistribution tables
    // work buffers
    size_t cap_slot_bytes = 0, cap_misc = 0;
    uint32_t* d_slot_xy = nullptr;
    SlotSO* d_slot_so = nullptr;  // [slot] {first sample index, sample stride} (RenderArgs::slot_so)
    uint32_t* d_rng = nullptr;
    float2* d_samples = nullptr;
    float4* d_L = nullptr;
    uint32_t* d_prim = nullptr;  // camera-ray hits per sample (k_primary), same indexing as d_samples
    uint32_t* d_bucket_ids = nullptr;
    uint32_t* d_bucket_base = nullptr;
    float* d_table = nullptr;
    void* d_lut = nullptr;       // splat filter-weight cells (splat_lut)
    unsigned long long* d_counters = nullptr;
    size_t cap_slots = 0, cap_samples = 0, cap_buckets = 0;
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};  // ev[4]: after k_primary
    bool primary_ran = false;  // the last dispatch launched k_primary (ev[4] recorded)
    uint32_t sched = 0;        // NART_SCHED_* bits of the current render (nart_render_stats::schedule)
    bool events = false;
    // megakernel work queue (launch_render)
    uint32_t* d_queue = nullptr;
    uint32_t* d_cost = nullptr;
    void* d_ilist = nullptr;   // dielectric-list columns beyond ILIST_REG (bounces > ILIST_REG)
    size_t cap_ilist = 0;
    void* d_gstack = nullptr;  // lean build: traversal-stack levels beyond the LDS (RenderArgs::gstack)
    size_t cap_gstack = 0;
    uint32_t* d_keys[2] = {nullptr, nullptr};
    uint32_t* d_vals[2] = {nullptr, nullptr};
    uint32_t* d_qhead = nullptr;
    void* d_sort_tmp = nullptr;
    size_t cap_sort_tmp = 0;
    uint32_t cap_queue = 0;
    // multi-device context (nart_hip_create_multi, host/multi_gpu.h): one single-device
    // sub-context per listed device; device 0 gathers and combines
    std::vector<nart_ctx*> subs;
    std::vector<int> devs;
    std::vector<hipStream_t> streams;
    std::vector<void*> sub_tiles;
    std::vector<size_t> sub_cap;
    std::vector<ncclComm_t> comms;
    bool gather_rccl = false;
    // RCCL requested implicitly (distinct devices) but unavailable: device-copy gather instead
    bool gather_fallback = false;
    // an RCCL gather failed: the communicator's state is unknown, every later render of this
    // context returns NART_E_RCCL (destroy it and create a new one)
    bool rccl_broken = false;
    int debug_fault = 0;     // nart_hip_debug_fault (tests only)
    uint32_t mem_share = 1;  // contexts of one multi-device context sharing this device ordinal
    // acceleration structure: built on the device (NART_BVH_BUILD=device) or the host; build time
    bool bvh_on_device = false;
    double bvh_ms = 0.0;
    uint32_t num_leaf_tris = 0;
    void *d_gather = nullptr, *d_byid = nullptr, *d_image = nullptr, *d_slab_map = nullptr;
    size_t cap_gather = 0, cap_byid = 0, cap_image = 0, cap_slab_map = 0;
};

namespace {

int fail(nart_ctx* c, int code, const std::string& m) {
    if (c) c->err = m;
    return code;
}
// On failure the error is also cleared from HIP's sticky last-error state, so that a context whose
// call failed (e.g. an allocation) renders normally afterwards.
#define HIPCHK(call)                                                                             \
    do {                                                                                         \
        hipError_t e_ = (call);                                                                  \
        if (e_ != hipSuccess) {                                                                  \
            (void)hipGetLastError();                                                             \
            return fail(ctx, e_ == hipErrorOutOfMemory ? NART_E_OOM : NART_E_HIP,                \
                        std::string(#call ": ") + hipGetErrorString(e_));                        \
        }                                                                                        \
    } while (0)

// Run-time switches, all read here.  Fallbacks a deployment can need: NART_BATCH_BYTES (per-batch
// memory budget), NART_BVH_BUILD=device, NART_GATHER=rccl|copy.  The others are test hooks that
// force one scheduling or kernel path of an otherwise automatic choice so that the GPU parity suite
// covers it (tests/test_gpu_*.py; DESIGN.md section 2 lists them); none changes an image.
const char* env_opt(const char* name) { return std::getenv(name); }
double env_num(const char* name, double def) {
    const char* e = env_opt(name);
    return e && *e ? std::atof(e) : def;
}

template <typename T>
int upload(nart_ctx* ctx, void*& dst, const T* src, size_t count) {
    size_t bytes = sizeof(T) * (count ? count : 1);
    HIPCHK(hipMalloc(&dst, bytes));
    if (count) HIPCHK(hipMemcpy(dst, src, sizeof(T) * count, hipMemcpyHostToDevice));
    return NART_OK;
}

// Feature mask of a scene (FT_*, path.h): every material kind, light kind, textured pattern and
// normal map the scene's records hold (a glass material's normal map is ignored, as the device
// record drops it: glassmaterial.cpp:3-9).  A path kernel built for a mask covering it compiles
// only that code; unknown kinds give FT_ALL (the generic build).
uint32_t scene_features(const nart_scene_blob* blob) {
    uint32_t f = 0;
    auto ptn = [&](const nart_pattern& p) {
        if (p.type != NART_PTN_CONSTANT) f |= FT_TEX;
    };
    for (uint32_t i = 0; i < blob->num_materials; ++i) {
        const nart_material& m = blob->materials[i];
        switch (m.type) {
            case NART_MAT_LAMBERT: f |= FT_LAMBERT; break;
            case NART_MAT_SPECULAR: f |= FT_SPECMAT; break;
            case NART_MAT_GLASS: f |= FT_GLASS; break;
            case NART_MAT_GLOSSY: f |= FT_GLOSSY; break;
            case NART_MAT_PLASTIC: f |= FT_PLASTIC; break;
            default: return FT_ALL;
        }
        for (const nart_pattern* p : {&m.rho_d, &m.rho_s, &m.tau, &m.eta, &m.alpha}) ptn(*p);
        if (m.type != NART_MAT_GLASS && m.has_normal) {
            f |= FT_NMAP;
            ptn(m.normal);
        }
    }
    for (uint32_t l = 0; l < blob->num_lights; ++l) {
        const nart_light& L = blob->lights[l];
        switch (L.type) {
            case NART_LIGHT_DISK: f |= FT_DISK; break;
            case NART_LIGHT_RING: f |= FT_RING; break;
            case NART_LIGHT_ENVIRONMENT: f |= FT_ENV; break;
            default: return FT_ALL;
        }
        ptn(L.Le);
    }
    return f;
}

DPattern dpat(const nart_pattern& p) {
    DPattern d;
    d.type = p.type;
    d.tex = p.texture;
    d.rough = p.is_roughness;
    d.v[0] = p.value[0];
    d.v[1] = p.value[1];
    d.v[2] = p.value[2];
    return d;
}

// Per-call light constants of disklight.cpp / ringlight.cpp, computed with the same float
// operations the reference executes on every call (vec4 * mat4 row-vector products).
DLight dlight(const nart_light& L) {
    DLight d;
    std::memset(&d, 0, sizeof(d));
    d.type = L.type;
    d.radius = L.radius;
    d.inner = L.inner_radius;
    d.intensity = L.intensity;
    d.Le = dpat(L.Le);
    std::memcpy(d.m, L.m, sizeof(d.m));
    f4 c = vec_mul_mat(F4(0.f, 0.f, 0.f, 1.f), L.m);
    f4 n = vec_mul_mat(F4(0.f, 0.f, -1.f, 0.f), L.m);
    f4 u = vec_mul_mat(F4(1.f, 0.f, 0.f, 0.f), L.m);
    f4 v = vec_mul_mat(F4(0.f, 1.f, 0.f, 0.f), L.m);
    d.center[0] = c.x; d.center[1] = c.y; d.center[2] = c.z;
    d.n[0] = n.x; d.n[1] = n.y; d.n[2] = n.z;
    d.D = dot(F3(c.x, c.y, c.z), F3(n.x, n.y, n.z));
    d.axu[0] = u.x; d.axu[1] = u.y; d.axu[2] = u.z; d.axu[3] = u.w;
    d.axv[0] = v.x; d.axv[1] = v.y; d.axv[2] = v.z; d.axv[3] = v.w;
    const float pi = ND_PI;
    if (L.type == NART_LIGHT_RING)
        d.pdf_area = 1.f / (pi * (1.f - ((L.inner_radius * L.inner_radius) / (L.radius * L.radius))) * L.radius * L.radius);
    else
        d.pdf_area = 1.f / (pi * L.radius * L.radius);
    d.r2 = L.radius * L.radius;
    d.ri2 = L.inner_radius * L.inner_radius;
    d.inner_ratio = L.inner_radius / L.radius;
    d.env = -1;
    return d;
}

// Guide table of one BinarySearch range v[0, n) (path.h guided_search): for each of the K cells of
// values [c/K, (c+1)/K) the range [ub(c/K), ub(last float of the cell)] of the upper bound (first
// index with v[j] > value), 16 bits each.  Only for non-decreasing, NaN-free ranges of < 2^16
// entries; otherwise false and the device runs the full search.
bool env_guide(const float* v, uint32_t n, uint32_t* out) {
    const uint32_t K = NART_ENV_GUIDE_K;
    if (n > 65535u) return false;
    for (uint32_t j = 0; j + 1 < n; ++j)
        if (!(v[j] <= v[j + 1])) return false;
    if (n && v[0] != v[0]) return false;
    auto ub = [&](float x) { return (uint32_t)(std::upper_bound(v, v + n, x) - v); };
    for (uint32_t c = 0; c < K; ++c) {
        const float lo = (float)c / (float)K;
        const float hi = c + 1 == K ? INFINITY : std::nextafter((float)(c + 1) / (float)K, 0.f);
        out[c] = ub(lo) | (ub(hi) << 16);
    }
    return true;
}

// Piecewise2DDistribution of an environment texture (texturepattern.cpp:3-70): marginal pdf of
// the rows (top row last), conditional pdf per row, and their CDFs, with the reference's float
// operation order.  Built on the host once per context.
int build_env(nart_ctx* ctx, const nart_texture& t, DEnvDist& d) {
    const uint32_t W = t.width, H = t.height;
    std::vector<float> mpdf(H), cpdf((size_t)W * H), mcdf(H + 1), ccdf((size_t)W * H + H);
    auto texel = [&](uint32_t row, uint32_t i) {  // |r| + |g| + |b| of the flipped row
        const uint16_t* q = t.rgba + ((size_t)(H - row - 1) * W + i) * 4;
        return std::fabs(nart_half_to_float(q[0])) + std::fabs(nart_half_to_float(q[1])) +
               std::fabs(nart_half_to_float(q[2]));
    };
    const float invW = 1.f / (float)W, invH = 1.f / (float)H;
    float fInt = 0.f;
    for (uint32_t j = 0; j < H; ++j) {
        mpdf[j] = 0.f;
        for (uint32_t i = 0; i < W; ++i) mpdf[j] += texel(j, i);
        mpdf[j] *= invW;
        fInt += mpdf[j];
    }
    fInt *= invH;
    for (uint32_t j = 0; j < H; ++j) {
        if (mpdf[j] != 0.f) {
            for (uint32_t i = 0; i < W; ++i) {
                cpdf[(size_t)j * W + i] = texel(j, i);
                cpdf[(size_t)j * W + i] /= mpdf[j];
            }
        } else {
            for (uint32_t i = 0; i < W; ++i) cpdf[(size_t)j * W + i] = 1.f;
        }
    }
    const float invFInt = 1.f / fInt;
    for (uint32_t j = 0; j < H; ++j) mpdf[j] *= invFInt;
    mcdf[0] = 0.f;
    mcdf[H] = 1.f;
    for (uint32_t i = 1; i < H; ++i) mcdf[i] = mcdf[i - 1] + (mpdf[i - 1] * invH);
    for (uint32_t i = 0; i < H; ++i) {
        ccdf[(size_t)i * (W + 1)] = 0.f;
        ccdf[(size_t)i * (W + 1) + W] = 1.f;
    }
    for (uint32_t j = 0; j < H; ++j)
        for (uint32_t i = 1; i < W; ++i)
            ccdf[(size_t)j * (W + 1) + i] = ccdf[(size_t)j * (W + 1) + i - 1] + (cpdf[(size_t)j * W + i - 1] * invW);
    // guide tables of the two searches (path.h guided_search): per cell of values [c/K, (c+1)/K)
    // the range [ub(c/K), ub(last float of the cell)] of the upper bound; built only over searched
    // ranges that are non-decreasing and NaN-free (otherwise the full search runs)
    const uint32_t K = NART_ENV_GUIDE_K;
    auto guide = env_guide;
    std::vector<uint32_t> mguide(K), cguide((size_t)K * H);
    bool guided = W <= 65535 && H <= 65535 && guide(mcdf.data(), H, mguide.data());
    for (uint32_t j = 0; guided && j < H; ++j) guided = guide(ccdf.data() + (size_t)j * (W + 1), W, cguide.data() + (size_t)j * K);
    void* bufs[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    const std::vector<float>* src[4] = {&mpdf, &cpdf, &mcdf, &ccdf};
    for (int k = 0; k < 4; ++k) {
        int rc = upload(ctx, bufs[k], src[k]->data(), src[k]->size());
        if (bufs[k]) ctx->env_bufs.push_back(bufs[k]);
        if (rc) return rc;
    }
    if (guided) {
        for (int k = 4; k < 6; ++k) {
            const std::vector<uint32_t>& g = k == 4 ? mguide : cguide;
            int rc = upload(ctx, bufs[k], g.data(), g.size());
            if (bufs[k]) ctx->env_bufs.push_back(bufs[k]);
            if (rc) return rc;
        }
    }
    d.mguide = (const uint32_t*)bufs[4];
    d.cguide = (const uint32_t*)bufs[5];
    d.w = W;
    d.h = H;
    d.invW = invW;
    d.invH = invH;
    d.mpdf = (const float*)bufs[0];
    d.cpdf = (const float*)bufs[1];
    d.mcdf = (const float*)bufs[2];
    d.ccdf = (const float*)bufs[3];
    return NART_OK;
}

// Camera medium: density grid upload + the width-1 MajorantGrid (media.cpp:47-130) on the host.
int build_medium(nart_ctx* ctx, const nart_medium& bm, DMedium& m) {
    std::memset(&m, 0, sizeof(m));
    if (!bm.present) return NART_OK;
    m.present = 1;
    m.rx = (uint8_t)bm.res[0];  // DensityGrid(uint8_t, uint8_t, uint8_t, ...) (scene.cpp:866-868)
    m.ry = (uint8_t)bm.res[1];
    m.rz = (uint8_t)bm.res[2];
    if (m.rx < 2 || m.ry < 2 || m.rz < 2)
        return fail(ctx, NART_E_UNSUPPORTED, "density grids need >= 2 points per axis (DensityGrid::LookUp reads past the grid)");
    for (int i = 0; i < 3; ++i) {
        m.bmin[i] = bm.bounds_min[i];
        m.bmax[i] = bm.bounds_max[i];
        m.Le[i] = bm.Le[i];
    }
    m.sigma_a = bm.sigma_a;
    m.sigma_s = bm.sigma_s;
    const uint32_t npts = bm.res[0] * bm.res[1] * bm.res[2];
    m.density = bm.density;  // host view for the majorant search below
    const float sigma_maj = bm.sigma_a + bm.sigma_s;
    const float mx = ((float)m.rx - 1.f) / 1.f, my = ((float)m.ry - 1.f) / 1.f, mz = ((float)m.rz - 1.f) / 1.f;
    auto u8min = [](uint32_t a, uint32_t b) { return b < a ? b : a; };
    const uint32_t x1 = u8min((uint8_t)(uint32_t)std::ceil(mx), m.rx);
    const uint32_t y1 = u8min((uint8_t)(uint32_t)std::ceil(my), m.ry);
    const uint32_t z1 = u8min((uint8_t)(uint32_t)std::ceil(mz), m.rz);
    float majorant = 0.f;
    for (uint32_t k = 0; k < z1; ++k)
        for (uint32_t j = 0; j < y1; ++j)
            for (uint32_t i = 0; i < x1; ++i) majorant = gmax(majorant, dg_at(m, m.density, i, j, k));
    for (int c = 0; c < 8; ++c)
        majorant = gmax(majorant, dg_lookup(m, m.density, F3((c & 4) ? 1.f : 0.f, (c & 2) ? 1.f : 0.f, (c & 1) ? 1.f : 0.f)));
    m.maj[0] = majorant * sigma_maj;
    m.maj[1] = sigma_maj;
    for (int i = 0; i < 3; ++i) {
        m.maj[2 + i] = bm.bounds_min[i];
        m.maj[5 + i] = bm.bounds_max[i];
    }
    // exact reciprocals of power-of-two divisors (x / 2^k and x * 2^-k round the same real value)
    auto pow2 = [](float x, float& inv) {
        int e = 0;
        if (!(x > 0.f) || !std::isfinite(x) || std::frexp(x, &e) != 0.5f) return false;
        inv = 1.f / x;
        return std::isnormal(inv) && std::frexp(inv, &e) == 0.5f;
    };
    for (int i = 0; i < 3; ++i)
        if (pow2(m.bmax[i] - m.bmin[i], m.inv_bs[i])) m.bs_pow2 |= 1u << i;
    for (int j = 0; j < 8; ++j)
        if (pow2(m.maj[j], m.inv_maj[j])) m.maj_pow2 |= 1u << j;
    if (m.rx == 2 && m.ry == 2 && m.rz == 2) {
        m.grid2 = 1;
        for (int i = 0; i < 8; ++i) m.dens8[i] = bm.density[i];
    }
    int rc = upload(ctx, ctx->d_density, bm.density, npts);
    m.density = (const float*)ctx->d_density;
    return rc;
}

int check_params(nart_ctx* ctx, const nart_render_params* p) {
    if (!p) return fail(ctx, NART_E_INVALID, "null params");
    if (p->integrator != NART_INTEGRATOR_PATH && p->integrator != NART_INTEGRATOR_VOLUME)
        return fail(ctx, NART_E_INVALID, "unknown integrator");
    if (!p->image_width || !p->image_height || !p->bucket_size || !p->spp)
        return fail(ctx, NART_E_INVALID, "imageWidth, imageHeight, bucketSize and spp must be > 0");
    if (!(p->filter_width > 0.f)) return fail(ctx, NART_E_INVALID, "filterWidth must be > 0");
    if (p->integrator == NART_INTEGRATOR_PATH && p->bounces > 32)
        return fail(ctx, NART_E_UNSUPPORTED, "bounces > 32 not supported by the path integrator");
    if (ctx->scene.num_lights == 0)
        return fail(ctx, NART_E_INVALID, "scene has no lights (reference throws in Scene::GetLight)");
    nart_session_geometry g;
    nart_session_geometry_of(p, &g);
    if (g.total_width > 65535 || g.total_height > 65535) return fail(ctx, NART_E_UNSUPPORTED, "image too large");
    return NART_OK;
}

// Per-sample state of one batch (LatinSquare sample, radiance, camera hit: 28 B per sample).  An
// MI355X holds 288 GB, so by default a batch may take half of the device memory free at the call
// (plus what this context already holds for it), at least 16 GiB: whole frames up to 4K x 512 spp
// (119 GB) render in one batch -- fewer launch tails than the former fixed 16 GiB (C5 469 -> 413
// ms, C4 5.27 -> 4.43 s per frame; profiles/r03a_bb_c4.log, r03a_bb_c5_s*.log).  NART_BATCH_BYTES
// overrides.
size_t batch_slot_limit(const nart_ctx* ctx, uint32_t spp) {
    size_t budget = (size_t)16 << 30;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
        const size_t held = ctx->cap_samples * (sizeof(float2) + sizeof(float4) + sizeof(uint32_t));
        budget = std::max(budget, (free_b + held) / 2);
        // sub-contexts that share an ordinal (a multi-device rehearsal) render concurrently and
        // each sees the same free memory: split the budget between them
        budget /= std::max<uint32_t>(1, ctx->mem_share);
    } else {
        (void)hipGetLastError();
    }
    if (const char* e = env_opt("NART_BATCH_BYTES")) budget = (size_t)std::strtoull(e, nullptr, 10);
    size_t per = 8 + (size_t)spp * (sizeof(float2) + sizeof(float4) + sizeof(uint32_t));
    size_t n = budget / per;
    return n < 256 ? 256 : n;
}

// hipMalloc that leaves no sticky error behind: a failed allocation must not make the next
// render's hipGetLastError() report it.
int dmalloc(nart_ctx* ctx, void** p, size_t bytes, const char* what) {
    const hipError_t e = hipMalloc(p, bytes);
    if (e == hipSuccess) return NART_OK;
    *p = nullptr;
    (void)hipGetLastError();
    return fail(ctx, e == hipErrorOutOfMemory ? NART_E_OOM : NART_E_HIP,
                std::string("hipMalloc ") + what + " (" + std::to_string(bytes) + " B): " + hipGetErrorString(e));
}

// Work buffers for a batch.  Each group's capacity is reset before its buffers are freed, so a
// failed allocation leaves a state in which the next call allocates again (never a stale
// capacity over null buffers).
int ensure(nart_ctx* ctx, size_t slots, uint32_t spp, size_t buckets) {
    const size_t samples = slots * spp;
    int rc = NART_OK;
    if (slots > ctx->cap_slots) {
        ctx->cap_slots = 0;
        for (void** b : {(void**)&ctx->d_slot_xy, (void**)&ctx->d_rng, (void**)&ctx->d_slot_so}) {
            if (*b) hipFree(*b);
            *b = nullptr;
        }
        if ((rc = dmalloc(ctx, (void**)&ctx->d_slot_xy, slots * 4, "slot pixels")) ||
            (rc = dmalloc(ctx, (void**)&ctx->d_slot_so, slots * sizeof(SlotSO), "slot sample table")) ||
            (rc = dmalloc(ctx, (void**)&ctx->d_rng, slots * 4, "slot RNG states")))
            return rc;
        ctx->cap_slots = slots;
    }
    if (samples > ctx->cap_samples) {
        ctx->cap_samples = 0;
        for (void** b : {(void**)&ctx->d_samples, (void**)&ctx->d_L, (void**)&ctx->d_prim}) {
            if (*b) hipFree(*b);
            *b = nullptr;
        }
        if ((rc = dmalloc(ctx, (void**)&ctx->d_samples, samples * sizeof(float2), "LatinSquare samples")) ||
            (rc = dmalloc(ctx, (void**)&ctx->d_L, samples * sizeof(float4), "per-sample radiance")) ||
            (rc = dmalloc(ctx, (void**)&ctx->d_prim, samples * sizeof(uint32_t), "camera-ray hits")))
            return rc;
        ctx->cap_samples = samples;
    }
    if (buckets > ctx->cap_buckets) {
        ctx->cap_buckets = 0;
        for (void** b : {(void**)&ctx->d_bucket_ids, (void**)&ctx->d_bucket_base}) {
            if (*b) hipFree(*b);
            *b = nullptr;
        }
        if ((rc = dmalloc(ctx, (void**)&ctx->d_bucket_ids, buckets * 4, "bucket ids")) ||
            (rc = dmalloc(ctx, (void**)&ctx->d_bucket_base, buckets * 4, "bucket bases")))
            return rc;
        ctx->cap_buckets = buckets;
    }
    return NART_OK;
}

// Work-queue buffers of the megakernel scheduler (queue, cost probe, radix-sort scratch).
int ensure_queue(nart_ctx* ctx, uint32_t n) {
    if (n <= ctx->cap_queue) return NART_OK;
    void** bufs[7] = {(void**)&ctx->d_queue, (void**)&ctx->d_cost, (void**)&ctx->d_keys[0], (void**)&ctx->d_keys[1],
                      (void**)&ctx->d_vals[0], (void**)&ctx->d_vals[1], (void**)&ctx->d_qhead};
    for (void** b : bufs) {
        if (*b) hipFree(*b);
        *b = nullptr;
    }
    if (ctx->d_sort_tmp) hipFree(ctx->d_sort_tmp);
    ctx->d_sort_tmp = nullptr;
    ctx->cap_queue = 0;
    for (int i = 0; i < 6; ++i) HIPCHK(hipMalloc(bufs[i], (size_t)n * 4));
    HIPCHK(hipMalloc(bufs[6], 256));
    size_t tmp = 0, t1 = 0, t2 = 0;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, t1, ctx->d_keys[0], ctx->d_keys[1], ctx->d_vals[0],
                                              ctx->d_vals[1], (int)n, 0, 1));
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, t2, ctx->d_keys[0], ctx->d_keys[1], ctx->d_vals[0],
                                              ctx->d_vals[1], (int)((n + 63) / 64), 0, 32));
    tmp = std::max(t1, t2);
    HIPCHK(hipMalloc(&ctx->d_sort_tmp, tmp + 256));
    ctx->cap_sort_tmp = tmp + 256;
    ctx->cap_queue = n;
    return NART_OK;
}

// LDS of one k_render block: traversal stack + as many top BVH nodes as fit while
// NART_RENDER_WAVES blocks share a CU's 160 KiB (NART_LDS_NODES overrides the node count).
uint32_t render_lds_nodes(const nart_ctx* ctx, size_t fixed = 0, uint32_t blocks_of_256 = 1) {
    const size_t stack = fixed ? fixed : (size_t)ctx->stack_depth * 256 * 8;
    const size_t budget = (size_t)160 * 1024 * blocks_of_256 / NART_RENDER_WAVES;
    size_t n = budget > stack ? (budget - stack) / sizeof(BVHNode) : 0;
    while (n && node_lds_bytes((uint32_t)n) > budget - stack) --n;  // NART_NODE_PAD padding
    return (uint32_t)std::min<size_t>(n, ctx->num_nodes);
}

// The ray-queue kernel's fixed LDS (stack + outboxes + results + id rings) fits one block per CU
// (stack_depth <= 24 at 512 lanes).  NART_RQ_LDS_LIMIT lowers the budget (tests of the fallback).
bool rq_fits(const nart_ctx* ctx) {
    const size_t limit = (size_t)std::min(env_num("NART_RQ_LDS_LIMIT", 160.0 * 1024), 160.0 * 1024);
    return rq_lds_bytes(ctx->stack_depth, NART_RQ_BLOCK) <= limit;
}

// ---------------------------------------------------------------- megakernel scheduling
// A pixel's samples are one serial chain (its RNG stream), so a frame can finish no earlier
// than its costliest pixels, and a wave of 64 costly pixels runs several times longer than one
// such pixel alone (the wave executes the union of its lanes' work).  With the work queue the
// grid is persistent: lanes take pixels from a queue ordered by a cost probe (one sample per
// pixel), the costliest pixels spread over all waves so that each holds only a few of them,
// and a lane whose pixel is done takes the next one instead of idling until its wave ends.
// The image is unchanged (each pixel's samples stay on its own RNG stream).
//   NART_QUEUE=0  one lane per pixel, no queue (the launch order is the slot order)
//   NART_QUEUE=1  persistent lanes, queue in slot order
//   NART_QUEUE=2  persistent lanes, queue ordered by the cost probe (default)

// Group (wave-sized run of 64 consecutive slots: a 16x4 strip of a bucket) costs, as keys of an
// ascending sort that puts the costliest group first; a partial last group always sorts last.
// per: cost entries per group (64: one per slot; fewer: the sampled probe, probe_sub).
__global__ void k_group_keys(const uint32_t* cost, uint32_t n, uint32_t* keys, uint32_t* vals, uint32_t per = 64) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t ng = (n + 63) / 64;
    if (g >= ng) return;
    uint64_t sum = 0;
    const uint32_t e = min(n, 64 * g + 64);
    if (per < 64) {  // a partial last group is keyed last below, whatever its entries hold
        if (e - 64 * g == 64)
            for (uint32_t i = per * g; i < per * g + per; ++i) sum += cost[i];
    } else {
        for (uint32_t i = 64 * g; i < e; ++i) sum += cost[i];
    }
    const uint32_t c = (uint32_t)min<uint64_t>(sum, 0xFFFFFFFEull);
    keys[g] = (e - 64 * g < 64) ? 0xFFFFFFFFu : 0xFFFFFFFEu - c;
    vals[g] = g;
}

// Two cost classes of groups for the wave-group refill order: keys[g] = 0 for the E costliest
// groups (ranks [0, E) of the cost-sorted list), 1 for the rest; vals = group ids in slot order,
// so a stable sort by the key keeps slot order inside each class.
__global__ void k_group_class(const uint32_t* sorted, uint32_t ng, uint32_t E, uint32_t* keys, uint32_t* vals) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= ng) return;
    keys[sorted[r]] = r < E ? 0u : 1u;
    vals[r] = r;
}

// Pixel list of the sorted groups (group order, slot order inside a group).
__global__ void k_expand_groups(const uint32_t* groups, uint32_t n, uint32_t* pixels) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    pixels[r] = 64 * groups[r / 64] + r % 64;
}

// Mark the k*W costliest pixels (ranks [0, E) of the class-sorted list) for the 1-bit partition.
__global__ void k_flag_top(const uint32_t* sorted, uint32_t n, uint32_t E, uint32_t* flag) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    flag[sorted[r]] = r < E ? 1u : 0u;
}

// Queue: in the first round of W waves, lanes j < k of wave w take the costly pixel of rank
// j*W + w (each wave holds k of them); every other position takes the remaining pixels in
// slot order (spatially coherent waves).
// With prio set (k_render_rq) the costly entries carry RQ_PRIO_BIT; with pairs = Q (2 or 4) each
// costly pixel goes to Q adjacent lanes (Qj .. Qj + Q - 1) with RQ_PAIR_BIT too, and the queue is
// n + (Q - 1)*k*W long.
__global__ void k_build_queue(const uint32_t* top, const uint32_t* rest, uint32_t n, uint32_t W, uint32_t k,
                              uint32_t prio, uint32_t pairs, uint32_t half, uint32_t quad, uint32_t* queue) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t per = pairs ? pairs : 1u, kk = per * k;  // first-round lanes of the costly pixels
    if (p >= n + (per - 1u) * k * W + (quad ? 2u * W : 0u)) return;
    const uint32_t g = 64u * W;
    if (p < g && quad) {
        // quad: each first-round wave's costliest pixel (ranks 0..W-1) on four lanes, its other k-1
        // costly pixels on pairs
        const uint32_t w = p / 64u, j = p % 64u, kq = kk + 2u;
        if (j < 4u) queue[p] = top[w] | prio | RQ_PAIR_BIT | RQ_QUAD_BIT;
        else if (j < kq) queue[p] = top[((j - 4u) / per + 1u) * W + w] | prio | RQ_PAIR_BIT;
        else queue[p] = rest[w * (64u - kq) + (j - kq)];
    } else if (p >= g && quad) {
        queue[p] = rest[(64u - kk - 2u) * W + (p - g)];
    } else if (p < g && half) {
        // half = BW, the waves of a ray-queue block (8 or 12: PB = 2 or 3 per SIMD): only its first 4
        // waves hold costly pixels (PB k each), so each SIMD has one priority wave
        const uint32_t BW = half, PB = BW / 4u;
        const uint32_t w = p / 64u, j = p % 64u, b = w / BW, i = w % BW, k2 = PB * kk;
        const uint32_t pw = b * 4u + i;  // priority wave index
        const uint32_t roff = b * BW * (64u - kk) + (i < 4u ? i * (64u - k2) : 4u * (64u - k2) + (i - 4u) * 64u);
        if (i < 4u && j < k2) queue[p] = top[(j / per) * (W / PB) + pw] | prio | (pairs ? RQ_PAIR_BIT : 0u);
        else queue[p] = rest[roff + (i < 4u ? j - k2 : j)];
    } else if (p < g) {
        const uint32_t w = p / 64u, j = p % 64u;
        queue[p] = j < kk ? (top[(j / per) * W + w] | prio | (pairs ? RQ_PAIR_BIT : 0u))
                          : rest[w * (64u - kk) + (j - kk)];
    } else {
        queue[p] = rest[(64u - kk) * W + (p - g)];
    }
}

// Pixel list (into `out`) of the wave-sized slot groups ordered by the probe costs in
// ctx->d_cost, costliest group first (ties keep slot order).
int sort_groups_by_cost(nart_ctx* ctx, uint32_t n, uint32_t* out, hipStream_t st);

// Sample-major bucket layout: slot `base + p` of a bucket of `cnt` traced pixels keeps sample s
// at base*spp + s*cnt + p (k_splat_col4's lanes then read neighbouring pixels' sample s from one
// line); pixel-major: at (base + p)*spp + s (k_splat_skew streams one pixel's samples).  One
// block per bucket of the batch.
__global__ void k_slot_table(const uint32_t* bucket_base, uint32_t nbk, uint32_t nslots, uint32_t spp, SlotSO* so,
                             bool pixel_major) {
    const uint32_t b = blockIdx.x;
    const uint32_t base = bucket_base[b], end = b + 1 < nbk ? bucket_base[b + 1] : nslots;
    for (uint32_t p = threadIdx.x; base + p < end; p += blockDim.x)
        so[base + p] = pixel_major ? SlotSO{(unsigned long long)(base + p) * spp, 1u, 0u}
                                   : SlotSO{(unsigned long long)base * spp + p, end - base, 0u};
}

__global__ void k_slot_rows(uint32_t n, uint32_t spp, SlotSO* so) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) so[i] = SlotSO{(unsigned long long)i * spp, 1u, 0u};
}

// Volume queue with the H costliest groups (sorted group ids, costliest first) spread S pixels per
// wave, the wave's other lanes idle (0xFFFFFFFF), then the remaining groups dense.
__global__ void k_sparse_groups(const uint32_t* groups, uint32_t n, uint32_t H, uint32_t S, uint32_t qlen,
                                uint32_t* queue) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= qlen) return;
    const uint32_t hot = H * (64u / S) * 64u;
    if (p < hot) {
        const uint32_t w = p / 64u, j = p % 64u, g = w / (64u / S), part = w % (64u / S);
        const uint32_t slot = 64u * groups[g] + part * S + j;
        queue[p] = (j < S && slot < n) ? slot : 0xFFFFFFFFu;
    } else {
        const uint32_t r = p - hot + 64u * H;  // rank in the dense group order
        queue[p] = 64u * groups[r / 64u] + r % 64u;
    }
}

__global__ void k_iota(uint32_t* v, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = i;
}

#ifndef NART_RQ_GROUP_LANES
#define NART_RQ_GROUP_LANES 2
#endif
// pixel work queue: 2 = cost probe + priority queue / wave-group refill (the schedule; 0, no
// queue, and 1, refill in slot order, were A/B forms)
constexpr int queue_mode() { return 2; }

int sort_groups_by_cost(nart_ctx* ctx, uint32_t n, uint32_t* out, hipStream_t st) {
    const uint32_t ng = (n + 63) / 64;
    hipLaunchKernelGGL(k_group_keys, dim3((ng + 255) / 256), dim3(256), 0, st, ctx->d_cost, n, ctx->d_keys[0],
                       ctx->d_vals[0]);
    size_t tmp = ctx->cap_sort_tmp;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(ctx->d_sort_tmp, tmp, ctx->d_keys[0], ctx->d_keys[1], ctx->d_vals[0],
                                              ctx->d_vals[1], (int)ng, 0, 32, st));
    hipLaunchKernelGGL(k_expand_groups, dim3((n + 255) / 256), dim3(256), 0, st, ctx->d_vals[1], n, out);
    HIPCHK(hipGetLastError());
    return NART_OK;
}

uint32_t lean_stack(const nart_ctx* ctx);
// traversal-phase quorum of throughput-bound ray-queue launches: the phase ends once the wave's
// queue is empty and at most this many lanes still trace (0/4/16/32: 134.7/123.5/123.0/129.9 vs
// 121.6 ms at 8 in round 2)
#ifndef NART_RQ_QUORUM
#define NART_RQ_QUORUM 8u
#endif

template <bool EXT, bool COUNT, bool ENV, uint32_t FM = FT_ALL, int WV = 2, bool PR = true>
int launch_render(nart_ctx* ctx, const RenderArgs& a_in, hipStream_t st) {
    auto kern = k_render<EXT, COUNT, ENV>;
    auto kern_rq = k_render_rq<EXT, COUNT, ENV, FM, WV, PR>;
    constexpr uint32_t RQB = RQ_BLOCK_OF(COUNT, WV);  // ray-queue block (kernels.h)
    RenderArgs a = a_in;
    if (EXT) {
        // the dielectric list's entries beyond ILIST_REG: one column per thread of the largest
        // launch below (whole 512-thread blocks over every slot)
        const size_t lanes = ((size_t)a.n_slots + 511) / 512 * 512;
        const size_t bytes = lanes * (ILIST_MAX - ILIST_REG) * sizeof(uint2);
        if (bytes > ctx->cap_ilist) {
            if (ctx->d_ilist) HIPCHK(hipFree(ctx->d_ilist));
            ctx->d_ilist = nullptr;
            ctx->cap_ilist = 0;
            if (hipMalloc(&ctx->d_ilist, bytes) != hipSuccess) return fail(ctx, NART_E_OOM, "hipMalloc dielectric lists");
            ctx->cap_ilist = bytes;
        }
        a.ilist_ext = static_cast<uint2*>(ctx->d_ilist);
        a.ilist_stride = (uint32_t)lanes;
    }
    static std::atomic<uint64_t> attr{0};  // dynamic LDS above the 64 KiB default, set once per device
    const uint64_t dbit = 1ull << (ctx->device & 63);
    if (!(attr.load() & dbit)) {
        for (const void* f : {(const void*)kern, (const void*)k_render<EXT, true, ENV>,
                              (const void*)kern_rq, (const void*)k_primary<COUNT, ENV, FM>})
            hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr.fetch_or(dbit);
    }
    // variant 0: ray-queue kernel; 3: k_render (one lane per pixel, the fallback below).
    // The ray-queue kernel's 512-lane blocks keep a stack_depth * 4 KiB traversal stack plus
    // 60 KiB of ray outboxes in LDS: a BVH deeper than 24 levels does not fit, and those scenes
    // run k_render (256-lane blocks, stack_depth * 2 KiB) instead -- same image.
    const bool rq = ctx->variant == 0 && rq_fits(ctx);
    ctx->fm_used = rq ? FM : FT_ALL;
    if (rq && FM != FT_ALL) ctx->sched |= NART_SCHED_SPECIALIZED;
    if (rq && WV == 3 && !PR) ctx->sched |= NART_SCHED_LEAN;
    // camera rays first, coherently (k_primary; leaving them to the path kernel measured C3 470 vs
    // 407 ms per frame, profiles/r02h_env_ab.log)
    const bool primary = true;

    // rounds of resident waves from which a launch counts as throughput-bound: ray-queue quorum 8
    // (else 0), no priority lanes or speculative pairs
    const double q_rounds = 3.0;
    RenderArgs b = a;
    b.lds_nodes = render_lds_nodes(ctx);
    const size_t lds = (size_t)ctx->stack_depth * 256 * 8 + node_lds_bytes(b.lds_nodes);
    RenderArgs brq = a;  // ray-queue kernel: outbox, results and id lists take part of the LDS
    if (rq && primary && ctx->d_prim && a.cost == nullptr) {
        // (staging the top BVH nodes in LDS, as the path kernel does, measured slower here: a
        // wave's coherent rays read the same node, which the L1 broadcasts: 9.7 vs 8.2 ms at 64 spp)
        // camera rays as wave packets (path.h traverse_packet; C3 -1.7 ms, C4 -31 ms per frame,
        // profiles/r04_primary_packet_ab.log); NART_PRIMARY_PACKET=0 (read per call): one ray per lane
        RenderArgs pa = a;
        pa.packet = env_num("NART_PRIMARY_PACKET", 1.0) != 0.0 ? 1u : 0u;
        hipLaunchKernelGGL((k_primary<COUNT, ENV, FM>), dim3((a.n_slots + 255) / 256), dim3(256),
                           (size_t)ctx->stack_depth * 256 * 8, st, ctx->scene, pa, ctx->d_prim);
        HIPCHK(hipGetLastError());
        if (ctx->events) {
            HIPCHK(hipEventRecord(ctx->ev[4], st));
            ctx->primary_ran = true;
        }
        ctx->sched |= NART_SCHED_PRIMARY;
        brq.prim = ctx->d_prim;
    }
    // one ray-queue block per CU (2 or 3 waves per SIMD); the lean build keeps lean_stack(ctx)
    // stack levels in LDS and the rest in a global column per thread
    const uint32_t skd = WV == 3 ? lean_stack(ctx) : ctx->stack_depth;
    brq.lds_nodes = render_lds_nodes(ctx, rq_lds_bytes(skd, RQB), NART_RENDER_WAVES);
    const size_t lds_rq = rq_lds_bytes(skd, RQB) + node_lds_bytes(brq.lds_nodes);
    const dim3 block(256);
    uint32_t blocks = (a.n_slots + 255) / 256;
    const int mode = queue_mode();
    int cus = 0, per_cu = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, 256, lds));
    const uint32_t resident_k = (uint32_t)std::max(1, cus * std::max(per_cu, 1));
    // rounds of resident waves (of k_render: the same figure for every build, so that the lean
    // build's choice, lean_fits, and this launch's thresholds agree)
    const double R = (double)a.n_slots / (64.0 * 4.0 * resident_k);
    // resident blocks of 256 lanes of the kernel this launch runs: the ray-queue kernel holds one
    // 512- or 768-lane block per CU, so its persistent grid and the waves the queue deals its
    // first round over are its own (the lean build has 1.5x k_render's resident lanes)
    int per_cu_rq = 0;
    if (rq) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_rq, (const void*)kern_rq, RQB, lds_rq));
    const uint32_t resident = rq ? (uint32_t)std::max(1, cus * std::max(per_cu_rq, 1)) * (RQB / 256) : resident_k;
    const uint32_t W = resident * 4;  // resident (persistent) waves
    // the ray-queue kernel takes kern's place (its own LDS layout); the cost probe keeps k_render
    auto launch = [&](uint32_t nblocks, const RenderArgs& args) -> int {
        if (rq) {
            // traversal-phase quorum: 8 on throughput-bound launches; 0 (every queued ray resolved
            // before the path phase) on small shards, whose costliest pixels' chains set the time
            // (1/8 C3 shard: 100.5 -> 96.0 ms)
            RenderArgs r2 = args;
            r2.lds_nodes = brq.lds_nodes;
            r2.prim = brq.prim;
            r2.stack_lds = skd;
            r2.rq_quorum = R >= q_rounds ? NART_RQ_QUORUM : 0u;
            const uint32_t per = RQB / 256;  // launches are counted in blocks of 256
            const uint32_t grid = (nblocks + per - 1) / per;
            const size_t threads = (size_t)grid * RQB;
            if (r2.stack_lds < 1 || r2.stack_lds > ctx->stack_depth || lds_rq > (size_t)160 * 1024)
                return fail(ctx, NART_E_INVALID, "ray-queue LDS layout out of range");
            // per-thread global columns, indexed by the global thread id: sized from this grid
            if (EXT && threads > r2.ilist_stride)
                return fail(ctx, NART_E_INVALID, "dielectric-list columns smaller than the launch");
            if (skd < ctx->stack_depth) {
                const size_t bytes = threads * (ctx->stack_depth - skd) * sizeof(int2);
                if (bytes > ctx->cap_gstack) {
                    if (ctx->d_gstack) HIPCHK(hipFree(ctx->d_gstack));
                    ctx->d_gstack = nullptr;
                    ctx->cap_gstack = 0;
                    if (hipMalloc(&ctx->d_gstack, bytes) != hipSuccess)
                        return fail(ctx, NART_E_OOM, "hipMalloc traversal stack columns");
                    ctx->cap_gstack = bytes;
                }
                r2.gstack = static_cast<int2*>(ctx->d_gstack);
            }
            hipLaunchKernelGGL(kern_rq, dim3(grid), dim3(RQB), lds_rq, st, ctx->scene, r2);
        } else {
            hipLaunchKernelGGL(kern, dim3(nblocks), block, lds, st, ctx->scene, args);
        }
        HIPCHK(hipGetLastError());
        return NART_OK;
    };
    if (mode > 0) {
        if (blocks > resident) {  // more pixels than resident lanes: persistent grid + queue
            const uint32_t n = a.n_slots;
            // room for the speculative groups' duplicates: qlen = n + (Q - 1) * k * W with Q * k <= 64
            int rc = ensure_queue(ctx, n + 63u * W);
            if (rc) return rc;
            const dim3 eg((n + 255) / 256);
            // costly pixels per first-round wave: few when the shard is small (their serial chains
            // bound the frame), all 64 (packed, launched first) when there are many rounds
            // Priority lanes for the costly pixels in the ray-queue kernel (NART_RQ_PRIO=0: off, 2:
            // also on launches of >= 3 rounds), run as speculative lane groups of Q lanes
            // (NART_RQ_PAIRS: 0 one lane per pixel, 1 or 2 pairs, 4 groups of four).  Only small
            // shards (< 3 rounds of resident waves), whose time is their costliest pixels' chains: on
            // throughput-bound launches the priority breaks and the speculative duplicates cost
            // throughput (1/2 C3 shard 238 -> 249 ms, C4 batches 3175 -> 3381 ms with them on)
            const int prio_env = (int)env_num("NART_RQ_PRIO", 1.0);
            const bool prio_on = prio_env == 2 || (prio_env == 1 && R < q_rounds);
            const int pe = (int)env_num("NART_RQ_PAIRS", NART_RQ_GROUP_LANES);
            const uint32_t Q = pe <= 0 ? 0u : (pe >= 4 ? 4u : 2u);
            // (the lean build has no priority lanes: it runs only where prio_on is false anyway)
            const uint32_t pbit = (rq && prio_on && PR) ? RQ_PRIO_BIT : 0u;
            // Half waves (default): the costly pixels only on the first 4 waves of each ray-queue
            // block (8 or 12 waves), PB = 2 or 3 shares each -- one such wave per SIMD -- and those
            // waves at a raised issue priority (s_setprio 2, NART_RQ_SETPRIO) while they hold priority
            // work, so the SIMD's other waves fill their stalls instead of sharing issue with them.
            // C3 1/8 shard, every rank: mean 84.2 -> 80.9 ms, worst 87-92 -> 86.0 ms
            // (profiles/r05h_chain_schedule_ab.log).  NART_RQ_HALF=0: dealt over every wave.
            const uint32_t BW = RQB / 64u, PB = BW / 4u;
            // costly pixels per first-round wave: few when the shard is small (their serial chains
            // bound the frame), all 64 (packed, launched first) when there are many rounds.  C3 1/8
            // shard, mean of the 8 ranks with half waves at k = 4/6/8/12/14/16 per two-wave block
            // share: 95.2/88.8/81.4/80.9/81.3/81.6 ms; three-wave blocks keep the same number of
            // costly pixels (k W constant: 8 per share).  The half layout is settled first, so a
            // configuration it does not fit falls back to k = 8 dealt over every wave.
            const uint32_t k_half = PB == 2u ? 12u : 8u;
            const bool half = pbit && rq && env_num("NART_RQ_HALF", 1.0) != 0.0 && (W % BW) == 0u && R < 3.0 &&
                              PB * ((Q && Q * k_half <= 64u) ? Q : 1u) * k_half <= 64u;
            uint32_t k = R >= 3.0 ? 32u : (half ? k_half : 8u);
            // ray-queue kernel: wave-group refill from 6 rounds of resident waves (C3 1/2 shard, 8
            // rounds: 241 -> 235 ms; C4 batches, ~9 rounds: 1385 -> 1566 Msamples/s).  Below that a
            // wave of costly groups outlasts the rest (1/4 shard, 4 rounds: 146 -> 211 ms; with the
            // groups cost-ordered still 156 vs 114 ms), and the probe-ordered pixel queue with
            // priority lanes stays.  The lean build (from 3 rounds where it runs: scenes without
            // glass) takes groups from there: C2 1/4 shard 32.2 -> 27.9 ms
            // (profiles/r06x_mid_shards.log)
            const double g_rounds = WV == 3 ? 3.0 : 6.0;
            if (R >= (rq ? g_rounds : 12.0) && mode == 2 && !env_opt("NART_QUEUE_K")) {
                // many rounds: the slot order (costly waves interleaved with cheap ones in time)
                // measured faster than any reordering; no probe.  The ray-queue kernel runs it on
                // a persistent grid whose waves take wave-sized slot groups in that order
                // (one wave per group, blocks retiring as a whole: 422 vs 407 ms, profiles/r02h_env_ab.log)
                const bool groups = rq;
                if (groups) {
                    HIPCHK(hipMemsetAsync(ctx->d_qhead, 0, sizeof(uint32_t), st));
                    b.ghead = ctx->d_qhead;
                    // group order (NART_RQ_ORDER): 0 slot order; 1 costliest group first (cost
                    // probe); 2 (default) the NART_RQ_TOPF % (default 10) costliest groups first,
                    // each class in slot order.  In slot order the costly groups (behind the
                    // glass) taken last left a tail: at 90 % of the C3 launch only 25 of 2,048
                    // waves were still running (WAVEPROF timeline).  C3 frame 445 -> 407 ms
                    // (probe included; order 1: 408, top 20 / 35 %: 408 / 408 ms)
                    // the lean build's slower waves leave a longer tail behind the costly groups taken
                    // late: fully cost-ordered groups (1) measured C3 227.5 vs 235-247 ms for the
                    // costliest 10 % first (2), 250 / 245 / 260 ms for 5 / 20 / 35 %, slot order 299
                    // (profiles/r06r_group_order_ab.log), C2 75 vs 77 ms; C4's environment-light
                    // frame keeps 2 (4K/128: 609 vs 624 ms, r06s_group_order_c4_c2.log).  The two-wave
                    // build's launches of 6-12 rounds (C3 1/2 shard, chain-bound) also take 1: worst
                    // rank 183-184 -> 167-169 ms (profiles/r06x_mid_shards.log)
                    const int order = (int)env_num("NART_RQ_ORDER", !ENV ? 1.0 : 2.0);
                    ctx->sched |= NART_SCHED_WAVE_GROUPS;
                    if (order == 1 || order == 2) {
                        // cost probe: the first sample of NART_PROBE_SUB (default 8) evenly spaced
                        // pixels of every 64-slot group (64: every pixel).  Only the group order
                        // depends on it (costliest NART_RQ_TOPF % first), and that order is not
                        // sensitive to the estimate (TOPF 10 / 20 / 35 %: 407 / 408 / 408 ms)
                        // Launches of fewer than NART_PROBE_SUB_ROUNDS (12) rounds of resident waves
                        // probe every pixel: there a costly group the sample missed and took late
                        // sets the tail (C4 1/8 shards, 8 rounds: worst rank 488-496 ms probing every
                        // pixel, 552-556 ms sampled; profiles/r05ah_c4_probe_ab.log)
                        const uint32_t ng = (n + 63) / 64;
                        const double sub_rounds = 12.0;
                        uint32_t sub = (uint32_t)env_num("NART_PROBE_SUB", R >= sub_rounds ? 8.0 : 64.0);
                        if (sub != 1u && sub != 2u && sub != 4u && sub != 8u && sub != 16u && sub != 32u) sub = 64u;
                        RenderArgs pb = b;
                        pb.spp = 1;
                        pb.cost = ctx->d_cost;
                        pb.ghead = nullptr;
                        pb.probe_sub = sub < 64u ? sub : 0u;
                        const uint32_t pblocks = sub < 64u ? (ng * sub + 255u) / 256u : blocks;
                        hipLaunchKernelGGL((k_render<EXT, true, ENV>), dim3(pblocks), block, lds, st, ctx->scene, pb);
                        const dim3 gg((ng + 255) / 256);
                        hipLaunchKernelGGL(k_group_keys, gg, block, 0, st, ctx->d_cost, n, ctx->d_keys[0], ctx->d_vals[0],
                                           sub);
                        size_t tmp = ctx->cap_sort_tmp;
                        HIPCHK(hipcub::DeviceRadixSort::SortPairs(ctx->d_sort_tmp, tmp, ctx->d_keys[0], ctx->d_keys[1],
                                                                  ctx->d_vals[0], ctx->d_vals[1], (int)ng, 0, 32, st));
                        if (order == 1) {
                            b.gorder = ctx->d_vals[1];
                        } else {
                            const double f = env_num("NART_RQ_TOPF", 10.0);
                            const uint32_t E = (uint32_t)std::min<double>(ng, std::max(0.0, f) * 0.01 * ng);
                            hipLaunchKernelGGL(k_group_class, gg, block, 0, st, ctx->d_vals[1], ng, E, ctx->d_keys[0],
                                               ctx->d_vals[0]);
                            tmp = ctx->cap_sort_tmp;
                            HIPCHK(hipcub::DeviceRadixSort::SortPairs(ctx->d_sort_tmp, tmp, ctx->d_keys[0], ctx->d_keys[1],
                                                                      ctx->d_vals[0], ctx->d_queue, (int)ng, 0, 1, st));
                            b.gorder = ctx->d_queue;
                        }
                    }
                    // launches are counted in blocks of 256 threads
                    blocks = std::min(blocks, resident);
                }
                return launch(blocks, b);
            }
            if (env_opt("NART_QUEUE_K")) k = (uint32_t)std::max(1.0, std::min(64.0, env_num("NART_QUEUE_K", 8.0)));
            const bool refill = k < 64u || mode == 1;
            if (mode == 1) {
                hipLaunchKernelGGL(k_iota, eg, block, 0, st, ctx->d_queue, n);
            } else {
                RenderArgs pb = b;  // cost probe: the first sample of every pixel
                pb.spp = 1;
                pb.cost = ctx->d_cost;
                hipLaunchKernelGGL((k_render<EXT, true, ENV>), dim3(blocks), block, lds, st, ctx->scene, pb);
                int rc2 = sort_groups_by_cost(ctx, n, k == 64u ? ctx->d_queue : ctx->d_cost, st);
                if (rc2) return rc2;
                size_t tmp = 0;
                if (k == 64u) {  // whole groups, costliest first (coherent waves, longest chains first)
                    b.queue = ctx->d_queue;
                    return launch(blocks, b);
                }
                HIPCHK(hipMemcpyAsync(ctx->d_vals[1], ctx->d_cost, (size_t)n * 4, hipMemcpyDeviceToDevice, st));
                // d_vals[1] = pixels by cost class; partition the rest (slot order) from the top k*W
                hipLaunchKernelGGL(k_flag_top, eg, block, 0, st, ctx->d_vals[1], n, k * W, ctx->d_keys[0]);
                hipLaunchKernelGGL(k_iota, eg, block, 0, st, ctx->d_cost, n);
                tmp = ctx->cap_sort_tmp;
                HIPCHK(hipcub::DeviceRadixSort::SortPairs(ctx->d_sort_tmp, tmp, ctx->d_keys[0], ctx->d_keys[1],
                                                          ctx->d_cost, ctx->d_vals[0], (int)n, 0, 1, st));
                const uint32_t pairs = (pbit && Q && Q * k <= 64u) ? Q : 0u;
                // (re-checked: NART_QUEUE_K may have changed k)
                const bool hw = half && PB * (pairs ? pairs : 1u) * k <= 64u;
                // NART_RQ_QUAD (A/B): each first-round wave's costliest pixel gets four lanes
                const bool quad = pbit && pairs == 2u && 2u * k + 2u <= 64u && env_num("NART_RQ_QUAD", 0.0) != 0.0;
                const uint32_t qlen = n + (pairs ? (pairs - 1u) * k * W : 0u) + (quad ? 2u * W : 0u);
                hipLaunchKernelGGL(k_build_queue, dim3((qlen + 255) / 256), block, 0, st, ctx->d_vals[1], ctx->d_vals[0],
                                   n, W, k, pbit, pairs, hw && !quad ? BW : 0u, quad ? 1u : 0u, ctx->d_queue);
                b.rq_setprio = pbit ? (uint32_t)std::max(0.0, env_num("NART_RQ_SETPRIO", hw ? 1.0 : 0.0)) : 0u;
                if (hw && !quad) ctx->sched |= NART_SCHED_HALF_WAVES;
                b.rq_prio = pbit ? 1u : 0u;
                b.rq_pairs = pairs;
                b.qlen = qlen;
                if (pbit) ctx->sched |= NART_SCHED_PRIORITY;
                if (pairs) ctx->sched |= NART_SCHED_SPEC_PAIRS;
            }
            b.queue = ctx->d_queue;
            if (refill) {
                HIPCHK(hipMemsetAsync(ctx->d_qhead, 0, sizeof(uint32_t), st));
                b.qhead = ctx->d_qhead;
                ctx->sched |= NART_SCHED_PROBE_QUEUE;
                // whole ray-queue blocks, so that every first-round lane's entry lies below qbase
                const uint32_t per = rq ? RQB / 256 : 1u;
                blocks = (resident + per - 1u) / per * per;
                b.qbase = blocks * 256;
            }
        }
    }
    return launch(blocks, b);
}

template <bool ENV>
int launch_render_maxl(nart_ctx* ctx, const RenderArgs& a, hipStream_t st) {
    // a path grows the dielectric list by at most one entry per bounce: the register list alone
    // serves bounces <= ILIST_REG; deeper ones (up to 32) spill it to the per-lane columns
    const bool c = ctx->counters;
    if (a.bounces <= ILIST_REG)
        return c ? launch_render<false, true, ENV>(ctx, a, st) : launch_render<false, false, ENV>(ctx, a, st);
    return c ? launch_render<true, true, ENV>(ctx, a, st) : launch_render<true, false, ENV>(ctx, a, st);
}

// Scene-specialised builds of the path kernels (k_render_rq, k_primary): glassSphere's (C3:
// Lambert + glass, one kind of area light, constant patterns), the Cornell box's (C2: Lambert,
// disk) and the textured environment-lit plastic of C4.  A render takes the first build whose mask
// covers the scene's (ctx->features); others, the counter pass and renders with bounces > ILIST_REG
// run the generic build.  Same operations per kind, so every build renders the same image
// (tests/test_gpu_specialize.py compares them on every suite scene).
constexpr uint32_t FM_DIFFUSE = FT_LAMBERT | FT_DISK;
constexpr uint32_t FM_GLASS = FT_LAMBERT | FT_GLASS | FT_DISK;
constexpr uint32_t FM_ENVTEX = FT_LAMBERT | FT_PLASTIC | FT_ENV | FT_TEX | FT_NMAP;

// Traversal-stack levels the lean build keeps in LDS: all of them where the 768-lane block's LDS
// then still stages 320 BVH nodes (or the whole BVH), else as many as leave room for them (>= 4;
// deeper levels go to per-thread global columns).  C3 (14 levels, 759 nodes): 8 levels and 352
// nodes; 7 / 8 / 10 levels measured 241 / 241 / 245 ms per frame, +-7 ms run to run
// (profiles/r06e_lean_stack_ab.log).  NART_LEAN_STACK (tests) forces a depth.
uint32_t lean_stack(const nart_ctx* ctx) {
    if (env_opt("NART_LEAN_STACK"))
        return std::max<uint32_t>(1u, std::min<uint32_t>(ctx->stack_depth, (uint32_t)env_num("NART_LEAN_STACK", 1.0)));
    const size_t nodes = std::min<size_t>(ctx->num_nodes, 320) * sizeof(BVHNode);
    uint32_t k = ctx->stack_depth;
    while (k > 4 && rq_lds_bytes(k, 768) + nodes > (size_t)160 * 1024) --k;
    return k;
}

// Rounds of resident waves a launch of n slots spans (launch_render's R): from 3 on the launch is
// throughput-bound and runs without priority lanes or speculative pairs.
double launch_rounds(nart_ctx* ctx, uint32_t n) {
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess) return 0.0;
    const size_t lds = (size_t)ctx->stack_depth * 256 * 8 + node_lds_bytes(render_lds_nodes(ctx));
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_render<false, false, false>, 256, lds) !=
        hipSuccess)
        return 0.0;
    const double W = (double)std::max(1, cus * std::max(per_cu, 1)) * 4.0;
    return (double)n / (64.0 * W);
}

// The lean three-waves-per-SIMD build (kernels.h WV = 3) for throughput-bound launches.  It raises
// throughput (C3 whole frame, 16 rounds of resident waves: path kernels 276.6 -> ~241 ms; C4 4K
// frame and its 1/8 shards, 8 rounds: 492 -> 456 ms) but each of its waves runs slower, which
// lengthens the serial sample chains of a scene's costliest pixels.  Glass scenes' chains (caustic
// paths behind the dielectric) set the time of their smaller launches, where the two-wave build
// stays faster (C3 1/2 and 1/4 shards, 8 and 4 rounds: 172-185 / 114 ms vs 202-206 / 131 ms lean;
// profiles/r06k_lean_rounds_ab.log), so they take it from 12 rounds on, other scenes from 3.
bool lean_fits(nart_ctx* ctx, const RenderArgs& a) {
    if (ctx->variant != 0 || !ctx->lean || !rq_fits(ctx)) return false;
    // glass scenes' small launches are bound by their costly pixels' chains, which the priority
    // lanes of the two-wave build shorten (C3 1/2, 1/4 shards: 183 / 115 ms two-wave vs 194 / 130
    // lean); scenes without glass or an environment light take the lean build from 1.5 rounds
    // (C2 1/8 shards, 2 rounds: mean 22.1 vs 23.9 ms, profiles/r06zg_c2_shard8.log)
    const double from = (ctx->features & FT_GLASS) ? 12.0 : (ctx->has_env ? 3.0 : 1.5);
    return launch_rounds(ctx, a.n_slots) >= env_num("NART_LEAN_ROUNDS", from);
}

int dispatch_megakernel(nart_ctx* ctx, const RenderArgs& a, hipStream_t st) {
    const uint32_t f = ctx->features;
    auto covers = [f](uint32_t m) { return (f & ~m) == 0u; };
    if (ctx->specialize && !ctx->counters && a.bounces <= ILIST_REG) {
        if (!ctx->has_env && covers(FM_DIFFUSE)) {
            if (lean_fits(ctx, a)) return launch_render<false, false, false, FM_DIFFUSE, 3, false>(ctx, a, st);
            return launch_render<false, false, false, FM_DIFFUSE>(ctx, a, st);
        }
        if (!ctx->has_env && covers(FM_GLASS)) {
            if (lean_fits(ctx, a)) return launch_render<false, false, false, FM_GLASS, 3, false>(ctx, a, st);
            // (small shards keep two waves per SIMD: the priority-lane build at three, 168 VGPRs with
            // 14 spilled, measured C3 1/8 shards worst 83-85 vs 79-81 ms, mean 79.5-79.8 vs 75.9-76.0;
            // profiles/r06l_three_wave_prio_ab.log)
            return launch_render<false, false, false, FM_GLASS>(ctx, a, st);
        }
        if (ctx->has_env && covers(FM_ENVTEX)) {
            if (lean_fits(ctx, a)) return launch_render<false, false, true, FM_ENVTEX, 3, false>(ctx, a, st);
            return launch_render<false, false, true, FM_ENVTEX>(ctx, a, st);
        }
    }
    return ctx->has_env ? launch_render_maxl<true>(ctx, a, st) : launch_render_maxl<false>(ctx, a, st);
}

// Volume integrator: k_render_volume_sm (lanes advance one tentative collision per iteration and
// start their next sample independently).  When the shard spans several rounds of resident
// waves, the costliest wave-sized pixel groups (cost probe: tentative collisions of 4 samples per
// pixel) are launched first.
int dispatch_volume(nart_ctx* ctx, const RenderArgs& a, hipStream_t st) {
    const dim3 block(256);
    const uint32_t blocks = (a.n_slots + 255) / 256;
    RenderArgs b = a;
    // small density grids (C5: 2x2x2) are read from LDS (1 % faster than L1-hitting global loads)
    const uint32_t nd = ctx->scene.medium.present ? ctx->scene.medium.rx * ctx->scene.medium.ry * ctx->scene.medium.rz : 0;
    b.lds_nodes = nd <= 4096u ? nd : 0u;
    const size_t dl = (size_t)b.lds_nodes * sizeof(float);
    // occupancy: launches of >= 8 rounds of resident waves use the 4-waves-per-SIMD build (C5 frame,
    // 10.5 rounds: 134 -> 122 ms); smaller ones keep the unconstrained build, whose lanes' serial
    // chains are shorter (C5 1/2, 1/4, 1/8 shards: 79 / 74 / 71 ms vs 83 / 80 / 76 with 4 waves;
    // profiles/r03h_vol_w4_ab.log)
    int cus = 0, per_cu = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_render_volume_sm<false, 1>, 256, dl));
    const uint32_t resident = (uint32_t)std::max(1, cus * std::max(per_cu, 1));
    const double w4_rounds = 8.0;
    const bool w4 = (double)blocks / (double)resident >= w4_rounds;
    uint32_t grid = blocks;
    if (queue_mode() == 2) {
        const uint32_t n = a.n_slots;
        if (blocks > resident && (double)n / (256.0 * resident) < 12.0 && a.spp > 4) {
            const uint32_t W = resident * 4;  // resident waves
            int rc = ensure_queue(ctx, n + 63u * W);
            if (rc) return rc;
            RenderArgs pb = b;
            pb.spp = 4;
            pb.cost = ctx->d_cost;
            hipLaunchKernelGGL((k_render_volume_sm<false, 1>), dim3(blocks), block, dl, st, ctx->scene, pb);
            rc = sort_groups_by_cost(ctx, n, ctx->d_queue, st);
            if (rc) return rc;
            b.queue = ctx->d_queue;
            ctx->sched |= NART_SCHED_VOL_QUEUE;
            // Sparse waves on shards of < NART_VOL_SPARSE_ROUNDS (default 2) rounds of resident
            // waves: the costliest groups (probe cost >= NART_VOL_SPARSE_F (4) x the median group's)
            // spread NART_VOL_SPARSE (16) pixels per wave, the other lanes idle.  A wave executes
            // the union of its lanes' divergent chains, and a frame's costliest volume pixels
            // cluster: C5's centre pixels take 30 ms alone at 1,024 spp, 69 ms as a wave of 64.
            // C5 1/8 shard 73.7 -> 65.3 ms; on larger shards (2+ rounds) the mostly idle sparse
            // waves hold slots the other groups need (1/2 shard 78 -> 127 ms), and 1-8 pixels per
            // wave measured worse (profiles/r04h_c5_sparse.log).  Only the order of work changes.
            const uint32_t S = (uint32_t)std::max(1.0, std::min(64.0, env_num("NART_VOL_SPARSE", 16.0)));
            const double f = env_num("NART_VOL_SPARSE_F", 4.0), max_rounds = env_num("NART_VOL_SPARSE_ROUNDS", 2.0);
            if (S < 64u && (64u % S) == 0u && (double)blocks / (double)resident < max_rounds) {
                const uint32_t ng = (n + 63) / 64;
                std::vector<uint32_t> keys(ng);
                HIPCHK(hipMemcpyAsync(keys.data(), ctx->d_keys[1], (size_t)ng * 4, hipMemcpyDeviceToHost, st));
                HIPCHK(hipStreamSynchronize(st));
                std::vector<uint32_t> costs;  // sorted descending (partial last group excluded)
                for (uint32_t g = 0; g < ng; ++g)
                    if (keys[g] != 0xFFFFFFFFu) costs.push_back(0xFFFFFFFEu - keys[g]);
                uint32_t H = 0;
                if (!costs.empty()) {
                    const double med = costs[costs.size() / 2];
                    while (H < costs.size() && (double)costs[H] >= f * med) ++H;
                }
                H = std::min<uint32_t>(H, 63u * W / (64u / S * 64u));  // queue room (ensure_queue)
                if (H) {
                    const uint32_t qlen = H * (64u / S) * 64u + (n - 64u * H);
                    hipLaunchKernelGGL(k_sparse_groups, dim3((qlen + 255) / 256), block, 0, st, ctx->d_vals[1], n, H, S,
                                       qlen, ctx->d_queue);
                    b.qlen = qlen;
                    grid = (qlen + 255) / 256;
                    ctx->sched |= NART_SCHED_VOL_SPARSE;
                }
            }
            HIPCHK(hipGetLastError());
        }
    }
    if (ctx->counters) hipLaunchKernelGGL((k_render_volume_sm<true, 1>), dim3(grid), block, dl, st, ctx->scene, b);
    else if (w4) hipLaunchKernelGGL((k_render_volume_sm<false, NART_VOL_WV>), dim3(grid), block, dl, st, ctx->scene, b);
    else hipLaunchKernelGGL((k_render_volume_sm<false, 1>), dim3(grid), block, dl, st, ctx->scene, b);
    HIPCHK(hipGetLastError());
    return NART_OK;
}

int dispatch_render(nart_ctx* ctx, const RenderArgs& a, int integrator, hipStream_t st) {
    if (integrator == NART_INTEGRATOR_VOLUME) return dispatch_volume(ctx, a, st);
    return dispatch_megakernel(ctx, a, st);
}

// Filter index of AddSample (render.cpp:43-49) as a function of d2 = distX^2 + distY^2:
// fi(d2) = min(63, uint8(RN(RN(sqrt(d2)) / fw) * 64)).  sqrt and / are correctly rounded and the
// scaling by 64 is exact, so below the uint8 wrap fi is a non-decreasing step function of d2 and
// fi(d2) >= k  <=>  d2 >= thr[k].  thr[0] = 0, thr[64] = inf; thr[k] is found by bisection over the
// float bit patterns with the same float operations.  A splat hit has |distX|, |distY| <= fw + 0.5,
// so the thresholds are exact for every hit when RN(sqrt(2) (fw + 0.5) / fw) * 64 stays below 256
// (fw > ~0.28); otherwise returns false and the splat keeps the direct computation.
static uint32_t filter_index_host(float d2, float fw) {
    volatile float dist = std::sqrt(d2);
    volatile float q = dist / fw;
    return std::min(63u, (uint32_t)(int32_t)(q * 64.f) & 0xFFu);
}

bool splat_thresholds(float fw, float thr[65]) {
    if (!(fw > 0.f)) return false;
    const float hmax = fw + 0.5f;
    const double worst = std::sqrt(2.0 * (double)hmax * hmax) / fw * 64.0;
    if (!(worst < 250.0)) return false;
    const float d2max = 2.f * hmax * hmax * 1.001f;
    uint32_t hi_bits;
    std::memcpy(&hi_bits, &d2max, 4);
    thr[0] = 0.f;
    thr[64] = __builtin_inff();
    for (uint32_t k = 1; k < 64; ++k) {
        uint32_t lo = 0, hi = hi_bits;  // f(lo) < k <= f(hi) unless no hit reaches index k
        if (filter_index_host(d2max, fw) < k) {
            thr[k] = __builtin_inff();
            continue;
        }
        while (hi - lo > 1) {
            const uint32_t mid = lo + (hi - lo) / 2;
            float m;
            std::memcpy(&m, &mid, 4);
            if (filter_index_host(m, fw) >= k) hi = mid;
            else lo = mid;
        }
        std::memcpy(&thr[k], &hi, 4);
        if (filter_index_host(0.f, fw) >= k) thr[k] = 0.f;
    }
    return true;
}

// Filter weight by d2 cell for the splat (k_splat_col4<.., true>): cell c covers the floats whose
// bits >> 16 equal b0 + c (128 cells per octave of d2).  Consecutive thresholds differ by at
// least a factor (64/63)^2 = 1.03 > 1 + 1/128, so a cell holds at most one threshold t: the
// filter index in the cell is base + (d2 >= t), base = fi(cell start).  Cell 0 lies wholly below
// thr[1] (index 0 for every smaller d2 too); the last cell starts past thr[63] (index 63 beyond).
// Stored per cell: {t (or inf), table[base], table[base + 1]}.  Returns false when the thresholds
// do not apply (then the splat keeps the sqrt estimate) or a cell would hold two of them.
bool splat_lut(const float thr[65], const float table[64], std::vector<float4>& lut, uint32_t& b0) {
    uint32_t u1, u63;
    std::memcpy(&u1, &thr[1], 4);
    std::memcpy(&u63, &thr[63], 4);
    if (!(thr[1] > 0.f) || !(thr[63] < __builtin_inff())) return false;
    b0 = (u1 >> 16) - 1;
    const uint32_t last = (u63 >> 16) + 1;
    const uint32_t n = last - b0 + 1;
    if (n > SPLAT_LUT_MAX) return false;
    lut.assign(n, make_float4(0.f, 0.f, 0.f, 0.f));
    for (uint32_t c = 0; c < n; ++c) {
        const uint32_t lo = (b0 + c) << 16, hi = lo | 0xFFFFu;
        float flo, fhi;
        std::memcpy(&flo, &lo, 4);
        std::memcpy(&fhi, &hi, 4);
        uint32_t base = 0, inside = 0;
        float t = __builtin_inff();
        for (uint32_t k = 1; k < 64; ++k) {
            if (thr[k] <= flo) base = k;
            else if (thr[k] <= fhi) {
                ++inside;
                t = thr[k];
            }
        }
        if (inside > 1) return false;
        lut[c] = make_float4(t, table[std::min(base, 63u)], table[std::min(base + inside, 63u)], 0.f);
    }
    return true;
}

// LatinSquare per traced pixel: float arrays in LDS up to 256 spp, LDS index shuffles up to 1024
// spp (scratch in Lout: 2*spp floats per lane of every launched block, within Lout's 4*spp per
// slot once there are >= 64 slots), the global-memory variant beyond.
int launch_latin(nart_ctx* ctx, const RenderArgs& ra, hipStream_t st) {
    // three-kernel form (k_latin_draws / _perm / _emit) when its scratch fits in Lout
    const uint32_t groups = (ra.n_slots + 63) / 64;
    LatinScratch ls;
    ls.n2 = (ra.spp + 1) / 2;
    // + padding rows per array: k_latin_perm / k_latin_emit load a batch of words ahead,
    // unconditionally
    const size_t words = (size_t)groups * 64 * ls.n2 + (size_t)std::max(NART_LATIN_PF, 2 * LATIN_EMIT_U * 16) * 64;
    const size_t stw = (size_t)((ra.n_slots + LATIN_EMIT_SLOTS - 1) / LATIN_EMIT_SLOTS) * LATIN_EMIT_SLOTS * ra.spp +
                       LATIN_ST_PAD;
    const bool three = ra.spp >= 2 && ra.spp <= 1024 && (4 * words + stw) * 4 <= ctx->cap_samples * sizeof(float4) &&
                       ra.spp > 64;  // C3 (256 spp): 6.7 -> 4.6 ms
    if (three) {
        uint32_t* base = reinterpret_cast<uint32_t*>(ra.Lout);
        ls.cx = base;
        ls.cy = base + words;
        ls.sx = base + 2 * words;
        ls.sy = base + 3 * words;
        ls.st = base + 4 * words;
        hipLaunchKernelGGL(k_latin_draws, dim3((ra.n_slots + 255) / 256), dim3(256), 0, st, ra, ls);
        if ((size_t)ls.n2 * 4 * 128 > 160 * 1024)  // one 64-lane block per CU: 80 lanes fill its LDS
            hipLaunchKernelGGL(k_latin_perm<80>, dim3((ra.n_slots + 79) / 80), dim3(80),
                               (size_t)ls.n2 * 2 * 80 * sizeof(uint16_t), st, ra, ls);
        else
            hipLaunchKernelGGL(k_latin_perm<64>, dim3(groups), dim3(64), (size_t)ls.n2 * 2 * 64 * sizeof(uint16_t),
                               st, ra, ls);
        hipLaunchKernelGGL(k_latin_emit, dim3((ra.n_slots + LATIN_EMIT_SLOTS - 1) / LATIN_EMIT_SLOTS), dim3(256),
                           (size_t)ra.spp * LATIN_EMIT_SLOTS * sizeof(uint32_t), st, ra, ls);
        HIPCHK(hipGetLastError());
        return NART_OK;
    }
    // (k_latin_idx at <= 256 spp measured slower: C3 11.0 vs 6.6 ms; the three-kernel form 4.6)
    if (ra.spp <= 256) {
        size_t lds = (size_t)ra.spp * 2 * 64 * sizeof(float);
        hipLaunchKernelGGL(k_latin_lds, dim3((ra.n_slots + 63) / 64), dim3(64), lds, st, ra);
    } else if (ra.spp <= 1024 && ra.n_slots >= 64) {
        size_t lds = (size_t)ra.spp * (ra.spp <= 512 ? 2 : 1) * 64 * sizeof(uint16_t);
        hipLaunchKernelGGL(k_latin_idx, dim3((ra.n_slots + 63) / 64), dim3(64), lds, st, ra, (float*)ra.Lout);
    } else {
        hipLaunchKernelGGL(k_latin, dim3((ra.n_slots + 255) / 256), dim3(256), 0, st, ra);
    }
    HIPCHK(hipGetLastError());
    return NART_OK;
}


// Render a bucket list into device tiles (list order).  Shared by all entry points.
int render_buckets(nart_ctx* ctx, const nart_render_params* p, const uint32_t* ids, uint32_t n, float* d_tiles,
                   hipStream_t st, nart_render_stats* stats) {
    int rc = check_params(ctx, p);
    if (rc) return rc;
    HIPCHK(hipSetDevice(ctx->device));
    nart_session_geometry g;
    nart_session_geometry_of(p, &g);
    const uint32_t nb_total = g.n_buckets_x * g.n_buckets_y;
    for (uint32_t i = 0; i < n; ++i)
        if (ids[i] >= nb_total) return fail(ctx, NART_E_INVALID, "bucket id out of range");
    // filter table [64] + filter-index thresholds [65] (splat_thresholds)
    float table[64 + 65];
    nart_filter_table(table);
    const bool thr_ok = splat_thresholds(p->filter_width, table + 64);
    if (!ctx->d_table) HIPCHK(hipMalloc(&ctx->d_table, sizeof(table)));
    HIPCHK(hipMemcpy(ctx->d_table, table, sizeof(table), hipMemcpyHostToDevice));
    std::vector<float4> lut;
    uint32_t lut_b0 = 0;
    const bool lut_ok = thr_ok && splat_lut(table + 64, table, lut, lut_b0);
    // skewed-time splat (k_splat_skew, pixel-major samples) where its preconditions hold, else
    // k_splat_col4 / k_splat over the sample-major layout
    // It runs one lane per tile column for ~W*B steps, so its time is one wave's latency once the
    // launch has fewer than ~2 waves per SIMD: small shards keep k_splat_col4 (C5 1/8 shard:
    // 54 ms skewed vs 23 ms col4; whole frame 72 vs 113 ms).  skew_min: waves per SIMD.
    const uint32_t B = p->bucket_size, tile = B + 2 * g.filter_bounds;
    const double skew_min = 2.0;
    int n_cus = 0;
    HIPCHK(hipDeviceGetAttribute(&n_cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    const double skew_waves = tile <= 64 ? (double)((n + 64 / tile - 1) / (64 / tile)) : 0.0;
    // splat mode -1 (default): 4 where the launch is large enough, else 3; an explicit 4 forces it.
    // Launches of 1-2 waves per SIMD split each bucket's tile rows into two bands (twice the waves
    // for ~2/3 of the steps each): C5 1/2 shard 60 -> 49 ms (k_splat_col4: 62); a whole frame keeps
    // one band (C5 73 vs 92 ms with two).  Below 1 wave per SIMD k_splat_col4 is faster (C5 1/4,
    // 1/8 shards: 36 / 23 ms vs 41 / 37 with two bands; profiles/r03k_skew_band_ab.log).
    // The two-band range is the volume integrator's only: for the path integrator the splat's
    // gain at the C3 1/2 shard (17 -> 12.5 ms) is within the path kernels' run-to-run spread under
    // the pixel-major layout (186-208 ms on one box; profiles/r03l_c3_half_shard_splat_ab.log).
    const double skew_from = p->integrator == NART_INTEGRATOR_VOLUME ? 0.5 * skew_min : skew_min;
    // Below that, k_splat_rows (mode 5: W lanes per tile column, five times k_splat_skew's
    // parallelism, each sample still fetched once per bucket) unless NART_SPLAT_SMALL=col4
    const char* ss = env_opt("NART_SPLAT_SMALL");
    const int small_mode = ss && std::strcmp(ss, "col4") == 0 ? 3 : 5;
    const int splat_mode =
        ctx->splat_mode >= 0 ? ctx->splat_mode : (skew_waves >= skew_from * 4.0 * n_cus ? 4 : small_mode);
    // NART_SKEW_BANDS (read per call): 1 or 2 forces the band count
    const char* be = env_opt("NART_SKEW_BANDS");
    const uint32_t skew_bands = be && std::atoi(be) > 0 ? (std::atoi(be) >= 2 ? 2u : 1u)
                                                          : (skew_waves >= skew_min * 4.0 * n_cus ? 1u : 2u);
    // skew: a pixel-major sample layout for k_splat_skew (mode 4) or k_splat_rows (mode 5)
    const bool skew = splat_mode >= 4 && lut_ok && (B & (B - 1)) == 0 && B <= 32 && tile <= 64 &&
                      g.filter_bounds >= 1 && g.filter_bounds <= 3;
    const bool rows = skew && splat_mode == 5;
    if (lut_ok) {
        if (!ctx->d_lut) HIPCHK(hipMalloc(&ctx->d_lut, SPLAT_LUT_MAX * sizeof(float4)));
        HIPCHK(hipMemcpy(ctx->d_lut, lut.data(), lut.size() * sizeof(float4), hipMemcpyHostToDevice));
    }
    const size_t n_cnt = 24;
    if (!ctx->d_counters) HIPCHK(hipMalloc(&ctx->d_counters, n_cnt * sizeof(unsigned long long)));
    if (ctx->counters) HIPCHK(hipMemsetAsync(ctx->d_counters, 0, n_cnt * sizeof(unsigned long long), st));
    if (!ctx->events) {
        for (auto& e : ctx->ev) HIPCHK(hipEventCreate(&e));
        ctx->events = true;
    }
    const size_t limit = batch_slot_limit(ctx, p->spp);
    const uint32_t tpx = g.tile_size * g.tile_size;
    double kernel_ms = 0.0, splat_ms = 0.0, latin_ms = 0.0, primary_ms = 0.0;
    uint32_t launches = 0;
    uint64_t traced = 0, counted = 0;
    uint32_t b0 = 0;
    ctx->sched = 0;
    std::vector<uint32_t> xy, base;
    while (b0 < n) {
        // gather a batch of buckets whose traced pixels fit the slot budget
        xy.clear();
        base.clear();
        uint32_t b1 = b0;
        while (b1 < n) {
            uint32_t id = ids[b1];
            uint32_t bx = id % g.n_buckets_x, by = id / g.n_buckets_x;
            uint32_t x0 = p->bucket_size * bx, y0 = p->bucket_size * by;
            uint32_t x1 = std::min(p->bucket_size * (bx + 1), g.total_width);   // render.cpp:163-168
            uint32_t y1 = std::min(p->bucket_size * (by + 1), g.total_height);
            size_t cnt = (size_t)(x1 - x0) * (y1 - y0);
            if (b1 > b0 && xy.size() + cnt > limit) break;
            base.push_back((uint32_t)xy.size());
            for (uint32_t y = y0; y < y1; ++y)
                for (uint32_t x = x0; x < x1; ++x) {
                    xy.push_back(x | (y << 16));
                    if (x < p->image_width && y < p->image_height) ++counted;
                }
            ++b1;
        }
        const uint32_t nslots = (uint32_t)xy.size(), nbk = b1 - b0;
        traced += (uint64_t)nslots * p->spp;
        rc = ensure(ctx, nslots, p->spp, nbk);
        if (rc) return rc;
        HIPCHK(hipMemcpyAsync(ctx->d_slot_xy, xy.data(), (size_t)nslots * 4, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(ctx->d_bucket_ids, ids + b0, (size_t)nbk * 4, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(ctx->d_bucket_base, base.data(), (size_t)nbk * 4, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_slot_table, dim3(nbk), dim3(256), 0, st, ctx->d_bucket_base, nbk, nslots, p->spp,
                           ctx->d_slot_so, skew);
        RenderArgs ra;
        ra.slot_xy = ctx->d_slot_xy;
        ra.slot_so = ctx->d_slot_so;
        ra.samples = ctx->d_samples;
        ra.rng0 = ctx->d_rng;
        ra.Lout = ctx->d_L;
        ra.n_slots = nslots;
        ra.spp = p->spp;
        ra.bounces = p->bounces;
        ra.W = p->image_width;
        ra.H = p->image_height;
        ra.totalW = g.total_width;
        ra.stack_depth = ctx->stack_depth;
        ra.lds_nodes = 0;
        ra.gamma = p->roughening_factor * p->roughening_factor;
        ra.counters = ctx->d_counters;
        HIPCHK(hipEventRecord(ctx->ev[3], st));
        rc = launch_latin(ctx, ra, st);
        if (rc) return rc;
        HIPCHK(hipEventRecord(ctx->ev[0], st));
        ctx->primary_ran = false;
        rc = dispatch_render(ctx, ra, p->integrator, st);
        if (rc) return rc;
        HIPCHK(hipEventRecord(ctx->ev[1], st));
        SplatArgs sa;
        sa.bucket_ids = ctx->d_bucket_ids;
        sa.bucket_base = ctx->d_bucket_base;
        sa.samples = ctx->d_samples;
        sa.Lout = ctx->d_L;
        sa.tiles = d_tiles + (size_t)b0 * tpx * 5;
        sa.table = ctx->d_table;
        sa.thr = thr_ok ? ctx->d_table + 64 : nullptr;
        sa.idx_scale = 64.f / p->filter_width;
        sa.n_buckets = nbk;
        sa.spp = p->spp;
        sa.B = p->bucket_size;
        sa.fb = g.filter_bounds;
        sa.tile = g.tile_size;
        sa.nbx = g.n_buckets_x;
        sa.totalW = g.total_width;
        sa.totalH = g.total_height;
        sa.fw = p->filter_width;
        sa.invB = (p->bucket_size & (p->bucket_size - 1)) == 0 ? 1.f / (float)p->bucket_size : 0.f;
        sa.lut = lut_ok ? static_cast<const float4*>(ctx->d_lut) : nullptr;
        sa.lut_b0 = lut_b0;
        sa.lut_n = (uint32_t)lut.size();
        {
            int ex = 0;
            float m = std::frexp(p->filter_width, &ex);
            sa.invFw = (m == 0.5f) ? 1.f / p->filter_width : 0.f;
        }
        uint64_t nthreads = (uint64_t)nbk * tpx;
        const dim3 sg((uint32_t)((nthreads + 255) / 256));
#ifndef NART_SPLAT_NP
#define NART_SPLAT_NP 4
#endif
        const uint64_t n4 = (uint64_t)nbk * g.tile_size * ((g.tile_size + NART_SPLAT_NP - 1) / NART_SPLAT_NP);
        // splat modes (all bit-identical): 4 skewed time, 3 four tile pixels per lane (power-of-two
        // buckets); 1 / 0 one tile pixel per lane with the threshold / direct filter-index arithmetic
        // (any bucket size; 2 selects 1 since the compare-only one-pixel kernel was retired)
        if (rows) {
            ctx->sched |= NART_SCHED_SPLAT_ROWS;
            const uint32_t U = g.tile_size * (2 * g.filter_bounds + 1), ub = std::max(1u, 512u / U);
            const uint32_t threads = (ub * U + 63) / 64 * 64, nblk = (nbk + ub - 1) / ub;
            const size_t lds = lut.size() * sizeof(float4) + 2u * ub * sizeof(uint32_t);
            if (g.filter_bounds == 1) hipLaunchKernelGGL((k_splat_rows<1>), dim3(nblk), dim3(threads), lds, st, sa);
            else if (g.filter_bounds == 2) hipLaunchKernelGGL((k_splat_rows<2>), dim3(nblk), dim3(threads), lds, st, sa);
            else hipLaunchKernelGGL((k_splat_rows<3>), dim3(nblk), dim3(threads), lds, st, sa);
        } else if (skew) {
            ctx->sched |= NART_SCHED_SPLAT_SKEW;
            const uint32_t nb = skew_bands;  // tile-row bands per bucket (k_splat_skew's NB)
            const uint32_t pb = 64u / g.tile_size, nblk = (nbk * nb + 4 * pb - 1) / (4 * pb);
            const size_t lds = lut.size() * sizeof(float4) + 8u * pb * sizeof(uint32_t);
            const int fbk = (int)g.filter_bounds * 2 + (int)nb - 1;
            if (fbk == 2) hipLaunchKernelGGL((k_splat_skew<1, 1>), dim3(nblk), dim3(256), lds, st, sa);
            else if (fbk == 3) hipLaunchKernelGGL((k_splat_skew<1, 2>), dim3(nblk), dim3(256), lds, st, sa);
            else if (fbk == 4) hipLaunchKernelGGL((k_splat_skew<2, 1>), dim3(nblk), dim3(256), lds, st, sa);
            else if (fbk == 5) hipLaunchKernelGGL((k_splat_skew<2, 2>), dim3(nblk), dim3(256), lds, st, sa);
            else if (fbk == 6) hipLaunchKernelGGL((k_splat_skew<3, 1>), dim3(nblk), dim3(256), lds, st, sa);
            else hipLaunchKernelGGL((k_splat_skew<3, 2>), dim3(nblk), dim3(256), lds, st, sa);
        } else if (sa.thr && sa.invB != 0.f && splat_mode >= 3)
        {
            if (sa.lut)
                hipLaunchKernelGGL((k_splat_col4<NART_SPLAT_NP, true>), dim3((uint32_t)((n4 + 255) / 256)), dim3(256), 0,
                                   st, sa);
            else
                hipLaunchKernelGGL((k_splat_col4<NART_SPLAT_NP, false>), dim3((uint32_t)((n4 + 255) / 256)), dim3(256),
                                   0, st, sa);
        }
        else if (sa.thr && splat_mode >= 1) hipLaunchKernelGGL(k_splat<1>, sg, dim3(256), 0, st, sa);
        else hipLaunchKernelGGL(k_splat<0>, sg, dim3(256), 0, st, sa);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ctx->ev[2], st));
        HIPCHK(hipEventSynchronize(ctx->ev[2]));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]));
        kernel_ms += ms;
        if (ctx->primary_ran) {
            HIPCHK(hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[4]));
            primary_ms += ms;
        }
        HIPCHK(hipEventElapsedTime(&ms, ctx->ev[1], ctx->ev[2]));
        splat_ms += ms;
        HIPCHK(hipEventElapsedTime(&ms, ctx->ev[3], ctx->ev[0]));
        latin_ms += ms;
        ++launches;
        b0 = b1;
    }
    if (stats) {
        stats->kernel_ms += kernel_ms;
        stats->splat_ms += splat_ms;
        stats->latin_ms += latin_ms;
        stats->primary_ms += primary_ms;
        stats->kernel_launches += launches;
        stats->schedule |= ctx->sched;
        stats->traced_samples += traced;
        stats->samples += counted * p->spp;
        if (ctx->counters) {
            unsigned long long c[8];
            HIPCHK(hipMemcpy(c, ctx->d_counters, sizeof(c), hipMemcpyDeviceToHost));
            stats->rays_extend += c[0];
            stats->rays_shadow += c[1];
            stats->node_visits += c[2];
            stats->tri_tests += c[3];
            stats->bounces += c[4];
            stats->octree_checks += c[5];
            stats->octree_replays += c[6];
        }
    }
    return NART_OK;
}

// ---------------------------------------------------------------- device-side BVH build
struct LbvhResult {
    uint32_t max_stack = 1, num_nodes = 0, num_leaf_tris = 0;
    int32_t root_code = -1;
};

// Linear BVH on the device (device/lbvh.h) over the triangles the reference octree can return
// (mask), into ctx->d_nodes / d_tri_isect / d_tri_perm.  ctx->d_tris must be resident.
int build_bvh_device(nart_ctx* ctx, const nart_scene_blob& blob, const std::vector<uint8_t>& mask,
                     const nart::RefOctree& oct, float pad, float margin, LbvhResult& out) {
    std::vector<uint32_t> vis, info;
    for (uint32_t g = 0; g < blob.num_triangles; ++g)
        if (mask[g]) vis.push_back(g);
    nart::octree_leaf_info(blob, oct, margin, info);
    const uint32_t m = (uint32_t)vis.size();
    out.num_leaf_tris = m;
    if (m == 0) {  // nothing the octree can return: never traversed (geometry_visible = 0)
        BVHNode dummy{};
        int rc = upload(ctx, ctx->d_nodes, &dummy, 0);
        if (!rc) rc = upload(ctx, ctx->d_tri_isect, (const float*)nullptr, 0);
        if (!rc) rc = upload(ctx, ctx->d_tri_perm, (const float*)nullptr, 0);
        return rc;
    }
    const int n = (int)((m + LBVH_LEAF - 1) / LBVH_LEAF);  // leaves
    const int ninner = n - 1;
    std::vector<void*> tmp;
    auto alloc = [&](void** p, size_t bytes) {
        const int rc = dmalloc(ctx, p, bytes ? bytes : 4, "BVH build scratch");
        if (!rc) tmp.push_back(*p);
        return rc;
    };
    auto cleanup = [&](int rc) {
        for (void* p : tmp) hipFree(p);
        return rc;
    };
    uint32_t *d_vis, *d_info, *d_keys[2], *d_vals[2], *d_lkey, *d_flag, *d_maxd, *d_ord[2];
    LbvhPrim *d_prims, *d_sorted;
    float* d_part;
    int2* d_child;
    int *d_pin, *d_pleaf, *d_remap;
    LbvhBox* d_box;
    const uint32_t nb = std::min<uint32_t>(1024, (m + 255) / 256);
    const size_t ni = (size_t)std::max(ninner, 1);
    int rc = NART_OK;
    if ((rc = alloc((void**)&d_vis, m * 4)) || (rc = alloc((void**)&d_info, blob.num_triangles * 4)) ||
        (rc = alloc((void**)&d_prims, m * sizeof(LbvhPrim))) || (rc = alloc((void**)&d_sorted, m * sizeof(LbvhPrim))) ||
        (rc = alloc((void**)&d_part, nb * 6 * 4)) || (rc = alloc((void**)&d_keys[0], m * 4)) ||
        (rc = alloc((void**)&d_keys[1], m * 4)) || (rc = alloc((void**)&d_vals[0], m * 4)) ||
        (rc = alloc((void**)&d_vals[1], m * 4)) || (rc = alloc((void**)&d_lkey, n * 4)) ||
        (rc = alloc((void**)&d_child, ni * sizeof(int2))) || (rc = alloc((void**)&d_pin, ni * 4)) ||
        (rc = alloc((void**)&d_pleaf, (size_t)n * 4)) || (rc = alloc((void**)&d_box, ni * sizeof(LbvhBox))) ||
        (rc = alloc((void**)&d_flag, ni * 4)) || (rc = alloc((void**)&d_maxd, 4)) ||
        (rc = alloc((void**)&d_ord[0], ni * 4)) || (rc = alloc((void**)&d_ord[1], ni * 4)) ||
        (rc = alloc((void**)&d_remap, ni * 4)))
        return cleanup(rc);
    if (hipMemcpy(d_vis, vis.data(), m * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_info, info.data(), blob.num_triangles * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(d_pin, 0xFF, ni * 4) != hipSuccess || hipMemset(d_pleaf, 0xFF, (size_t)n * 4) != hipSuccess ||
        hipMemset(d_flag, 0, ni * 4) != hipSuccess || hipMemset(d_maxd, 0, 4) != hipSuccess)
        return cleanup(fail(ctx, NART_E_HIP, "BVH build: upload"));
    const dim3 blk(256);
    const uint32_t gm = (m + 255) / 256, gn = ((uint32_t)n + 255) / 256, gi = ((uint32_t)ni + 255) / 256;
    hipLaunchKernelGGL(k_lbvh_prims, dim3(gm), blk, 0, 0, (const nart_triangle*)ctx->d_tris, d_vis, m, d_prims);
    hipLaunchKernelGGL(k_lbvh_bounds, dim3(nb), blk, 0, 0, d_prims, m, d_part);
    hipLaunchKernelGGL(k_lbvh_bounds_final, dim3(1), dim3(64), 0, 0, d_part, nb);
    hipLaunchKernelGGL(k_lbvh_morton, dim3(gm), blk, 0, 0, d_prims, m, d_part, d_keys[0], d_vals[0]);
    size_t ts = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, ts, d_keys[0], d_keys[1], d_vals[0], d_vals[1], (int)m, 0, 30) !=
        hipSuccess)
        return cleanup(fail(ctx, NART_E_HIP, "BVH build: sort size"));
    void* d_ts = nullptr;
    if ((rc = alloc(&d_ts, ts))) return cleanup(rc);
    if (hipcub::DeviceRadixSort::SortPairs(d_ts, ts, d_keys[0], d_keys[1], d_vals[0], d_vals[1], (int)m, 0, 30) !=
        hipSuccess)
        return cleanup(fail(ctx, NART_E_HIP, "BVH build: sort"));
    hipLaunchKernelGGL(k_lbvh_gather, dim3(gm), blk, 0, 0, d_prims, d_vals[1], m, d_sorted);
    hipLaunchKernelGGL(k_lbvh_leaf_keys, dim3(gn), blk, 0, 0, d_keys[1], m, n, d_lkey);
    if (ninner > 0) {
        hipLaunchKernelGGL(k_lbvh_karras, dim3(gi), blk, 0, 0, d_lkey, n, d_child, d_pin, d_pleaf);
        hipLaunchKernelGGL(k_lbvh_refit, dim3(gn), blk, 0, 0, d_sorted, m, n, d_child, d_pin, d_pleaf, d_box, d_flag);
        hipLaunchKernelGGL(k_lbvh_depth, dim3(gi), blk, 0, 0, d_pin, ninner, d_keys[0], d_vals[0], d_maxd);
        size_t ts2 = 0;
        if (hipcub::DeviceRadixSort::SortPairs(nullptr, ts2, d_keys[0], d_keys[1], d_vals[0], d_ord[0], ninner, 0, 8) !=
            hipSuccess)
            return cleanup(fail(ctx, NART_E_HIP, "BVH build: sort size"));
        void* d_ts2 = nullptr;
        if ((rc = alloc(&d_ts2, ts2))) return cleanup(rc);
        if (hipcub::DeviceRadixSort::SortPairs(d_ts2, ts2, d_keys[0], d_keys[1], d_vals[0], d_ord[0], ninner, 0, 8) !=
            hipSuccess)
            return cleanup(fail(ctx, NART_E_HIP, "BVH build: sort"));
        hipLaunchKernelGGL(k_lbvh_remap, dim3(gi), blk, 0, 0, d_ord[0], ninner, d_remap);
    }
    if ((rc = dmalloc(ctx, &ctx->d_nodes, ni * sizeof(BVHNode), "BVH nodes")) ||
        (rc = dmalloc(ctx, &ctx->d_tri_isect, (size_t)m * 64, "triangle records")) ||
        (rc = dmalloc(ctx, &ctx->d_tri_perm, ((size_t)m * 3 + NART_TRI_PAD) * 64, "permuted triangle records")))
        return cleanup(rc);
    if (ninner > 0)
        hipLaunchKernelGGL(k_lbvh_emit, dim3(gi), blk, 0, 0, d_ord[0], ninner, d_child, d_remap, d_box, d_sorted, m, pad,
                           (BVHNode*)ctx->d_nodes);
    hipLaunchKernelGGL(k_lbvh_tris, dim3(gm), blk, 0, 0, (const nart_triangle*)ctx->d_tris, d_sorted, m, d_info,
                       (float*)ctx->d_tri_isect);
    hipLaunchKernelGGL(k_lbvh_perm, dim3(gm), blk, 0, 0, (const float*)ctx->d_tri_isect, m, (float*)ctx->d_tri_perm);
    uint32_t maxd = 0;
    if (hipGetLastError() != hipSuccess || hipMemcpy(&maxd, d_maxd, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return cleanup(fail(ctx, NART_E_HIP, "BVH build: kernels"));
    out.num_nodes = (uint32_t)std::max(ninner, 0);
    out.max_stack = ninner > 0 ? maxd + 1 : 1;
    out.root_code = ninner > 0 ? 0 : ~(int32_t)(m - 1);  // one leaf of m <= LBVH_LEAF triangles
    return cleanup(NART_OK);
}

}  // namespace

#include "host/multi_gpu.h"

extern "C" {

int nart_hip_create(const nart_scene_blob* blob, int device_id, nart_ctx** out) {
    if (!blob || !out) return NART_E_INVALID;
    nart_ctx* ctx = new (std::nothrow) nart_ctx();
    if (!ctx) return NART_E_OOM;
    *out = nullptr;
    ctx->device = device_id;
    if (const char* v = env_opt("NART_VARIANT")) {
        const int var = std::atoi(v);
        if (var == 0 || var == 3) ctx->variant = var;
    }
    if (const char* v = env_opt("NART_SPLAT_MODE")) ctx->splat_mode = std::max(-1, std::min(5, std::atoi(v)));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device_id || device_id < 0) {
        delete ctx;
        return NART_E_HIP;
    }
    int rc = NART_OK;
    auto bail = [&](int code) {
        nart_hip_destroy(ctx);
        return code;
    };
    if (hipSetDevice(device_id) != hipSuccess) return bail(NART_E_HIP);
    // dynamic LDS above the 64 KiB default: LatinSquare arrays (128 KiB at 256 spp)
    if (hipFuncSetAttribute((const void*)k_latin_lds, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
        hipSuccess)
        return bail(NART_E_HIP);
    if (hipFuncSetAttribute((const void*)k_latin_idx, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
        hipSuccess)
        return bail(NART_E_HIP);
    if (hipFuncSetAttribute((const void*)k_latin_perm<64>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
            hipSuccess ||
        hipFuncSetAttribute((const void*)k_latin_perm<80>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
            hipSuccess ||
        hipFuncSetAttribute((const void*)k_latin_emit, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
            hipSuccess)
        return bail(NART_E_HIP);
    // reference octree visibility (Q14) + device BVH
    std::vector<uint8_t> mask;
    bool root_leaf = false;
    uint32_t n_chunks = 0;
    nart::RefOctree oct;
    nart::reference_visibility(*blob, mask, root_leaf, n_chunks, &oct);
    float maxabs = 1.f;
    for (uint32_t g = 0; g < blob->num_triangles; ++g) {
        const nart_triangle& T = blob->triangles[g];
        for (int k = 0; k < 3; ++k)
            maxabs = std::max(maxabs, std::max(std::fabs(T.v0[k]), std::max(std::fabs(T.v1[k]), std::fabs(T.v2[k]))));
    }
    for (int k = 12; k < 15; ++k) maxabs = std::max(maxabs, std::fabs(blob->camera.m[k]));
    for (int k = 3; k < 16; k += 4) maxabs = std::max(maxabs, std::fabs(blob->camera.m[k]));
    // hit points deviate from the reference's slab arithmetic by far less than 2^-14 * scene
    // scale (|o| + |t d| <= 3 * maxabs, errors of a few ulps): octree.h oc_clear
    const float pad = maxabs * 6.103515625e-05f + 1e-6f, margin = maxabs * 6.103515625e-05f;
    if ((rc = upload(ctx, ctx->d_tris, blob->triangles, blob->num_triangles))) return bail(rc);
    // NART_BVH_BUILD=device: linear BVH built on the GPU (device/lbvh.h); default: binned SAH on
    // the host (host/bvh_build.cpp) -- same node / record format, same images
    const char* bb = env_opt("NART_BVH_BUILD");
    ctx->bvh_on_device = bb && std::string(bb) == "device";
    const auto tb0 = std::chrono::steady_clock::now();
    LbvhResult lb;
    if (ctx->bvh_on_device) {
        if ((rc = build_bvh_device(ctx, *blob, mask, oct, pad, margin, lb))) return bail(rc);
    } else {
        nart::BuiltBVH bvh;
        nart::build_bvh(*blob, mask, pad, bvh);
        nart::annotate_octree_leaves(*blob, oct, margin, bvh);
        lb.max_stack = bvh.max_stack;
        lb.num_nodes = (uint32_t)bvh.nodes.size();
        lb.root_code = bvh.root_code;
        lb.num_leaf_tris = (uint32_t)(bvh.tri_isect.size() / 16);
        if ((rc = upload(ctx, ctx->d_nodes, bvh.nodes.data(), bvh.nodes.size()))) return bail(rc);
        if ((rc = upload(ctx, ctx->d_tri_isect, bvh.tri_isect.data(), bvh.tri_isect.size()))) return bail(rc);
        // vertex block of every triangle test record, permuted for each ray major axis, followed
        // by the plane {n, dot(v0, n)}: one 64-B record, so a test issues its four loads at once
        const size_t nt = bvh.tri_isect.size() / 16;
        std::vector<float> perm((3 * nt + NART_TRI_PAD) * 16);  // + padding records (trav_step's record groups)
        for (int m = 0; m < 3; ++m) {
            const int kx = (m + 1) % 3, ky = (m + 2) % 3, kz = m;
            for (size_t i = 0; i < nt; ++i) {
                const float* r = &bvh.tri_isect[i * 16];
                const float* v[3] = {r + 4, r + 7, r + 10};  // v0, v1, v2 (words 4-12)
                float* o = &perm[((size_t)m * nt + i) * 16];
                for (int k = 0; k < 3; ++k) {
                    o[3 * k + 0] = v[k][kx];
                    o[3 * k + 1] = v[k][ky];
                    o[3 * k + 2] = v[k][kz];
                }
                o[9] = r[13];   // global index
                o[10] = r[14];  // octree leaf | inside bit
                o[11] = r[15];  // grazing threshold
                for (int k = 0; k < 4; ++k) o[12 + k] = r[k];  // plane (words 0-3)
            }
        }
        if ((rc = upload(ctx, ctx->d_tri_perm, perm.data(), perm.size()))) return bail(rc);
    }
    ctx->bvh_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb0).count();
    ctx->stack_depth = std::max<uint32_t>(lb.max_stack + 1, 2);
    if ((size_t)ctx->stack_depth * 256 * 8 > (size_t)160 * 1024) return bail(NART_E_UNSUPPORTED);  // LDS stack
    ctx->num_nodes = lb.num_nodes;
    ctx->num_leaf_tris = lb.num_leaf_tris;
    std::vector<uint32_t> tri_mesh(blob->num_triangles);
    std::vector<DMesh> meshes(blob->num_meshes);
    for (uint32_t m = 0; m < blob->num_meshes; ++m) {
        meshes[m].material = blob->meshes[m].material;
        meshes[m].priority = blob->meshes[m].priority & 0xFFu;
        for (uint32_t i = 0; i < blob->meshes[m].num_tris; ++i) tri_mesh[blob->meshes[m].first_tri + i] = m;
    }
    if (blob->num_meshes >= (1u << 24)) return bail(NART_E_UNSUPPORTED);
    if ((rc = upload(ctx, ctx->d_tri_mesh, tri_mesh.data(), tri_mesh.size()))) return bail(rc);
    if ((rc = upload(ctx, ctx->d_meshes, meshes.data(), meshes.size()))) return bail(rc);
    std::vector<DMaterial> mats(blob->num_materials);
    for (uint32_t i = 0; i < blob->num_materials; ++i) {
        const nart_material& m = blob->materials[i];
        DMaterial& d = mats[i];
        d.type = m.type;
        d.has_normal = (m.type == NART_MAT_GLASS) ? 0 : m.has_normal;  // glassmaterial.cpp:3-9
        d.rho_d = dpat(m.rho_d);
        d.rho_s = dpat(m.rho_s);
        d.tau = dpat(m.tau);
        d.eta = dpat(m.eta);
        d.alpha = dpat(m.alpha);
        d.normal = dpat(m.normal);
    }
    if ((rc = upload(ctx, ctx->d_mats, mats.data(), mats.size()))) return bail(rc);
    // per mesh: bxdf_eta of its one-lobe constant-pattern BSDF (the compact dielectric list,
    // kernels.h IList): B_LAMBERT -> 0, every other one-lobe kind -> the material's eta value
    std::vector<float> mesh_eta(blob->num_meshes);
    for (uint32_t m = 0; m < blob->num_meshes; ++m) {
        const uint32_t mi = blob->meshes[m].material;
        mesh_eta[m] = (mi >= mats.size() || mats[mi].type == NART_MAT_LAMBERT) ? 0.f : mats[mi].eta.v[0];
    }
    if ((rc = upload(ctx, ctx->d_mesh_eta, mesh_eta.data(), mesh_eta.size()))) return bail(rc);
    std::vector<DLight> lights;
    std::vector<DEnvDist> envs;
    for (uint32_t l = 0; l < blob->num_lights; ++l) {
        lights.push_back(dlight(blob->lights[l]));
        const nart_light& L = blob->lights[l];
        if (L.type == NART_LIGHT_ENVIRONMENT) ctx->has_env = true;
        if (L.type == NART_LIGHT_ENVIRONMENT && L.Le.type == NART_PTN_TEXTURE) {
            DEnvDist d;
            if ((rc = build_env(ctx, blob->textures[L.Le.texture], d))) return bail(rc);
            lights.back().env = (int32_t)envs.size();
            envs.push_back(d);
        }
    }
    if ((rc = upload(ctx, ctx->d_envs, envs.data(), envs.size()))) return bail(rc);
    if ((rc = upload(ctx, ctx->d_lights, lights.data(), lights.size()))) return bail(rc);
    ctx->features = scene_features(blob);
    std::vector<DTexture> texs(blob->num_textures);
    size_t pool = 0;
    for (uint32_t t = 0; t < blob->num_textures; ++t) {
        texs[t].w = blob->textures[t].width;
        texs[t].h = blob->textures[t].height;
        texs[t].offset = pool;
        pool += (size_t)texs[t].w * texs[t].h * 4;
    }
    std::vector<uint16_t> tex_pool(pool ? pool : 1);
    for (uint32_t t = 0; t < blob->num_textures; ++t)
        std::memcpy(&tex_pool[texs[t].offset], blob->textures[t].rgba, (size_t)texs[t].w * texs[t].h * 8);
    if ((rc = upload(ctx, ctx->d_texs, texs.data(), texs.size()))) return bail(rc);
    if ((rc = upload(ctx, ctx->d_tex_pool, tex_pool.data(), tex_pool.size()))) return bail(rc);

    DScene& S = ctx->scene;
    std::memset(&S, 0, sizeof(S));
    S.nodes = (const BVHNode*)ctx->d_nodes;
    S.tri_isect = (const float4*)ctx->d_tri_isect;
    S.tri_perm = (const float4*)ctx->d_tri_perm;
    S.tris = (const nart_triangle*)ctx->d_tris;
    S.tri_mesh = (const uint32_t*)ctx->d_tri_mesh;
    S.meshes = (const DMesh*)ctx->d_meshes;
    S.mats = (const DMaterial*)ctx->d_mats;
    S.mesh_eta = (const float*)ctx->d_mesh_eta;
    S.lights = (const DLight*)ctx->d_lights;
    S.texs = (const DTexture*)ctx->d_texs;
    S.tex_pool = (const uint16_t*)ctx->d_tex_pool;
    S.envs = (const DEnvDist*)ctx->d_envs;
    if ((rc = build_medium(ctx, blob->medium, S.medium))) return bail(rc);
    S.num_lights = blob->num_lights;
    S.num_tris = blob->num_triangles;
    S.num_leaf_tris = lb.num_leaf_tris;
    S.root = lb.root_code;
    S.geometry_visible = (!root_leaf && lb.num_leaf_tris > 0) ? 1 : 0;
    std::memcpy(S.cam_m, blob->camera.m, sizeof(S.cam_m));
    // glm::tan(glm::radians(fov)) with the host libm, as the reference (pinholecamera.cpp:20)
    S.cam_tan = std::tan(blob->camera.fov * (float)0.01745329251994329576923690768489);
    // reference octree + replay heap pool: entries of 64 heaps (one per lane of a replaying
    // wave, octree.h oc_replay), held only while a wave replays; up to 512 entries within 256 MiB
    // (NART_OC_POOL overrides the count: tests force a single entry)
    if ((rc = upload(ctx, ctx->d_oc_nodes, oct.nodes.data(), oct.nodes.size()))) return bail(rc);
    if ((rc = upload(ctx, ctx->d_oc_chunks, oct.chunks.data(), oct.chunks.size()))) return bail(rc);
    if ((rc = upload(ctx, ctx->d_oc_tris, oct.tris.data(), oct.tris.size()))) return bail(rc);
    if ((rc = upload(ctx, ctx->d_tri_leaf, oct.tri_leaf.data(), oct.tri_leaf.size()))) return bail(rc);
    S.oc_nodes = (const OcNode*)ctx->d_oc_nodes;
    S.oc_chunks = (const uint32_t*)ctx->d_oc_chunks;
    S.oc_tris = (const uint32_t*)ctx->d_oc_tris;
    S.tri_leaf = (const int32_t*)ctx->d_tri_leaf;
    S.oc_root = oct.root;
    S.oc_cap = (uint32_t)std::max<size_t>(oct.nodes.size(), 1);
    S.oc_pool = (uint32_t)std::max<size_t>(1, std::min<size_t>(512, (256ull << 20) / (64ull * 8ull * S.oc_cap)));
    if (const char* v = env_opt("NART_OC_POOL")) S.oc_pool = (uint32_t)std::max(1, std::atoi(v));
    S.oc_scale = maxabs;
    S.oc_exact = 1;
    // NART_OCTREE_EXACT: 0 off (A/B timing only), 2 every query replays the octree search (tests)
    if (const char* v = env_opt("NART_OCTREE_EXACT")) S.oc_exact = std::max(0, std::min(2, std::atoi(v)));
    if (hipMalloc(&ctx->d_oc_lock, sizeof(uint32_t) * S.oc_pool) != hipSuccess ||
        hipMemset(ctx->d_oc_lock, 0, sizeof(uint32_t) * S.oc_pool) != hipSuccess ||
        hipMalloc(&ctx->d_oc_heap, sizeof(unsigned long long) * 64 * S.oc_pool * S.oc_cap) != hipSuccess)
        return bail(NART_E_OOM);
    S.oc_lock = (uint32_t*)ctx->d_oc_lock;
    S.oc_heap = (unsigned long long*)ctx->d_oc_heap;
    *out = ctx;
    return NART_OK;
}

void nart_hip_destroy(nart_ctx* ctx) {
    if (!ctx) return;
    if (!ctx->subs.empty()) {  // multi-device context
        const RcclApi& R = rccl_api();
        for (ncclComm_t c : ctx->comms)
            if (c && R.ok) R.CommDestroy(c);
        for (size_t d = 0; d < ctx->subs.size(); ++d) {
            hipSetDevice(ctx->devs[d]);
            if (d < ctx->sub_tiles.size() && ctx->sub_tiles[d]) hipFree(ctx->sub_tiles[d]);
            if (d < ctx->streams.size() && ctx->streams[d]) hipStreamDestroy(ctx->streams[d]);
        }
        hipSetDevice(ctx->devs[0]);
        for (void* b : {ctx->d_gather, ctx->d_byid, ctx->d_image, ctx->d_slab_map})
            if (b) hipFree(b);
        for (nart_ctx* c : ctx->subs) nart_hip_destroy(c);
        delete ctx;
        return;
    }
    hipSetDevice(ctx->device);
    void* bufs[] = {ctx->d_nodes, ctx->d_tri_isect, ctx->d_tri_perm, ctx->d_tris, ctx->d_tri_mesh, ctx->d_meshes, ctx->d_mesh_eta, ctx->d_mats,
                    ctx->d_lights, ctx->d_texs, ctx->d_tex_pool, ctx->d_slot_xy, ctx->d_slot_so, ctx->d_rng, ctx->d_samples, ctx->d_prim,
                    ctx->d_L, ctx->d_bucket_ids, ctx->d_bucket_base, ctx->d_table, ctx->d_lut, ctx->d_counters, ctx->d_envs, ctx->d_density,
                    ctx->d_oc_nodes, ctx->d_oc_chunks, ctx->d_oc_tris, ctx->d_tri_leaf, ctx->d_oc_lock, ctx->d_oc_heap,
                    ctx->d_queue, ctx->d_cost, ctx->d_keys[0], ctx->d_keys[1], ctx->d_vals[0], ctx->d_vals[1],
                    ctx->d_qhead, ctx->d_sort_tmp, ctx->d_ilist, ctx->d_gstack};
    for (void* b : bufs)
        if (b) hipFree(b);
    for (void* b : {ctx->d_gather, ctx->d_image})  // nart_hip_render_device's tiles and image
        if (b) hipFree(b);
    for (void* b : ctx->env_bufs) hipFree(b);
    if (ctx->events)
        for (auto& e : ctx->ev) hipEventDestroy(e);
    delete ctx;
}

const char* nart_hip_last_error(const nart_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int nart_hip_set_counters(nart_ctx* ctx, int enable) {
    if (!ctx) return NART_E_INVALID;
    ctx->counters = enable != 0;
    for (nart_ctx* c : ctx->subs) c->counters = ctx->counters;
    return NART_OK;
}

int nart_hip_set_splat_mode(nart_ctx* ctx, int mode) {
    if (!ctx) return NART_E_INVALID;
    for (nart_ctx* c : ctx->subs)
        if (int rc = nart_hip_set_splat_mode(c, mode)) return fail(ctx, rc, c->err);
    if (mode < -1 || mode > 5)
        return fail(ctx, NART_E_UNSUPPORTED, "splat mode must be -1 (automatic) or 0-5 (5 skewed-time tile rows, 4 skewed-time "
                                             "tile columns, 3 four pixels per lane, 1-0 one pixel per lane; the "
                                             "LDS-staged and tile-column-sweep modes were retired, DESIGN.md)");
    ctx->splat_mode = mode;
    return NART_OK;
}

int nart_hip_set_specialize(nart_ctx* ctx, int mode) {
    if (!ctx || mode < 0 || mode > 2) return NART_E_INVALID;
    ctx->specialize = mode != 0;
    ctx->lean = mode == 2;
    for (nart_ctx* c : ctx->subs) {
        c->specialize = ctx->specialize;
        c->lean = ctx->lean;
    }
    return NART_OK;
}

int nart_hip_scene_features_of(const nart_scene_blob* scene, uint32_t* features) {
    if (!scene || !features) return NART_E_INVALID;
    *features = scene_features(scene);
    return NART_OK;
}

int nart_hip_scene_features(const nart_ctx* ctx, uint32_t* features, uint32_t* build) {
    if (!ctx) return NART_E_INVALID;
    const nart_ctx* c = ctx->subs.empty() ? ctx : ctx->subs[0];
    if (features) *features = c->features;
    if (build) *build = c->fm_used;
    return NART_OK;
}

int nart_hip_set_variant(nart_ctx* ctx, int variant) {
    if (!ctx) return NART_E_INVALID;
    for (nart_ctx* c : ctx->subs)
        if (int rc = nart_hip_set_variant(c, variant)) return fail(ctx, rc, c->err);
    if (variant != 0 && variant != 3)
        return fail(ctx, NART_E_UNSUPPORTED, "variant must be 0 (megakernel with a wave ray queue) or 3 (megakernel, "
                                             "one lane per pixel); the wavefront variant 1 and the traversal-quorum "
                                             "variant 2 were retired (DESIGN.md)");
    ctx->variant = variant;
    return NART_OK;
}

int nart_hip_render_buckets_async(nart_ctx* ctx, const nart_render_params* p, const uint32_t* bucket_ids,
                                  uint32_t n_buckets, nart_pixel* d_tiles, void* stream, nart_render_stats* stats) {
    if (!ctx || !bucket_ids || !d_tiles) return NART_E_INVALID;
    if (!ctx->subs.empty())
        return fail(ctx, NART_E_UNSUPPORTED, "render_buckets_async takes a single-device context (one per rank)");
    auto t0 = std::chrono::steady_clock::now();
    int rc = render_buckets(ctx, p, bucket_ids, n_buckets, reinterpret_cast<float*>(d_tiles), (hipStream_t)stream, stats);
    if (stats) stats->render_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int nart_hip_combine_async(nart_ctx* ctx, const nart_render_params* p, const nart_pixel* d_tiles, nart_pixel* d_image,
                           void* stream) {
    if (!ctx || !p || !d_tiles || !d_image) return NART_E_INVALID;
    if (!ctx->subs.empty()) return nart_hip_combine_async(ctx->subs[0], p, d_tiles, d_image, stream);
    HIPCHK(hipSetDevice(ctx->device));
    nart_session_geometry g;
    nart_session_geometry_of(p, &g);
    CombineArgs ca;
    ca.tiles = reinterpret_cast<const float*>(d_tiles);
    ca.image = reinterpret_cast<float*>(d_image);
    ca.W = p->image_width;
    ca.H = p->image_height;
    ca.B = p->bucket_size;
    ca.fb = g.filter_bounds;
    ca.tile = g.tile_size;
    ca.nbx = g.n_buckets_x;
    ca.nby = g.n_buckets_y;
    ca.totalW = g.total_width;
    ca.totalH = g.total_height;
    uint64_t n = (uint64_t)g.total_width * g.total_height;
    hipLaunchKernelGGL(k_combine, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ca);
    HIPCHK(hipGetLastError());
    return NART_OK;
}

int nart_hip_render(nart_ctx* ctx, const nart_render_params* p, nart_pixel* image, nart_render_stats* stats) {
    if (!ctx || !p || !image) return NART_E_INVALID;
    auto t0 = std::chrono::steady_clock::now();
    if (!ctx->subs.empty()) {
        const int rc = render_multi(ctx, p, image, stats);
        if (stats) stats->render_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return rc;
    }
    int rc = check_params(ctx, p);
    if (rc) return rc;
    HIPCHK(hipSetDevice(ctx->device));
    nart_session_geometry g;
    nart_session_geometry_of(p, &g);
    const uint32_t nb = g.n_buckets_x * g.n_buckets_y;
    std::vector<uint32_t> ids(nb);
    for (uint32_t i = 0; i < nb; ++i) ids[i] = i;
    size_t tile_bytes = (size_t)nb * g.tile_size * g.tile_size * sizeof(nart_pixel);
    size_t img_bytes = (size_t)g.total_width * g.total_height * sizeof(nart_pixel);
    void *d_tiles = nullptr, *d_img = nullptr;
    HIPCHK(hipMalloc(&d_tiles, tile_bytes));
    if (hipMalloc(&d_img, img_bytes) != hipSuccess) {
        hipFree(d_tiles);
        return fail(ctx, NART_E_OOM, "hipMalloc image");
    }
    rc = render_buckets(ctx, p, ids.data(), nb, (float*)d_tiles, 0, stats);
    if (!rc) rc = nart_hip_combine_async(ctx, p, (const nart_pixel*)d_tiles, (nart_pixel*)d_img, 0);
    if (!rc && hipMemcpy(image, d_img, img_bytes, hipMemcpyDeviceToHost) != hipSuccess)
        rc = fail(ctx, NART_E_HIP, "copy image");
    hipFree(d_tiles);
    hipFree(d_img);
    if (stats) stats->render_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int nart_hip_render_device(nart_ctx* ctx, const nart_render_params* p, const nart_pixel** d_image,
                           nart_render_stats* stats) {
    if (!ctx || !p || !d_image) return NART_E_INVALID;
    auto t0 = std::chrono::steady_clock::now();
    int rc = NART_OK;
    if (!ctx->subs.empty()) {
        rc = render_multi(ctx, p, nullptr, stats);  // tiles gathered to device 0, combined there
        if (!rc) *d_image = static_cast<const nart_pixel*>(ctx->d_image);
    } else {
        if ((rc = check_params(ctx, p))) return rc;
        HIPCHK(hipSetDevice(ctx->device));
        nart_session_geometry g;
        nart_session_geometry_of(p, &g);
        const uint32_t nb = g.n_buckets_x * g.n_buckets_y;
        std::vector<uint32_t> ids(nb);
        for (uint32_t i = 0; i < nb; ++i) ids[i] = i;
        const size_t tile_bytes = (size_t)nb * g.tile_size * g.tile_size * sizeof(nart_pixel);
        const size_t img_bytes = (size_t)g.total_width * g.total_height * sizeof(nart_pixel);
        if ((rc = ensure_dev(ctx, ctx->device, ctx->d_gather, ctx->cap_gather, tile_bytes, "tiles")) ||
            (rc = ensure_dev(ctx, ctx->device, ctx->d_image, ctx->cap_image, img_bytes, "image")))
            return rc;
        rc = render_buckets(ctx, p, ids.data(), nb, static_cast<float*>(ctx->d_gather), 0, stats);
        if (!rc) rc = nart_hip_combine_async(ctx, p, static_cast<const nart_pixel*>(ctx->d_gather),
                                            static_cast<nart_pixel*>(ctx->d_image), 0);
        if (!rc && hipStreamSynchronize(0) != hipSuccess) rc = fail(ctx, NART_E_HIP, "render");
        if (!rc) *d_image = static_cast<const nart_pixel*>(ctx->d_image);
    }
    if (stats) stats->render_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int nart_hip_render_samples(nart_ctx* ctx, const nart_render_params* p, uint32_t x0, uint32_t y0, uint32_t w,
                            uint32_t h, float* out) {
    if (!ctx || !p || !out) return NART_E_INVALID;
    if (!ctx->subs.empty()) {  // per-sample debugging runs on the first device
        const int rc = nart_hip_render_samples(ctx->subs[0], p, x0, y0, w, h, out);
        return rc ? fail(ctx, rc, ctx->subs[0]->err) : NART_OK;
    }
    int rc = check_params(ctx, p);
    if (rc) return rc;
    HIPCHK(hipSetDevice(ctx->device));
    nart_session_geometry g;
    nart_session_geometry_of(p, &g);
    if (x0 + w > g.total_width || y0 + h > g.total_height) return fail(ctx, NART_E_INVALID, "rect out of range");
    std::vector<uint32_t> xy;
    for (uint32_t y = y0; y < y0 + h; ++y)
        for (uint32_t x = x0; x < x0 + w; ++x) xy.push_back(x | (y << 16));
    uint32_t n = (uint32_t)xy.size();
    rc = ensure(ctx, n, p->spp, 1);
    if (rc) return rc;
    HIPCHK(hipMemcpy(ctx->d_slot_xy, xy.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_slot_rows, dim3((n + 255) / 256), dim3(256), 0, 0, n, p->spp, ctx->d_slot_so);
    const size_t n_cnt = 24;
    if (!ctx->d_counters) HIPCHK(hipMalloc(&ctx->d_counters, n_cnt * sizeof(unsigned long long)));
    if (ctx->counters) HIPCHK(hipMemset(ctx->d_counters, 0, n_cnt * sizeof(unsigned long long)));
    RenderArgs ra;
    ra.slot_xy = ctx->d_slot_xy;
    ra.slot_so = ctx->d_slot_so;
    ra.samples = ctx->d_samples;
    ra.rng0 = ctx->d_rng;
    ra.Lout = ctx->d_L;
    ra.n_slots = n;
    ra.spp = p->spp;
    ra.bounces = p->bounces;
    ra.W = p->image_width;
    ra.H = p->image_height;
    ra.totalW = g.total_width;
    ra.stack_depth = ctx->stack_depth;
    ra.lds_nodes = 0;
    ra.gamma = p->roughening_factor * p->roughening_factor;
    ra.counters = ctx->d_counters;
    rc = launch_latin(ctx, ra, 0);
    if (rc) return rc;
    {
        rc = dispatch_render(ctx, ra, p->integrator, 0);
        if (rc) return rc;
    }
    HIPCHK(hipMemcpy(out, ctx->d_L, (size_t)n * p->spp * sizeof(float4), hipMemcpyDeviceToHost));
    return NART_OK;
}

int nart_hip_bvh_info(const nart_scene_blob* blob, nart_bvh_info* out) {
    if (!blob || !out) return NART_E_INVALID;
    std::vector<uint8_t> mask;
    bool root_leaf = false;
    uint32_t n_chunks = 0;
    nart::reference_visibility(*blob, mask, root_leaf, n_chunks, nullptr);
    nart::BuiltBVH bvh;
    nart::build_bvh(*blob, mask, 0.f, bvh);
    out->num_nodes = (uint32_t)bvh.nodes.size();
    out->stack_depth = std::max<uint32_t>(bvh.max_stack + 1, 2);  // as nart_hip_create
    out->num_leaf_tris = bvh.num_leaf_tris;
    out->reserved = 0;
    return NART_OK;
}

int nart_hip_env_search(const float* v, uint32_t n, const float* values, uint32_t m, uint32_t* full,
                        uint32_t* guided) {
    if (!v || !values || !full || !guided || !n) return NART_E_INVALID;
    std::vector<uint32_t> g(NART_ENV_GUIDE_K);
    const bool ok = env_guide(v, n, g.data());
    for (uint32_t i = 0; i < m; ++i) {
        full[i] = binary_search(values[i], v, 0, n);
        guided[i] = guided_search(values[i], v, 0, n, ok ? g.data() : nullptr);
    }
    return ok ? 1 : 0;
}

int nart_hip_splat_lut(float filter_width, float* cells4, uint32_t* n_cells, uint32_t* b0) {
    if (!cells4 || !n_cells || !b0) return NART_E_INVALID;
    float table[64 + 65];
    nart_filter_table(table);
    std::vector<float4> lut;
    if (!splat_thresholds(filter_width, table + 64) || !splat_lut(table + 64, table, lut, *b0)) return NART_E_INVALID;
    std::memcpy(cells4, lut.data(), lut.size() * sizeof(float4));
    *n_cells = (uint32_t)lut.size();
    return NART_OK;
}

int nart_hip_splat_thresholds(float filter_width, float* thr65) {
    if (!thr65) return NART_E_INVALID;
    return splat_thresholds(filter_width, thr65) ? NART_OK : NART_E_INVALID;
}

int nart_hip_eval_sincos(nart_ctx* ctx, const float* x, uint32_t n, float* s, float* c) {
    if (!ctx || !x || !s || !c) return NART_E_INVALID;
    if (!ctx->subs.empty()) return nart_hip_eval_sincos(ctx->subs[0], x, n, s, c);
    HIPCHK(hipSetDevice(ctx->device));
    float *dx = nullptr, *ds = nullptr, *dc = nullptr;
    HIPCHK(hipMalloc(&dx, (size_t)n * 4 + 4));
    HIPCHK(hipMalloc(&ds, (size_t)n * 4 + 4));
    HIPCHK(hipMalloc(&dc, (size_t)n * 4 + 4));
    HIPCHK(hipMemcpy(dx, x, (size_t)n * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_sincos, dim3((n + 255) / 256), dim3(256), 0, 0, dx, n, ds, dc);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(s, ds, (size_t)n * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(c, dc, (size_t)n * 4, hipMemcpyDeviceToHost));
    hipFree(dx);
    hipFree(ds);
    hipFree(dc);
    return NART_OK;
}

int nart_hip_context_bvh(const nart_ctx* ctx, nart_bvh_info* out, double* build_ms) {
    if (!ctx || !out) return NART_E_INVALID;
    const nart_ctx* c = ctx->subs.empty() ? ctx : ctx->subs[0];
    out->num_nodes = c->num_nodes;
    out->stack_depth = c->stack_depth;
    out->num_leaf_tris = c->num_leaf_tris;
    out->reserved = c->bvh_on_device ? 1u : 0u;
    if (build_ms) *build_ms = c->bvh_ms;
    return NART_OK;
}

int nart_hip_device_count(int* count) {
    if (!count) return NART_E_INVALID;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        *count = 0;
        return NART_E_HIP;
    }
    *count = n;
    return NART_OK;
}

int nart_hip_shard_buckets(uint32_t n_buckets_x, uint32_t n_buckets, uint32_t n_devices, uint32_t device_index,
                           uint32_t* ids, uint32_t* count) {
    if (!count || !n_devices || !n_buckets_x || device_index >= n_devices) return NART_E_INVALID;
    const std::vector<uint32_t> v = shard_ids(n_buckets_x, n_buckets, n_devices, device_index);
    if (ids) std::memcpy(ids, v.data(), v.size() * sizeof(uint32_t));
    *count = (uint32_t)v.size();
    return NART_OK;
}

int nart_hip_create_multi(const nart_scene_blob* blob, const int* device_ids, int n_devices, nart_ctx** out) {
    if (!blob || !out || !device_ids || n_devices < 1 || n_devices > 64) return NART_E_INVALID;
    *out = nullptr;
    const char* gm = env_opt("NART_GATHER");
    const bool force_rccl = gm && std::string(gm) == "rccl";
    const bool force_copy = gm && std::string(gm) == "copy";
    if (n_devices == 1 && !force_rccl) return nart_hip_create(blob, device_ids[0], out);
    nart_ctx* ctx = new (std::nothrow) nart_ctx();
    if (!ctx) return NART_E_OOM;
    ctx->device = device_ids[0];
    auto bail = [&](int code) {
        nart_hip_destroy(ctx);
        return code;
    };
    bool distinct = true;
    for (int i = 0; i < n_devices; ++i)
        for (int j = 0; j < i; ++j) distinct = distinct && device_ids[i] != device_ids[j];
    for (int d = 0; d < n_devices; ++d) {
        nart_ctx* sub = nullptr;
        if (int rc = nart_hip_create(blob, device_ids[d], &sub)) return bail(rc);
        ctx->subs.push_back(sub);
        ctx->devs.push_back(device_ids[d]);
        ctx->sub_tiles.push_back(nullptr);
        ctx->sub_cap.push_back(0);
        hipStream_t st = nullptr;
        if (hipSetDevice(device_ids[d]) != hipSuccess || hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess)
            return bail(NART_E_HIP);
        ctx->streams.push_back(st);
    }
    for (int d = 0; d < n_devices; ++d)
        for (int j = 0; j < n_devices; ++j) ctx->subs[d]->mem_share += (j != d && device_ids[j] == device_ids[d]) ? 1u : 0u;
    ctx->gather_rccl = force_rccl || (distinct && !force_copy);
    if (ctx->gather_rccl) {
        const RcclApi& R = rccl_api();
        bool ok = R.ok && distinct;
        if (ok) {
            ctx->comms.assign(n_devices, nullptr);
            if (R.CommInitAll(ctx->comms.data(), n_devices, device_ids) != ncclSuccess) {
                ctx->comms.clear();
                (void)hipGetLastError();
                ok = false;
            }
        }
        if (!ok) {
            // NART_GATHER=rccl demands RCCL; otherwise the device-copy gather serves the same
            // image (nart_hip_context_devices reports the fallback)
            if (force_rccl) return bail(NART_E_RCCL);
            ctx->gather_rccl = false;
            ctx->gather_fallback = true;
        }
    }
    if (!ctx->gather_rccl) {
        // device copies to device 0 (peer access where the devices differ)
        hipSetDevice(device_ids[0]);
        for (int d = 1; d < n_devices; ++d)
            if (device_ids[d] != device_ids[0]) {
                int can = 0;
                if (hipDeviceCanAccessPeer(&can, device_ids[0], device_ids[d]) == hipSuccess && can)
                    hipDeviceEnablePeerAccess(device_ids[d], 0);
                (void)hipGetLastError();  // already enabled is fine
            }
    }
    *out = ctx;
    return NART_OK;
}

int nart_hip_context_devices(const nart_ctx* ctx, int* n_devices, int* uses_rccl) {
    if (!ctx || !n_devices) return NART_E_INVALID;
    *n_devices = ctx->subs.empty() ? 1 : (int)ctx->subs.size();
    if (uses_rccl) *uses_rccl = ctx->gather_rccl ? 1 : (ctx->gather_fallback ? 2 : 0);
    return NART_OK;
}

int nart_hip_debug_fault(nart_ctx* ctx, int fault) {
    if (!ctx || fault < 0 || fault > 1) return NART_E_INVALID;
    ctx->debug_fault = fault;
    return NART_OK;
}

}  // extern "C"
