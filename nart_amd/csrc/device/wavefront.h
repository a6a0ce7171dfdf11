// Wavefront variant of the path tracer: ray queues + path state in HBM.
//
// Per iteration two kernels run:
//   k_wf_trace  every queued ray (extension = closest hit, shadow = any hit) of the iteration
//               through one traversal loop; writes hit records / occlusion bytes per slot.
//   k_wf_shade  every live slot, in slot order: (a) adds last bounce's deferred EstimateDirect term using the
//               shadow results, (b) stores the sample that ended last bounce and starts the one
//               whose camera ray was just traced, (c) shades this bounce's hit (BSDF,
//               EstimateDirect, continuation, Russian roulette) and emits the next rays
//               (extension + up to two shadow rays) into the next iteration's queues.
// A slot is one traced pixel; it walks its pixel's spp samples in order on one RNG stream, so
// every RNG draw and float operation happens in exactly the order of the megakernel (and of
// the reference's Li_alpha, pathintegrator.cpp:147-251).  Shadow rays only gate an additive
// term, so they are traced one iteration after the shading that spawned them, alongside the
// continuation ray, and the term is added first thing in the next shade -- before anything
// else touches L.  The camera ray and light loop of a new sample use no RNG, so a new sample's
// camera ray is issued in the same iteration as the previous sample's last shadow rays.
// Queue appends are wave-aggregated (shuffle prefix sum, one atomic per wave).
#pragma once

#include "kernels.h"

namespace nd {

// slot flag bits (WFState::u.w)
#define WF_BSDF_MASK 0xFFu        // persistent BSDF `flags` of Li_alpha
#define WF_LIGHTHIT (1u << 8)     // the current sample's camera ray hit a light first
#define WF_PENDING (1u << 9)      // deferred EstimateDirect term to add (have_ed)
#define WF_USE1 (1u << 10)        // shadow ray 1 traced for it
#define WF_USE2 (1u << 11)        // shadow ray 2 traced for it
#define WF_FINISH (1u << 12)      // the current sample ended: store it before shading the new ray
#define WF_RETIRE (1u << 13)      // ... and it was the pixel's last sample
#define WF_NEXT_LIGHT (1u << 14)  // the next sample's camera ray hit a light first
#define WF_DEAD (1u << 15)        // all samples of the pixel stored

enum { RK_EXT = 0, RK_SH1 = 1, RK_SH2 = 2 };

struct WFState {
    uint4* u;         // rng, sample index, bounce, flags
    float4* L;        // L.xyz, alpha
    float4* beta;     // beta.xyz, eta_sampled
    float4* misc;     // Le.xyz of the camera ray in flight, alphaTweak
    float4* c1;       // EstimateDirect BSDF-sampled term (xyz)
    float4* c2;       // EstimateDirect light-sampled term (xyz)
    float4* betak;    // beta the deferred term is weighted with (xyz)
    float4* ray_o;    // [3][n] origin.xyz, tmax   (extension, shadow 1, shadow 2)
    float4* ray_d;    // [3][n] direction.xyz
    uint2* hit;       // extension result: t bits, scene triangle index or NO_HIT
    uint8_t* occ;     // [3][n] shadow results (rows 1, 2)
    uint32_t* ln;     // nested-dielectric list length
    uint32_t* lid;    // [MAXL][n] meshID | priority << 24
    float* leta;      // [MAXL][n]
};

struct WFArgs {
    RenderArgs R;
    WFState st;
    uint32_t* rq_ext[2];  // extension-ray queues by iteration parity: slot
    uint32_t* rq_sh[2];   // shadow-ray queues by iteration parity: slot << 2 | kind
    uint32_t* counts;     // [p] extension rays, [2 + p] shadow rays, [4 + p] live slots of parity p
};

// Wave-aggregated append: each active lane reserves `n` consecutive entries; one atomic per wave.
// Must be reached by every active lane of the wave.
ND uint32_t wave_append(uint32_t* counter, uint32_t n) {
    const int lane = __lane_id();
    uint32_t incl = n;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t v = __shfl_up(incl, off, 64);
        if (lane >= off) incl += v;
    }
    const uint64_t active = __ballot(1);
    const int last = 63 - __clzll((long long)active);
    const uint32_t total = __shfl(incl, last, 64);
    uint32_t base = 0;
    if (lane == last && total) base = atomicAdd(counter, total);
    base = __shfl(base, last, 64);
    return base + incl - n;
}

ND uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Camera ray + light loop of a new sample (pathintegrator.cpp:167-182 at bounce 0).
ND void gen_camera(const DScene& S, const RenderArgs& A, uint32_t slot, uint32_t s, f3& o, f3& d, float& tmax,
                   f3& Le, bool& lightHit) {
    const uint32_t xy = A.slot_xy[slot];
    const float2 sm = A.samples[sample_index(A, slot, s)];
    Ray r = cast_ray(S, F2(sm.x, sm.y), A.W, A.H, xy & 0xFFFFu, xy >> 16);
    o = r.o;
    d = r.d;
    tmax = __builtin_inff();
    lightHit = false;
    Le = F3(0.f, 0.f, 0.f);
    for (uint32_t j = 0; j < S.num_lights; ++j) {
        float lt = __builtin_inff();
        f3 Li = light_li(S, S.lights[j], o, d, nullptr, lt);
        if (lt < tmax) {
            Le = Li;
            tmax = lt;
            lightHit = true;
        }
    }
}

// Light loop of a continuation ray: only the bound matters (alpha is already 1 past bounce 0,
// and Le is only used by a bounce-0 miss).
ND float light_tmax(const DScene& S, f3 o, f3 d) {
    float tmax = __builtin_inff();
    for (uint32_t j = 0; j < S.num_lights; ++j) {
        float lt = __builtin_inff();
        light_li(S, S.lights[j], o, d, nullptr, lt);
        if (lt < tmax) tmax = lt;
    }
    return tmax;
}

ND void put_ray(const WFArgs& A, uint32_t kind, uint32_t slot, f3 o, f3 d, float tmax) {
    const size_t i = (size_t)kind * A.R.n_slots + slot;
    A.st.ray_o[i] = make_float4(o.x, o.y, o.z, tmax);
    A.st.ray_d[i] = make_float4(d.x, d.y, d.z, 0.f);
}

// ---------------------------------------------------------------- init: sample 0 of every slot
__global__ __launch_bounds__(256) void k_wf_init(DScene S, WFArgs A) {
    const uint32_t gsize = gridDim.x * blockDim.x;
    const RenderArgs& R = A.R;
    for (uint32_t base = blockIdx.x * blockDim.x; base < R.n_slots; base += gsize) {
        const uint32_t slot = base + threadIdx.x;
        const bool live = slot < R.n_slots && R.bounces > 0;
        if (slot < R.n_slots && R.bounces == 0) {
            // every sample ends before its first light loop (pathintegrator.cpp:165)
            for (uint32_t s = 0; s < R.spp; ++s) R.Lout[sample_index(R, slot, s)] = make_float4(0.f, 0.f, 0.f, 0.f);
            A.st.u[slot] = make_uint4(0u, R.spp, 0u, WF_DEAD);
        }
        if (live) {
            f3 o, d, Le;
            float tmax;
            bool lh;
            gen_camera(S, R, slot, 0, o, d, tmax, Le, lh);
            put_ray(A, RK_EXT, slot, o, d, tmax);
            A.st.u[slot] = make_uint4(R.rng0[slot], 0u, 0u, lh ? WF_LIGHTHIT : 0u);
            A.st.L[slot] = make_float4(0.f, 0.f, 0.f, lh ? 1.f : 0.f);
            A.st.beta[slot] = make_float4(1.f, 1.f, 1.f, 1.f);
            A.st.misc[slot] = make_float4(Le.x, Le.y, Le.z, 1.f);
            A.st.ln[slot] = 0;
        }
        const uint32_t ri = wave_append(&A.counts[0], live ? 1u : 0u);
        if (live) A.rq_ext[0][ri] = slot;
        const uint32_t nlive = wave_sum(live ? 1u : 0u);
        if (__lane_id() == 0 && nlive) atomicAdd(&A.counts[4], nlive);
    }
}

// ---------------------------------------------------------------- trace
template <bool COUNT>
__global__ __launch_bounds__(256) void k_wf_trace(DScene S, WFArgs A, uint32_t it) {
    extern __shared__ __attribute__((aligned(16))) int s_dyn[];
    int* sc = reinterpret_cast<int*>(reinterpret_cast<int2*>(s_dyn) + threadIdx.x);
    const uint32_t cur = it & 1u, nxt = cur ^ 1u;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        A.counts[nxt] = 0;  // queues of the next iteration, filled by k_wf_shade(it)
        A.counts[2 + nxt] = 0;
        A.counts[4 + nxt] = 0;
    }
    // extension rays first, then shadow rays: a wave holds one query type except at the seam
    const uint32_t ne = A.counts[cur];
    const uint32_t n = ne + A.counts[2 + cur];
    const uint32_t gsize = gridDim.x * blockDim.x;
    const size_t N = A.R.n_slots;
    TraceCounters cnt = {0u, 0u, 0u, 0u};
    uint32_t n_ext = 0, n_sh = 0, n_hit = 0;
    // Persistent lanes with dynamic ray fetching: a lane whose ray is resolved takes its next
    // ray (grid-stride order) before the next traversal step, instead of idling until the
    // slowest ray of its wave is done.
    uint32_t next = blockIdx.x * blockDim.x + threadIdx.x;
    bool busy = false;
    uint32_t slot = 0, kind = 0;
    Ray r;
    Trav t;
    for (;;) {
        while (!busy && next < n) {
            const uint32_t tag = next < ne ? (A.rq_ext[cur][next] << 2) : A.rq_sh[cur][next - ne];
            next += gsize;
            slot = tag >> 2;
            kind = tag & 3u;
            const float4 o = A.st.ray_o[kind * N + slot];
            const float4 d = A.st.ray_d[kind * N + slot];
            r = make_ray(F3(o.x, o.y, o.z), F3(d.x, d.y, d.z));
            if (S.geometry_visible) {
                trav_begin(S, r, o.w, kind != RK_EXT, t);
                busy = true;
            } else {  // nothing to hit
                if (kind == RK_EXT) A.st.hit[slot] = make_uint2(__float_as_uint(o.w), NO_HIT);
                else A.st.occ[kind * N + slot] = 0;
                if (COUNT) {
                    n_ext += kind == RK_EXT ? 1u : 0u;
                    n_sh += kind == RK_EXT ? 0u : 1u;
                }
            }
        }
        if (__ballot(busy) == 0) break;
        if (busy && trav_step<COUNT>(S, r, t, sc, nullptr, blockDim.x, cnt, nullptr, 0)) {
            busy = false;
            oc_resolve<COUNT>(S, r, t.tmax, t.any, t.risky, t.bestInfo, fminf(t.t2, oc_cull(S, t.bestT)), t.bestT, t.bestG, cnt);
            const bool hit = t.bestG != NO_HIT;
            if (kind == RK_EXT) {
                A.st.hit[slot] = make_uint2(__float_as_uint(t.bestT), t.bestG);
                if (COUNT) {
                    ++n_ext;
                    n_hit += hit ? 1u : 0u;
                }
            } else {
                A.st.occ[kind * N + slot] = hit ? 1 : 0;
                if (COUNT) ++n_sh;
            }
        }
    }
    if (COUNT) {
        const uint32_t e = wave_sum(n_ext), sh = wave_sum(n_sh), nv = wave_sum(cnt.nodes), tt = wave_sum(cnt.tris);
        const uint32_t hh = wave_sum(n_hit);
        if (__lane_id() == 0) {
            atomicAdd(&A.R.counters[0], (unsigned long long)e);
            atomicAdd(&A.R.counters[1], (unsigned long long)sh);
            atomicAdd(&A.R.counters[2], (unsigned long long)nv);
            atomicAdd(&A.R.counters[3], (unsigned long long)tt);
            atomicAdd(&A.R.counters[4], (unsigned long long)hh);
        }
        atomicAdd(&A.R.counters[5], (unsigned long long)cnt.oc_checks);
        atomicAdd(&A.R.counters[6], (unsigned long long)cnt.oc_replays);
    }
}

// ---------------------------------------------------------------- shade one slot
// Returns the rays emitted (bit 0 extension, bit 1 shadow 1, bit 2 shadow 2); their origin,
// direction and bound are already stored in the slot's ray rows.
template <int MAXL>
ND uint32_t shade_slot(const DScene& S, const WFArgs& A, uint32_t slot, const uint4 u) {
    const RenderArgs& R = A.R;
    const WFState& T = A.st;
    const size_t N = R.n_slots;
    const float nL = (float)S.num_lights;
    uint32_t rng = u.x, s = u.y, bounce = u.z, fl = u.w;
    const float4 L4 = T.L[slot], B4 = T.beta[slot], M4 = T.misc[slot];
    f3 L = F3(L4.x, L4.y, L4.z), beta = F3(B4.x, B4.y, B4.z), Le = F3(M4.x, M4.y, M4.z);
    float alpha = L4.w, eta_sampled = B4.w, alphaTweak = M4.w;
    uint32_t ln = T.ln[slot];
    bool list_dirty = false;

    // (a) L += EstimateDirect(...) * beta, EstimateDirect = ((0 + c1) + c2) * numLights
    if (fl & WF_PENDING) {
        f3 Led = F3(0.f, 0.f, 0.f);
        if ((fl & WF_USE1) && !T.occ[N + slot]) {
            const float4 c = T.c1[slot];
            Led = add(Led, F3(c.x, c.y, c.z));
        }
        if ((fl & WF_USE2) && !T.occ[2 * N + slot]) {
            const float4 c = T.c2[slot];
            Led = add(Led, F3(c.x, c.y, c.z));
        }
        const float4 bk = T.betak[slot];
        L = add(L, mul(muls(Led, nL), F3(bk.x, bk.y, bk.z)));
        fl &= ~(WF_PENDING | WF_USE1 | WF_USE2);
    }
    // (b) the sample that ended last bounce is complete: store it, start the traced one
    if (fl & WF_FINISH) {
        R.Lout[sample_index(R, slot, s)] = make_float4(L.x, L.y, L.z, alpha);
        ++s;
        if (fl & WF_RETIRE) {  // pixel done
            T.u[slot] = make_uint4(rng, s, bounce, WF_DEAD);
            return 0u;
        }
        const bool lh = (fl & WF_NEXT_LIGHT) != 0;
        L = F3(0.f, 0.f, 0.f);
        alpha = lh ? 1.f : 0.f;
        eta_sampled = 1.f;
        beta = F3(1.f, 1.f, 1.f);
        fl = lh ? WF_LIGHTHIT : 0u;
        alphaTweak = 1.f;
        bounce = 0;
        ln = 0;
        list_dirty = true;
    }
    IList<MAXL> list;
    list.n = ln;
#pragma unroll
    for (int k = 0; k < MAXL; ++k)
        if (k < (int)ln) {
            list.id[k] = T.lid[(size_t)k * N + slot];
            list.eta[k] = T.leta[(size_t)k * N + slot];
        }

    // (c) this bounce
    uint32_t emit = 0;
    bool sample_end = false, pending = false;
    const uint2 h = T.hit[slot];
    if (h.y == NO_HIT) {
        // escaped: at bounce 0 the light seen directly is the result; past bounce 0 the
        // reference repeats the same miss until its loop ends (no RNG, no state change)
        if (bounce == 0 && (fl & WF_LIGHTHIT)) L = Le;
        sample_end = true;
    } else {
        const float4 o4 = T.ray_o[slot], d4 = T.ray_d[slot];
        const Ray cur = make_ray(F3(o4.x, o4.y, o4.z), F3(d4.x, d4.y, d4.z));
        Isect is;
        fill_isect(S, cur, h.y, is);
        BSDF bsdf;
        create_bsdf(S, is, alphaTweak, bsdf);
        uint32_t flags = fl & WF_BSDF_MASK;
        bool use1 = false, use2 = false, cont = false, have_ed = false;
        float eta_outer = 1.f;
        f3 betak = F3(0.f, 0.f, 0.f), no = F3(0.f, 0.f, 0.f), nd = F3(0.f, 0.f, 1.f);
        if (list.valid(is.meshID, is.priority, eta_outer)) {
            if (bounce == 0) alpha = 1.f;
            const f3 wo = to_local(bsdf, neg(cur.d));
            // ---- EstimateDirect (pathintegrator.cpp:38-121)
            const DLight& Lg = S.lights[f2u8(gmin(rng_float(rng), ND_ONE_MINUS_EPS) * nL)];
            float sPdf = 0.f, lPdf = 0.f;
            const float sx = rng_float(rng);
            const float sy = rng_float(rng);
            const float bsmp = rng_float(rng);
            uint32_t dflags = 0;
            f3 wi;
            const f3 f = bsdf_sample_f(bsdf, wo, wi, bsmp, F2(sx, sy), sPdf, dflags, true, eta_outer, nullptr, nullptr);
            if (sPdf > 0.f) {
                const float flip = wi.z > 0.f ? 1.f : -1.f;
                const f3 wW = to_world(bsdf, wi);
                float lt = __builtin_inff();
                const f3 Li = light_li(S, Lg, is.p, wW, &lPdf, lt);
                float weight = 1.f;
                bool add1 = true;
                if (!(dflags & F_SPECULAR)) {
                    weight = (sPdf * sPdf) / (sPdf * sPdf + lPdf * lPdf);
                    add1 = lPdf > 0.f;
                }
                if (add1) {
                    const f3 c1 = divs(muls(muls(mul(f, Li), gabs(wi.z)), weight), sPdf);
                    // an all-zero term cannot change the sum: skip its shadow ray
                    use1 = !(c1.x == 0.f && c1.y == 0.f && c1.z == 0.f);
                    if (use1) {
                        T.c1[slot] = make_float4(c1.x, c1.y, c1.z, 0.f);
                        put_ray(A, RK_SH1, slot, add(is.p, muls(muls(is.gn, SHADOW_BIAS), flip)), wW, lt);
                    }
                }
            }
            lPdf = 0.f;
            const float lx = rng_float(rng);
            const float ly = rng_float(rng);
            f3 wiW;
            float lt2 = __builtin_inff();
            const f3 Li2 = light_sample_li(S, Lg, is.p, wiW, F2(lx, ly), lPdf, lt2);
            const f3 wi2 = to_local(bsdf, wiW);
            if (lPdf > 0.f) {
                float sp2;
                const f3 fv = bsdf_f_pdf(bsdf, wo, wi2, true, eta_outer, sp2);
                if (sp2 > 0.f) {
                    const float weight = (lPdf * lPdf) / (sp2 * sp2 + lPdf * lPdf);
                    const f3 c2 = divs(muls(muls(mul(fv, Li2), gabs(wi2.z)), weight), lPdf);
                    use2 = !(c2.x == 0.f && c2.y == 0.f && c2.z == 0.f);
                    if (use2) {
                        const float flip2 = wi2.z > 0.f ? 1.f : -1.f;
                        T.c2[slot] = make_float4(c2.x, c2.y, c2.z, 0.f);
                        put_ray(A, RK_SH2, slot, add(is.p, muls(muls(is.gn, SHADOW_BIAS), flip2)), wiW, lt2);
                    }
                }
            }
            betak = beta;
            have_ed = true;
            // ---- continuation (pathintegrator.cpp:199-220)
            const float a = rng_float(rng);
            const float b = rng_float(rng);
            const float bs2 = rng_float(rng);
            float cpdf = 0.f, alpha_i = 0.f;
            f3 wic;
            const f3 fc = bsdf_sample_f(bsdf, wo, wic, bs2, F2(a, b), cpdf, flags, false, eta_outer, &alpha_i,
                                        &eta_sampled);
            if (cpdf > 0.f) {
                alphaTweak = (1.f - (R.gamma * alpha_i)) * alphaTweak;
                beta = mul(beta, muls(divs(fc, cpdf), gabs(wic.z)));
                const float flip = wic.z > 0.f ? 1.f : -1.f;
                no = add(is.p, muls(muls(is.gn, SHADOW_BIAS), flip));
                nd = to_world(bsdf, wic);
                cont = true;
            }
        } else {
            // lower-priority interface: step through (pathintegrator.cpp:223-229)
            no = add(is.p, muls(cur.d, SHADOW_BIAS));
            nd = cur.d;
            flags = F_TRANSMISSIVE;
            const float bs2 = rng_float(rng);
            eta_sampled = bsdf_sample_eta(bsdf, bs2);
            cont = true;
        }
        if (cont) {
            if (flags & F_TRANSMISSIVE) {
                list.update(is.meshID, is.priority, eta_sampled);
                list_dirty = true;
            }
            // Russian roulette (pathintegrator.cpp:236-246)
            const float q = gmax((beta.x + beta.y + beta.z) * 0.33333f, 0.f);
            if (bounce > 3) {
                if (q >= rng_float(rng)) beta = divs(beta, q);
                else cont = false;
            }
        }
        ++bounce;
        if (have_ed) {
            if (use1 || use2) {
                pending = true;
                T.betak[slot] = make_float4(betak.x, betak.y, betak.z, 0.f);
                fl |= WF_PENDING | (use1 ? WF_USE1 : 0u) | (use2 ? WF_USE2 : 0u);
                emit |= (use1 ? 2u : 0u) | (use2 ? 4u : 0u);
            } else {
                L = add(L, mul(muls(F3(0.f, 0.f, 0.f), nL), betak));
            }
        }
        fl = (fl & ~WF_BSDF_MASK) | (flags & WF_BSDF_MASK);
        if (cont && bounce < R.bounces) {
            put_ray(A, RK_EXT, slot, no, nd, light_tmax(S, no, nd));
            emit |= 1u;
        } else {
            sample_end = true;
        }
    }

    if (sample_end) {
        if (pending) {
            // the term is added next iteration; the next sample's camera ray goes out now
            fl |= WF_FINISH;
            if (s + 1 < R.spp) {
                f3 o, d, LeN;
                float tmax;
                bool lh;
                gen_camera(S, R, slot, s + 1, o, d, tmax, LeN, lh);
                put_ray(A, RK_EXT, slot, o, d, tmax);
                Le = LeN;
                if (lh) fl |= WF_NEXT_LIGHT;
                emit |= 1u;
            } else {
                fl |= WF_RETIRE;
            }
        } else {
            R.Lout[sample_index(R, slot, s)] = make_float4(L.x, L.y, L.z, alpha);
            ++s;
            if (s >= R.spp) {  // pixel done
                T.u[slot] = make_uint4(rng, s, bounce, WF_DEAD);
                return 0u;
            }
            f3 o, d, LeN;
            float tmax;
            bool lh;
            gen_camera(S, R, slot, s, o, d, tmax, LeN, lh);
            put_ray(A, RK_EXT, slot, o, d, tmax);
            Le = LeN;
            L = F3(0.f, 0.f, 0.f);
            alpha = lh ? 1.f : 0.f;
            eta_sampled = 1.f;
            beta = F3(1.f, 1.f, 1.f);
            fl = lh ? WF_LIGHTHIT : 0u;
            alphaTweak = 1.f;
            bounce = 0;
            list.n = 0;
            list_dirty = true;
            emit |= 1u;
        }
    }

    T.u[slot] = make_uint4(rng, s, bounce, fl);
    T.L[slot] = make_float4(L.x, L.y, L.z, alpha);
    T.beta[slot] = make_float4(beta.x, beta.y, beta.z, eta_sampled);
    T.misc[slot] = make_float4(Le.x, Le.y, Le.z, alphaTweak);
    if (list_dirty) {
        T.ln[slot] = list.n;
#pragma unroll
        for (int k = 0; k < MAXL; ++k)
            if (k < (int)list.n) {
                T.lid[(size_t)k * N + slot] = list.id[k];
                T.leta[(size_t)k * N + slot] = list.eta[k];
            }
    }
    return emit;
}

// ---------------------------------------------------------------- shade
// Slots are visited in index order (coalesced state rows); retired pixels are skipped.  Every
// live slot has exactly one traced ray set to consume per iteration.
template <int MAXL>
__global__ __launch_bounds__(256) void k_wf_shade(DScene S, WFArgs A, uint32_t it) {
    const uint32_t cur = it & 1u, nxt = cur ^ 1u;
    if (A.counts[4 + cur] == 0) return;
    const uint32_t N = A.R.n_slots;
    const uint32_t gsize = gridDim.x * blockDim.x;
    for (uint32_t base = blockIdx.x * blockDim.x; base < N; base += gsize) {
        const uint32_t slot = base + threadIdx.x;
        uint32_t emit = 0;
        if (slot < N) {
            const uint4 u = A.st.u[slot];
            if (!(u.w & WF_DEAD)) emit = shade_slot<MAXL>(S, A, slot, u);
        }
        const uint32_t ri = wave_append(&A.counts[nxt], emit & 1u);
        if (emit & 1u) A.rq_ext[nxt][ri] = slot;
        const uint32_t nsh = ((emit >> 1) & 1u) + ((emit >> 2) & 1u);
        uint32_t si = wave_append(&A.counts[2 + nxt], nsh);
        if (emit & 2u) A.rq_sh[nxt][si++] = (slot << 2) | RK_SH1;
        if (emit & 4u) A.rq_sh[nxt][si] = (slot << 2) | RK_SH2;
        const uint32_t nlive = wave_sum(emit ? 1u : 0u);
        if (__lane_id() == 0 && nlive) atomicAdd(&A.counts[4 + nxt], nlive);
    }
}

}  // namespace nd
