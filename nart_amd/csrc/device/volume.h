// Volume integrator (volumeintegrator.cpp:3-84): delta tracking through the camera medium's
// width-1 majorant grid (media.h:128-181, media.cpp:3-324), isotropic scattering
// (UniformSampleSphere, sampling.cpp:33-45), escape to the lights.  No surfaces are
// intersected: the reference's integrator never calls Scene::Intersect.
//
// One lane per traced pixel walks its spp samples in order on its RNG stream (the same slot
// layout as k_render); the kernel needs no BVH.  Small density grids are staged in LDS.
#pragma once

#include "kernels.h"

namespace nd {

ND f3 uniform_sample_sphere(f2 smp) {  // sampling.cpp:33-45 (pdf unused by the caller)
    const float theta = glibc_acosf(1.f - (2.f * smp.x));
    const float phi = smp.y * ND_TWO_PI;
    float cosTheta, sinTheta, cosPhi, sinPhi;
    glibc_sincosf(theta, sinTheta, cosTheta);
    glibc_sincosf(phi, sinPhi, cosPhi);
    return F3(sinTheta * cosPhi, sinTheta * sinPhi, cosTheta);
}

NHD float dg_at(const DMedium& m, const float* dens, uint32_t x, uint32_t y, uint32_t z) {  // media.cpp:3-7
    return dens[(m.rx * m.ry * z) + (m.rx * y) + x];
}
// dens: the grid (m.density, or its LDS copy)
NHD float dg_lookup(const DMedium& m, const float* dens, f3 p) {  // media.cpp:10-45
    const float x = gmin(gmax(0.f, p.x), 0.999f) * (float)((int)m.rx - 1);
    const uint32_t loX = (uint8_t)(uint32_t)x, hiX = (uint8_t)(loX + 1);
    const float xD = (x - (float)loX);
    const float y = gmin(gmax(0.f, p.y), 0.999f) * (float)((int)m.ry - 1);
    const uint32_t loY = (uint8_t)(uint32_t)y, hiY = (uint8_t)(loY + 1);
    const float yD = (y - (float)loY);
    const float z = gmin(gmax(0.f, p.z), 0.999f) * (float)((int)m.rz - 1);
    const uint32_t loZ = (uint8_t)(uint32_t)z, hiZ = (uint8_t)(loZ + 1);
    const float zD = (z - (float)loZ);
    const float x0 = gmix(dg_at(m, dens, loX, loY, loZ), dg_at(m, dens, hiX, loY, loZ), xD);
    const float x1 = gmix(dg_at(m, dens, loX, loY, hiZ), dg_at(m, dens, hiX, loY, hiZ), xD);
    const float x2 = gmix(dg_at(m, dens, loX, hiY, loZ), dg_at(m, dens, hiX, hiY, loZ), xD);
    const float x3 = gmix(dg_at(m, dens, loX, hiY, hiZ), dg_at(m, dens, hiX, hiY, hiZ), xD);
    const float y0 = gmix(x0, x2, yD);
    const float y1 = gmix(x1, x3, yD);
    return gmix(y0, y1, zD);
}

// DensityGrid::LookUp on a 2x2x2 grid (m.grid2): every lookup reads corners lo = 0, hi = 1 of
// each axis (x = clamp(p, 0, 0.999) * (2 - 1) truncates to 0), so the densities come from the
// kernel arguments; the arithmetic is dg_lookup's, operation for operation.
NHD float dg_lookup2(const DMedium& m, f3 p) {
    const float xD = gmin(gmax(0.f, p.x), 0.999f) * 1.f - 0.f;
    const float yD = gmin(gmax(0.f, p.y), 0.999f) * 1.f - 0.f;
    const float zD = gmin(gmax(0.f, p.z), 0.999f) * 1.f - 0.f;
    const float* d = m.dens8;  // index 4z + 2y + x (dg_at with rx = ry = 2)
    const float x0 = gmix(d[0], d[1], xD);
    const float x1 = gmix(d[4], d[5], xD);
    const float x2 = gmix(d[2], d[3], xD);
    const float x3 = gmix(d[6], d[7], xD);
    const float y0 = gmix(x0, x2, yD);
    const float y1 = gmix(x1, x3, yD);
    return gmix(y0, y1, zD);
}

struct MajIter {  // RayMajorantIterator (media.cpp:138-255) for a width-1 grid
    float tCurrent, tMax;
    uint32_t idx;
    f3 next;
    // The grid direction, not the crossing distances: crossDistance_i = |((1 / gD_i) * 1) * bs_i|
    // (inf for gD_i == 0) is only ever read through nextCrossing_i after Next() stores it there,
    // and a ray in a one-cell grid leaves the medium at that first crossing, so the reciprocals
    // are formed when a later Next() reads the stored entry (cross_at), not per ray: three
    // correctly rounded divisions fewer per scattering event, the same values when needed.
    f3 gD;
    uint32_t pend;     // 1 + the axis whose next entry holds a not yet formed crossDistance, or 0
    uint32_t stepPos;  // bit i: step[i] > 0 (only the sign of the step is ever used)
};

// crossDistance_i of the iterator constructor (media.cpp:172-177)
NHD float cross_at(const DMedium& m, const MajIter& it, int i) {
    const float g = comp(it.gD, i), bsi = m.bmax[i] - m.bmin[i];
    return g == 0.f ? __builtin_inff() : gabs(((1.f / g) * 1.f) * bsi);
}

// Medium::SampleRay (media.cpp:281-324) + the iterator constructor.
ND bool medium_sample_ray(const DMedium& m, f3 o, f3 d, MajIter& it) {
    float tMin = -__builtin_inff(), tMax = __builtin_inff();
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const f3 n = F3(i == 0 ? 1.f : 0.f, i == 1 ? 1.f : 0.f, i == 2 ? 1.f : 0.f);
        float slabMin = (m.bmin[i] - dot(o, n)) / dot(d, n);
        float slabMax = (m.bmax[i] - dot(o, n)) / dot(d, n);
        if (slabMin > slabMax) {
            const float t = slabMin;
            slabMin = slabMax;
            slabMax = t;
        }
        if (slabMin > tMax || tMin > slabMax) return false;
        tMin = gmax(tMin, slabMin);
        tMax = gmin(tMax, slabMax);
    }
    const f3 bmin = F3(m.bmin[0], m.bmin[1], m.bmin[2]), bmax = F3(m.bmax[0], m.bmax[1], m.bmax[2]);
    it.tMax = tMax;
    it.tCurrent = gmax(0.f, tMin);
    f3 pE = add(o, muls(d, it.tCurrent));
    f3 pX = add(o, muls(d, tMax));
    const f3 bs = sub(bmax, bmin);
    pE = sub(pE, bmin);
    pE = m.bs_pow2 == 7u ? F3(pE.x * m.inv_bs[0], pE.y * m.inv_bs[1], pE.z * m.inv_bs[2])
                         : F3(pE.x / bs.x, pE.y / bs.y, pE.z / bs.z);
    pE = F3(gmax(gmin(pE.x, 0.999999f), 0.f), gmax(gmin(pE.y, 0.999999f), 0.f), gmax(gmin(pE.z, 0.999999f), 0.f));
    pE = muls(pE, 1.f);
    it.idx = 0;
    pX = sub(pX, bmin);
    pX = m.bs_pow2 == 7u ? F3(pX.x * m.inv_bs[0], pX.y * m.inv_bs[1], pX.z * m.inv_bs[2])
                         : F3(pX.x / bs.x, pX.y / bs.y, pX.z / bs.z);
    pX = F3(gmax(gmin(pX.x, 0.999999f), 0.f), gmax(gmin(pX.y, 0.999999f), 0.f), gmax(gmin(pX.z, 0.999999f), 0.f));
    pX = muls(pX, 1.f);
    f3 gD = normalize(sub(pX, pE));
    if (pX.x == pE.x && pX.y == pE.y && pX.z == pE.z) gD = F3(1.f, 0.f, 0.f);
    it.gD = gD;  // crossDistance: cross_at, when Next() needs it
    it.pend = 0;
    float t3[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float pe = comp(pE, i), g = comp(gD, i);
        if (comp(d, i) >= 0.f) t3[i] = gabs((ceilf(pe + 0.00001f) - pe) / g);
        else t3[i] = gabs((floorf(pe - 0.00001f) - pe) / g);
        if (g == 0.f) t3[i] = __builtin_inff();
    }
    it.next = muls(mul(F3(t3[0], t3[1], t3[2]), bs), 1.f);
    it.stepPos = (gD.x < 0.f ? 0u : 1u) | (gD.y < 0.f ? 0u : 2u) | (gD.z < 0.f ? 0u : 4u);
    return true;
}

ND bool maj_next(const DMedium& m, MajIter& it, float& sigma, float& t0, float& t1, uint32_t* used = nullptr) {  // media.cpp:214-255
    if (it.tCurrent + 0.0001f > it.tMax) return false;
    if (it.pend) {  // the crossDistance the previous call stored in nextCrossing
        const int a = (int)it.pend - 1;
        const float c = cross_at(m, it, a);
        it.next.x = a == 0 ? c : it.next.x;
        it.next.y = a == 1 ? c : it.next.y;
        it.next.z = a == 2 ? c : it.next.z;
        it.pend = 0;
    }
    uint32_t choice = 0;
    if (it.next.x < it.next.y) choice += 4;
    if (it.next.x < it.next.z) choice += 2;
    if (it.next.y < it.next.z) choice += 1;
    // choiceMap {2, 1, 0, 1, 2, 0, 0, 0}
    const int index = (choice == 0 || choice == 4) ? 2 : (choice == 1 || choice == 3) ? 1 : 0;
    const float dt = index == 0 ? it.next.x : index == 1 ? it.next.y : it.next.z;
    if (it.idx > 7) return false;  // past the Medium object: undefined in the reference
    // selects only (an indexed form made the compiler keep the iterator in scratch memory)
    float sm = m.maj[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) sm = (int)it.idx == j ? m.maj[j] : sm;
    sigma = sm;
    if (used) *used = it.idx;
    t0 = it.tCurrent;
    t1 = it.tCurrent + dt;
    // nextCrossing -= dt; nextCrossing[index] = crossDistance[index] (formed by the next call)
    it.next.x -= dt;
    it.next.y -= dt;
    it.next.z -= dt;
    it.pend = (uint32_t)index + 1u;
    it.idx += (it.stepPos >> index) & 1u;
    it.tCurrent += dt;
    return true;
}

// VolumeIntegrator::Li_alpha (volumeintegrator.cpp:3-84) with SampleT_maj (media.h:128-181)
// inlined -- T_maj only feeds an unused callback argument, so its exp() factors are not evaluated
// -- as a per-lane state machine.  Running each sample to completion (the round-1 kernel, retired
// in round 5) made a wave wait for its slowest lane at every sample: sum_s max_lane(collisions),
// several times the mean for the roughly geometric collision counts.  Here one loop iteration
// advances every lane by one tentative collision (plus whatever cheap steps lead up to it: a new
// sample, a new ray segment, the next majorant segment), and a lane whose sample ends starts its
// next sample at once, so the wave costs about max_lane sum_s(collisions).  Each lane performs
// exactly the reference's RNG draws and float operations in its order: bit-identical.
// WV: minimum waves per SIMD requested from the register allocator (dispatch_volume: 4 on
// throughput-bound launches, 1 on small shards)
#ifndef NART_VOL_WV
#define NART_VOL_WV 4  // waves per SIMD of the throughput-bound launches (dispatch_volume)
#endif
template <bool COUNT, int WV>
__global__ __launch_bounds__(256, WV) void k_render_volume_sm(DScene S, RenderArgs A) {
    // A.lds_nodes != 0: the density grid (that many floats) is staged in LDS
    extern __shared__ float s_dens[];
    // glibc logf's (invc, logc) table: one LDS read per tentative collision instead of a
    // 16-way select of double pairs (~80 VALU instructions)
    __shared__ double2 s_logf[16];
    if (threadIdx.x < 16) {
        double invc, logc;
        logf_table((int)threadIdx.x, invc, logc);
        s_logf[threadIdx.x] = make_double2(invc, logc);
    }
    // the medium stays in the kernel arguments (a local copy with its density pointer swapped
    // lived in scratch memory: every field read in the loop was a scratch load)
    const float* dens = S.medium.density;
    if (A.lds_nodes) {
        for (uint32_t i = threadIdx.x; i < A.lds_nodes; i += blockDim.x) s_dens[i] = S.medium.density[i];
        dens = s_dens;
    }
    __syncthreads();
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t qlen = A.qlen ? A.qlen : A.n_slots;  // queue entries (sparse waves: > n_slots)
    if (gid >= qlen) return;
    uint32_t slot = A.queue ? A.queue[gid] : gid;
    if (slot == 0xFFFFFFFFu) return;  // an idle lane of a sparse wave (dispatch_volume)
    uint32_t px = 0, py = 0, rng = 0;
    SlotSO so;
    const float2* smp = nullptr;
    float4* out = nullptr;
    // The lane's next LatinSquare samples.  Pixel-major rows (stride 1): four samples per 32-B load
    // pair, issued when the last sample of the previous quad starts -- so a sample never waits for
    // its own load, and each read of a line no other lane shares serves four samples (the single
    // 8-B loads re-fetched a lane's line for every sample once other lanes' lines and the sky's
    // texels had evicted it: 212 GB fetched per C5 launch for 17 GB of samples; with no sample
    // loads at all the launch fetched 0.4 GB, profiles/r06m_volume_ablation.log; pairs: 91 GB).
    // Other layouts: one sample ahead, in nq.xy.
    float4 nq = make_float4(0.f, 0.f, 0.f, 0.f), nq1 = nq;
    bool pairs = false;
    // Results of pixel-major rows go out four at a time (64 contiguous bytes per lane, one line
    // sector written whole instead of four partial 16-B writes: 80 GB written per C5 launch for
    // 34 GB of results), staged in s_out[k][thread]
    __shared__ float4 s_outq[4][256];
    auto take = [&](uint32_t sl) {
        slot = sl;
        const uint32_t xy = A.slot_xy[sl];
        px = xy & 0xFFFFu;
        py = xy >> 16;
        rng = A.rng0[sl];
        so = A.slot_so[sl];
        smp = A.samples + so.first;
        out = A.Lout + so.first;
    };
    take(slot);
    pairs = so.stride == 1u && (so.first & 3u) == 0u && (A.spp & 3u) == 0u;
    if (pairs) {
        nq = reinterpret_cast<const float4*>(smp)[0];
        nq1 = reinterpret_cast<const float4*>(smp)[1];
    } else {
        nq = make_float4(smp[0].x, smp[0].y, 0.f, 0.f);
    }
    const DMedium& m = S.medium;
    const f3 beta = F3(1.f, 1.f, 1.f);
    enum { P_SAMPLE, P_RAY, P_MAJ, P_COLL, P_ESC, P_SCAT };
    uint32_t work = 0, s = 0, bounce = 0;
    // a sample's Li_alpha: staged and written in fours (pixel-major rows), else at once
    auto emit = [&](float4 v) {
        if (!pairs) {
            out[(size_t)s * so.stride] = v;
            return;
        }
        s_outq[s & 3u][threadIdx.x] = v;
        if ((s & 3u) == 3u) {
            float4* o4 = out + (s & ~3u);
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) o4[j] = s_outq[j][threadIdx.x];
        }
    };
    int ph = P_SAMPLE;
    f3 o = F3(0.f, 0.f, 0.f), d = o, ro = o, rd = o, L = o;
    float uMode = 0.f, sigma = 1.f, tMin = 0.f, t1 = 0.f;
    uint32_t sidx = 0;  // majorant entry of the current segment (sigma = m.maj[sidx])
    MajIter it;
    for (;;) {
        bool finish = false;
        // The scattering phase's UniformSampleSphere (volumeintegrator.cpp:44-47) and the escape
        // phase's environment lookup (environmentlight.cpp:9-28) both begin with an acosf: one
        // evaluation per lane per iteration serves the lane's phase.  The escape phase therefore
        // runs at the top of the iteration after the one that chose it (and the lane starts its
        // next sample in that same iteration, as before): each lane's operations and their order
        // are unchanged.
        const bool scat = ph == P_SCAT, esc = ph == P_ESC;
        float sa = 0.f, sb = 0.f, theta = 0.f;
        if (scat) {
            sa = rng_float(rng);
            sb = rng_float(rng);
        }
        if (scat || esc) theta = glibc_acosf(scat ? 1.f - (2.f * sa) : d.z);
        if (esc) {
            float lightTMax = __builtin_inff();
            f3 Le = F3(0.f, 0.f, 0.f);
            for (uint32_t j = 0; j < S.num_lights; ++j) {
                float lt = __builtin_inff();
                const f3 Li = light_li(S, uniform_light(S, j), o, d, nullptr, lt, theta);
                if (lt < lightTMax) {
                    Le = Li;
                    lightTMax = lt;
                }
            }
            L = add(L, mul(Le, beta));
            emit(make_float4(L.x, L.y, L.z, 1.f));
            ++s;
            ph = P_SAMPLE;
        }
        if (ph == P_SAMPLE) {
            if (s >= A.spp) break;
            float2 sm;
            if (pairs) {
                const float4 h = (s & 2u) ? nq1 : nq;
                sm = (s & 1u) ? make_float2(h.z, h.w) : make_float2(h.x, h.y);
                // the last sample of a quad starts: load the next quad (the last quad reloads itself)
                if ((s & 3u) == 3u) {
                    const float4* q = reinterpret_cast<const float4*>(smp) + ((s + 1u < A.spp ? s + 1u : s - 3u) >> 1);
                    nq = q[0];
                    nq1 = q[1];
                }
            } else {
                sm = make_float2(nq.x, nq.y);
                const float2 n1 = smp[(size_t)(s + 1u < A.spp ? s + 1u : s) * so.stride];
                nq = make_float4(n1.x, n1.y, 0.f, 0.f);
            }
            const Ray r = cast_ray(S, F2(sm.x, sm.y), A.W, A.H, px, py);
            o = r.o;
            d = r.d;
            L = F3(0.f, 0.f, 0.f);
            bounce = 0;
            ph = P_RAY;
        }
        if (scat) {  // the rest of UniformSampleSphere (sampling.cpp:33-45)
            const float phi = sb * ND_TWO_PI;
            float cosTheta, sinTheta, cosPhi, sinPhi;
            glibc_sincosf(theta, sinTheta, cosTheta);
            glibc_sincosf(phi, sinPhi, cosPhi);
            d = F3(sinTheta * cosPhi, sinTheta * sinPhi, cosTheta);
            ph = P_RAY;
        }
        if (ph == P_RAY) {  // top of VolumeIntegrator's bounce loop
            (void)rng_float(rng);  // u: passed to SampleT_maj, unused there
            uMode = rng_float(rng);
            if (m.present && medium_sample_ray(m, o, d, it)) {
                ro = o;
                rd = d;
                ph = P_MAJ;
            } else {
                ph = P_ESC;
            }
        }
        if (ph == P_MAJ) {
            float t0;
            if (maj_next(m, it, sigma, t0, t1, &sidx)) {
                tMin = t0;
                ph = P_COLL;
            } else {
                ph = P_ESC;
            }
        }
        if (ph == P_COLL) {
            ++work;
            // sigma a power of two for every lane of the wave: multiply by its exact reciprocal
            const bool sp2 = __ballot(!((m.maj_pow2 >> sidx) & 1u)) == 0;
            float isig = m.inv_maj[0];
#pragma unroll
            for (int j = 1; j < 8; ++j) isig = (int)sidx == j ? m.inv_maj[j] : isig;
            const float lg = -glibc_logf_with(1.f - rng_float(rng), [&](int i, double& invc, double& logc) {
                const double2 e = s_logf[i];
                invc = e.x;
                logc = e.y;
            });
            float t;
            if (sp2) t = tMin + lg * isig;
            else t = tMin + lg / sigma;
            if (!(t < t1)) {
                ph = P_MAJ;
            } else {
                const f3 p = add(ro, muls(rd, t));
                if (p.x < m.bmin[0] || p.y < m.bmin[1] || p.z < m.bmin[2] || p.x > m.bmax[0] || p.y > m.bmax[1] ||
                    p.z > m.bmax[2]) {
                    ph = P_ESC;
                } else {
                    const f3 bmin = F3(m.bmin[0], m.bmin[1], m.bmin[2]);
                    const f3 bs = sub(F3(m.bmax[0], m.bmax[1], m.bmax[2]), bmin);
                    const f3 q0 = sub(p, bmin);
                    const f3 qn = m.bs_pow2 == 7u ? F3(q0.x * m.inv_bs[0], q0.y * m.inv_bs[1], q0.z * m.inv_bs[2])
                                                  : F3(q0.x / bs.x, q0.y / bs.y, q0.z / bs.z);
                    const float density = m.grid2 ? dg_lookup2(m, qn) : dg_lookup(m, dens, qn);
                    const float ca = m.sigma_a * density, cs = m.sigma_s * density;
                    float pAbsorb, pScatter;
                    if (sp2) {
                        pAbsorb = ca * isig;
                        pScatter = cs * isig;
                    } else {
                        pAbsorb = ca / sigma;
                        pScatter = cs / sigma;
                    }
                    if (uMode < pAbsorb) {
                        L = add(L, mul(muls(F3(m.Le[0], m.Le[1], m.Le[2]), density), beta));
                        finish = true;
                    } else if (uMode < pAbsorb + pScatter) {
                        if (bounce++ > A.bounces) {
                            finish = true;
                        } else {
                            o = p;
                            ph = P_SCAT;
                        }
                    } else {
                        uMode = rng_float(rng);  // null collision
                        tMin = t;
                    }
                }
            }
        }
        if (finish) {
            emit(make_float4(L.x, L.y, L.z, 1.f));
            ++s;
            ph = P_SAMPLE;
        }
    }
    if (A.cost) {
        A.cost[gid] = work + A.spp;
        return;
    }
    if (COUNT) atomicAdd(&A.counters[0], (unsigned long long)A.spp);
}

}  // namespace nd
