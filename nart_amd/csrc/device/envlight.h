// Light::Li / Light::Sample_Li dispatch for the device path: disk and ring area lights and the
// lat-long environment light (environmentlight.cpp:9-79) with its Piecewise2DDistribution
// importance sampling (texturepattern.cpp:3-170).  acosf / atan2f / sinf / cosf are the glibc
// restatements of dmath.h, so the mapping rounds exactly as the reference's libm.
#pragma once

namespace nd {

#define ENV_TMAX 2139095040.0f  // (float)0x7f7fffff (environmentlight.cpp:26, 59)

// TexturePattern::Pdf / ConstantPattern::Pdf of the env light's Le (texturepattern.cpp:160-170)
ND float env_ptn_pdf(const DScene& S, const DLight& L, f2 st) {
    if (L.Le.type == NART_PTN_CONSTANT || L.env < 0) return 1.f;
    return env_pdf(cst(S.envs)[L.env], F2(gmin(st.x, 0.9999f), gmin(st.y, 0.9999f)));
}

// Light::Li (disklight.cpp:12-23, ringlight.cpp:13-24, environmentlight.cpp:9-28).
// ENV = false compiles the environment branch out (scenes without one): it costs registers.
// theta_in: acosf(wi.z) already formed by the caller (k_render_volume_sm shares that evaluation
// with its scattering phase), or NAN to form it here
template <bool ENV = true, uint32_t FM = FT_ALL>
ND f3 light_li(const DScene& S, const DLight& L, f3 p, f3 wi, float* pdf, float& tMax,
               float theta_in = __builtin_nanf("")) {
    if (ENV && L.type == NART_LIGHT_ENVIRONMENT) {
        const float theta = theta_in == theta_in ? theta_in : glibc_acosf(wi.z);
        float phi = glibc_atan2f(wi.y, wi.x) + ND_PI;
        if (phi > ND_TWO_PI) phi -= ND_TWO_PI;
        if (phi < 0.f) phi += ND_TWO_PI;
        const f2 est = F2(1.f - (phi * ND_ONE_OVER_TWO_PI), 1.f - (theta * ND_ONE_OVER_PI));
        if (pdf) {
            *pdf = env_ptn_pdf(S, L, est);
            *pdf *= ND_ONE_OVER_PI * 0.25f / gabs(glibc_sinf(theta));
        }
        tMax = ENV_TMAX;
        return muls(ptn_value<FM>(S, L.Le, est), L.intensity);
    }
    f2 st = F2(0.f, 0.f);
    float lp = area_pdf<FM>(L, p, wi, st, tMax);
    if (lp > 0.f) {
        if (pdf) *pdf = lp;
        return muls(ptn_value<FM>(S, L.Le, st), L.intensity);
    }
    return F3(0.f, 0.f, 0.f);
}

// A light record at a wave-uniform index (the light loops' j), read through the constant address
// space (cst, dscene.h): the compiler then reads its fields with scalar loads.
ND const DLight& uniform_light(const DScene& S, uint32_t j) { return cst(S.lights)[j]; }

// The light loop of an extension ray (pathintegrator.cpp:171-182) when its Le cannot reach L: Le
// is used only when the camera ray escapes (pathintegrator.cpp:252-256, Q7), so for every other
// ray the loop needs just the bound tMax (and whether it was lowered), which this sets exactly as
// light_li does -- without the radiance: for the environment light the acosf / atan2f and the
// texture fetch, a dependent global load.
template <bool ENV = true, uint32_t FM = FT_ALL>
ND void light_bound(const DLight& L, f3 p, f3 wi, float& tMax) {
    if (ENV && L.type == NART_LIGHT_ENVIRONMENT) {
        tMax = ENV_TMAX;
        return;
    }
    f2 st = F2(0.f, 0.f);
    (void)area_pdf<FM>(L, p, wi, st, tMax);
}

// Light::Sample_Li (disklight.cpp:25-60, ringlight.cpp:26-64)
template <bool ENV = true, uint32_t FM = FT_ALL>
ND f3 light_sample_li(const DScene& S, const DLight& L, f3 p, f3& wi, f2 sample, float& pdf, float& tMax) {
    if (ENV && L.type == NART_LIGHT_ENVIRONMENT) {
        // Pattern::Sample (constantpattern.cpp:3-14, texturepattern.cpp:130-158)
        f2 ps = sample;
        f3 Lv;
        if (!(FM & FT_TEX) || L.Le.type == NART_PTN_CONSTANT) {
            pdf = 1.f;
            Lv = F3(L.Le.v[0], L.Le.v[1], L.Le.v[2]);
        } else {
            if (L.env < 0) pdf = 1.f;
            else ps = env_sample(cst(S.envs)[L.env], sample, pdf);  // leaves pdf as is on a zero row
            Lv = tex_fetch(S, L.Le.tex, ps.x, ps.y, L.Le.rough);
        }
        Lv = muls(Lv, L.intensity);
        const float theta = (1.f - ps.y) * ND_PI;
        float phi = (1.f - ps.x) * 2.f * ND_PI;
        phi += ND_PI;
        if (phi > ND_TWO_PI) phi -= ND_TWO_PI;
        if (phi < 0.f) phi += ND_TWO_PI;
        float st, ct, sp, cp;
        glibc_sincosf(theta, st, ct);
        glibc_sincosf(phi, sp, cp);
        wi = F3(cp * st, sp * st, ct);
        pdf *= ND_ONE_OVER_PI * 0.25f / gabs(st);
        tMax = ENV_TMAX;
        return Lv;
    }
    f4 ds;
    if ((FM & FT_RING) && L.type == NART_LIGHT_RING) {
        f2 r = uniform_sample_ring(sample, pdf, L.inner_ratio);
        ds = F4(r.x * L.radius, r.y * L.radius, 0.f, 1.f);
    } else {
        f2 r = uniform_sample_disk(sample);
        ds = F4(r.x * L.radius, r.y * L.radius, 0.f, 1.f);
    }
    float u = ((ds.x + 1.f) * 0.5f) / L.radius;
    float v = ((ds.y + 1.f) * 0.5f) / L.radius;
    f2 st = F2(u, 1.f - v);
    ds = vec_mul_mat(ds, L.m);
    f3 n = load3(L.n);
    wi = sub(xyz(ds), p);
    float dist = sqrtf(wi.x * wi.x + wi.y * wi.y + wi.z * wi.z);
    wi = normalize(wi);
    if ((FM & FT_RING) && L.type == NART_LIGHT_RING) pdf /= (ND_PI * L.radius * L.radius);
    else pdf = L.pdf_area;
    float wiDotN = dot(neg(wi), n);
    if (wiDotN <= 0.f) {
        pdf = 0.f;
        return F3(0.f, 0.f, 0.f);
    }
    pdf = pdf * ((dist * dist) / wiDotN);
    tMax = dist;
    return muls(ptn_value<FM>(S, L.Le, st), L.intensity);
}

}  // namespace nd
