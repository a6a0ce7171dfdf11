// Light::Li / Light::Sample_Li dispatch for the device path (disk and ring area lights).
// The environment light (environmentlight.cpp:9-79) needs glibc-exact acosf/atan2f ports;
// until those land, nart_hip_create rejects scenes with an environment light
// (NART_E_UNSUPPORTED) instead of rendering them with a different libm.
#pragma once

namespace nd {

// Light::Li (disklight.cpp:12-23, ringlight.cpp:117-128)
ND f3 light_li(const DScene& S, const DLight& L, f3 p, f3 wi, float* pdf, float& tMax) {
    f2 st = F2(0.f, 0.f);
    float lp = area_pdf(L, p, wi, st, tMax);
    if (lp > 0.f) {
        if (pdf) *pdf = lp;
        return muls(ptn_value(S, L.Le, st), L.intensity);
    }
    return F3(0.f, 0.f, 0.f);
}

// Light::Sample_Li (disklight.cpp:25-60, ringlight.cpp:130-168)
ND f3 light_sample_li(const DScene& S, const DLight& L, f3 p, f3& wi, f2 sample, float& pdf, float& tMax) {
    f4 ds;
    if (L.type == NART_LIGHT_RING) {
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
    if (L.type == NART_LIGHT_RING) pdf /= (ND_PI * L.radius * L.radius);
    else pdf = L.pdf_area;
    float wiDotN = dot(neg(wi), n);
    if (wiDotN <= 0.f) {
        pdf = 0.f;
        return F3(0.f, 0.f, 0.f);
    }
    pdf = pdf * ((dist * dist) / wiDotN);
    tMax = dist;
    return muls(ptn_value(S, L.Le, st), L.intensity);
}

}  // namespace nd
