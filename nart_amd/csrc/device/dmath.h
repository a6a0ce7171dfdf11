// Device arithmetic for the nart render path (gfx950).
//
// Every operation reproduces the reference's float semantics bit for bit:
//  * GLM 0.9.9.8 scalar code paths (association order of dot/normalize/mat*vec, ternary
//    min/max, abs(x) = x >= 0 ? x : -x, fract, mod, mix);
//  * correctly rounded f32 division and sqrt (hipcc default
//    -fhip-fp32-correctly-rounded-divide-sqrt) and no FMA contraction (-ffp-contract=off);
//  * sinf/cosf are glibc 2.35's algorithm (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c,
//    sincosf.h: double-precision range reduction + polynomials), verified bit-exact against
//    the host libm over every float in [-7, 7] (tests/test_libm_parity.py).
//
// Third-party notices.  The sinf/cosf/logf ports restate algorithms and constant tables of the
// GNU C Library 2.35 (sysdeps/ieee754/flt-32; those files are Copyright (C) 2017-2022 Free
// Software Foundation, Inc. and Arm Ltd., licensed under the GNU Lesser General Public License
// v2.1 or later).  The acosf/atanf/atan2f ports restate fdlibm's single-precision algorithms as
// shipped in glibc ("Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
// Developed at SunPro, a Sun Microsystems, Inc. business.  Permission to use, copy, modify, and
// distribute this software is freely granted, provided that this notice is preserved.").
// They are needed to reproduce the reference's glm::sin/cos/acos/atan/log results bit for bit.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define ND __device__ __forceinline__
#define NHD __host__ __device__ __forceinline__

namespace nd {

struct f2 { float x, y; };
struct f3 { float x, y, z; };
struct f4 { float x, y, z, w; };

NHD f2 F2(float x, float y) { f2 r; r.x = x; r.y = y; return r; }
NHD f3 F3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
NHD f4 F4(float x, float y, float z, float w) { f4 r; r.x = x; r.y = y; r.z = z; r.w = w; return r; }
NHD f3 add(f3 a, f3 b) { return F3(a.x + b.x, a.y + b.y, a.z + b.z); }
NHD f3 sub(f3 a, f3 b) { return F3(a.x - b.x, a.y - b.y, a.z - b.z); }
NHD f3 mul(f3 a, f3 b) { return F3(a.x * b.x, a.y * b.y, a.z * b.z); }
NHD f3 muls(f3 a, float s) { return F3(a.x * s, a.y * s, a.z * s); }
NHD f3 divs(f3 a, float s) { return F3(a.x / s, a.y / s, a.z / s); }
NHD f3 neg(f3 a) { return F3(-a.x, -a.y, -a.z); }
NHD float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
NHD float dot4(f4 a, f4 b) { return (a.x * b.x + a.y * b.y) + (a.z * b.z + a.w * b.w); }
NHD f3 cross(f3 x, f3 y) { return F3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y); }
NHD f3 normalize(f3 v) { float s = 1.f / sqrtf(dot(v, v)); return muls(v, s); }
NHD f4 normalize4(f4 v) { float s = 1.f / sqrtf(dot4(v, v)); return F4(v.x * s, v.y * s, v.z * s, v.w * s); }
NHD float gmin(float a, float b) { return (b < a) ? b : a; }
NHD float gmax(float a, float b) { return (a < b) ? b : a; }
NHD float gabs(float x) { return x >= 0.f ? x : -x; }
NHD float gfract(float x) { return x - floorf(x); }
NHD float gmod(float a, float b) { return a - b * floorf(a / b); }
NHD float gmix(float x, float y, float a) { return x * (1.f - a) + y * a; }
NHD float comp(f3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
// row vector * glm::mat4 (m[c*4+r]): r_i = m[i][0]v0 + m[i][1]v1 + m[i][2]v2 + m[i][3]v3
NHD f4 vec_mul_mat(f4 v, const float* m) {
    f4 r;
    r.x = ((m[0] * v.x + m[1] * v.y) + m[2] * v.z) + m[3] * v.w;
    r.y = ((m[4] * v.x + m[5] * v.y) + m[6] * v.z) + m[7] * v.w;
    r.z = ((m[8] * v.x + m[9] * v.y) + m[10] * v.z) + m[11] * v.w;
    r.w = ((m[12] * v.x + m[13] * v.y) + m[14] * v.z) + m[15] * v.w;
    return r;
}
NHD f3 xyz(f4 v) { return F3(v.x, v.y, v.z); }

// static_cast<uint32_t>(float) as the reference's x86-64 build evaluates it
// (cvttss2si to 64 bits, low 32 bits; NaN / out of range -> 0).
NHD uint32_t f2u32(float f) {
    if (f >= 0.f && f < 4294967296.f) return (uint32_t)f;
    if (!(f > -9.2233715e18f && f < 9.2233715e18f)) return 0u;
    return (uint32_t)(int64_t)f;
}
NHD uint8_t f2u8(float f) { return (uint8_t)f2u32(f); }

// glm constants: genType(<double literal>)
#define ND_PI ((float)3.14159265358979323846264338327950288)
#define ND_TWO_PI ((float)6.28318530717958647692528676655900576)
#define ND_ONE_OVER_PI ((float)0.318309886183790671537767526745028724)
#define ND_ONE_OVER_TWO_PI ((float)0.159154943091895335768883763372514362)
#define ND_EPS 1.1920928955078125e-07f
#define ND_ONE_MINUS_EPS (1.f - 1.1920928955078125e-07f)

// ---------------------------------------------------------------- glibc sinf / cosf
struct SinCosT {
    double sign[4];
    double hpi_inv, hpi, c0, c1, c2, c3, c4, s1, s2, s3;
};

// __sincosf_table (glibc sysdeps/ieee754/flt-32/s_sincosf_data.c), !TOINT_INTRINSICS:
// entry 1 is entry 0 with the cosine polynomial negated (multiplying by +-1 is exact).
NHD SinCosT sincos_table(int k) {
    const double c = k ? -1.0 : 1.0;
    SinCosT t = {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, c * 0x1p0,
                 c * -0x1.ffffffd0c621cp-2, c * 0x1.55553e1068f19p-5, c * -0x1.6c087e89a359dp-10,
                 c * 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13};
    return t;
}
NHD uint32_t abstop12(float x) { return (__builtin_bit_cast(uint32_t, x) >> 20) & 0x7ff; }
NHD float sinf_poly(double x, double x2, const SinCosT* p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = p->s2 + x2 * p->s3;
        double x7 = x3 * x2;
        double s = x + x3 * p->s1;
        return (float)(s + x7 * s1);
    }
    double x4 = x2 * x2;
    double c2 = p->c3 + x2 * p->c4;
    double c1 = p->c0 + x2 * p->c1;
    double x6 = x4 * x2;
    double c = c1 + x4 * p->c2;
    return (float)(c + x6 * c2);
}
NHD double reduce_fast(double x, const SinCosT* p, int* np) {
    double r = x * p->hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return x - n * p->hpi;
}
// sinf and cosf of one argument (glibc's sinf / cosf / sincosf share this reduction), without
// branches: a wave whose lanes fall on both sides of glibc's |y| < pi/4 test used to run both
// paths.  For 2^-12 <= |y| < 0.75 (abstop12(y) < abstop12(pi/4)) glibc evaluates the polynomials
// on y itself, which is exactly the reduced path with n = 0 (x - 0 * pi/2 = x, sign +1, table
// 0); below 2^-12 it returns y and 1.  The cosine polynomial of table 1 is table 0's with every
// coefficient negated, i.e. exactly the negated value, so both polynomials are evaluated once
// and assigned by the parity of n.  Valid for |y| < 120 (the reference only evaluates angles in
// [0, 2*pi]); larger inputs would need glibc's reduce_large, which the render path never reaches.
NHD void glibc_sincosf(float y, float& sn, float& cs) {
    const SinCosT t0 = sincos_table(0);
    int n;
    const double x = reduce_fast((double)y, &t0, &n);
    const double sg = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;  // t0.sign[n & 3]
    const double x2 = x * x;
    const float ps = sinf_poly(x * sg, x2, &t0, 0);  // sine polynomial (either table)
    float pc = sinf_poly(x * sg, x2, &t0, 1);        // cosine polynomial, table 0
    pc = (n & 2) ? -pc : pc;                          // table 1
    const bool tiny = abstop12(y) < abstop12(0x1p-12f);
    sn = tiny ? y : ((n & 1) ? pc : ps);
    cs = tiny ? 1.0f : ((n & 1) ? ps : pc);
}
NHD float glibc_sinf(float y) {
    float s, c;
    glibc_sincosf(y, s, c);
    return s;
}
NHD float glibc_cosf(float y) {
    float s, c;
    glibc_sincosf(y, s, c);
    return c;
}

// ---------------------------------------------------------------- RNG (rng.h:8-59)
ND uint32_t xorshift(uint32_t y) {
    y ^= (y << 13);
    y ^= (y >> 17);
    y ^= (y << 5);
    return y;
}
// ---------------------------------------------------------------- glibc 2.35 acosf / atanf / atan2f
// sysdeps/ieee754/flt-32/{e_acosf,s_atanf,e_atan2f}.c: the fdlibm single-precision algorithms,
// plain float arithmetic (no FMA contraction on x86-64).  Restated so the environment light's
// lat-long mapping (environmentlight.cpp:9-28) rounds exactly as the reference's libm does;
// tests/native/libm_port_check.cpp compares them with this host's glibc.
NHD float fbits(uint32_t u) { return __builtin_bit_cast(float, u); }
NHD uint32_t ubits(float f) { return __builtin_bit_cast(uint32_t, f); }

NHD float acosf_rpoly(float z) {
    const float pS0 = fbits(0x3e2aaaabu), pS1 = fbits(0xbea6b090u), pS2 = fbits(0x3e4e0aa8u),
                pS3 = fbits(0xbd241146u), pS4 = fbits(0x3a4f7f04u), pS5 = fbits(0x3811ef08u),
                qS1 = fbits(0xc019d139u), qS2 = fbits(0x4001572du), qS3 = fbits(0xbf303361u),
                qS4 = fbits(0x3d9dc62eu);
    float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    float q = 1.0f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    return p / q;
}
// The three argument ranges of the main path (|x| < 0.5, x < -0.5, x > 0.5) share one
// polynomial-quotient evaluation on the range's z, one sqrt and one division, selected per lane
// instead of branched (a wave holding all three ranges ran three quotients, two sqrts and four
// divisions); each lane's result is its range's expression, operation for operation.
NHD float glibc_acosf(float x) {
    const float pi = fbits(0x40490fdau), pio2_hi = fbits(0x3fc90fdau), pio2_lo = fbits(0x33a22168u);
    const int32_t hx = (int32_t)ubits(x);
    const int32_t ix = hx & 0x7fffffff;
    if (ix == 0x3f800000) return hx > 0 ? 0.0f : pi + 2.0f * pio2_lo;
    if (ix > 0x3f800000) return (x - x) / (x - x);
    if (ix <= 0x32800000) return pio2_hi + pio2_lo;  // |x| < 2^-26 (inside |x| < 0.5)
    const bool mid = ix < 0x3f000000, neg = hx < 0;   // |x| < 0.5; else x < -0.5 / x > 0.5
    const float z = mid ? x * x : (neg ? (1.0f + x) * 0.5f : (1.0f - x) * 0.5f);
    const float r = acosf_rpoly(z);
    const float s = sqrtf(z);
    const float df = fbits(ubits(s) & 0xfffff000u);
    const float c = (z - df * df) / (s + df);
    const float a_mid = pio2_hi - (x - (pio2_lo - x * r));
    const float a_neg = pi - 2.0f * (s + (r * s - pio2_lo));
    const float a_pos = 2.0f * (df + (r * s + c));
    return mid ? a_mid : (neg ? a_neg : a_pos);
}

NHD float glibc_atanf(float x) {
    const float atanhi[4] = {fbits(0x3eed6338u), fbits(0x3f490fdau), fbits(0x3f7b985eu), fbits(0x3fc90fdau)};
    const float atanlo[4] = {fbits(0x31ac3769u), fbits(0x33222168u), fbits(0x33140fb4u), fbits(0x33a22168u)};
    const float aT0 = fbits(0x3eaaaaabu), aT1 = fbits(0xbe4ccccdu), aT2 = fbits(0x3e124925u),
                aT3 = fbits(0xbde38e38u), aT4 = fbits(0x3dba2e6eu), aT5 = fbits(0xbd9d8795u),
                aT6 = fbits(0x3d886b35u), aT7 = fbits(0xbd6ef16bu), aT8 = fbits(0x3d4bda59u),
                aT9 = fbits(0xbd15a221u), aT10 = fbits(0x3c8569d7u);
    const int32_t hx = (int32_t)ubits(x);
    const int32_t ix = hx & 0x7fffffff;
    if (ix >= 0x4c000000) {  // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x31000000) return x;  // |x| < 2^-29
    // the argument reduction's four quotients as one division of selected operands (per lane
    // the same numerator and denominator expressions; lanes of the |x| < 0.4375 range discard it)
    const int id = ix < 0x3ee00000 ? -1 : ix < 0x3f300000 ? 0 : ix < 0x3f980000 ? 1 : ix < 0x401c0000 ? 2 : 3;
    const float ax = fabsf(x);
    const float num = id == 0 ? 2.0f * ax - 1.0f : id == 1 ? ax - 1.0f : id == 2 ? ax - 1.5f : -1.0f;
    const float den = id == 0 ? 2.0f + ax : id == 1 ? ax + 1.0f : id == 2 ? 1.0f + 1.5f * ax : ax;
    const float q = num / den;
    x = id < 0 ? x : q;
    float z = x * x;
    float w = z * z;
    float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    const float small = x - x * (s1 + s2);
    const float hi = id == 0 ? atanhi[0] : id == 1 ? atanhi[1] : id == 2 ? atanhi[2] : atanhi[3];
    const float lo = id == 0 ? atanlo[0] : id == 1 ? atanlo[1] : id == 2 ? atanlo[2] : atanlo[3];
    z = hi - ((x * (s1 + s2) - lo) - x);
    return id < 0 ? small : (hx < 0 ? -z : z);
}

NHD float glibc_atan2f(float y, float x) {
    const float tiny = 1.0e-30f, pi_o_4 = fbits(0x3f490fdbu), pi_o_2 = fbits(0x3fc90fdbu),
                pi = fbits(0x40490fdbu), pi_lo = fbits(0xb3bbbd2eu);
    const int32_t hx = (int32_t)ubits(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)ubits(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return glibc_atanf(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        if (m <= 1) return y;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            if (m == 0) return pi_o_4 + tiny;
            if (m == 1) return -pi_o_4 - tiny;
            if (m == 2) return 3.0f * pi_o_4 + tiny;
            return -3.0f * pi_o_4 - tiny;
        }
        if (m == 0) return 0.0f;
        if (m == 1) return -0.0f;
        if (m == 2) return pi + tiny;
        return -pi - tiny;
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else z = glibc_atanf(fabsf(y / x));
    if (m == 0) return z;
    if (m == 1) return fbits(ubits(z) ^ 0x80000000u);
    if (m == 2) return pi - (z - pi_lo);
    return (z - pi_lo) - pi;
}

// glibc 2.35 logf (sysdeps/ieee754/flt-32/e_logf.c, table e_logf_data.c, 16 intervals), in
// the form x86-64 glibc runs on FMA/AVX2 hosts (the __logf_fma ifunc: the double-precision
// steps contracted to fused multiply-adds).  SampleExponentialDecay (sampling.cpp:60-62).
// glibc's 16 (invc, logc) pairs, entry i selected without a memory table
NHD void logf_table(int i, double& invc, double& logc) {
    struct LogfT { double invc, logc; };
    const LogfT T[16] = {
        {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
        {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
        {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
        {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
        {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
        {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
        {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
        {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};
    invc = i == 0 ? T[0].invc : 0.0;
    logc = i == 0 ? T[0].logc : 0.0;
#pragma unroll
    for (int j = 1; j < 16; ++j)
        if (i == j) {
            invc = T[j].invc;
            logc = T[j].logc;
        }
}
// logf with the table entry supplied by lookup(i, invc, logc)
template <typename Lookup>
NHD float glibc_logf_with(float x, Lookup lookup) {
    const double Ln2 = 0x1.62e42fefa39efp-1, A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2,
                 A2 = -0x1.ffffef20a4123p-2;
    uint32_t ix = ubits(x);
    if (ix == 0x3f800000u) return 0.f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2 == 0) return -__builtin_inff();
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return __builtin_nanf("");
        ix = ubits(x * 0x1p23f);  // subnormal
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) % 16);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    double invc, logc;
    lookup(i, invc, logc);
    const double z = (double)fbits(iz);
    const double r = __builtin_fma(z, invc, -1.0);
    const double y0 = __builtin_fma((double)k, Ln2, logc);
    const double r2 = r * r;
    double y = __builtin_fma(r, A1, A2);
    y = __builtin_fma(r2, A0, y);
    y = __builtin_fma(r2, y, r + y0);
    return (float)y;
}
NHD float glibc_logf(float x) {
    return glibc_logf_with(x, [](int i, double& invc, double& logc) { logf_table(i, invc, logc); });
}

ND float rng_float(uint32_t& y) {
    y = xorshift(y);
    float f = (float)(uint32_t)(y * 0x9E3779BBu) * 2.3283064365386963e-10f;
    return gmin(ND_ONE_MINUS_EPS, f);
}
ND uint32_t rng_int(uint32_t& y, uint32_t max) {
    y = xorshift(y);
    return (uint32_t)(((uint64_t)(uint32_t)(y * 0x9E3779B9u) * ((uint64_t)max + 1)) >> 32);
}

// ---------------------------------------------------------------- sampling.cpp
ND f2 uniform_sample_disk(f2 s) {  // sampling.cpp:5-16
    float r = sqrtf(s.x);
    float theta = s.y * ND_TWO_PI;
    float c, sn;
    glibc_sincosf(theta, sn, c);
    return F2(r * c, r * sn);
}
ND f2 uniform_sample_ring(f2 s, float& pdf, float inner) {  // sampling.cpp:18-31
    float r = sqrtf(gmix(inner, 1.f, s.x));
    float theta = s.y * ND_TWO_PI;
    float c, sn;
    glibc_sincosf(theta, sn, c);
    pdf = 1.f / (ND_PI * (1.f - inner));
    return F2(r * c, r * sn);
}
ND f3 cosine_sample_hemisphere(f2 s, float& pdf) {  // sampling.cpp:47-58
    f2 d = uniform_sample_disk(s);
    float z = sqrtf(1.f - (d.x * d.x + d.y * d.y));
    pdf = z * ND_ONE_OVER_PI;
    return F3(d.x, d.y, z);
}

}  // namespace nd
