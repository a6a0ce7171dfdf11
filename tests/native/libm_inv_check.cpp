// Host build of the device acosf / atanf / atan2f ports (nart_amd/csrc/device/dmath.h) against
// this host's glibc.  TEST HELPER.
//   libm_inv_check acos STRIDE        every STRIDE-th float bit pattern in [-1, 1] (and beyond)
//   libm_inv_check atan STRIDE        every STRIDE-th bit pattern of both signs
//   libm_inv_check atan2 N SEED       N random (y, x) pairs: unit vectors, wide exponents, specials
//   libm_inv_check log STRIDE         every STRIDE-th positive float bit pattern
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>

#include "../../nart_amd/csrc/device/dmath.h"

static bool same(float a, float b) { return std::memcmp(&a, &b, 4) == 0 || (a != a && b != b); }

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const char* fn = argv[1];
    unsigned long n = 0, bad = 0;
    if (!std::strcmp(fn, "log")) {  // every STRIDE-th positive pattern up to +inf, and -1, -0
        unsigned stride = (unsigned)std::strtoul(argv[2], nullptr, 10);
        for (unsigned b = 0; b <= 0x7f800000u; b += stride) {
            float x;
            std::memcpy(&x, &b, 4);
            float r = nd::glibc_logf(x), h = logf(x);
            if (!same(r, h)) {
                if (bad < 5) std::printf("mismatch log(%a) port=%a glibc=%a\n", x, r, h);
                ++bad;
            }
            ++n;
        }
    } else if (!std::strcmp(fn, "acos") || !std::strcmp(fn, "atan")) {
        unsigned stride = (unsigned)std::strtoul(argv[2], nullptr, 10);
        bool acos = !std::strcmp(fn, "acos");
        unsigned top = acos ? 0x3f800010u : 0x7f800001u;
        for (unsigned b = 0; b <= top; b += stride) {
            for (int sgn = 0; sgn < 2; ++sgn) {
                float x;
                unsigned u = b | (sgn ? 0x80000000u : 0u);
                std::memcpy(&x, &u, 4);
                float r = acos ? nd::glibc_acosf(x) : nd::glibc_atanf(x);
                float h = acos ? acosf(x) : atanf(x);
                if (!same(r, h)) {
                    if (bad < 5) std::printf("mismatch %s(%a) port=%a glibc=%a\n", fn, x, r, h);
                    ++bad;
                }
                ++n;
            }
        }
    } else {
        unsigned long N = std::strtoul(argv[2], nullptr, 10);
        uint64_t st = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 1;
        auto next = [&]() { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; };
        const float specials[] = {0.f, -0.f, 1.f, -1.f, INFINITY, -INFINITY, 1e-38f, -1e-38f, 1e-45f, 3e38f};
        for (unsigned long i = 0; i < N; ++i) {
            float y, x;
            uint64_t r = next();
            int mode = (int)(r & 3);
            if (mode == 0) {  // unit vector components (the env light's use)
                double a = (double)(next() >> 11) * 0x1p-53 * 6.283185307179586, c = (double)(next() >> 11) * 0x1p-53;
                float z = (float)(2 * c - 1), s = sqrtf(1 - z * z);
                x = s * (float)std::cos(a);
                y = s * (float)std::sin(a);
            } else if (mode == 1) {  // arbitrary bit patterns
                uint32_t a = (uint32_t)next(), b = (uint32_t)next();
                std::memcpy(&y, &a, 4);
                std::memcpy(&x, &b, 4);
            } else if (mode == 2) {  // close exponents
                uint32_t a = (uint32_t)next() & 0x83ffffffu, b = (uint32_t)next() & 0x83ffffffu;
                a |= 0x3c000000u;
                b |= 0x3c000000u;
                std::memcpy(&y, &a, 4);
                std::memcpy(&x, &b, 4);
            } else {
                y = specials[next() % 10] * ((next() & 1) ? 1.f : 0.5f);
                uint32_t b = (uint32_t)next();
                std::memcpy(&x, &b, 4);
                if (next() & 1) std::swap(x, y);
            }
            float p = nd::glibc_atan2f(y, x), h = atan2f(y, x);
            if (!same(p, h)) {
                if (bad < 5) std::printf("mismatch atan2(%a, %a) port=%a glibc=%a\n", y, x, p, h);
                ++bad;
            }
            ++n;
        }
    }
    std::printf("checked %lu values, %lu mismatches\n", n, bad);
    return bad ? 1 : 0;
}
