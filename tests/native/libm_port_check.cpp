// Host build of the device libm port (nart_amd/csrc/device/dmath.h) compared against this
// host's glibc sinf/cosf over a strided sweep of float bit patterns.  TEST HELPER.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../nart_amd/csrc/device/dmath.h"

int main(int argc, char** argv) {
    unsigned stride = argc > 1 ? (unsigned)std::atoi(argv[1]) : 1;
    float lim = argc > 2 ? std::atof(argv[2]) : 7.0f;
    unsigned long n = 0, bad = 0;
    unsigned top;
    std::memcpy(&top, &lim, 4);
    for (unsigned b = 0; b <= top; b += stride) {
        float x;
        std::memcpy(&x, &b, 4);
        for (int sgn = 0; sgn < 2; ++sgn) {
            float v = sgn ? -x : x;
            float s = nd::glibc_sinf(v), c = nd::glibc_cosf(v);
            float hs = sinf(v), hc = cosf(v);
            if (std::memcmp(&s, &hs, 4) || std::memcmp(&c, &hc, 4)) {
                if (bad < 5) std::printf("mismatch x=%a port=(%a,%a) glibc=(%a,%a)\n", v, s, c, hs, hc);
                ++bad;
            }
            ++n;
        }
    }
    std::printf("checked %lu values, %lu mismatches\n", n, bad);
    return bad ? 1 : 0;
}
