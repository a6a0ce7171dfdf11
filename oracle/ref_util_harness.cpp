// TEST INFRASTRUCTURE ONLY.  C entry point into the reference's own BinarySearch
// (src/core/util.cpp:4-20, compiled from /root/reference by oracle/Makefile's `ref` target into
// oracle/_ref/libref_util.so).  util.cpp is the one source file on the render path that needs
// none of the dependencies missing from this image (GLM, OpenEXR/Imath, oneTBB, nlohmann), so
// it is the only part of the reference that runs here; tests/test_oracle_ref.py pins the
// oracle's restatement (and tests/golden/binary_search.npz) to it.
#include <cstdint>
#include <vector>

#include "util.h"  // the reference's header (-I <reference>/include/nart/core)

extern "C" uint32_t ref_binary_search(float value, const float* v, uint32_t n, uint32_t start, uint32_t end) {
    const std::vector<float> cdf(v, v + n);
    return BinarySearch(value, cdf, start, end);
}
