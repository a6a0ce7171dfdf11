// OpenEXR PIZ chunk decompression (exr_piz.cpp).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace nart {

// Decode one PIZ chunk of `lines` scanlines, `width` samples each, channels in file (sorted)
// order with EXR pixel types (0 UINT, 1 HALF, 2 FLOAT), into the uncompressed scanline layout
// (per line, per channel, little-endian samples).  False on malformed data.
bool piz_decode(const uint8_t* src, size_t n, const int* chan_types, int nchan, uint32_t width, uint32_t lines,
                std::vector<uint8_t>& raw);

}  // namespace nart
