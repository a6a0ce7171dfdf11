// OpenEXR PIZ decompression (wavelet + Huffman), restated from the published format
// (OpenEXR 3.2 ImfPizCompressor / ImfHuf / ImfWav): the reference reads PIZ textures through
// Imf::RgbaInputFile (texturepattern.cpp:111-128) -- cameraLens and glassIceWater use them.
//
// A PIZ chunk (up to 32 scanlines) holds: the [min, max] byte range of a 65536-bit bitmap of the
// 16-bit values present, that bitmap range, a 32-bit Huffman payload length, the Huffman-coded
// 16-bit words of every channel plane, wavelet-transformed per plane.  Decoding reverses the
// Huffman code, the 2D Haar-like wavelet (14- or 16-bit variant by the value range), maps
// values back through the bitmap's reverse LUT and interleaves planes into scanlines.
//
// Third-party notice.  The Huffman decoder (code-length unpacking with the zero-run codes, the
// canonical code table, the decoding table) and the wavelet decoder restate OpenEXR's
// ImfHuf.cpp and ImfWav.cpp, whose constants and structure they keep:
//   Copyright (c) 2002-2012, Industrial Light & Magic, a division of Lucas Digital Ltd. LLC.
//   Copyright (c) Contributors to the OpenEXR Project.  All rights reserved.
//   SPDX-License-Identifier: BSD-3-Clause.
//   Redistribution and use in source and binary forms, with or without modification, are
//   permitted provided that the following conditions are met: (1) redistributions of source code
//   must retain the above copyright notice, this list of conditions and the following disclaimer;
//   (2) redistributions in binary form must reproduce the above copyright notice, this list of
//   conditions and the following disclaimer in the documentation and/or other materials provided
//   with the distribution; (3) neither the name of the copyright holder nor the names of its
//   contributors may be used to endorse or promote products derived from this software without
//   specific prior written permission.  THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND
//   CONTRIBUTORS "AS IS" AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO, THE
//   IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR A PARTICULAR PURPOSE ARE DISCLAIMED. IN NO
//   EVENT SHALL THE COPYRIGHT HOLDER OR CONTRIBUTORS BE LIABLE FOR ANY DIRECT, INDIRECT,
//   INCIDENTAL, SPECIAL, EXEMPLARY, OR CONSEQUENTIAL DAMAGES (INCLUDING, BUT NOT LIMITED TO,
//   PROCUREMENT OF SUBSTITUTE GOODS OR SERVICES; LOSS OF USE, DATA, OR PROFITS; OR BUSINESS
//   INTERRUPTION) HOWEVER CAUSED AND ON ANY THEORY OF LIABILITY, WHETHER IN CONTRACT, STRICT
//   LIABILITY, OR TORT (INCLUDING NEGLIGENCE OR OTHERWISE) ARISING IN ANY WAY OUT OF THE USE OF
//   THIS SOFTWARE, EVEN IF ADVISED OF THE POSSIBILITY OF SUCH DAMAGE.
#include "exr_piz.h"

#include <cstring>
#include <vector>

namespace nart {
namespace {

constexpr int HUF_ENCBITS = 16;
constexpr int HUF_DECBITS = 14;
constexpr int HUF_ENCSIZE = (1 << HUF_ENCBITS) + 1;
constexpr int HUF_DECSIZE = 1 << HUF_DECBITS;
constexpr int HUF_DECMASK = HUF_DECSIZE - 1;
constexpr int SHORT_ZEROCODE_RUN = 59;
constexpr int LONG_ZEROCODE_RUN = 63;
constexpr int SHORTEST_LONG_RUN = 2 + LONG_ZEROCODE_RUN - SHORT_ZEROCODE_RUN;
constexpr int USHORT_RANGE = 1 << 16;
constexpr int BITMAP_SIZE = USHORT_RANGE >> 3;

struct HufDec {
    int len = 0;
    int lit = 0;
    std::vector<int> p;  // long codes sharing this 14-bit prefix
};

inline int huf_length(int64_t code) { return int(code & 63); }
inline int64_t huf_code(int64_t code) { return code >> 6; }

struct BitReader {
    const uint8_t* in;
    const uint8_t* end;       // end of the coded bits (loop control)
    const uint8_t* hard_end;  // end of the buffer (a run-length byte may sit past `end`)
    uint64_t c = 0;
    int lc = 0;
    bool get_char() {
        if (in >= hard_end) return false;
        c = (c << 8) | *in++;
        lc += 8;
        return true;
    }
};

// canonical code table from code lengths (ImfHuf hufCanonicalCodeTable)
void canonical_codes(std::vector<int64_t>& hcode) {
    int64_t n[59] = {0};
    for (int i = 0; i < HUF_ENCSIZE; ++i) n[hcode[i]] += 1;
    int64_t c = 0;
    for (int i = 58; i > 0; --i) {
        int64_t nc = (c + n[i]) >> 1;
        n[i] = c;
        c = nc;
    }
    for (int i = 0; i < HUF_ENCSIZE; ++i) {
        int l = int(hcode[i]);
        if (l > 0) hcode[i] = l | (n[l]++ << 6);
    }
}

bool unpack_enc_table(const uint8_t*& p, const uint8_t* end, int im, int iM, std::vector<int64_t>& hcode) {
    hcode.assign(HUF_ENCSIZE, 0);
    BitReader br{p, end, end};
    auto get_bits = [&](int nb, int& v) {
        while (br.lc < nb)
            if (!br.get_char()) return false;
        br.lc -= nb;
        v = int((br.c >> br.lc) & ((1 << nb) - 1));
        return true;
    };
    for (; im <= iM; im++) {
        int l;
        if (!get_bits(6, l)) return false;
        hcode[im] = l;
        if (l == LONG_ZEROCODE_RUN) {
            int z;
            if (!get_bits(8, z)) return false;
            int zerun = z + SHORTEST_LONG_RUN;
            if (im + zerun > iM + 1) return false;
            while (zerun--) hcode[im++] = 0;
            im--;
        } else if (l >= SHORT_ZEROCODE_RUN) {
            int zerun = l - SHORT_ZEROCODE_RUN + 2;
            if (im + zerun > iM + 1) return false;
            while (zerun--) hcode[im++] = 0;
            im--;
        }
    }
    p = br.in;
    canonical_codes(hcode);
    return true;
}

bool build_dec_table(const std::vector<int64_t>& hcode, int im, int iM, std::vector<HufDec>& hdec) {
    hdec.assign(HUF_DECSIZE, HufDec());
    for (; im <= iM; im++) {
        int64_t c = huf_code(hcode[im]);
        int l = huf_length(hcode[im]);
        if (c >> l) return false;
        if (l > HUF_DECBITS) {
            HufDec& pl = hdec[size_t(c >> (l - HUF_DECBITS))];
            if (pl.len) return false;
            pl.lit++;
            pl.p.push_back(im);
        } else if (l) {
            size_t base = size_t(c << (HUF_DECBITS - l));
            for (int64_t i = int64_t(1) << (HUF_DECBITS - l); i > 0; i--, base++) {
                HufDec& pl = hdec[base];
                if (pl.len || !pl.p.empty()) return false;
                pl.len = l;
                pl.lit = im;
            }
        }
    }
    return true;
}

bool huf_decode(const std::vector<int64_t>& hcode, const std::vector<HufDec>& hdec, const uint8_t* in,
                const uint8_t* in_end, int64_t ni, int rlc, size_t no, uint16_t* out) {
    uint16_t* const outb = out;
    uint16_t* const oe = out + no;
    BitReader br{in, in + (ni + 7) / 8, in_end};
    auto emit = [&](int po) {
        if (po == rlc) {
            if (br.lc < 8 && !br.get_char()) return false;
            br.lc -= 8;
            unsigned cs = unsigned((br.c >> br.lc) & 0xff);
            if (out + cs > oe || out - 1 < outb) return false;
            const uint16_t s = out[-1];
            while (cs-- > 0) *out++ = s;
        } else {
            if (out >= oe) return false;
            *out++ = uint16_t(po);
        }
        return true;
    };
    while (br.in < br.end) {
        br.get_char();
        while (br.lc >= HUF_DECBITS) {
            const HufDec& pl = hdec[size_t((br.c >> (br.lc - HUF_DECBITS)) & HUF_DECMASK)];
            if (pl.len) {
                br.lc -= pl.len;
                if (!emit(pl.lit)) return false;
            } else {
                if (pl.p.empty()) return false;
                int j;
                for (j = 0; j < pl.lit; j++) {
                    const int l = huf_length(hcode[pl.p[j]]);
                    while (br.lc < l && br.in < br.end) br.get_char();
                    if (br.lc >= l &&
                        uint64_t(huf_code(hcode[pl.p[j]])) == ((br.c >> (br.lc - l)) & ((uint64_t(1) << l) - 1))) {
                        br.lc -= l;
                        if (!emit(pl.p[j])) return false;
                        break;
                    }
                }
                if (j == pl.lit) return false;
            }
        }
    }
    const int i = int((8 - ni) & 7);
    br.c >>= i;
    br.lc -= i;
    while (br.lc > 0) {
        const HufDec& pl = hdec[size_t((br.c << (HUF_DECBITS - br.lc)) & HUF_DECMASK)];
        if (!pl.len) return false;
        br.lc -= pl.len;
        if (!emit(pl.lit)) return false;
    }
    return size_t(out - outb) == no;
}

uint32_t rd32(const uint8_t* p) { return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24); }

bool huf_uncompress(const uint8_t* compressed, size_t n, uint16_t* raw, size_t nraw) {
    if (n == 0) return nraw == 0;
    if (n < 20) return false;
    const int im = int(rd32(compressed)), iM = int(rd32(compressed + 4));
    const int64_t nBits = int64_t(rd32(compressed + 12));
    if (im < 0 || im >= HUF_ENCSIZE || iM < 0 || iM >= HUF_ENCSIZE) return false;
    const uint8_t* ptr = compressed + 20;
    std::vector<int64_t> hcode;
    if (!unpack_enc_table(ptr, compressed + n, im, iM, hcode)) return false;
    if (nBits > 8 * int64_t(compressed + n - ptr)) return false;
    std::vector<HufDec> hdec;
    if (!build_dec_table(hcode, im, iM, hdec)) return false;
    return huf_decode(hcode, hdec, ptr, compressed + n, nBits, iM, nraw, raw);
}

inline void wdec14(uint16_t l, uint16_t h, uint16_t& a, uint16_t& b) {
    const int16_t ls = int16_t(l), hs = int16_t(h);
    const int hi = hs;
    const int ai = ls + (hi & 1) + (hi >> 1);
    const int16_t as = int16_t(ai), bs = int16_t(ai - hi);
    a = uint16_t(as);
    b = uint16_t(bs);
}
inline void wdec16(uint16_t l, uint16_t h, uint16_t& a, uint16_t& b) {
    const int m = l, d = h;
    const int bb = (m - (d >> 1)) & 0xffff;
    const int aa = (d + bb - 0x8000) & 0xffff;
    b = uint16_t(bb);
    a = uint16_t(aa);
}

void wav2_decode(uint16_t* in, int nx, int ox, int ny, int oy, uint16_t mx) {
    const bool w14 = mx < (1 << 14);
    auto dec = [&](uint16_t l, uint16_t h, uint16_t& a, uint16_t& b) {
        if (w14) wdec14(l, h, a, b);
        else wdec16(l, h, a, b);
    };
    const int n = nx > ny ? ny : nx;
    int p = 1, p2;
    while (p <= n) p <<= 1;
    p >>= 1;
    p2 = p;
    p >>= 1;
    while (p >= 1) {
        uint16_t* py = in;
        uint16_t* const ey = in + oy * (ny - p2);
        const int oy1 = oy * p, oy2 = oy * p2, ox1 = ox * p, ox2 = ox * p2;
        uint16_t i00, i01, i10, i11;
        for (; py <= ey; py += oy2) {
            uint16_t* px = py;
            uint16_t* const ex = py + ox * (nx - p2);
            for (; px <= ex; px += ox2) {
                uint16_t* p01 = px + ox1;
                uint16_t* p10 = px + oy1;
                uint16_t* p11 = p10 + ox1;
                dec(*px, *p10, i00, i10);
                dec(*p01, *p11, i01, i11);
                dec(i00, i01, *px, *p01);
                dec(i10, i11, *p10, *p11);
            }
            if (nx & p) {
                uint16_t* p10 = px + oy1;
                dec(*px, *p10, i00, *p10);
                *px = i00;
            }
        }
        if (ny & p) {
            uint16_t* px = py;
            uint16_t* const ex = py + ox * (nx - p2);
            for (; px <= ex; px += ox2) {
                uint16_t* p01 = px + ox1;
                dec(*px, *p01, i00, *p01);
                *px = i00;
            }
        }
        p2 = p;
        p >>= 1;
    }
}

}  // namespace

bool piz_decode(const uint8_t* src, size_t n, const int* chan_types, int nchan, uint32_t width, uint32_t lines,
                std::vector<uint8_t>& raw) {
    // channel planes: HALF = 1 word per sample, UINT / FLOAT = 2 words
    std::vector<size_t> start(nchan), words(nchan);
    size_t total = 0;
    for (int c = 0; c < nchan; ++c) {
        words[c] = chan_types[c] == 1 ? 1 : 2;
        start[c] = total;
        total += size_t(width) * lines * words[c];
    }
    std::vector<uint16_t> tmp(total ? total : 1);
    if (n < 4) return false;
    const uint16_t minNZ = uint16_t(src[0] | (src[1] << 8)), maxNZ = uint16_t(src[2] | (src[3] << 8));
    size_t q = 4;
    if (maxNZ >= BITMAP_SIZE) return false;
    std::vector<uint8_t> bitmap(BITMAP_SIZE, 0);
    if (minNZ <= maxNZ) {
        const size_t len = size_t(maxNZ) - minNZ + 1;
        if (q + len > n) return false;
        std::memcpy(&bitmap[minNZ], src + q, len);
        q += len;
    }
    std::vector<uint16_t> lut(USHORT_RANGE, 0);
    int k = 0;
    for (int i = 0; i < USHORT_RANGE; ++i)
        if (i == 0 || (bitmap[i >> 3] & (1 << (i & 7)))) lut[k++] = uint16_t(i);
    const uint16_t maxValue = uint16_t(k - 1);
    if (q + 4 > n) return false;
    const uint32_t length = rd32(src + q);
    q += 4;
    if (q + length > n) return false;
    if (!huf_uncompress(src + q, length, tmp.data(), total)) return false;
    for (int c = 0; c < nchan; ++c)
        for (size_t j = 0; j < words[c]; ++j)
            wav2_decode(tmp.data() + start[c] + j, int(width), int(words[c]), int(lines), int(width * words[c]), maxValue);
    for (size_t i = 0; i < total; ++i) tmp[i] = lut[tmp[i]];
    raw.resize(total * 2);
    size_t o = 0;
    for (uint32_t y = 0; y < lines; ++y)
        for (int c = 0; c < nchan; ++c) {
            const uint16_t* row = tmp.data() + start[c] + size_t(y) * width * words[c];
            for (size_t x = 0; x < size_t(width) * words[c]; ++x) {
                raw[o++] = uint8_t(row[x] & 0xff);
                raw[o++] = uint8_t(row[x] >> 8);
            }
        }
    return true;
}

}  // namespace nart
