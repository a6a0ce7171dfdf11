"""Independent (test-side) restatement of OpenEXR's PIZ codec for one scanline chunk, written from
the published format: a bitmap of the 16-bit values present and its reverse LUT, a canonical
Huffman code whose 6-bit code-length table carries zero-run codes (59-62 short runs, 63 + 8 bits
a long run) and whose largest symbol is the run-length code (8 more bits: repeats of the previous
value), then the 2D Haar-like wavelet per 16-bit plane (14-bit or 16-bit variant by the value
range), then the LUT, then the planes interleaved back into scanlines.

It shares no code with the product's decoder (nart_amd/csrc/host/exr_piz.cpp): Huffman symbols are
decoded by code length against the canonical ranges (not a 14-bit table), and each wavelet level is
applied to whole arrays with numpy.  tests/test_ingestion_independent.py compares the two on the
reference's PIZ textures texel for texel.  Pure Python: meant for chunks, not whole 4K textures.
"""
import struct

import numpy as np

USHORT_RANGE = 1 << 16
BITMAP_SIZE = USHORT_RANGE >> 3
SHORT_ZEROCODE_RUN, LONG_ZEROCODE_RUN = 59, 63
SHORTEST_LONG_RUN = 2 + LONG_ZEROCODE_RUN - SHORT_ZEROCODE_RUN
ENCSIZE = (1 << 16) + 1


class _Bits:
    """MSB-first bit reader over a byte string."""

    def __init__(self, data, pos=0):
        self.data, self.pos, self.acc, self.n = data, pos, 0, 0

    def get(self, nb):
        while self.n < nb:
            self.acc = (self.acc << 8) | self.data[self.pos]
            self.pos += 1
            self.n += 8
        self.n -= nb
        v = (self.acc >> self.n) & ((1 << nb) - 1)
        self.acc &= (1 << self.n) - 1
        return v


def _code_lengths(data, pos, im, iM):
    lens = {}
    br = _Bits(data, pos)
    s = im
    while s <= iM:
        length = br.get(6)
        if length == LONG_ZEROCODE_RUN:
            s += br.get(8) + SHORTEST_LONG_RUN
        elif length >= SHORT_ZEROCODE_RUN:
            s += length - SHORT_ZEROCODE_RUN + 2
        else:
            if length:
                lens[s] = length
            s += 1
    assert s == iM + 1, "code-length table overruns the symbol range"
    return lens, br.pos


def _canonical(lens):
    """{length: (first code, [symbols in code order])}: codes of a length are consecutive in
    symbol order, and longer codes start below shorter ones' (OpenEXR's assignment)."""
    count = [0] * 59
    for ln in lens.values():
        count[ln] += 1
    start = [0] * 59
    c = 0
    for ln in range(58, 0, -1):
        start[ln] = c
        c = (c + count[ln]) >> 1
    table = {}
    for sym in sorted(lens):
        table.setdefault(lens[sym], []).append(sym)
    return {ln: (start[ln], syms) for ln, syms in table.items()}


def huffman_decode(data, nout):
    im, iM, _tlen, nbits, _ = struct.unpack_from("<IIIII", data, 0)
    lens, pos = _code_lengths(data, 20, im, iM)
    canon = _canonical(lens)
    maxlen = max(canon) if canon else 0
    out = np.empty(nout, np.uint16)
    k = 0
    br = _Bits(data, pos)
    used = 0
    rlc = iM  # the largest symbol is the run-length code
    while used < nbits:
        code, ln = 0, 0
        while True:
            code = (code << 1) | br.get(1)
            ln += 1
            used += 1
            e = canon.get(ln)
            if e is not None and e[0] <= code < e[0] + len(e[1]):
                sym = e[1][code - e[0]]
                break
            assert ln < maxlen and used < nbits, "invalid Huffman code"
        if sym == rlc:
            run = br.get(8)
            used += 8
            out[k:k + run] = out[k - 1]
            k += run
        else:
            out[k] = sym
            k += 1
    assert k == nout, (k, nout)
    return out


def _wdec14(l, h):
    ls, hs = l.astype(np.int16).astype(np.int32), h.astype(np.int16).astype(np.int32)
    ai = ls + (hs & 1) + (hs >> 1)
    return (ai & 0xFFFF).astype(np.uint16), ((ai - hs) & 0xFFFF).astype(np.uint16)


def _wdec16(l, h):
    m, d = l.astype(np.int32), h.astype(np.int32)
    bb = (m - (d >> 1)) & 0xFFFF
    aa = (d + bb - 0x8000) & 0xFFFF
    return aa.astype(np.uint16), bb.astype(np.uint16)


def wavelet_decode(plane, mx):
    """In-place inverse wavelet of a (ny, nx) uint16 plane."""
    dec = _wdec14 if mx < (1 << 14) else _wdec16
    ny, nx = plane.shape
    n = min(nx, ny)
    p = 1
    while p <= n:
        p <<= 1
    p >>= 1
    p2, p = p, p >> 1
    while p >= 1:
        ys = np.arange(0, ny - p2 + 1, p2)
        xs = np.arange(0, nx - p2 + 1, p2)
        Y, X = np.meshgrid(ys, xs, indexing="ij")
        a, b = plane[Y, X], plane[Y, X + p]
        c, d = plane[Y + p, X], plane[Y + p, X + p]
        i00, i10 = dec(a, c)
        i01, i11 = dec(b, d)
        plane[Y, X], plane[Y, X + p] = dec(i00, i01)
        plane[Y + p, X], plane[Y + p, X + p] = dec(i10, i11)
        if nx & p:  # the column after the last 2x2 block
            xe = xs[-1] + p2 if len(xs) else 0
            a, c = plane[ys, xe], plane[ys + p, xe]
            plane[ys, xe], plane[ys + p, xe] = dec(a, c)
        if ny & p:  # the row after the last 2x2 block
            ye = ys[-1] + p2 if len(ys) else 0
            a, b = plane[ye, xs], plane[ye, xs + p]
            plane[ye, xs], plane[ye, xs + p] = dec(a, b)
        p2, p = p, p >> 1


def piz_chunk(data, types, width, lines):
    """Decode one PIZ chunk: types = pixel type per channel in file (alphabetical) order (1 HALF,
    0 UINT, 2 FLOAT); returns the chunk's raw scanline bytes (as the uncompressed layout)."""
    words = [1 if t == 1 else 2 for t in types]
    total = sum(width * lines * w for w in words)
    mn, mx = struct.unpack_from("<HH", data, 0)
    q = 4
    bitmap = np.zeros(BITMAP_SIZE, np.uint8)
    if mn <= mx:
        bitmap[mn:mx + 1] = np.frombuffer(data, np.uint8, mx - mn + 1, q)
        q += mx - mn + 1
    present = np.unpackbits(bitmap, bitorder="little").astype(bool)
    present[0] = True
    lut = np.flatnonzero(present).astype(np.uint16)
    maxvalue = len(lut) - 1
    (length,) = struct.unpack_from("<i", data, q)
    q += 4
    tmp = huffman_decode(data[q:q + length], total)
    planes, off = [], 0
    for w in words:
        plane = tmp[off:off + width * lines * w].reshape(lines, width * w).copy()
        for j in range(w):
            sub = plane[:, j::w].copy()
            wavelet_decode(sub, maxvalue)
            plane[:, j::w] = sub
        planes.append(lut[plane])
        off += width * lines * w
    rows = []
    for y in range(lines):
        for plane in planes:
            rows.append(plane[y].astype("<u2").tobytes())
    return b"".join(rows)
