"""Independent (test-side) OpenEXR scanline reader: NONE / RLE / ZIPS / ZIP, HALF / FLOAT / UINT
channels, as Imf::RgbaInputFile presents them to the reference (texturepattern.cpp:111-128):
R, G, B, A as halves, a missing A reads as 1, a luminance-only (Y) file reads as gray.

Written from the published OpenEXR file layout (magic, attribute header, chlist, offset table,
per-chunk {y, size, data}) and its ZIP codec (zlib, then the byte predictor and the two-half
interleave); it shares no code with the product's reader (nart_amd/csrc/host/scene_host.cpp), so
comparing the two checks the ingestion of the reference's textures instead of self-comparing.
PIZ is restated separately (tests/exr_piz_py.py) and used here chunk by chunk.
"""
import struct
import zlib

import numpy as np

NONE, RLE, ZIPS, ZIP, PIZ = 0, 1, 2, 3, 4
HALF_ONE = 0x3C00


def _cstr(buf, pos):
    end = buf.index(b"\0", pos)
    return buf[pos:end].decode("latin-1"), end + 1


def parse_header(buf):
    assert buf[:4] == b"\x76\x2f\x31\x01", "not an OpenEXR file"
    version = struct.unpack_from("<I", buf, 4)[0]
    assert version & 0x200 == 0, "tiled files are not used by the reference's textures"
    pos, attrs = 8, {}
    while buf[pos] != 0:
        name, pos = _cstr(buf, pos)
        typ, pos = _cstr(buf, pos)
        size = struct.unpack_from("<i", buf, pos)[0]
        pos += 4
        attrs[name] = (typ, buf[pos:pos + size])
        pos += size
    pos += 1
    chans = []
    cl = attrs["channels"][1]
    q = 0
    while cl[q] != 0:
        nm, q = _cstr(cl, q)
        ptype, _lin, xs, ys = struct.unpack_from("<iB3xii", cl, q)
        q += 16
        chans.append((nm, ptype, xs, ys))
    comp = attrs["compression"][1][0]
    xmin, ymin, xmax, ymax = struct.unpack("<iiii", attrs["dataWindow"][1])
    return {"channels": chans, "compression": comp, "window": (xmin, ymin, xmax, ymax)}, pos


def _unzip(data, raw_size):
    t = np.frombuffer(zlib.decompress(data), np.uint8).astype(np.int32)
    # predictor: t[i] = t[i-1] + t[i] - 128 (mod 256), a running sum
    d = t.copy()
    d[1:] -= 128
    t = (np.cumsum(d) & 0xFF).astype(np.uint8)
    half = (raw_size + 1) // 2
    out = np.empty(raw_size, np.uint8)
    out[0::2] = t[:half]
    out[1::2] = t[half:raw_size]
    return out.tobytes()


def _unrle(data, raw_size):
    out = bytearray()
    i = 0
    while i < len(data):
        c = struct.unpack_from("b", data, i)[0]
        i += 1
        if c < 0:
            out += data[i:i - c]
            i += -c
        else:
            out += bytes([data[i]]) * (c + 1)
            i += 1
    assert len(out) == raw_size
    # RLE also applies the predictor and interleave
    t = np.frombuffer(bytes(out), np.uint8).astype(np.int32)
    d = t.copy()
    d[1:] -= 128
    t = (np.cumsum(d) & 0xFF).astype(np.uint8)
    half = (raw_size + 1) // 2
    res = np.empty(raw_size, np.uint8)
    res[0::2] = t[:half]
    res[1::2] = t[half:raw_size]
    return res.tobytes()


def read_rgba_halves(path, max_rows=None):
    """(H, W, 4) uint16 half bit patterns in R, G, B, A order, top row first.  max_rows: decode
    only the chunks that start above that row (the rest stays zero; PIZ in pure Python is slow)."""
    buf = open(path, "rb").read()
    hdr, pos = parse_header(buf)
    comp = hdr["compression"]
    if comp not in (NONE, RLE, ZIPS, ZIP, PIZ):
        raise NotImplementedError("compression %d" % comp)
    xmin, ymin, xmax, ymax = hdr["window"]
    w, h = xmax - xmin + 1, ymax - ymin + 1
    lines = {ZIP: 16, PIZ: 32}.get(comp, 1)
    nchunks = (h + lines - 1) // lines
    offsets = struct.unpack_from("<%dQ" % nchunks, buf, pos)
    chans = sorted(hdr["channels"], key=lambda c: c[0])
    size = {0: 4, 1: 2, 2: 4}
    planes = {c[0]: np.zeros((h, w), np.uint16 if c[1] == 1 else (np.float32 if c[1] == 2 else np.uint32))
              for c in chans}
    for off in offsets:
        y, n = struct.unpack_from("<ii", buf, off)
        data = buf[off + 8:off + 8 + n]
        y0 = y - ymin
        if max_rows is not None and y0 >= max_rows:
            continue
        nl = min(lines, h - y0)
        raw = nl * w * sum(size[c[1]] for c in chans)
        if n < raw:
            if comp == PIZ:
                from exr_piz_py import piz_chunk
                data = piz_chunk(data, [c[1] for c in chans], w, nl)
            else:
                data = _unzip(data, raw) if comp in (ZIPS, ZIP) else (_unrle(data, raw) if comp == RLE else data)
        assert len(data) == raw
        q = 0
        for ln in range(nl):
            for nm, ptype, _xs, _ys in chans:
                nb = w * size[ptype]
                dt = {0: "<u4", 1: "<u2", 2: "<f4"}[ptype]
                planes[nm][y0 + ln] = np.frombuffer(data[q:q + nb], dt)
                q += nb
    out = np.zeros((h, w, 4), np.uint16)

    def as_half(a):
        if a.dtype == np.uint16:
            return a
        return a.astype(np.float32).astype(np.float16).view(np.uint16)

    if "R" in planes or "G" in planes or "B" in planes:
        for k, nm in enumerate("RGB"):
            out[..., k] = as_half(planes[nm]) if nm in planes else 0
    elif "Y" in planes:
        for k in range(3):
            out[..., k] = as_half(planes["Y"])
    out[..., 3] = as_half(planes["A"]) if "A" in planes else HALF_ONE
    return out, hdr


def read_rgba(path):
    halves, _ = read_rgba_halves(path)
    return halves.view(np.float16).astype(np.float32)
