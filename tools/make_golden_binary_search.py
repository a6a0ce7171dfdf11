"""Golden vectors for BinarySearch (src/core/util.cpp:4-20) from the reference's own code.

Runs the reference's util.cpp, compiled in place by `make -C oracle ref` (oracle/_ref/, never
committed), over CDF inversion cases shaped like the environment light's (texturepattern.cpp:
72-102: the marginal CDF [0, h] and conditional rows [v(w+1), v(w+1)+w] of one array, values in
[0, 1-eps]), plus edge cases: values equal to CDF entries, flat segments (zero-pdf rows and
texels), start == end.  Writes tests/golden/binary_search.npz (inputs and expected indices).
    python tools/make_golden_binary_search.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import oracle  # noqa: E402


def cases(rng):
    """(cdf array, list of (value, start, end))"""
    out = []
    for w, h, zero_frac in [(16, 8, 0.0), (37, 5, 0.3), (128, 64, 0.1), (3, 2, 0.5), (1, 1, 0.0), (255, 4, 0.9)]:
        tex = rng.random((h, w)).astype(np.float32) * (rng.random((h, w)) >= zero_frac)
        tex[rng.integers(0, h)] = 0.0  # a zero row: flat marginal segment, constant conditional
        cdf = [np.float32(0.0)]
        mpdf = tex.mean(axis=1).astype(np.float32)
        tot = np.float32(mpdf.sum()) or np.float32(1.0)
        for j in range(1, h):  # marginal CDF, float32 running sum
            cdf.append(np.float32(cdf[-1] + np.float32(mpdf[j - 1] / tot / h)))
        cdf.append(np.float32(1.0))
        rows = []
        for j in range(h):
            r = [np.float32(0.0)]
            s = np.float32(tex[j].sum()) or np.float32(1.0)
            for i in range(1, w):
                r.append(np.float32(r[-1] + np.float32(tex[j, i - 1] / s / w)))
            r.append(np.float32(1.0))
            rows += r
        arr = np.array(cdf + rows, np.float32)
        q = []
        vals = np.concatenate([rng.random(200, np.float32) * np.float32(1 - 2 ** -24), arr[arr < 1.0],
                               np.float32([0.0, 1 - 2 ** -24])])
        for v in vals:
            q.append((v, 0, h))  # marginal: BinarySearch(s.y, marginalCdf, 0, height)
            j = int(rng.integers(0, h))
            q.append((v, h + 1 + j * (w + 1), h + 1 + j * (w + 1) + w))  # one conditional row
        q += [(np.float32(0.5), 3, 3), (np.float32(0.0), 0, 0), (np.float32(0.25), 1, 2)]
        out.append((arr, q))
    return out


def main():
    f = oracle.ref_binary_search() or (oracle.build_ref() and oracle.ref_binary_search())
    if f is None:
        raise SystemExit("reference util.cpp not available (needs /root/reference)")
    rng = np.random.default_rng(20261016)
    arrays, offs, vals, starts, ends, want, which = [], [0], [], [], [], [], []
    for k, (arr, q) in enumerate(cases(rng)):
        arrays.append(arr)
        offs.append(offs[-1] + len(arr))
        for v, s, e in q:
            vals.append(v)
            starts.append(s)
            ends.append(e)
            which.append(k)
            want.append(f(v, arr, s, e))
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "binary_search.npz"),
                        cdfs=np.concatenate(arrays), offsets=np.array(offs, np.int64),
                        values=np.array(vals, np.float32), starts=np.array(starts, np.uint32),
                        ends=np.array(ends, np.uint32), which=np.array(which, np.int32),
                        expected=np.array(want, np.uint32))
    print("%d cases" % len(want))


if __name__ == "__main__":
    main()
