"""The oracle pinned to the reference's own code where the reference can run here.

Only src/core/util.cpp (BinarySearch, the environment light's CDF inversion,
texturepattern.cpp:72-102) compiles without the dependencies this image lacks; it is built in
place by `make -C oracle ref` into oracle/_ref/.  The committed golden vectors
(tests/golden/binary_search.npz, tools/make_golden_binary_search.py) hold its outputs, so the pin
also holds where the reference checkout is absent."""
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "binary_search.npz")


def test_binary_search_matches_reference_golden(built):
    z = np.load(GOLDEN, allow_pickle=False)
    cdfs, offs = z["cdfs"], z["offsets"]
    got = np.array([oracle.binary_search(v, cdfs[offs[k]:offs[k + 1]], s, e)
                    for v, s, e, k in zip(z["values"], z["starts"], z["ends"], z["which"])], np.uint32)
    assert len(got) > 20000
    bad = np.flatnonzero(got != z["expected"])
    assert bad.size == 0, "%d of %d differ, first at %d" % (bad.size, len(got), bad[:1])


def test_binary_search_matches_reference_live(built):
    ref = oracle.ref_binary_search() or (oracle.build_ref() and oracle.ref_binary_search())
    if ref is None:
        pytest.skip("reference util.cpp not available (no /root/reference and no prebuilt oracle/_ref)")
    rng = np.random.default_rng(5)
    for trial in range(60):
        n = int(rng.integers(1, 300))
        steps = rng.random(n).astype(np.float32) * (rng.random(n) > rng.random())  # flat runs
        cdf = np.concatenate([[0], np.cumsum(steps, dtype=np.float32)]).astype(np.float32)
        cdf /= cdf[-1] if cdf[-1] > 0 else np.float32(1)
        cdf[-1] = 1.0
        vals = np.concatenate([rng.random(64, np.float32) * np.float32(1 - 2 ** -24), cdf[:-1]])
        for v in vals:
            s = int(rng.integers(0, n))
            e = int(rng.integers(s, n + 1))
            for a, b in ((0, n), (s, e)):
                assert oracle.binary_search(v, cdf, a, b) == ref(v, cdf, a, b), (trial, v, a, b)


def _guided(v, cdf, start, end, K=64):
    """Restatement of render.hip build_env's guide table + path.h guided_search (the device's
    shortcut), in numpy float32: per cell [c/K, (c+1)/K) the range of the upper bound
    ub(x) = first j in [start, end) with cdf[j] > x, then a search of that range; ub - 1."""
    seg = cdf[start:end]
    f32 = np.float32
    c = min(K - 1, int(f32(v) * f32(K)))
    lo = f32(c) / f32(K)
    hi = np.inf if c + 1 == K else np.nextafter(f32(c + 1) / f32(K), f32(0))
    a = int(np.searchsorted(seg, lo, side="right"))
    b = int(np.searchsorted(seg, hi, side="right"))
    lo_i, hi_i = start + a, start + b
    while lo_i < hi_i:
        mid = lo_i + ((hi_i - lo_i) >> 1)
        if cdf[mid] > f32(v):
            hi_i = mid
        else:
            lo_i = mid + 1
    return (lo_i - 1) & 0xFFFFFFFF


def test_guided_search_equals_reference_binary_search(built):
    """The premise of the device's guide tables (environment-lit scenes):
    the reference's BinarySearch (util.cpp:4-20) returns ub - 1 for the upper bound ub of the
    searched range, whichever probes it takes -- checked against the reference's own compiled
    util.cpp (or the golden-pinned oracle restatement) on CDFs with flat runs, values at CDF
    entries and at guide-cell boundaries, and searched sub-ranges as the conditional CDFs use."""
    ref = oracle.ref_binary_search() or oracle.binary_search
    rng = np.random.default_rng(11)
    for trial in range(40):
        n = int(rng.integers(1, 400))
        steps = rng.random(n).astype(np.float32) * (rng.random(n) > rng.random())  # flat runs
        cdf = np.concatenate([[0], np.cumsum(steps, dtype=np.float32)]).astype(np.float32)
        cdf /= cdf[-1] if cdf[-1] > 0 else np.float32(1)
        cdf[-1] = 1.0
        cells = (np.arange(64, dtype=np.float32) / np.float32(64)).astype(np.float32)
        vals = np.concatenate([rng.random(48, np.float32) * np.float32(1 - 2 ** -24), cdf[:-1], cells,
                               np.nextafter(cells[1:], np.float32(0))]).astype(np.float32)
        for v in vals:
            assert _guided(v, cdf, 0, n) == ref(v, cdf, 0, n), (trial, float(v))
            s = int(rng.integers(0, n))
            e = int(rng.integers(s + 1, n + 1))
            assert _guided(v, cdf, s, e) == ref(v, cdf, s, e), (trial, float(v), s, e)
