"""The three-kernel LatinSquare (k_latin_draws / k_latin_perm / k_latin_emit, device/kernels.h)
restated in numpy and checked against the oracle's LatinSquare (sampling.cpp:72-86) on CPU.

The decomposition rests on two facts the GPU kernels rely on: the shuffle's transpositions
(i, c_i) depend only on the RNG stream, and a jittered stratum value depends only on the stream
position that drew it, so sample j = (val_x(sigma_x[j]), val_y(sigma_y[j])) with val_x(k) from
the state after draw 2k+1 and val_y(k) one xorshift step later.  Odd spp exercise the u16-pair
packing's half-used last word."""
import numpy as np
import pytest

import oracle

M32 = 0xFFFFFFFF


def _xorshift(y):
    y ^= (y << 13) & M32
    y ^= y >> 17
    y ^= (y << 5) & M32
    return y


def _uniform_float(y):  # rng.h:15-35 on the state after the draw
    f = np.float32(np.float32((y * 0x9E3779BB) & M32) * np.float32(2.3283064365386963e-10))
    return min(np.float32(1.0) - np.float32(1.1920928955078125e-07), f)


def _latin_three_kernels(seed, n):
    rng = (seed + 2463534242) & M32
    # k_latin_draws: st[k] = state after draw 2k+1; then the 2n shuffle choices
    st = []
    for _ in range(n):
        rng = _xorshift(rng)
        st.append(rng)
        rng = _xorshift(rng)
    cx, cy = [], []
    for i in range(n):
        rng = _xorshift(rng)
        cx.append((((rng * 0x9E3779B9) & M32) * (n - i)) >> 32)  # UniformInt32(n - 1 - i)
        rng = _xorshift(rng)
        cy.append((((rng * 0x9E3779B9) & M32) * (n - i)) >> 32)
    # k_latin_perm: the swaps replayed on stratum indices
    sx, sy = list(range(n)), list(range(n))
    for i in range(n):
        sx[i], sx[cx[i]] = sx[cx[i]], sx[i]
        sy[i], sy[cy[i]] = sy[cy[i]], sy[i]
    # k_latin_emit: values recomputed from the states
    inv = np.float32(1.0) / np.float32(n)
    out = np.zeros((n, 2), np.float32)
    for j in range(n):
        kx, ky = sx[j], sy[j]
        out[j, 0] = np.float32(np.float32(np.float32(kx) + _uniform_float(st[kx])) * inv)
        out[j, 1] = np.float32(np.float32(np.float32(ky) + _uniform_float(_xorshift(st[ky]))) * inv)
    return out, rng


@pytest.mark.parametrize("n", [2, 3, 17, 64, 257, 300])
def test_three_kernel_latin_square_matches_reference_order(built, n):
    for seed in (0, 12345, 1921 * 700 + 811):
        want, want_state = oracle.latin_square(seed, n)
        got, state = _latin_three_kernels(seed, n)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (seed, n)
        assert state == want_state


def _perm_batched(c, n, PF=16):
    """k_latin_perm's replay (NART_LATIN_HALF): serial swaps in batches of 2 PF, except that a
    full batch starting at or after m = ceil(n/2) runs as three stages (B_i = A[i]; in step order
    r_i = A[c_i], A[c_i] = B_i; A[i] = r_i), the partial last batch serially."""
    A = list(range(n + 2))
    m, i2 = (n + 1) // 2, 0
    while 2 * (i2 + PF) <= n:
        idx = range(2 * i2, 2 * i2 + 2 * PF)
        if 2 * i2 >= m:
            bv = [A[i] for i in idx]
            rv = []
            for q, i in enumerate(idx):
                rv.append(A[c[i]])
                A[c[i]] = bv[q]
            for q, i in enumerate(idx):
                A[i] = rv[q]
        else:
            for i in idx:
                A[i], A[c[i]] = A[c[i]], A[i]
        i2 += PF
    for i in range(2 * i2, n):
        A[i], A[c[i]] = A[c[i]], A[i]
    return A[:n]


@pytest.mark.parametrize("n", [31, 32, 64, 65, 96, 100, 129, 256, 257, 511, 512, 1023, 1024])
def test_second_half_three_stage_shuffle_matches_serial(n):
    """For i >= ceil(n/2) the choices c_i <= n-1-i fall below the batch, so the three-stage form
    of k_latin_perm's second half equals the serial swaps, on random and on RNG-drawn choices."""
    r = np.random.default_rng(n)
    for t in range(40):
        if t % 2:
            c = [int(r.integers(0, n - i)) for i in range(n)]
        else:  # the pixel's own draws (sampling.cpp:81-84), x then y
            rng = (t * 7919 + 2463534242) & M32
            for _ in range(2 * n):
                rng = _xorshift(rng)
            c = []
            for i in range(n):
                rng = _xorshift(rng)
                c.append((((rng * 0x9E3779B9) & M32) * (n - i)) >> 32)
                rng = _xorshift(rng)
        want = list(range(n))
        for i in range(n):
            want[i], want[c[i]] = want[c[i]], want[i]
        assert _perm_batched(c, n) == want
