"""The skewed-time splat's schedule (k_splat_skew, device/kernels.h) checked on CPU against the
order in which AddSample reaches each tile pixel (render.cpp:23-70), as the gather kernels
visit it (k_splat / k_splat_col4: the tile pixel's source window in raster order, the bucket's
last column as an extra column after each row and its last row as an extra row after all rows).

The simulation replays the kernel's loop for every lane (tile column) and band: at step t the
lane's only candidate source is the sx in [tx-2R, tx] with sx = t (mod 2R+1); a pass over a
source row adds to the window rows [sy, sy+2R]; the extra-column pass follows the lane's last
source of a row; the last-row wrap passes run after the loop.  Every tile pixel of the band must
receive exactly the gather order's (source, kind) sequence, and no lane may have two sources
at one step."""
import pytest


def gather_order(tx, ty, B, R, bw, bh):
    sxlo, sxhi = max(0, tx - 2 * R), min(bw - 1, tx)
    sylo, syhi = max(0, ty - 2 * R), min(bh - 1, ty)
    wrapx = bw == B and tx <= 2 * R + 1 and bw - 1 > sxhi
    wrapy = bh == B and ty <= 2 * R + 1 and bh - 1 > syhi
    seq = []
    for sy in range(sylo, syhi + 1):
        seq += [(sy, sx, "n") for sx in range(sxlo, sxhi + 1)]
        if wrapx:
            seq.append((sy, bw - 1, "x"))
    if wrapy:
        seq += [(bh - 1, sx, "y") for sx in range(sxlo, sxhi + 1)]
        if wrapx:
            seq.append((bh - 1, bw - 1, "y"))
    return seq


def skew_order(tx, B, R, bw, bh, NB, band):
    """{tile row: [(sy, sx, kind), ...]} that lane tx of this band delivers, in delivery order."""
    W, T = 2 * R + 1, B + 2 * R
    rpb = (T + NB - 1) // NB
    tr0, tr1 = band * rpb, min(T, band * rpb + rpb)
    sr0, sr1 = max(0, tr0 - 2 * R), min(bh - 1, tr1 - 1)
    tmax = W * (min(B, rpb + 2 * R) - 1) + (B - 1)
    xwrap_lane = bw == B and tx <= 2 * R + 1 and bw - 1 > tx
    got = {ty: [] for ty in range(tr0, tr1)}
    seen_steps = set()
    for t0 in range(tmax + 1):
        t = t0 + W * sr0
        d = (tx - t) % W
        sx = tx - d
        assert (t - sx) % W == 0
        sy = (t - sx) // W
        if sx < 0 or sx >= bw or sy < sr0 or sy > sr1:
            continue
        assert t not in seen_steps  # one source per lane and step
        seen_steps.add(t)
        for ty in range(sy, sy + 2 * R + 1):
            if tr0 <= ty < tr1:
                got[ty].append((sy, sx, "n"))
        if xwrap_lane and sx == tx:
            for ty in range(sy, sy + 2 * R + 1):
                if tr0 <= ty < tr1:
                    got[ty].append((sy, bw - 1, "x"))
    if tr0 == 0 and bh == B:
        nr = min(2 * R + 2, B - 1)
        for sx in range(max(0, tx - 2 * R), min(bw - 1, tx) + 1):
            for ty in range(nr):
                got[ty].append((B - 1, sx, "y"))
        if xwrap_lane:
            for ty in range(nr):
                got[ty].append((B - 1, bw - 1, "y"))
    return got


@pytest.mark.parametrize("B,R", [(16, 2), (16, 1), (16, 3), (8, 2), (4, 2), (32, 1)])
@pytest.mark.parametrize("ragged", [False, True])
@pytest.mark.parametrize("NB", [1, 2])
def test_skew_schedule_is_addsample_order(B, R, ragged, NB):
    T = B + 2 * R
    bw, bh = (B - 3, B - 5) if ragged and B > 5 else (B, B)
    for band in range(NB):
        for tx in range(T):
            got = skew_order(tx, B, R, bw, bh, NB, band)
            for ty, seq in got.items():
                want = gather_order(tx, ty, B, R, bw, bh)
                # the y-wrap rows are the first band's: nr = min(2R+2, B-1) rows, which the
                # gather kernels reach as ty <= 2R+1 with bh-1 > ty
                assert seq == want, (B, R, bw, bh, NB, band, tx, ty)
