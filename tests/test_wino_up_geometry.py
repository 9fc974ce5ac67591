"""Host-side bound check for the Winograd kernel's fused upsample-add staging
(fvc_conv_wino.hip, UP form): the low-resolution rows and columns one fix-up reads must fit its
LDS area (kLowRows = 4 rows, kLowCols = 20 columns). Restates the kernel's index arithmetic
(fvc_up_index_scaled: float32 scale (in-1)/(out-1), src = scale * d, floor, clamp) in numpy float32
for every fix-up the kernel can issue (2 new rows of a continuing item, the 4-row window of a
chunk's first item, every 32-column group) at every even size up to 4352."""
import numpy as np

K_LOW_ROWS, K_LOW_COLS = 4, 20


def up_i0_i1(d, n_in, n_out):
    scale = np.float32(n_in - 1) / np.float32(n_out - 1) if n_out > 1 else np.float32(0)
    src = (scale * d.astype(np.float32)).astype(np.float32)
    i0 = np.floor(src).astype(np.int64)
    i0 = np.minimum(i0, n_in - 1)
    i1 = i0 + (i0 < n_in - 1)
    return i0, i1


def test_fixup_rows_fit_lds():
    worst = 0
    for H in range(2, 4354, 2):
        hl = H // 2
        tiles = (H + 1) // 2
        ty = np.arange(tiles)
        for r0, nr in ((2 * ty + 1, 2), (2 * ty - 1, 4)):
            rf = np.maximum(r0, 0)
            rl = np.minimum(r0 + nr - 1, H - 1)
            ok = rf <= rl
            lo, _ = up_i0_i1(rf[ok], hl, H)
            _, hi = up_i0_i1(rl[ok], hl, H)
            if hi.size:
                worst = max(worst, int((hi - lo + 1).max()))
    assert worst <= K_LOW_ROWS, worst


def test_fixup_columns_fit_lds():
    worst = 0
    for W in range(2, 4354, 2):
        wl = W // 2
        g = np.arange((W + 31) // 32)
        cf = np.maximum(32 * g - 1, 0)
        cl = np.minimum(32 * g + 32, W - 1)
        lo, _ = up_i0_i1(cf, wl, W)
        _, hi = up_i0_i1(cl, wl, W)
        worst = max(worst, int((hi - lo + 1).max()))
    assert worst <= K_LOW_COLS, worst


def test_every_tap_inside_the_staged_span():
    """Each output pixel's two source rows / columns lie inside its fix-up's staged span (the
    kernel indexes `low` by i - lr0 / i - lc0 without a bound check)."""
    for n in (2, 4, 30, 36, 70, 98, 120, 136, 544, 960, 1088, 1920, 2176, 3840):
        nl = n // 2
        d = np.arange(n)
        i0, i1 = up_i0_i1(d, nl, n)
        assert (i0 >= 0).all() and (i1 <= nl - 1).all() and (i1 - i0 <= 1).all()
        # columns: every group's span covers its 34 ring columns' taps
        for g in range((n + 31) // 32):
            cols = np.arange(max(32 * g - 1, 0), min(32 * g + 32, n - 1) + 1)
            a0, a1 = up_i0_i1(cols, nl, n)
            lc0 = a0.min()
            assert (a1 - lc0 < K_LOW_COLS).all() and (a0 >= lc0).all()
