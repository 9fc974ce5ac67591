"""CPU emulation of the split-precision conv arithmetic against float64 (VERDICT r4 #2 / #5 gate).

Emulates, for a 64 -> 64 3x3 layer (seeded Warp_net ResBlock weights) and SpyNet's 7x7 layers:
* direct x3 (conv_x3_kernel): x and 2^kw-scaled w split exactly into fp16 hi + lo * 2^-11,
  main = sum w_hi x_hi, corr = sum (w_lo x_hi + w_hi x_lo), each MFMA's K-block summed exactly and
  rounded once to fp32 into an fp32 accumulator;
* Winograd F(m x m, 3 x 3) / 1-D F(m, r) in the same split arithmetic: input transform in fp32,
  V split (scaled by a power of two so |V| stays below the fp16 range), U = G g G^T in double,
  scaled and split, M per position as above, output transform in fp32;
and prints max |y - y64| / max |y64| (the tests' "of scale" measure) and the mean.

python scripts/wino_accuracy.py
"""
import os
import sys
from fractions import Fraction as Fr

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

F16 = np.float16
F32 = np.float32


def split(v, scale_exp=0):
    """v (float32/64) * 2^scale_exp -> (hi, lo) float64 values of the fp16 halves (lo in units 2^-11)."""
    v = np.asarray(v, np.float64) * 2.0 ** scale_exp
    v32 = v.astype(F32)
    hi = v32.astype(F16).astype(np.float64)
    lo = ((v32.astype(np.float64) - hi) * 2048.0).astype(F32).astype(F16).astype(np.float64)
    return hi, lo


def kblock_dot(a, b, kb):
    """sum over the last axis of a[..., K] * b[..., K] with exact K-block sums rounded to fp32 and
    accumulated in fp32 (MFMA model). a: [M, K], b: [K, N] -> [M, N]."""
    M, K = a.shape
    acc = np.zeros((M, b.shape[1]), F32)
    for k0 in range(0, K, kb):
        acc = (acc + (a[:, k0:k0 + kb] @ b[k0:k0 + kb]).astype(F32)).astype(F32)
    return acc


def toom(m, r, pts):
    """Correlation F(m, r) matrices from interpolation points (+ infinity): A^T, G, B^T as float64;
    G solved exactly (sympy) from the bilinear identity."""
    import sympy
    n = m + r - 1
    P = [Fr(p) for p in pts]

    def prod_poly(roots):
        poly = [Fr(1)]
        for a in roots:
            poly = [Fr(0)] + poly
            for k in range(len(poly) - 1):
                poly[k] -= a * poly[k + 1]
        return poly
    AT = [[P[j] ** i for j in range(n - 1)] + [Fr(1 if i == m - 1 else 0)] for i in range(m)]
    BT = [prod_poly([P[l] for l in range(n - 1) if l != j]) + [Fr(0)] for j in range(n - 1)] + [prod_poly(P)]
    G = sympy.Matrix(n, r, lambda j, k: sympy.Symbol(f"g{j}_{k}"))
    R = lambda x: sympy.Rational(x.numerator, x.denominator)  # noqa: E731
    eqs = [sum(R(AT[i][j]) * G[j, k] * R(BT[j][l]) for j in range(n)) - (1 if l == i + k else 0)
           for i in range(m) for k in range(r) for l in range(n)]
    sol = sympy.solve(eqs, list(G), dict=True)[0]
    Gm = np.array(G.subs(sol).tolist(), dtype=np.float64)
    return (np.array([[float(x) for x in row] for row in AT]), Gm,
            np.array([[float(x) for x in row] for row in BT]))


def conv64(x, w):
    """float64 reference correlation, zero padding (k-1)/2: x [C, H, W], w [O, C, k, k]."""
    C, H, W = x.shape
    k = w.shape[-1]
    p = k // 2
    xp = np.pad(x, ((0, 0), (p, p), (p, p)))
    cols = np.stack([xp[:, i:i + H, j:j + W] for i in range(k) for j in range(k)], 1)  # [C, k*k, H, W]
    return np.einsum("ocq,cqhw->ohw", w.reshape(w.shape[0], C, k * k), cols)


def kw_exp(wmax):
    return 14 - int(np.frexp(wmax)[1])


def direct_x3(x, w, kb=16):
    O, C, k, _ = w.shape
    H, W = x.shape[1:]
    p = k // 2
    kw = kw_exp(np.abs(w).max())
    wh, wl = split(w, kw)
    xh, xl = split(x)
    xph, xpl = np.pad(xh, ((0, 0), (p, p), (p, p))), np.pad(xl, ((0, 0), (p, p), (p, p)))
    # K order: tap-major, channel-minor (as the kernel's k-steps: (tap, 8 channels) blocks)
    colh = np.stack([xph[:, i:i + H, j:j + W] for i in range(k) for j in range(k)], 0).reshape(k * k * C, H * W)
    coll = np.stack([xpl[:, i:i + H, j:j + W] for i in range(k) for j in range(k)], 0).reshape(k * k * C, H * W)
    Wh = wh.transpose(0, 2, 3, 1).reshape(O, k * k * C)
    Wl = wl.transpose(0, 2, 3, 1).reshape(O, k * k * C)
    main = kblock_dot(Wh, colh, kb)
    cor = kblock_dot(Wl, colh, kb)
    cor = (cor + kblock_dot(Wh, coll, kb)).astype(F32)
    y = (main + cor * F32(1 / 2048)).astype(F32) * F32(2.0 ** -kw)
    return y.reshape(O, H, W)


def fp32_direct(x, w, kb=2):
    """fp32-MFMA kernel model: fp32 products, K-block sums rounded to fp32."""
    O, C, k, _ = w.shape
    H, W = x.shape[1:]
    p = k // 2
    xp = np.pad(x, ((0, 0), (p, p), (p, p))).astype(F32).astype(np.float64)
    col = np.stack([xp[:, i:i + H, j:j + W] for i in range(k) for j in range(k)], 0).reshape(k * k * C, H * W)
    Wm = w.astype(F32).astype(np.float64).transpose(0, 2, 3, 1).reshape(O, k * k * C)
    # products rounded to fp32, accumulated in fp32 (FMA chain model)
    acc = np.zeros((O, H * W), F32)
    for k0 in range(0, col.shape[0], kb):
        acc = (acc + (Wm[:, k0:k0 + kb] @ col[k0:k0 + kb]).astype(F32)).astype(F32)
    return acc.reshape(O, H, W)


def wino2d(x, w, mh, mw, pts_h, pts_w, kb=32, vscale=None):
    """Winograd F(mh x mw, 3 x 3) in split precision (kb = channels per MFMA K block)."""
    O, C, r, _ = w.shape
    H, W = x.shape[1:]
    ATh, Gh, BTh = toom(mh, r, pts_h)
    ATw, Gw, BTw = toom(mw, r, pts_w)
    nh, nw = mh + r - 1, mw + r - 1
    th, tw = -(-H // mh), -(-W // mw)
    p = r // 2
    xp = np.zeros((C, th * mh + r - 1, tw * mw + r - 1), F32)
    xp[:, p:p + H, p:p + W] = x
    # input patches [C, th, tw, nh, nw]
    patches = np.stack([np.stack([xp[:, a * mh:a * mh + nh, b * mw:b * mw + nw] for b in range(tw)], 1)
                        for a in range(th)], 1)
    # V = B^T d B in fp32: rows first (the kernel's E), then columns
    BTh32, BTw32 = BTh.astype(F32), BTw.astype(F32)
    E = np.einsum("ij,ctajk->ctaik", BTh32, patches.astype(F32)).astype(F32)
    V = np.einsum("ctaik,lk->ctail", E, BTw32).astype(F32)   # [C, th, tw, nh, nw]
    vmax = float(np.abs(V).max())
    if vscale is None:
        vscale = 0
        while vmax * 2.0 ** vscale >= 32768:
            vscale -= 1
    U = np.einsum("ij,ocjk,lk->ocil", Gh, w, Gw)               # [O, C, nh, nw] float64
    kw = kw_exp(np.abs(U).max())
    uh, ul = split(U, kw)
    vh, vl = split(V, vscale)
    T = th * tw
    M = np.zeros((O, T, nh, nw), F32)
    for i in range(nh):
        for j in range(nw):
            a_h, a_l = uh[:, :, i, j], ul[:, :, i, j]              # [O, C]
            b_h = vh[:, :, :, i, j].reshape(C, T)
            b_l = vl[:, :, :, i, j].reshape(C, T)
            main = kblock_dot(a_h, b_h, kb)
            cor = (kblock_dot(a_l, b_h, kb) + kblock_dot(a_h, b_l, kb)).astype(F32)
            M[:, :, i, j] = (cor * F32(1 / 2048) + main).astype(F32)
    Z = np.einsum("otij,lj->otil", M, ATw.astype(F32)).astype(F32)
    Y = np.einsum("ki,otil->otkl", ATh.astype(F32), Z).astype(F32) * F32(2.0 ** (-kw - vscale))
    Y = Y.reshape(O, th, tw, mh, mw).transpose(0, 1, 3, 2, 4).reshape(O, th * mh, tw * mw)
    return Y[:, :H, :W], vscale


def wino_rows(x, w, m, pts, kb=32, vscale=None):
    """1-D Winograd F(m, k) along rows (columns of the image), direct over the k kernel rows:
    per output row and position j, M[j] = sum over (kernel row dy, channel) of U[dy][j] V[dy][j]."""
    O, C, k, _ = w.shape
    H, W = x.shape[1:]
    AT, G, BT = toom(m, k, pts)
    n = m + k - 1
    tw = -(-W // m)
    p = k // 2
    xp = np.zeros((C, H + k - 1, tw * m + k - 1), F32)
    xp[:, p:p + H, p:p + W] = x
    # V[c, row, tile, j] = sum_l BT[j][l] xp[c, row, tile*m + l] (fp32)
    pat = np.stack([xp[:, :, b * m:b * m + n] for b in range(tw)], 2)      # [C, Hp, tw, n]
    V = np.einsum("jl,crtl->crtj", BT.astype(F32), pat.astype(F32)).astype(F32)
    vmax = float(np.abs(V).max())
    if vscale is None:
        vscale = 0
        while vmax * 2.0 ** vscale >= 32768:
            vscale -= 1
    U = np.einsum("jq,ocdq->ocdj", G, w)                                     # [O, C, dy, n]
    kw = kw_exp(np.abs(U).max())
    uh, ul = split(U, kw)
    vh, vl = split(V, vscale)
    M = np.zeros((O, H, tw, n), F32)
    for j in range(n):
        # K = (dy, c): rows y + dy of the padded input
        a_h = uh[:, :, :, j].transpose(0, 2, 1).reshape(O, k * C)
        a_l = ul[:, :, :, j].transpose(0, 2, 1).reshape(O, k * C)
        b_h = np.stack([vh[:, dy:dy + H, :, j] for dy in range(k)], 0).reshape(k * C, H * tw)
        b_l = np.stack([vl[:, dy:dy + H, :, j] for dy in range(k)], 0).reshape(k * C, H * tw)
        main = kblock_dot(a_h, b_h, kb)
        cor = (kblock_dot(a_l, b_h, kb) + kblock_dot(a_h, b_l, kb)).astype(F32)
        M[..., j] = (cor * F32(1 / 2048) + main).astype(F32).reshape(O, H, tw)
    Y = np.einsum("ij,ohtj->ohti", AT.astype(F32), M).astype(F32) * F32(2.0 ** (-kw - vscale))
    return Y.reshape(O, H, tw * m)[:, :, :W], vscale


def report(name, y, y64):
    s = np.abs(y64).max()
    e = np.abs(y.astype(np.float64) - y64)
    print(f"  {name:34s} max {e.max() / s:.2e}  mean {e.mean() / s:.2e}  of scale", flush=True)
    return e.max() / s


def main():
    from fastvideocodec_amd.weights import seeded_torch_state_dict
    sd = seeded_torch_state_dict()
    w = sd["warpnet.conv0.conv1.weight"].numpy().astype(np.float64)
    rng = np.random.default_rng(0)
    H = W = 48
    print("64->64 3x3 (warpnet.conv0.conv1, seeded), 48x48, relu(N(0, s)) inputs")
    for s in (1e-2, 1.0, 30.0):
        x = np.maximum(rng.normal(0, s, (64, H, W)), 0).astype(F32)
        y64 = conv64(x.astype(np.float64), w)
        print(f" input scale {s}")
        report("direct x3 (conv_x3_kernel)", direct_x3(x, w), y64)
        report("fp32 FMA chain (conv_mfma_f32)", fp32_direct(x, w), y64)
        report("F(2x2,3x3) 0,1,-1 (conv_wino_kernel)", wino2d(x, w, 2, 2, [0, 1, -1], [0, 1, -1])[0], y64)
        report("F(2x4) rows 0,1,-1 cols 0,1,-1,2,-2", wino2d(x, w, 2, 4, [0, 1, -1], [0, 1, -1, 2, -2])[0], y64)
        report("F(2x4) cols 0,1,-1,1/2,-2", wino2d(x, w, 2, 4, [0, 1, -1], [0, 1, -1, Fr(1, 2), -2])[0], y64)
        report("F(4x4) 0,1,-1,2,-2 (Lavin)", wino2d(x, w, 4, 4, [0, 1, -1, 2, -2], [0, 1, -1, 2, -2])[0], y64)
        report("F(4x4) 0,1,-1,1/2,-2", wino2d(x, w, 4, 4, [0, 1, -1, Fr(1, 2), -2], [0, 1, -1, Fr(1, 2), -2])[0], y64)
        report("F(4x4) 0,1,-1,1/2,-1/2", wino2d(x, w, 4, 4, [0, 1, -1, Fr(1, 2), Fr(-1, 2)],
                                                 [0, 1, -1, Fr(1, 2), Fr(-1, 2)])[0], y64)


def main_spynet():
    from fastvideocodec_amd.weights import seeded_torch_state_dict
    sd = seeded_torch_state_dict()
    rng = np.random.default_rng(1)
    H, W = 24, 48
    for name in ("opticFlow.moduleBasic.3.conv2.weight", "opticFlow.moduleBasic.3.conv3.weight"):
        w = sd[name].numpy().astype(np.float64)
        x = np.maximum(rng.normal(0, 1.0, (w.shape[1], H, W)), 0).astype(F32)
        y64 = conv64(x.astype(np.float64), w)
        print(f"{name} {tuple(w.shape)} (pretrained SpyNet), {H}x{W}, relu(N(0,1)) inputs")
        report("direct x3 (conv_x3_kernel)", direct_x3(x, w), y64)
        report("fp32 FMA chain (conv_mfma_f32)", fp32_direct(x, w), y64)
        report("rows F(2,7) 0,1,-1,2,-2,1/2,-1/2", wino_rows(x, w, 2, [0, 1, -1, 2, -2, Fr(1, 2), Fr(-1, 2)])[0], y64)
        report("rows F(2,7) 0,1,-1,2,-2,3,1/2", wino_rows(x, w, 2, [0, 1, -1, 2, -2, 3, Fr(1, 2)])[0], y64)
        report("rows F(1+... ) check: F(1,7) 0..", wino_rows(x, w, 1, [0, 1, -1, 2, -2, Fr(1, 2)])[0], y64)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "spynet":
        main_spynet()
        sys.exit(0)
    main()
