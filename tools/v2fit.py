"""Minimax fits of the frm semantics v2 builtin kernels.

Each kernel is a polynomial in float64 fitted by Lawson's algorithm (iteratively reweighted
least squares converging to the minimax solution) on a dense grid, with the coefficients then
rounded to f32 one at a time (the remaining ones refitted after each rounding). The error of
the f32 Horner evaluation (fma emulated in float64) is reported against float64 math.

    python tools/v2fit.py            # print every kernel's coefficients and errors
"""
import math
import sys

import numpy as np

f32 = np.float32


def fma32(a, b, c):
    # f32 fma emulated in float64: a*b is exact in float64, the sum may round twice (rare
    # one-ulp differences; the bit-exact definition lives in the oracle's C)
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)


def lawson(basis, target, weight, iters=300):
    """min over c of max |weight * (basis @ c - target)|; basis is (n_points, n_coef)."""
    A = basis * weight[:, None]
    b = target * weight
    w = np.full(len(b), 1.0 / len(b))
    best = None
    for _ in range(iters):
        sw = np.sqrt(w)
        c, *_ = np.linalg.lstsq(A * sw[:, None], b * sw, rcond=None)
        e = np.abs(A @ c - b)
        m = e.max()
        if best is None or m < best[0]:
            best = (m, c)
        w = w * (e + 1e-300)
        w /= w.sum()
    return best[1], best[0]


def fit_rounded(xs, basis_fn, target, weight, fixed=()):
    """Fit all coefficients, round the highest-order one to f32, refit the rest, ... so that
    each rounding is compensated by the lower-order coefficients. `fixed` pins leading
    low-order coefficients (e.g. the constant 1 of 2^f)."""
    B = basis_fn(xs)
    n = B.shape[1]
    coefs = [None] * n
    for i, v in fixed:
        coefs[i] = float(f32(v))
    free = [i for i in range(n) if coefs[i] is None]
    while free:
        tgt = target.copy()
        for i in range(n):
            if coefs[i] is not None:
                tgt = tgt - coefs[i] * B[:, i]
        c, _ = lawson(B[:, free], tgt, weight)
        hi = free[-1]  # highest-order free coefficient
        coefs[hi] = float(f32(c[-1]))
        free = free[:-1]
    return [f32(c) for c in coefs]


def horner32(coefs, x):
    """Horner in f32 with fma, coefs low -> high."""
    p = np.full_like(x, coefs[-1])
    for c in coefs[-2::-1]:
        p = fma32(p, x, np.full_like(x, c))
    return p


def ulp32(v):
    v = np.abs(v.astype(np.float64))
    e = np.floor(np.log2(np.maximum(v, 2.0**-126)))
    return 2.0 ** (e - 23)


# ---------------------------------------------------------------------------------------
def fit_sin(deg_u):
    """sin(pi r) = r * S(r^2), r in [0, 1/2]; relative error."""
    r = np.linspace(1e-6, 0.5, 20001)
    u = r * r
    tgt = np.sin(np.pi * r) / r
    c = fit_rounded(u, lambda u: np.vander(u, deg_u + 1, increasing=True), tgt, r / np.sin(np.pi * r))
    return c


def fit_cos(deg_u):
    """cos(pi r) = C(r^2), r in [0, 1/2]; absolute error, C(0) = 1 exactly."""
    r = np.linspace(0.0, 0.5, 20001)
    u = r * r
    c = fit_rounded(u, lambda u: np.vander(u, deg_u + 1, increasing=True), np.cos(np.pi * r),
                    np.ones_like(r), fixed=((0, 1.0),))
    return c


def fit_acos(deg):
    """acos(a) = sqrt(1 - a) * P(a), a in [0, 1]; relative error of acos."""
    a = np.linspace(0.0, 1.0 - 1e-9, 40001)
    tgt = np.arccos(a) / np.sqrt(1.0 - a)
    return fit_rounded(a, lambda a: np.vander(a, deg + 1, increasing=True), tgt, np.ones_like(a) / tgt)


def fit_atan(deg_s):
    """atan(a) = a + a s Q(s), s = a^2, a in [0, 1]; relative error of atan."""
    a = np.linspace(1e-6, 1.0, 40001)
    s = a * a
    tgt = (np.arctan(a) - a) / (a * s)
    w = (a * s) / np.arctan(a)
    return fit_rounded(s, lambda s: np.vander(s, deg_s + 1, increasing=True), tgt, w)


def fit_log2(deg):
    """log2(1 + f) = f Q(f), f in [sqrt(1/2) - 1, sqrt(2) - 1]; relative error."""
    f = np.linspace(math.sqrt(0.5) - 1.0, math.sqrt(2.0) - 1.0, 40001)
    f = f[np.abs(f) > 1e-7]
    tgt = np.log2(1.0 + f) / f
    return fit_rounded(f, lambda f: np.vander(f, deg + 1, increasing=True), tgt, 1.0 / tgt)


def fit_exp2(deg):
    """2^f = 1 + f P(f), f in [-1/2, 1/2]; relative error."""
    f = np.linspace(-0.5, 0.5, 40001)
    f = f[np.abs(f) > 1e-7]
    tgt = (np.exp2(f) - 1.0) / f
    return fit_rounded(f, lambda f: np.vander(f, deg, increasing=True), tgt, f / np.exp2(f))


# ---------------------------------------------------------------------------------------
def err_report():
    rng = np.random.default_rng(1)
    out = {}
    for deg in (3, 4):
        c = fit_sin(deg)
        r = np.linspace(0, 0.5, 1 << 20).astype(f32)
        u = (r * r).astype(f32)
        s = (r * horner32(c, u)).astype(f32)
        e = np.abs(s.astype(np.float64) - np.sin(np.pi * r.astype(np.float64)))
        out[f"sin u-deg{deg}"] = (c, e.max())
    for deg in (3, 4, 5):
        c = fit_cos(deg)
        r = np.linspace(0, 0.5, 1 << 20).astype(f32)
        u = (r * r).astype(f32)
        v = horner32(c, u)
        e = np.abs(v.astype(np.float64) - np.cos(np.pi * r.astype(np.float64)))
        out[f"cos u-deg{deg}"] = (c, e.max())
    for deg in (5, 6, 7):
        c = fit_acos(deg)
        a = np.linspace(0, 1, 1 << 20).astype(f32)
        v = (np.sqrt((f32(1) - a)).astype(f32) * horner32(c, a)).astype(f32)
        ref = np.arccos(a.astype(np.float64))
        e = np.abs(v - ref) / np.maximum(ref, 1e-30)
        out[f"acos deg{deg} (rel)"] = (c, e[ref > 0].max())
    for deg in (4, 5, 6):
        c = fit_atan(deg)
        a = np.linspace(0, 1, 1 << 20).astype(f32)
        s = (a * a).astype(f32)
        v = fma32((a * s).astype(f32), horner32(c, s), a)
        ref = np.arctan(a.astype(np.float64))
        e = np.abs(v - ref) / np.maximum(ref, 1e-30)
        out[f"atan s-deg{deg} (rel)"] = (c, e[ref > 0].max())
    for deg in (5, 6, 7, 8):
        c = fit_log2(deg)
        f = np.linspace(math.sqrt(0.5) - 1, math.sqrt(2) - 1, 1 << 20).astype(f32)
        v = (f * horner32(c, f)).astype(f32)
        ref = np.log2(1.0 + f.astype(np.float64))
        e = np.abs(v - ref) / np.maximum(np.abs(ref), 1e-30)
        out[f"log2 deg{deg} (rel)"] = (c, e[np.abs(ref) > 0].max())
    for deg in (4, 5):
        c = fit_exp2(deg)
        f = np.linspace(-0.5, 0.5, 1 << 20).astype(f32)
        v = fma32(f, horner32(c, f), np.ones_like(f))
        ref = np.exp2(f.astype(np.float64))
        e = np.abs(v - ref) / ref
        out[f"exp2 deg{deg} (rel)"] = (c, e.max())
    return out


if __name__ == "__main__":
    for k, (c, e) in err_report().items():
        print(f"{k:22s} max err {e:.3e} ({e / 2**-24:.2f} x 2^-24)  coefs " +
              ", ".join(f"{float(x).hex()}" for x in c))
    sys.exit(0)
