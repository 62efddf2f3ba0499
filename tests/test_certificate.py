"""The winner certificate's quotient-free form (cpt_path.hpp cert_inside) restated in numpy and
checked against the exact slab test it stands in for (bvh.cu:181-200 with IEEE f32 quotients,
as cpt_path.hpp slab_reject<true> computes them): whenever the quotient-free form certifies a
box at tmax = t, the exact test passes it.  numpy's float32 arithmetic is IEEE round-to-nearest,
and the fma is exact here in float64 (P - 2^-21 |P| needs at most 45 significant bits) before its
one rounding to float32.  Cases: random boxes and rays, and distances t placed within a few ulps
of each box plane's exact quotient (the only place the two forms can disagree)."""
import numpy as np

F = np.float32
TMAX_DEFAULT = F(1e30)


def exact_passes(a, b, o, d, t, tmin):
    """Not slab_reject: a, b (..., 3) box planes, o, d (..., 3) ray, t the winner's distance."""
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        t0 = (a - o) / d
        t1 = (b - o) / d
    use = d != 0
    lo = np.where(use, np.minimum(t0, t1), F(-2e30)).max(axis=-1)
    hi = np.where(use, np.maximum(t0, t1), F(2e30)).min(axis=-1)
    lo = np.maximum(lo, F(-2e30))
    hi = np.minimum(hi, F(2e30))
    return ~((lo > hi) | (lo > t) | (hi < tmin))


def cert_inside(a, b, o, d, t):
    s_a = a - o
    s_b = b - o
    with np.errstate(over="ignore", invalid="ignore"):
        P = (t[..., None] * d).astype(F)
        p64 = P.astype(np.float64)
        T = (p64 - np.abs(p64) * 2.0 ** -21).astype(F)
        U = (p64 + np.abs(p64) * 2.0 ** -21).astype(F)
        ok = (d == 0) | ((s_a <= T) & (s_b >= U) & (np.abs(P) >= F(2.0 ** -100)))
    return ok.all(axis=-1)


def _cases(rng, n):
    c = rng.uniform(-30, 30, (n, 3)).astype(F)
    ext = np.exp(rng.uniform(np.log(1e-3), np.log(10), (n, 3))).astype(F)
    a, b = (c - ext).astype(F), (c + ext).astype(F)
    # a few platform-like slabs: unbounded in x and z, +-1e-4 in y
    plat = rng.random(n) < 0.1
    a[plat, 0] = F(-5e30); b[plat, 0] = F(5e30)
    a[plat, 2] = F(-5e30); b[plat, 2] = F(5e30)
    a[plat, 1] = c[plat, 1] - F(1e-4); b[plat, 1] = c[plat, 1] + F(1e-4)
    o = rng.uniform(-60, 60, (n, 3)).astype(F)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(F)
    # axis-parallel rays (d == 0 on an axis: skipped by the reference)
    zero = rng.random((n, 3)) < 0.03
    d[zero] = F(0)
    return a, b, o, d


def _near_plane_t(rng, a, b, o, d):
    """t within a few ulps of one of the six planes' exact quotients."""
    n = a.shape[0]
    ax = rng.integers(0, 3, n)
    side = rng.random(n) < 0.5
    plane = np.where(side, a[np.arange(n), ax], b[np.arange(n), ax])
    dd = d[np.arange(n), ax]
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        q = ((plane - o[np.arange(n), ax]) / dd).astype(F)
    k = rng.integers(-16, 17, n).astype(np.int32)
    t = (q.view(np.int32) + np.where(q >= 0, k, -k)).view(F)
    return t


def test_certificate_implies_exact_pass():
    rng = np.random.default_rng(20261018)
    tmin = F(1e-3)
    n_cert = n_total = 0
    for it in range(8):
        a, b, o, d = _cases(rng, 250_000)
        if it % 2 == 0:
            t = _near_plane_t(rng, a, b, o, d)
        else:
            # the box's own range along the ray, sampled: mostly inside, some just outside
            with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
                t0 = (a - o) / d
                t1 = (b - o) / d
            lo = np.where(d != 0, np.minimum(t0, t1), F(-2e30)).max(axis=1)
            hi = np.where(d != 0, np.maximum(t0, t1), F(2e30)).min(axis=1)
            u = rng.uniform(-0.05, 1.05, a.shape[0])
            t = (lo.astype(np.float64) + u * (hi.astype(np.float64) - lo)).astype(F)
        good = np.isfinite(t) & (t > tmin) & (t < TMAX_DEFAULT)
        a, b, o, d, t = a[good], b[good], o[good], d[good], t[good]
        cert = cert_inside(a, b, o, d, t)
        exact = exact_passes(a, b, o, d, t, tmin)
        bad = cert & ~exact
        assert not bad.any(), (a[bad][:3], b[bad][:3], o[bad][:3], d[bad][:3], t[bad][:3])
        n_cert += int(cert.sum())
        n_total += int(exact.sum())
    # the quotient-free form decides almost every passing box by itself
    assert n_cert > 0.5 * n_total


def test_certificate_decides_interior_hits():
    """Hits well inside their box (the common case: a sphere hit is at least its radius times a
    small factor inside its bounding cube on most axes) are certified without the exact test."""
    rng = np.random.default_rng(7)
    a, b, o, d = _cases(rng, 200_000)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        t0 = (a - o) / d
        t1 = (b - o) / d
    lo = np.where(d != 0, np.minimum(t0, t1), F(-2e30)).max(axis=1)
    hi = np.where(d != 0, np.maximum(t0, t1), F(2e30)).min(axis=1)
    t = (0.5 * (lo.astype(np.float64) + hi)).astype(F)
    good = (hi > lo) & (lo > 1.0) & (hi < 1e4) & ((hi - lo) > 1e-3 * hi)
    a, b, o, d, t = a[good], b[good], o[good], d[good], t[good]
    cert = cert_inside(a, b, o, d, t)
    assert exact_passes(a, b, o, d, t, F(1e-3)).all()
    assert cert.mean() > 0.999
