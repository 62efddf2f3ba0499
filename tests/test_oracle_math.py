"""Accuracy of the oracle's deterministic transcendentals.

The reference's libdevice pow/sinf/cosf/asinf/atanf cannot be run here; the restatement
evaluates them in double and rounds.  These checks bound that restatement against numpy's
double-precision libm: the float results must equal the correctly rounded float of the
libm double result except in rare near-tie cases, and never be more than 1 ulp off.
"""
import numpy as np
import pytest

RNG = np.random.default_rng(7)


def _ulp_diff(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, np.int64(-(2 ** 31)) - a, a)
    b = np.where(b < 0, np.int64(-(2 ** 31)) - b, b)
    return np.abs(a - b)


def _check(got, want, min_exact=0.9999):
    want = want.astype(np.float32)
    d = _ulp_diff(got, want)
    assert d.max() <= 1, f"max ulp diff {d.max()}"
    assert (d == 0).mean() >= min_exact, f"exact fraction {(d == 0).mean()}"


def test_sin_cos_phi_range(oracle_mod):
    # phi = (float)(2*M_PI*x2), x2 in (0,1]: the lobe's argument range (material.cu:25)
    x = (RNG.random(200000) * 2 * np.pi).astype(np.float32)
    _check(oracle_mod.math_batch(1, x), np.sin(x.astype(np.float64)))
    _check(oracle_mod.math_batch(2, x), np.cos(x.astype(np.float64)))


def test_sin_cos_wide_range(oracle_mod):
    x = ((RNG.random(100000) - 0.5) * 2e4).astype(np.float32)
    _check(oracle_mod.math_batch(1, x), np.sin(x.astype(np.float64)))
    _check(oracle_mod.math_batch(2, x), np.cos(x.astype(np.float64)))


def test_asin_atan(oracle_mod):
    x = (RNG.random(200000) * 2 - 1).astype(np.float32)
    _check(oracle_mod.math_batch(3, x), np.arcsin(x.astype(np.float64)))
    y = (np.tan((RNG.random(200000) - 0.5) * np.pi)).astype(np.float32)
    _check(oracle_mod.math_batch(4, y), np.arctan(y.astype(np.float64)))
    edge = np.array([-1, 1, 0, -0.0, 1e-30, -1e-30, np.inf, -np.inf], dtype=np.float32)
    got = oracle_mod.math_batch(4, edge)
    np.testing.assert_array_equal(got, np.arctan(edge.astype(np.float64)).astype(np.float32))
    got = oracle_mod.math_batch(3, np.array([-1, 1, 0, 0.5, -0.5], dtype=np.float32))
    np.testing.assert_array_equal(got, np.arcsin(np.array([-1, 1, 0, 0.5, -0.5])).astype(np.float32))
    assert np.isnan(oracle_mod.math_batch(3, np.array([1.5, np.nan], dtype=np.float32))).all()


def test_pow_lobe_exponents(oracle_mod):
    # z = pow(x1, 1/alpha), x1 = curand_uniform in (0,1], alpha = 1000^s or 2 (material.cu:24,45)
    x = (RNG.random(200000).astype(np.float32) + np.float32(2 ** -33)).astype(np.float32)
    for alpha in (2.0, 31.6227766, 1000.0, 1e6, 1e12):
        got = oracle_mod.math_batch(5, x, np.full_like(x, alpha))
        want = np.power(x.astype(np.float64), 1.0 / np.float64(np.float32(alpha)))
        _check(got, want)


def test_powf(oracle_mod):
    s = (RNG.random(100000) * 6).astype(np.float32)
    got = oracle_mod.math_batch(0, np.full_like(s, 1000.0), s)
    _check(got, np.power(1000.0, s.astype(np.float64)))
    b = (RNG.random(100000) * 2 - 0.5).astype(np.float32)        # schlick: pow(1 - cos, 5)
    got = oracle_mod.math_batch(0, b, np.full_like(b, 5.0))
    _check(got, np.power(b.astype(np.float64), 5.0))


@pytest.mark.parametrize("x,y,want", [(0.0, 5.0, 0.0), (1.0, 123.0, 1.0), (2.0, 0.0, 1.0), (-2.0, 5.0, -32.0),
                                      (-2.0, 4.0, 16.0)])
def test_pow_special(oracle_mod, x, y, want):
    assert oracle_mod.lib().or_pow(x, y) == pytest.approx(want, rel=1e-15, abs=0)
    assert np.isnan(oracle_mod.lib().or_pow(-2.0, 0.5))


def test_pow5_schlick(oracle_mod):
    # (1 - cosine)^5 in schlick (ray_tracing_math.hpp:68): cosine in [-1, 1], and the specials
    x = (RNG.random(200000) * 2).astype(np.float32)
    _check(oracle_mod.math_batch(9, x), np.power(x.astype(np.float64), 5))
    edge = np.array([0.0, 1.0, 2.0, 1e-30, 3e7, np.inf], np.float32)
    with np.errstate(over="ignore"):
        np.testing.assert_array_equal(oracle_mod.math_batch(9, edge), np.power(edge.astype(np.float64), 5).astype(np.float32))
    assert np.isnan(oracle_mod.math_batch(9, np.array([np.nan], np.float32))).all()
