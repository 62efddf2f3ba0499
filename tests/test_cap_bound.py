"""The cylinder cap test's bound (cpt_capi.cpp cap_disk_bound, cpt_path.hpp cap_test): the
kernels decide the reference's `sqrtf(q) < radius` (object.cu:52-77) as `q <= bound`.  Host
only: the bound comes from libcpt.so's test hook, the truth from numpy's correctly rounded
float32 sqrt, over radii of every magnitude and q at and around each bound."""
import ctypes

import numpy as np

from cpppathtracer_amd import _lib


def _bound(r):
    out = ctypes.c_float()
    assert _lib.load().cpt_cap_disk_bound(ctypes.c_float(float(r)), ctypes.byref(out)) == 0
    return np.float32(out.value)


def _radii():
    rng = np.random.default_rng(11)
    r = [np.float32(x) for x in (1.0, 2.0, 0.5, 3.0, 1e-3, 7.25, 100.0, 1e19, 3e38)]
    r += [np.float32(2.0) ** k for k in range(-149, 128, 7)]                   # powers of two
    r += list((rng.random(300) * 20).astype(np.float32))                       # scene-sized
    r += list(np.exp(rng.uniform(-100, 87, 300)).astype(np.float32))          # any magnitude
    r += list(np.frombuffer(rng.integers(1, 0x7f800000, 200, dtype=np.uint32).astype(np.uint32).tobytes(),
                            dtype=np.float32))                                 # any bit pattern
    return [x for x in r if np.isfinite(x) and x > 0]


def test_bound_decides_like_sqrt():
    for r in _radii():
        c = _bound(r)
        bits = np.array([c], np.float32).view(np.int32)[0]
        near = np.arange(bits - 40, bits + 41, dtype=np.int64)
        near = near[(near >= 0) & (near < 0x7f800000)].astype(np.int32).view(np.float32)
        rng = np.random.default_rng(int(np.array([r], np.float32).view(np.uint32)[0]))
        wide = (np.float32(r) * np.float32(r) * rng.uniform(0, 4, 200)).astype(np.float32)
        q = np.concatenate([near, wide, np.array([0.0, np.inf], np.float32)]).astype(np.float32)
        want = np.sqrt(q) < np.float32(r)
        got = q <= c
        assert (want == got).all(), (r, c, q[want != got][:5])
        wn = np.sqrt(near) < np.float32(r)
        assert wn[near <= c].all() and not wn[near > c].any()   # c is the largest such float


def test_degenerate_radii():
    for r in (0.0, -1.0, -0.0, float("nan")):
        c = _bound(r)
        q = np.array([0.0, 1e-45, 1.0, np.inf], np.float32)
        assert not (q <= c).any()
    assert _bound(float("inf")) == np.finfo(np.float32).max
