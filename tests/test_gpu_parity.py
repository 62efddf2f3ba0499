"""GPU parity: the HIP kernels in libcpt.so vs the CPU oracle, bit for bit.

The integrator is integer RNG + IEEE float arithmetic with FMA contraction off on both
sides and deterministic transcendentals, so the bar here is exact equality of the
per-pixel radiance sums, the XORWOW end states and the traversal counters — stronger than
the north star's RMSE < 1e-4 (which test_gpu_full_size checks at full size).
"""
import numpy as np
import pytest

from cpppathtracer_amd import camera_get_copy, scenes, types

pytestmark = pytest.mark.gpu
RNG = np.random.default_rng(11)


# ------------------------------------------------------------------------------ math
@pytest.mark.parametrize("op", [1, 2, 3, 4])
def test_unary_math_bitexact(gpu, oracle_mod, op):
    x = np.concatenate([
        (RNG.random(300000) * 2 * np.pi).astype(np.float32),
        ((RNG.random(100000) - 0.5) * 2e4).astype(np.float32),
        (RNG.random(100000) * 2 - 1).astype(np.float32),
        np.tan((RNG.random(100000) - 0.5) * np.pi).astype(np.float32),
        np.array([0, -0.0, 1, -1, 1e-30, -1e-38, 1e-45, np.inf, -np.inf, np.nan, 3.4e38], np.float32),
    ])
    g = gpu.math_batch(op, x)
    o = oracle_mod.math_batch(op, x)
    np.testing.assert_array_equal(g.view(np.uint32), o.view(np.uint32))


def test_pow5_bitexact(gpu, oracle_mod):
    # schlick's (1 - cosine)^5 (op 9): GPU and oracle evaluate the same three double products
    x = np.concatenate([(RNG.random(400000) * 2).astype(np.float32),
                        ((RNG.random(100000) - 0.5) * 1e3).astype(np.float32),
                        np.array([0, -0.0, 1, 2, 1e-30, 1e-45, np.inf, -np.inf, np.nan, 3.4e38], np.float32)])
    np.testing.assert_array_equal(gpu.math_batch(9, x).view(np.uint32), oracle_mod.math_batch(9, x).view(np.uint32))


@pytest.mark.parametrize("op", [0, 5])
def test_binary_pow_bitexact(gpu, oracle_mod, op):
    a = np.concatenate([RNG.random(200000).astype(np.float32) + np.float32(2 ** -33),
                        (RNG.random(50000) * 2 - 0.5).astype(np.float32),
                        np.array([0, 1, -2, np.nan, np.inf, 1e-40], np.float32)])
    b = np.concatenate([(RNG.random(200000) * 6).astype(np.float32),
                        np.full(50000, 5.0, np.float32),
                        np.array([5, 3, 5, 2, 2, 0.5], np.float32)])
    if op == 0:
        a[:200000] = 1000.0
    else:
        b = np.abs(b) + np.float32(1.0)
    g = gpu.math_batch(op, a, b)
    o = oracle_mod.math_batch(op, a, b)
    np.testing.assert_array_equal(g.view(np.uint32), o.view(np.uint32))


def test_ieee_div_sqrt(gpu):
    a = (RNG.standard_normal(500000) * 10.0 ** RNG.integers(-30, 30, 500000)).astype(np.float32)
    b = (RNG.standard_normal(500000) * 10.0 ** RNG.integers(-30, 30, 500000)).astype(np.float32)
    np.testing.assert_array_equal(gpu.math_batch(7, a, b).view(np.uint32), (a / b).view(np.uint32))
    with np.errstate(over="ignore"):   # quotients past f32 range round to inf, as on the GPU
        want = (a.astype(np.float64) / b.astype(np.float64)).astype(np.float32)
    np.testing.assert_array_equal(gpu.math_batch(6, a, b).view(np.uint32), want.view(np.uint32))
    s = np.abs(a)
    np.testing.assert_array_equal(gpu.math_batch(8, s).view(np.uint32), np.sqrt(s).view(np.uint32))


@pytest.mark.parametrize("which,n", [(0, 1 << 32), (1, 1 << 32), (2, 1 << 32)])
def test_exact_quotient_selftest(gpu, which, n):
    """qdiv(a, RN64(1/d)) == IEEE f32 a/d (cpt_device.hpp): 4.3e9 hashed pairs per family,
    compared on the device against the hardware v_div_* sequence."""
    cnt, pairs = gpu.selftest_qdiv(which, n, seed=which + 1)
    assert cnt == 0, [(float(a), float(d), float(a) / float(d)) for a, d in pairs]


def test_rcp_d_exhaustive(gpu):
    """rcp_d (v_rcp_f64 + two Newton steps, cpt_device.hpp) == the IEEE 1.0 / (double)d for
    every one of the 2^32 float bit patterns d (+-0, +-inf, NaN and subnormals included)."""
    cnt, pairs = gpu.selftest_qdiv(3, 1 << 32)
    assert cnt == 0, [float(d) for _, d in pairs]


def test_rcp_exhaustive(gpu):
    """rcp_f (v_rcp_f32 + one Newton step, cpt_device.hpp) == the IEEE 1.0f / d for every
    float pattern d with 2^-126 <= |d| < 2^126 (and 0, inf, NaN), and rcp_f(sqrtf(d)) ==
    1.0f / sqrtf(d) for all 2^32 patterns (normalize and to_world take that form)."""
    cnt, pairs = gpu.selftest_qdiv(4, 1 << 32)
    assert cnt == 0, [float(d) for _, d in pairs]


def test_sqrt_nn_exhaustive(gpu):
    """sqrt_nn (v_sqrt_f32 + the +-1 ulp residual correction without the tiny-argument scaling,
    cpt_device.hpp) == the IEEE sqrtf for every float pattern of its domain: +-0, |x| >= 2^-96,
    inf, NaN (the BSDF's 1 - z*z and squared lengths of near-unit vectors).  Outside it: v_sqrt_f32
    gives a negative subnormal's square root as -0 where sqrtf gives NaN."""
    cnt, pairs = gpu.selftest_qdiv(5, 1 << 32)
    assert cnt == 0, [float(d) for _, d in pairs]


def test_dn_weight_exhaustive(gpu):
    """The display weight (cpt_kernels.hip dn_weight: the short table exp + rounding guard) ==
    its slow form dn_weight_slow (the round-4 sequence, itself equal to the oracle's
    min(dm_exp(-(double)d2 / M_PI), 1.0) on every float in [0, 2341]:
    test_exact_identities.py::test_denoise_weight_exhaustive) for all 2^31 non-negative float
    patterns: 0, subnormals, (0, 330) where the short exp decides, the >= 330 shortcut, inf and
    every NaN.  Also records how rarely the guard falls back (path_tracer.cu:219-233)."""
    cnt, pairs = gpu.selftest_qdiv(6, 1 << 31)
    assert cnt == 0, [float(a) for a, _ in pairs]
    # the guard's fallbacks over [0, 274): the normal-float results (above 274.5 the weight is a
    # subnormal float and always takes the slow form)
    lim = int(np.float32(274.0).view(np.uint32))
    fallbacks, _ = gpu.selftest_qdiv(7, lim)
    assert fallbacks < 1e-5 * lim, fallbacks


def test_lobe_pow_exhaustive(gpu, oracle_mod):
    """The BSDF lobe's z = (float)pow(x_1, inv_alpha) through its short form (cpt_device.hpp
    lobe_pow: sqrtf for Diffuse's 1/2, fm::pow_unit + rounding guard for the others) == the full
    double sequence dm::pow, rounded to float, for every float x in [0, 1] at every exponent the
    S4 and S1000 materials use, at 1/2, and at the edges of the short form's domain (round 6;
    material.cu:24,43-45,78,85,104).  The full sequence equals the oracle's dm_pow
    (test_binary_pow_bitexact); tests/test_fastmath.py restates the short form on the host."""
    from conftest import lobe_exponents
    n = int(np.float32(1.0).view(np.uint32)) + 1
    ys = sorted(set(lobe_exponents(oracle_mod, "s4") + lobe_exponents(oracle_mod, "s1000")))
    for y in ys + [0.5, 1.0, 0.999, 0.25, 2.0 ** -40, 1.5]:
        seed = int(np.float64(y).view(np.uint64))
        cnt, xs = gpu.selftest_qdiv(8, n, seed=seed)
        assert cnt == 0, (y, [float(x) for x, _ in xs])
    # the guard's fallbacks over the normal floats of (0, 1] at the materials' exponents
    # (subnormal x always takes the full pow: the lobe's x_1 >= 2^-33 never is one)
    for y in ys:
        fell, _ = gpu.selftest_qdiv(9, n, seed=int(np.float64(y).view(np.uint64)))
        assert fell - 0x00800000 < 1e-5 * n, (y, fell)


def test_lobe_sincos_exhaustive(gpu):
    """The lobe's sinf/cosf of phi = (float)(2 pi x_2) through the short table form + rounding
    guard (cpt_device.hpp lobe_sincos) == the full dm::sincosf_ sequence, both results, for all
    2^32 float patterns (outside [0, 2 pi] the guard always hands over), and how rarely the guard
    fires on [0, 2 pi] (material.cu:26-27,47-48)."""
    cnt, xs = gpu.selftest_qdiv(10, 1 << 32)
    assert cnt == 0, [float(x) for x, _ in xs]
    n = int(np.float32(2 * np.pi).view(np.uint32)) + 1
    fell, _ = gpu.selftest_qdiv(11, n)
    assert fell - 0x00800000 < 1e-5 * n, fell


def test_miss_atan_asin_exhaustive(gpu):
    """The sky fetch's atanf(d.y / d.x) and asinf(d.z) through fm::atan_ratio + rounding guard
    (cpt_device.hpp miss_atanf, miss_asinf; round 6) == the full dm::atanf_ / dm::asinf_
    sequences (themselves the oracle's: test_unary_math_bitexact) for all 2^32 float patterns,
    and how rarely the guards fire (path_tracer.cu:119-120)."""
    cnt, xs = gpu.selftest_qdiv(12, 1 << 32)
    assert cnt == 0, [float(x) for x, _ in xs]
    fell, _ = gpu.selftest_qdiv(13, 1 << 32)
    # +-0 and the 2 (2^23 - 1) subnormals (atan x = x, asin x = x: subnormal floats), the
    # infinities and NaNs (2^24 - 2 patterns) always take the full sequences
    assert fell - 2 * 0x00800000 - (1 << 24) < 1e-5 * (1 << 32), fell


def test_winner_certificate_quotient_free(gpu):
    """The ordered walk's quotient-free winner certificate (cpt_path.hpp cert_inside, round 6) as
    compiled for the device never certifies a box the exact slab test rejects (bvh.cu:181-200 with
    the exact quotients, slab_reject<true>): 2^32 hashed cases, half of them with the distance
    within 16 ulps of a box plane's exact quotient (where it must stay inconclusive) and the rest
    at random distances; both sides are exercised (r06: 19.8 M of the 108 M passing cases
    certified).  tests/test_certificate.py restates it on the host and checks that hits well
    inside their box are certified."""
    n = 1 << 32
    bad, ids = gpu.selftest_qdiv(14, n, seed=20261018)
    assert bad == 0, ids
    certified, _ = gpu.selftest_qdiv(15, n, seed=20261018)
    passing, _ = gpu.selftest_qdiv(16, n, seed=20261018)
    assert passing > 1e7 and certified > 0.1 * passing, (certified, passing)


# ------------------------------------------------------------------------------- rng
@pytest.mark.parametrize("w,rows", [(64, list(range(64))), (3840, [0, 1, 7, 1079, 2159]),
                                    (333, [5, 3, 200, 3])])
def test_rng_init_bitexact(gpu, oracle_mod, w, rows):
    gpu.set_frame(w, max(rows) + 1, rows)
    gpu.init_rng(1234)
    g = gpu.read_rng()
    o = oracle_mod.init_rng(1234, w, np.array(rows, np.int32), threads=8)
    np.testing.assert_array_equal(g, o)


# ------------------------------------------------------------------------- integrator
def _run_both(gpu, oracle_mod, sky, objs, W, H, spp, depth, rows=None, seed=1234, aux=False, env=True,
              path="megakernel"):
    rows = np.arange(H, dtype=np.int32) if rows is None else np.asarray(rows, np.int32)
    cam = camera_get_copy(scenes.camera_for(W, H))
    gpu.set_scene(objs)
    gpu.set_env(sky if env else None)
    gpu.set_frame(W, H, rows)
    gpu.init_rng(seed)
    gpu.reset_stats()
    stats = not _timed(path)
    gpu.render(cam, spp, depth, aux=aux, stats=stats, sync=True, **_kw(path))
    g_acc, g_rng = gpu.read_accum(), gpu.read_rng()
    g_st = gpu.stats() if stats else None
    if stats and _kw(path)["ordered"]:
        g_st["fallbacks"] = gpu.raw_counters()[5]
    g_aux = gpu.read_aux() if aux else None
    rng = oracle_mod.init_rng(seed, W, rows, threads=8)
    o_acc, o_st, o_n, o_d = oracle_mod.render(objs, cam, sky if env else None, rows, spp, depth, rng,
                                             want_aux=aux, threads=8)
    if _kw(path)["ordered"]:
        # node/prim counts of the ordered walk come from the oracle's diagnostic restatement of
        # that walk; its image must equal the reference walk's too
        rng2 = oracle_mod.init_rng(seed, W, rows, threads=8)
        oracle_mod.set_walk(True)
        try:
            w_acc, w_st, _, _ = oracle_mod.render(objs, cam, sky if env else None, rows, spp, depth, rng2, threads=8)
            w_st["fallbacks"] = oracle_mod.last_fallbacks()
        finally:
            oracle_mod.set_walk(False)
        np.testing.assert_array_equal(w_acc.view(np.uint32), o_acc.view(np.uint32))
        np.testing.assert_array_equal(rng2, rng)
        o_st = dict(o_st, walk=w_st)
    return (g_acc, g_rng, g_st, g_aux), (o_acc, rng, o_st, (o_n, o_d))


def _kw(path):
    path, *opts = path.split("+")
    base, _, mode = path.partition(":")
    kw = dict(path=base, ordered={"": False, "ordered": True, "plain": "plain"}[mode])
    if "timed" in opts:
        kw["schedule"] = "cost" if base == "megakernel" else "tiles"
    if "cons" in opts:
        kw["consolidate"] = True
    return kw


def _timed(path):
    """"<path>+timed": the instantiation bench.py times — no STATS counters, and for the
    megakernel the cost schedule (pilot pass + heaviest-tiles-first order).  "+cons" forces the
    tail-consolidating megakernel, which the library picks by itself for ranks of more than 1 and
    at most 4 pixels per lane at >= 512 spp (strong-scaled row tiles); these small test renders would otherwise run
    the plain one, the kernel the N = 1 bench times."""
    return "+timed" in path


CASES = [
    ("s3", 64, 64, 4, 4),
    ("s3", 67, 33, 3, 8),
    ("s4", 64, 48, 4, 16),
    ("s4", 40, 40, 2, 32),
    ("s1000", 64, 36, 2, 16),
    ("s1000", 96, 54, 1, 8),
]


# "<path>:ordered" = the near-first octant walk (CPT_TRAVERSAL_ORDERED): same closest hits,
# so the same images, RNG end states and segment/hit/miss counts.  "<path>:plain" tests each
# leaf where the walk meets it (CPT_TRAVERSAL_PLAIN_LEAVES): its node/prim counts equal the
# oracle's diagnostic restatement of the ordered walk (oracle.set_walk), including the number
# of segments whose winner certificate failed (reference-walk fallback).  The default
# ordered walk runs on 4-wide nodes and parks leaves for wave-wide rounds.
PATHS = ["megakernel", "wavefront", "megakernel:ordered", "wavefront:ordered", "megakernel:plain",
         "wavefront:plain", "megakernel+timed", "megakernel:ordered+timed", "wavefront:ordered+timed",
         "megakernel:ordered+cons", "megakernel:ordered+timed+cons"]


def _check_stats(gs, os_, path):
    if gs is None:   # "+timed": images and RNG states only
        return
    path = path.split("+")[0]
    if path.endswith(":plain"):
        for k in ("segments", "hits", "misses"):
            assert gs[k] == os_[k], k
        assert gs == os_["walk"]
    elif path.endswith(":ordered"):
        # the default ordered walk (4-wide nodes, postponed leaves) finds the same closest
        # hits, so segments/hits/misses and the winner certificates match; its node and
        # primitive counts are its own (wide nodes; leaves whose box the parent rejected are
        # never tested)
        for k in ("segments", "hits", "misses"):
            assert gs[k] == os_[k], k
        assert gs["fallbacks"] == os_["walk"]["fallbacks"]
        assert (gs["nodes"] > 0) == (os_["walk"]["nodes"] > 0)
    else:
        assert gs == os_


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("name,W,H,spp,depth", CASES)
def test_render_bitexact(gpu, oracle_mod, sky, name, W, H, spp, depth, path):
    objs = scenes.SCENES[name]()
    (ga, gr, gs, _), (oa, orng, os_, _) = _run_both(gpu, oracle_mod, sky, objs, W, H, spp, depth, path=path)
    np.testing.assert_array_equal(gr, orng)
    _check_stats(gs, os_, path)
    np.testing.assert_array_equal(ga.view(np.uint32), oa.view(np.uint32))
    assert np.isfinite(ga).all() and (ga[:, 3] == spp).all()


@pytest.mark.parametrize("path", PATHS)
def test_exact_ties_between_primitives(gpu, oracle_mod, sky, path):
    """Every primitive duplicated with a different material (and the copies shuffled through
    the object list): all hits are exact ties between two primitives, and the reference keeps
    the one its right-first DFS tests first (strict `temp < tmax`, object.cu).  The ordered
    walk must pick the same one through its reference-rank tie rule."""
    objs = scenes.scene_s1000(n=60)
    twins = objs.copy()
    mats = twins["material"].copy()
    twins["material"] = np.roll(mats, 7)
    both = np.concatenate([objs, twins]).astype(types.OBJECT_DTYPE)   # concatenate drops the padded layout
    perm = np.random.default_rng(5).permutation(both.size)
    both = np.ascontiguousarray(both[perm])
    (ga, gr, gs, _), (oa, orng, os_, _) = _run_both(gpu, oracle_mod, sky, both, 64, 40, 2, 8, path=path)
    np.testing.assert_array_equal(gr, orng)
    _check_stats(gs, os_, path)
    np.testing.assert_array_equal(ga.view(np.uint32), oa.view(np.uint32))


@pytest.mark.parametrize("path", PATHS)
def test_render_aux_bitexact(gpu, oracle_mod, sky, path):
    objs = scenes.scene_s4()
    (ga, gr, gs, (gn, gd)), (oa, orng, os_, (on, od)) = _run_both(gpu, oracle_mod, sky, objs, 48, 32, 2, 8, aux=True,
                                                                  path=path)
    np.testing.assert_array_equal(gn.view(np.uint32), on.view(np.uint32))
    np.testing.assert_array_equal(gd, od)
    assert (gd == np.float32(1e30)).all()   # depth quirk (a18): TraceRay gets the ray by value


@pytest.mark.parametrize("path", PATHS)
def test_row_subset_and_order(gpu, oracle_mod, sky, path):
    """Any row list (tiles, interleaved blocks, unsorted, repeated) gives per-row results
    identical to the monolithic render: a pixel's stream depends only on (seed, x, y)."""
    objs = scenes.scene_s1000()
    W, H = 48, 40
    (ga, gr, _, _), _ = _run_both(gpu, oracle_mod, sky, objs, W, H, 2, 8, path=path)
    rows = [39, 0, 17, 17, 5]
    (sa, sr, _, _), (oa, orng, _, _) = _run_both(gpu, oracle_mod, sky, objs, W, H, 2, 8, rows=rows, path=path)
    np.testing.assert_array_equal(sa, oa)
    full = ga.reshape(H, W, 4)
    np.testing.assert_array_equal(sa.reshape(len(rows), W, 4), full[rows])


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("depth", [0, 1])
def test_tiny_depths(gpu, oracle_mod, sky, depth, path):
    objs = scenes.scene_s4()
    (ga, gr, gs, _), (oa, orng, os_, _) = _run_both(gpu, oracle_mod, sky, objs, 32, 16, 3, depth, path=path)
    np.testing.assert_array_equal(gr, orng)
    np.testing.assert_array_equal(ga.view(np.uint32), oa.view(np.uint32))
    _check_stats(gs, os_, path)


@pytest.mark.parametrize("path", PATHS)
def test_empty_scene_and_no_env(gpu, oracle_mod, sky, path):
    empty = np.zeros(0, dtype=types.OBJECT_DTYPE)
    (ga, gr, gs, _), (oa, orng, os_, _) = _run_both(gpu, oracle_mod, sky, empty, 32, 16, 2, 8, path=path)
    np.testing.assert_array_equal(ga.view(np.uint32), oa.view(np.uint32))
    np.testing.assert_array_equal(gr, orng)
    assert gs is None or gs["hits"] == 0
    _check_stats(gs, os_, path)
    (ga, gr, gs, _), (oa, orng, os_, _) = _run_both(gpu, oracle_mod, sky, scenes.scene_s3(), 32, 16, 2, 8, env=False)
    np.testing.assert_array_equal(ga.view(np.uint32), oa.view(np.uint32))


@pytest.mark.parametrize("path", ["megakernel", "megakernel:ordered", "megakernel:plain", "megakernel:ordered+timed",
                                  "megakernel:ordered+timed+cons"])
def test_single_object_and_cylinders(gpu, oracle_mod, sky, path):
    objs = scenes.scene_s1000(n=3)
    for sl in (slice(0, 1), slice(1, 2), slice(0, 4)):
        o = np.ascontiguousarray(objs[sl])
        (ga, gr, gs, _), (oa, orng, os_, _) = _run_both(gpu, oracle_mod, sky, o, 40, 24, 2, 8, path=path)
        np.testing.assert_array_equal(ga.view(np.uint32), oa.view(np.uint32))
        _check_stats(gs, os_, path)


@pytest.mark.parametrize("path", PATHS)
def test_accumulate_and_spp0(gpu, oracle_mod, sky, path):
    objs = scenes.scene_s3()
    W, H = 32, 32
    cam = camera_get_copy(scenes.camera_for(W, H))
    gpu.set_scene(objs)
    gpu.set_env(sky)
    gpu.set_frame(W, H)
    gpu.init_rng(99)
    kw = _kw(path)
    gpu.render(cam, 0, 4, sync=True, **kw)
    assert (gpu.read_accum() == 0).all()
    gpu.render(cam, 2, 4, sync=True, **kw)
    gpu.render(cam, 3, 4, accumulate=True, sync=True, **kw)
    a = gpu.read_accum()
    rng = oracle_mod.init_rng(99, W, np.arange(H, dtype=np.int32))
    acc, _, _, _ = oracle_mod.render(objs, cam, sky, np.arange(H, dtype=np.int32), 2, 4, rng)
    acc, _, _, _ = oracle_mod.render(objs, cam, sky, np.arange(H, dtype=np.int32), 3, 4, rng, accum=acc,
                                     accumulate=True)
    np.testing.assert_array_equal(a.view(np.uint32), acc.view(np.uint32))
    assert (a[:, 3] == 5).all()


def test_invalid_arguments(gpu):
    from cpppathtracer_amd import CptError
    cam = camera_get_copy(scenes.camera_for(16, 16))
    gpu.set_scene(scenes.scene_s3())
    gpu.set_frame(16, 16)
    gpu.init_rng(1)
    with pytest.raises(CptError):
        gpu.render(cam, 1, 33)
    with pytest.raises(CptError):
        gpu.render(camera_get_copy(scenes.camera_for(8, 16)), 1, 4)
    with pytest.raises(CptError):
        gpu.set_frame(16, 16, [16])


@pytest.mark.parametrize("path", ["megakernel", "wavefront", "megakernel:ordered", "megakernel:plain",
                                  "megakernel:ordered+timed"])
def test_update_object_refit(gpu, oracle_mod, sky, path):
    """SceneBVH::UpdateObject (bvh.cu:122-157): the leaf takes the new object, its ancestors'
    boxes are refit and the topology is kept.  Moves a sphere far out (boxes grow), shrinks a
    cylinder, swaps a material; the render after the edits matches the oracle's refit BVH."""
    objs = scenes.scene_s1000(n=40)
    W, H, spp, depth = 48, 32, 2, 8
    cam = camera_get_copy(scenes.camera_for(W, H))
    edits = []
    sph = int(np.flatnonzero(objs["type"] == 0)[3])
    o = objs[sph].copy()
    o["center"][1] += 25.0
    o["center"][0] -= 40.0
    edits.append((sph, o))
    cyl = np.flatnonzero(objs["type"] == 2)
    if cyl.size:
        o = objs[int(cyl[0])].copy()
        o["radius"] *= 0.5
        o["height"] *= 1.5
        edits.append((int(cyl[0]), o))
    o = objs[5].copy()
    o["material"] = objs[7]["material"]
    edits.append((5, o))
    gpu.set_scene(objs)
    for i, ob in edits:
        gpu.update_object(i, ob)
    gpu.set_env(sky)
    gpu.set_frame(W, H)
    gpu.init_rng(11)
    gpu.reset_stats()
    stats = not _timed(path)
    gpu.render(cam, spp, depth, stats=stats, sync=True, **_kw(path))
    ga = gpu.read_accum()
    gs = gpu.stats() if stats else None
    if stats and _kw(path)["ordered"]:
        gs["fallbacks"] = gpu.raw_counters()[5]
    rows = np.arange(H, dtype=np.int32)
    rng = oracle_mod.init_rng(11, W, rows, threads=8)
    oa, os_ = oracle_mod.render_edited(objs, edits, cam, sky, rows, spp, depth, rng, threads=8)
    if _kw(path)["ordered"]:
        oracle_mod.set_walk(True)
        try:
            _, w_st = oracle_mod.render_edited(objs, edits, cam, sky, rows, spp, depth,
                                               oracle_mod.init_rng(11, W, rows, threads=8), threads=8)
            w_st["fallbacks"] = oracle_mod.last_fallbacks()
        finally:
            oracle_mod.set_walk(False)
        os_ = dict(os_, walk=w_st)
    np.testing.assert_array_equal(ga.view(np.uint32), oa.view(np.uint32))
    np.testing.assert_array_equal(gpu.read_rng(), rng)
    _check_stats(gs, os_, path)


@pytest.mark.parametrize("path", ["megakernel:ordered", "wavefront:ordered", "megakernel:plain",
                                  "megakernel:ordered+timed"])
def test_ordered_walk_platform_only_and_multiple_platforms(gpu, oracle_mod, sky, path):
    """Walk-tree edge cases: a scene that is only a platform (no tree left after splicing),
    and several platforms (floor, a ceiling plane, a duplicate floor) mixed with primitives."""
    objs = scenes.scene_s1000(n=20)
    floor = objs[objs["type"] == 1][0].copy()
    only = np.ascontiguousarray(np.array([floor], dtype=types.OBJECT_DTYPE))
    (ga, gr, gs, _), (oa, orng, os_, _) = _run_both(gpu, oracle_mod, sky, only, 32, 16, 2, 8, path=path)
    np.testing.assert_array_equal(ga.view(np.uint32), oa.view(np.uint32))
    _check_stats(gs, os_, path)
    ceil = floor.copy()
    ceil["y_pos"] = 60.0
    twin = floor.copy()
    twin["material"] = objs[3]["material"]
    many = np.concatenate([objs, np.array([ceil, twin], dtype=types.OBJECT_DTYPE)]).astype(types.OBJECT_DTYPE)
    (ga, gr, gs, _), (oa, orng, os_, _) = _run_both(gpu, oracle_mod, sky, many, 48, 32, 2, 8, path=path)
    np.testing.assert_array_equal(gr, orng)
    np.testing.assert_array_equal(ga.view(np.uint32), oa.view(np.uint32))
    _check_stats(gs, os_, path)


def _chain_scene(n=90):
    """Spheres on a geometric progression along x: the SAH peels one sphere off per split, so
    the walk tree is a chain whose 4-wide form needs more than the device's 32 stack entries."""
    objs = np.zeros(n + 1, dtype=types.OBJECT_DTYPE)
    objs[0] = scenes.scene_s4()[0]                     # the floor
    mat = scenes.scene_s4()[1]["material"]
    for k in range(n):
        objs[k + 1] = types.make_object(types.SPHERE, mat, center=(-40.0 + 1.12 ** k, 10.0, 0.0),
                                         radius=0.05 * 1.12 ** k)
    return objs


def test_wide_walk_structure_and_deep_tree_fallback(gpu, oracle_mod, sky):
    """The default ordered walk runs on 4-wide nodes for S1000; a walk tree too deep for the
    per-lane LDS stack keeps the binary octant orders (cpt_get_walk_info n_wide == 0), with the
    same bit-exact images."""
    gpu.set_scene(scenes.scene_s1000())
    info = gpu.walk_info()
    assert info["n_wide"] > 0 and info["n_unb"] == 1 and info["n_walk"] == 2000
    objs = _chain_scene()
    gpu.set_scene(objs)
    assert gpu.walk_info()["n_wide"] == 0
    for path in ("megakernel:ordered", "megakernel", "megakernel:ordered+timed"):
        (ga, gr, gs, _), (oa, orng, os_, _) = _run_both(gpu, oracle_mod, sky, objs, 48, 32, 2, 8, path=path)
        np.testing.assert_array_equal(gr, orng)
        np.testing.assert_array_equal(ga.view(np.uint32), oa.view(np.uint32))
        _check_stats(gs, os_, path)


LDS_TREE_NODES = 512   # cpt_path.hpp: wide nodes staged in LDS; the rest are read from global memory


@pytest.mark.parametrize("path", ["megakernel:ordered", "megakernel:ordered+timed", "megakernel:ordered+timed+cons",
                                  "wavefront:ordered", "wavefront:ordered+timed"])
def test_wide_walk_beyond_lds_image(gpu, oracle_mod, sky, path):
    """A 4-wide tree larger than the LDS image (S1000's generator with 3000 primitives): the
    walk reads the top LDS_TREE_NODES nodes from LDS and the others from the image in global
    memory (cpt_path.hpp load_wide_node).  Images, RNG end states, segment/hit/miss counts and
    certificate fallbacks equal the oracle's (bvh.cu:167-205 is the reference walk)."""
    objs = scenes.scene_s1000(n=3000)
    gpu.set_scene(objs)
    info = gpu.walk_info()
    assert info["n_wide"] > LDS_TREE_NODES, info
    (ga, gr, gs, _), (oa, orng, os_, _) = _run_both(gpu, oracle_mod, sky, objs, 64, 36, 2, 16, path=path)
    np.testing.assert_array_equal(gr, orng)
    _check_stats(gs, os_, path)
    np.testing.assert_array_equal(ga.view(np.uint32), oa.view(np.uint32))
    assert_hbm_part_walked(gpu, path, 64, 36, 16)


def assert_hbm_part_walked(gpu, path, W, H, depth):
    """The render above really read wide nodes past the LDS image (raw counter 6, the HYB
    branch of load_wide_node): a "+timed" path has no counters, so its counting
    instantiation renders the same frame once more."""
    if _timed(path):
        cam = camera_get_copy(scenes.camera_for(W, H))
        gpu.init_rng(5)
        gpu.reset_stats()
        kw = _kw(path.split("+")[0])
        gpu.render(cam, 1, depth, stats=True, sync=True, **kw)
    global_nodes = int(gpu.raw_counters()[6])
    assert global_nodes > 0, "no wide-node visit read the image in global memory"


def test_hbm_read_probe(gpu):
    """cpt_measure_read_bandwidth (the bench's measured roofline ceiling) returns a sane GB/s
    for a 1 GiB buffer: above 1 TB/s, below the 8 TB/s spec (with 5% slack for timer noise)."""
    gbps = gpu.measure_read_bandwidth(1 << 30, 5)
    assert 1000.0 < gbps < 8400.0, gbps


@pytest.mark.parametrize("ordered", [True, False])
def test_previous_pass_schedule(gpu, oracle_mod, sky, ordered):
    """CPT_SCHEDULE_PREVIOUS (the DispatchRay loop's order: tiles heaviest first by the last
    pass's RNG draws, no pilot): five accumulated 1-spp renders, the first in row-major order and
    the others in the order the draws gave, equal the oracle's 5-pass render bit for bit; a
    re-seeded context (its draw baseline reset) stays exact."""
    objs = scenes.scene_s1000(n=300)
    W, H = 72, 40
    cam = camera_get_copy(scenes.camera_for(W, H))
    rows = np.arange(H, dtype=np.int32)
    gpu.set_scene(objs)
    gpu.set_env(sky)
    gpu.set_frame(W, H)
    for seed in (1234, 77):
        gpu.init_rng(seed)
        for k in range(5):
            gpu.render(cam, 1, 8, accumulate=k > 0, ordered=ordered, schedule="previous", sync=True)
        rng = oracle_mod.init_rng(seed, W, rows, threads=8)
        oa, _, _, _ = oracle_mod.render(objs, cam, sky, rows, 5, 8, rng, threads=8)
        np.testing.assert_array_equal(gpu.read_rng(), rng)
        np.testing.assert_array_equal(gpu.read_accum().view(np.uint32), oa.view(np.uint32))
