"""Parity at BASELINE.json's full sizes (C4 1920x1080, C5 3840x2160) through size-independent
properties, plus oracle spot checks on evenly spaced rows (the oracle is scalar; a full frame
is left to bench.py's on-device walk comparison and tools/walk_parity.py)."""
import numpy as np
import pytest

from cpppathtracer_amd import camera_get_copy, scenes, tiling

pytestmark = pytest.mark.gpu


def _frame(gpu, sky, objs, W, H, rows=None, seed=1234):
    gpu.set_scene(objs)
    gpu.set_env(sky)
    gpu.set_frame(W, H, rows)
    gpu.init_rng(seed)
    return camera_get_copy(scenes.camera_for(W, H))


def _render(gpu, cam, spp, depth, **kw):
    gpu.render(cam, spp, depth, sync=True, **kw)
    return gpu.read_accum(), gpu.read_rng()


@pytest.mark.parametrize("W,H", [(1920, 1080), (3840, 2160)])
def test_fullsize_walks_agree_and_rows_match_oracle(gpu, oracle_mod, sky, W, H):
    objs = scenes.scene_s1000()
    cam = _frame(gpu, sky, objs, W, H)
    ref_acc, ref_rng = _render(gpu, cam, 1, 16)
    gpu.init_rng(1234)
    ord_acc, ord_rng = _render(gpu, cam, 1, 16, ordered=True)
    np.testing.assert_array_equal(ord_acc.view(np.uint32), ref_acc.view(np.uint32))
    np.testing.assert_array_equal(ord_rng, ref_rng)
    gpu.init_rng(1234)
    plain_acc, _ = _render(gpu, cam, 1, 16, ordered="plain")
    np.testing.assert_array_equal(plain_acc.view(np.uint32), ref_acc.view(np.uint32))
    rows = np.linspace(0, H - 1, 6).astype(np.int32)
    rng = oracle_mod.init_rng(1234, W, rows, threads=16)
    o_acc, _, _, _ = oracle_mod.render(objs, cam, sky, rows, 1, 16, rng, threads=16)
    got = ref_acc.reshape(H, W, 4)[rows].reshape(-1, 4)
    np.testing.assert_array_equal(got.view(np.uint32), o_acc.view(np.uint32))
    np.testing.assert_array_equal(ref_rng.reshape(6, H, W)[:, rows].reshape(6, -1), rng)


def test_fullsize_pass_split_and_determinism(gpu, sky):
    """2 passes in one render == 1 pass + 1 accumulated pass (the stream continues), and a
    repeated render is identical (no races in the refill queue)."""
    W, H = 1920, 1080
    cam = _frame(gpu, sky, scenes.scene_s1000(), W, H)
    a2, r2 = _render(gpu, cam, 2, 16, ordered=True)
    gpu.init_rng(1234)
    _render(gpu, cam, 1, 16, ordered=True)
    a11, r11 = _render(gpu, cam, 1, 16, ordered=True, accumulate=True)
    np.testing.assert_array_equal(a11.view(np.uint32), a2.view(np.uint32))
    np.testing.assert_array_equal(r11, r2)
    gpu.init_rng(1234)
    again, _ = _render(gpu, cam, 2, 16, ordered=True)
    np.testing.assert_array_equal(again.view(np.uint32), a2.view(np.uint32))


def test_fullsize_row_tiling_is_exact(gpu, sky):
    """Every rank's rows of a 4-way and a 3-way partition equal the monolithic frame's."""
    W, H = 1920, 1080
    objs = scenes.scene_s1000()
    cam = _frame(gpu, sky, objs, W, H)
    full, full_rng = _render(gpu, cam, 1, 16, ordered=True)
    full = full.reshape(H, W, 4)
    for world in (3, 4):
        for rank in range(world):
            rows = tiling.partition_rows(H, world, rank)
            _frame(gpu, sky, objs, W, H, rows)
            part, _ = _render(gpu, cam, 1, 16, ordered=True)
            np.testing.assert_array_equal(part.reshape(rows.size, W, 4).view(np.uint32), full[rows].view(np.uint32))


def test_fullsize_wavefront_equals_megakernel(gpu, sky):
    W, H = 1920, 1080
    cam = _frame(gpu, sky, scenes.scene_s4(), W, H)
    mk, mk_rng = _render(gpu, cam, 1, 16, ordered=True)
    gpu.init_rng(1234)
    wf, wf_rng = _render(gpu, cam, 1, 16, ordered=True, path="wavefront")
    np.testing.assert_array_equal(wf.view(np.uint32), mk.view(np.uint32))
    np.testing.assert_array_equal(wf_rng, mk_rng)


@pytest.mark.parametrize("config,spp", [("c2", 8), ("c3", 8), ("c4", 8), ("c2", 64), ("c4", 64)])
def test_fullsize_configs_timed_kernel_rows_match_oracle(gpu, oracle_mod, sky, config, spp):
    """BASELINE.json's C2 / C3 / C4 at full size through the instantiation bench.py times
    (ordered walk, cost schedule, no counters), 8 passes: six evenly spaced rows and their
    XORWOW end states equal the oracle's bit for bit.  At 64 passes the long-chain take applies
    (ranges shrinking with the ids left, cpt_tuning.hpp TAKE_TAPER): every pixel of the frame
    must then have been taken exactly once, so every pass count is spp."""
    cfg = scenes.CONFIGS[config]
    W, H, depth = cfg["width"], cfg["height"], cfg["depth"]
    objs = scenes.SCENES[cfg["scene"]]()
    cam = _frame(gpu, sky, objs, W, H)
    acc, rng_end = _render(gpu, cam, spp, depth, ordered=True, schedule="cost")
    np.testing.assert_array_equal(acc[:, 3], np.full(W * H, spp, np.float32))
    rows = np.linspace(0, H - 1, 6).astype(np.int32)
    rng = oracle_mod.init_rng(1234, W, rows, threads=16)
    o_acc, _, _, _ = oracle_mod.render(objs, cam, sky, rows, spp, depth, rng, threads=16)
    got = acc.reshape(H, W, 4)[rows].reshape(-1, 4)
    np.testing.assert_array_equal(got.view(np.uint32), o_acc.view(np.uint32))
    np.testing.assert_array_equal(rng_end.reshape(6, H, W)[:, rows].reshape(6, -1), rng)
