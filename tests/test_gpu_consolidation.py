"""Tail consolidation (k_megakernel<..., CONS>, cpt_kernels.hip): the default kernel of
ranks holding more than 1 and at most 4 pixels per lane (N = 2..7 at 1080p, C5 at N = 8).  Its hand-overs must either finish every chain bit for bit or end the render with
an error -- never with silently missing pixels (cpt.h CPT_ERR_DEVICE; the reference at least
logs its CUDA errors, path_tracer.cu:279-283).
"""
import numpy as np
import pytest

from cpppathtracer_amd import CptError, camera_get_copy, scenes
from cpppathtracer_amd._lib import CPT_ERR_DEVICE

pytestmark = pytest.mark.gpu


def _setup(gpu, sky, objs, W, H, seed):
    gpu.set_scene(objs)
    gpu.set_env(sky)
    gpu.set_frame(W, H)
    gpu.init_rng(seed)
    return camera_get_copy(scenes.camera_for(W, H))


def _oracle(oracle_mod, sky, objs, W, H, spp, depth, seed):
    rows = np.arange(H, dtype=np.int32)
    rng = oracle_mod.init_rng(seed, W, rows, threads=8)
    acc, _, _, _ = oracle_mod.render(objs, scenes_cam(W, H), sky, rows, spp, depth, rng, threads=8)
    return acc, rng


def scenes_cam(W, H):
    return camera_get_copy(scenes.camera_for(W, H))


@pytest.mark.parametrize("W,H,schedule", [(136, 8, "tiles"), (136, 8, "cost"), (72, 40, "tiles"), (72, 40, "cost")])
def test_partial_last_workgroup_bitexact(gpu, oracle_mod, sky, W, H, schedule):
    """Tile counts that leave the last workgroup partly filled (17 and 45 tiles of 64 pixels for
    16 waves of 1024-lane workgroups): with the dynamic dequeue, a level-0 wave of that
    workgroup can find the queue empty before its siblings have counted their chains; it must
    keep waiting for them (s_q[3], the waves still taking) instead of leaving their hand-overs
    with no keeper."""
    objs = scenes.scene_s1000(n=200)
    spp, depth, seed = 24, 8, 77
    cam = _setup(gpu, sky, objs, W, H, seed)
    gpu.render(cam, spp, depth, ordered=True, schedule=schedule, consolidate=True, sync=True)
    acc, rng = gpu.read_accum(), gpu.read_rng()
    oacc, orng = _oracle(oracle_mod, sky, objs, W, H, spp, depth, seed)
    np.testing.assert_array_equal(rng, orng)
    np.testing.assert_array_equal(acc.view(np.uint32), oacc.view(np.uint32))
    assert (acc[:, 3] == spp).all()


def _expect_device_error(gpu, cam, spp, depth):
    with pytest.raises(CptError) as e:
        gpu.render(cam, spp, depth, ordered=True, schedule="cost", consolidate=True, sync=True)
    assert e.value.status == CPT_ERR_DEVICE, e.value
    return str(e.value)


def test_lost_live_count_is_reported(gpu, oracle_mod, sky):
    """A phantom live chain (the count the keeper waits on can never reach zero): the keeper's
    idle-spin limit trips and the render fails with CPT_ERR_DEVICE instead of returning OK."""
    objs = scenes.scene_s1000(n=200)
    W, H, spp, depth, seed = 64, 48, 16, 8, 5
    cam = _setup(gpu, sky, objs, W, H, seed)
    try:
        gpu.set_debug_consolidation(flags=1, keeper_spin_log2=8)
        msg = _expect_device_error(gpu, cam, spp, depth)
        assert "keeper" in msg, msg
    finally:
        gpu.set_debug_consolidation(0)
    # the error was reported once and cleared; a normal render is bit-exact again
    gpu.init_rng(seed)
    gpu.render(cam, spp, depth, ordered=True, schedule="cost", consolidate=True, sync=True)
    oacc, orng = _oracle(oracle_mod, sky, objs, W, H, spp, depth, seed)
    np.testing.assert_array_equal(gpu.read_accum().view(np.uint32), oacc.view(np.uint32))
    np.testing.assert_array_equal(gpu.read_rng(), orng)


def test_unpublished_handover_is_reported(gpu, oracle_mod, sky):
    """Hand-overs whose publication flag never arrives: the taking lane gives up after the
    (lowered) wait, does not read the slot, and the render fails with CPT_ERR_DEVICE."""
    objs = scenes.scene_s1000(n=200)
    W, H, spp, depth, seed = 64, 48, 48, 8, 6
    cam = _setup(gpu, sky, objs, W, H, seed)
    try:
        gpu.set_debug_consolidation(flags=2, publish_wait_log2=4)
        msg = _expect_device_error(gpu, cam, spp, depth)
        assert "never published" in msg, msg
    finally:
        gpu.set_debug_consolidation(0)
    gpu.synchronize()   # nothing left over


def test_error_is_reported_by_a_later_sync(gpu, sky):
    """An asynchronous render's device error surfaces at the next synchronising call."""
    objs = scenes.scene_s1000(n=200)
    W, H, spp, depth = 64, 48, 16, 8
    cam = _setup(gpu, sky, objs, W, H, 9)
    try:
        gpu.set_debug_consolidation(flags=1, keeper_spin_log2=8)
        gpu.render(cam, spp, depth, ordered=True, schedule="cost", consolidate=True)   # async: OK
        with pytest.raises(CptError) as e:
            gpu.synchronize()
        assert e.value.status == CPT_ERR_DEVICE
    finally:
        gpu.set_debug_consolidation(0)
    gpu.synchronize()
