"""Row-banded display path on the GPU (cpt_denoise_mix_band, cpppathtracer_amd.display).

Each simulated rank is its own context on cuda:0 rendering its band plus the 3-row halo; the
stitched BGRA8 frame must equal the single-GPU display path byte for byte (the committed
golden, and cpt_denoise_mix on the same frame)."""
import ctypes
import os

import numpy as np
import pytest

from cpppathtracer_amd import camera_get_copy, scenes, tiling

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
pytestmark = pytest.mark.gpu


def _banded(sky, objs, W, H, world, idxs, depth=8, ordered=False):
    from cpppathtracer_amd import Renderer
    from cpppathtracer_amd.display import BandedDisplay
    cam = camera_get_copy(scenes.camera_for(W, H))
    g = np.zeros((world, tiling.max_band_rows(H, world), W, 4), np.uint8)
    for rank in range(world):
        with Renderer(0) as r:
            r.set_scene(objs)
            r.set_env(sky)
            d = BandedDisplay(r, W, H, 1234, rank, world)
            for idx in idxs:
                band = d.dispatch(cam, idx, depth, ordered=ordered)
            g[rank, : band.shape[0]] = band
    return tiling.stitch_bands(g, H, W, world)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_gpu_banded_display_equals_golden(gpu, sky, world):
    z = np.load(os.path.join(GOLDEN, "display_s4_64x48_3frames.npz"))
    np.testing.assert_array_equal(_banded(sky, scenes.scene_s4(), 64, 48, world, (2, 3, 4)), z["bgra"])


@pytest.mark.parametrize("ordered", [False, True])
def test_gpu_banded_display_equals_full_frame(gpu, sky, ordered):
    """BVH scene, a height that is not a multiple of 16, both walks."""
    W, H = 80, 53
    objs = scenes.scene_s1000()
    cam = camera_get_copy(scenes.camera_for(W, H))
    gpu.set_scene(objs)
    gpu.set_env(sky)
    gpu.set_frame(W, H)
    gpu.init_rng(1234)
    for idx in (2, 3):
        gpu.render(cam, 1, 8, aux=True, sync=True, ordered=ordered)
        full = gpu.denoise_mix(idx)
    np.testing.assert_array_equal(_banded(sky, objs, W, H, 3, (2, 3), ordered=ordered), full)


def test_gpu_band_needs_halo_rows(gpu, sky):
    from cpppathtracer_amd.renderer import CptError
    W, H = 64, 48
    gpu.set_scene(scenes.scene_s4())
    gpu.set_env(sky)
    gpu.set_frame(W, H, np.arange(16, 32, dtype=np.int32))   # the band alone, no halo
    gpu.init_rng(1234)
    gpu.render(camera_get_copy(scenes.camera_for(W, H)), 1, 8, aux=True, sync=True)
    with pytest.raises(CptError):
        gpu.denoise_mix_band(2, 16, 32)
    with pytest.raises(CptError):
        gpu.denoise_mix_band(2, 40, 64)   # past H'


def test_gpu_banded_display_16_wide(gpu, sky):
    """A 16-column frame through band contexts (round 6, advisor r05): k_denoise_rows' halo lanes
    past 2 W' wrap beyond the next row; they must read nothing outside the context's rows (the
    guard), and the stitched frame equals the full-frame display path byte for byte.  The Mix
    mean read back is sized from the library's band (cpt_display_band) and checked against a
    buffer too small for it (cpt_read_mix's capacity)."""
    from cpppathtracer_amd import Renderer
    from cpppathtracer_amd.renderer import CptError
    W, H = 16, 100
    objs = scenes.scene_s4()
    cam = camera_get_copy(scenes.camera_for(W, H))
    gpu.set_scene(objs)
    gpu.set_env(sky)
    gpu.set_frame(W, H)
    gpu.init_rng(1234)
    for idx in (2, 3):
        gpu.render(cam, 1, 8, aux=True, sync=True)
        full = gpu.denoise_mix(idx)
    full_mix = gpu.read_mix()
    assert gpu.display_band() == (0, 16 * (H // 16))
    np.testing.assert_array_equal(_banded(sky, objs, W, H, 3, (2, 3)), full)
    with Renderer(0) as r:
        r.set_scene(objs)
        r.set_env(sky)
        from cpppathtracer_amd.display import BandedDisplay
        d = BandedDisplay(r, W, H, 1234, 1, 3)
        for idx in (2, 3):
            d.dispatch(cam, idx, 8)
        y0, y1 = r.display_band()
        assert (y0, y1) == (d.y0, d.y1)
        np.testing.assert_array_equal(r.read_mix().view(np.uint32),
                                      full_mix[y0 * W: y1 * W].view(np.uint32))
        small = np.zeros(((y1 - y0) * W - 1, 3), np.float32)
        with pytest.raises(CptError):
            r._check(r._L.cpt_read_mix(r._ctx, ctypes.c_void_p(small.ctypes.data), small.size))
