"""Row-banded multi-rank display path (SURVEY.md §8(e), next tier) on the CPU.

The oracle stands in for each rank's GPU: a rank renders its band plus the 3-row halo
(tiling.display_rows) at 1 spp with first-hit normal/depth, runs Denoising + Mix on its band
(oracle.denoise_mix_band, the restatement of cpt_denoise_mix_band), and the BGRA8 bands are
all-gathered over gloo.  The stitched frame must equal the single-GPU display path's bytes:
the committed golden (display_s4_64x48_3frames.npz, 3 DispatchRay frames) and the
full-frame oracle on other sizes."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cpppathtracer_amd import scenes, texture_io, tiling

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _band_frames(oracle_mod, sky, objs, W, H, world, rank, idxs, depth=8):
    """One rank's display: returns its band's BGRA8 rows after the dispatches `idxs`."""
    cam = oracle_mod.camera_get_copy(scenes.camera_for(W, H))
    y0, y1 = tiling.display_band(H, world, rank)
    rows = tiling.display_rows(H, world, rank)
    rng = oracle_mod.init_rng(1234, W, rows)
    mix = np.zeros(((y1 - y0) * W, 3), np.float32)
    out = np.zeros((y1 - y0, W, 4), np.uint8)
    for idx in idxs:
        acc, _, nrm, dep = oracle_mod.render(objs, cam, sky, rows, 1, depth, rng, want_aux=True)
        if y1 > y0:
            oracle_mod.denoise_mix_band(acc, nrm, dep, mix, out, W, H, int(rows[0]), y0, y1, idx)
    return out


def _full_frames(oracle_mod, sky, objs, W, H, idxs, depth=8):
    cam = oracle_mod.camera_get_copy(scenes.camera_for(W, H))
    rows = np.arange(H, dtype=np.int32)
    rng = oracle_mod.init_rng(1234, W, rows)
    mix = np.zeros((W * H, 3), np.float32)
    out = np.zeros((H, W, 4), np.uint8)
    for idx in idxs:
        acc, _, nrm, dep = oracle_mod.render(objs, cam, sky, rows, 1, depth, rng, want_aux=True)
        oracle_mod.denoise_mix(acc, nrm, dep, mix, out, W, H, idx)
    return out


def test_display_bands_cover_launch_once():
    for H in (48, 50, 1080, 2160, 17):
        he = 16 * (H // 16)
        for world in (1, 2, 3, 4, 8):
            bands = [tiling.display_band(H, world, r) for r in range(world)]
            assert bands[0][0] == 0 and bands[-1][1] == he
            assert all(bands[r][1] == bands[r + 1][0] for r in range(world - 1))
            for r, (y0, y1) in enumerate(bands):
                rows = tiling.display_rows(H, world, r)
                if y1 > y0:
                    assert rows[0] == max(0, y0 - 3) and rows[-1] == min(he, y1 + 3) - 1


@pytest.mark.parametrize("world", [2, 3, 5])
def test_band_stitch_equals_golden_display(oracle_mod, sky, world):
    """Bands computed independently (no shared buffers) stitch into the golden frame."""
    z = np.load(os.path.join(GOLDEN, "display_s4_64x48_3frames.npz"))
    W, H = 64, 48
    objs = scenes.scene_s4()
    bands = [_band_frames(oracle_mod, sky, objs, W, H, world, r, (2, 3, 4)) for r in range(world)]
    g = np.zeros((world, tiling.max_band_rows(H, world), W, 4), np.uint8)
    for r, b in enumerate(bands):
        g[r, : b.shape[0]] = b
    np.testing.assert_array_equal(tiling.stitch_bands(g, H, W, world), z["bgra"])


def test_band_stitch_equals_full_frame_bvh_scene(oracle_mod, sky):
    """A frame whose height is not a multiple of 16 (rows past H' stay 0), BVH scene."""
    W, H, world = 48, 37, 2
    objs = scenes.scene_s1000()
    full = _full_frames(oracle_mod, sky, objs, W, H, (2, 3))
    g = np.zeros((world, tiling.max_band_rows(H, world), W, 4), np.uint8)
    for r in range(world):
        b = _band_frames(oracle_mod, sky, objs, W, H, world, r, (2, 3))
        g[r, : b.shape[0]] = b
    np.testing.assert_array_equal(tiling.stitch_bands(g, H, W, world), full)


def _worker(rank, world, port, q):
    import oracle
    from cpppathtracer_amd.display import BandedDisplay
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        W, H = 64, 48
        sky = texture_io.load_cptex()
        band = _band_frames(oracle, sky, scenes.scene_s4(), W, H, world, rank, (2, 3, 4))
        # the GPU ranks' gather (BandedDisplay.gather), here over gloo with host tensors
        disp = BandedDisplay.__new__(BandedDisplay)
        disp.width, disp.height, disp.rank, disp.world = W, H, rank, world
        disp.band_rows = tiling.max_band_rows(H, world)
        frame = disp.gather(band)
        if rank == 0:
            q.put(frame)
        dist.barrier()
    except Exception as e:  # report instead of leaving the parent waiting on the queue
        q.put(repr(e))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_banded_display_gloo_ranks(world):
    z = np.load(os.path.join(GOLDEN, "display_s4_64x48_3frames.npz"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    assert not isinstance(frame, str), frame
    assert all(p.exitcode == 0 for p in procs)
    np.testing.assert_array_equal(frame, z["bgra"])
