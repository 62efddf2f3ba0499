"""Row tiling behind the drop-in API (SURVEY.md §8(b) `SetDevices(n)`, §8(e)).

* cpt_gather_rows: tiles rendered by separate contexts, gathered into one frame context, equal
  the monolithic render (accumulator and first-hit normals);
* PathTracer::SetDevices(n) through examples/headless_render.cpp: C5's 3840x2160 frame on 2 and
  8 contexts (all on device 0 here: a device may repeat) equals the single-context render bit
  for bit and the oracle on sampled rows; the DispatchRay display path over 2 contexts
  reproduces the golden BGRA8 frames.
"""
import os
import subprocess

import numpy as np
import pytest

from cpppathtracer_amd import CptError, Renderer, camera_get_copy, scenes, tiling

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _headless():
    from cpppathtracer_amd import build
    return build.build_examples()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_rows_equals_monolithic(gpu, sky, world):
    objs = scenes.scene_s1000(n=300)
    W, H, spp, depth, seed = 80, 44, 3, 12, 21
    cam = camera_get_copy(scenes.camera_for(W, H))
    gpu.set_scene(objs)
    gpu.set_env(sky)
    gpu.set_frame(W, H)
    gpu.init_rng(seed)
    gpu.render(cam, spp, depth, aux=True, ordered=True, schedule="cost", sync=True)
    mono, (mono_n, mono_d) = gpu.read_accum(), gpu.read_aux()
    tiles = []
    try:
        for rank in range(world):
            t = Renderer(0)
            tiles.append(t)
            t.set_scene(objs)
            t.set_env(sky)
            t.set_frame(W, H, tiling.partition_rows(H, world, rank))
            t.init_rng(seed)
            t.render(cam, spp, depth, aux=True, ordered=True, schedule="cost")   # asynchronous
        with Renderer(0) as frame:
            frame.set_frame(W, H)
            for t in tiles:
                frame.gather_rows(t)
            acc, (nrm, dep) = frame.read_accum(), frame.read_aux()
            # a destination that does not hold the source's rows is refused
            with Renderer(0) as part:
                part.set_frame(W, H, tiling.partition_rows(H, world, 0))
                with pytest.raises(CptError):
                    part.gather_rows(tiles[1])
    finally:
        for t in tiles:
            t.close()
    np.testing.assert_array_equal(acc.view(np.uint32), mono.view(np.uint32))
    np.testing.assert_array_equal(nrm.view(np.uint32), mono_n.view(np.uint32))
    np.testing.assert_array_equal(dep, mono_d)


def _run(args, tmp_path, name):
    out = tmp_path / name
    r = subprocess.run([_headless(), *args, "--out", str(out)], cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return np.fromfile(out, dtype=np.float32), r.stdout


def test_set_devices_c5_frame(oracle_mod, sky, tmp_path):
    """C5's frame (3840x2160, S1000, depth 16) at 2 spp: SetDevices(2) and SetDevices(8) equal
    the single-device image bit for bit, and the oracle on rows from every partition."""
    W, H, spp, depth = 3840, 2160, 2, 16
    base = ["--scene", "s1000", "--width", str(W), "--height", str(H), "--spp", str(spp), "--depth", str(depth),
            "--seed", "1234"]
    mono, _ = _run(base, tmp_path, "d1.bin")
    for n in (2, 8):
        got, stdout = _run(base + ["--devices", str(n)], tmp_path, f"d{n}.bin")
        assert f"on {n} device context(s)" in stdout, stdout
        np.testing.assert_array_equal(got.view(np.uint32), mono.view(np.uint32))
        os.remove(tmp_path / f"d{n}.bin")
    rows = np.array([0, 7, 8, 15, 16, 1079, 1080, 2151, 2159], dtype=np.int32)
    cam = oracle_mod.camera_get_copy(scenes.camera_for(W, H))
    rng = oracle_mod.init_rng(1234, W, rows, threads=8)
    acc, _, _, _ = oracle_mod.render(scenes.scene_s1000(), cam, sky, rows, spp, depth, rng, threads=8)
    want = (acc[:, :3] / acc[:, 3:4]).astype(np.float32)
    got_rows = mono.reshape(H, W, 3)[rows].reshape(-1, 3)
    np.testing.assert_array_equal(got_rows.view(np.uint32), want.view(np.uint32))


def test_set_devices_dispatch_pipeline(tmp_path):
    """InitPipeline + DispatchRay x3 over 2 row-tile contexts: each pass's tiles (with their
    first-hit normals) are gathered before the denoise + mix, so the BGRA8 frame is the golden
    single-device frame (path_tracer.cu:256-306)."""
    out = tmp_path / "frame.bin"
    r = subprocess.run([_headless(), "--scene", "s4", "--width", "64", "--height", "48", "--depth", "8",
                        "--dispatch", "3", "--bgra", str(out), "--devices", "2"], cwd=REPO, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    z = np.load(os.path.join(GOLDEN, "display_s4_64x48_3frames.npz"))
    np.testing.assert_array_equal(np.fromfile(out, dtype=np.uint8).reshape(48, 64, 4), z["bgra"])
