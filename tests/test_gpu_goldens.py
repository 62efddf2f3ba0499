"""GPU against the committed goldens, the display path, and the C++ drop-in API.

* the HIP megakernel reproduces every golden fixture bit for bit (config 1 in full);
* Denoising + Mix (cpt_denoise_mix) reproduces the oracle's display frames byte for byte;
* the reference-shaped C++ API (include/cpppathtracer, examples/headless_render.cpp) renders
  the same radiance as the oracle and runs the asynchronous DispatchRay pipeline.
"""
import ast
import hashlib
import os
import subprocess

import numpy as np
import pytest

from cpppathtracer_amd import camera_get_copy, scenes

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CASES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz") and f[0] in "cs" and "spp" in f)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", CASES)
def test_gpu_matches_golden(gpu, sky, name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    m = ast.literal_eval(str(z["meta"]))
    W, H = m["width"], m["height"]
    gpu.set_scene(scenes.SCENES[m["scene"]]())
    gpu.set_env(sky)
    gpu.set_frame(W, H)
    gpu.init_rng(m["seed"])
    gpu.reset_stats()
    gpu.render(camera_get_copy(scenes.camera_for(W, H)), m["spp"], m["depth"], aux=True, stats=True, sync=True)
    acc, rng = gpu.read_accum(), gpu.read_rng()
    nrm, _ = gpu.read_aux()
    st = gpu.stats()
    assert [st[k] for k in ("segments", "nodes", "prims", "hits", "misses")] == z["stats"].tolist()
    if "accum" in z:
        np.testing.assert_array_equal(acc.view(np.uint32), z["accum"].view(np.uint32))
        np.testing.assert_array_equal(rng, z["rng"])
    assert sha(acc) == str(z["accum_sha256"])
    assert sha(rng) == str(z["rng_sha256"])
    assert sha(nrm) == str(z["normal_sha256"])


def test_gpu_display_path(gpu, sky):
    z = np.load(os.path.join(GOLDEN, "display_s4_64x48_3frames.npz"))
    W, H = 64, 48
    gpu.set_scene(scenes.scene_s4())
    gpu.set_env(sky)
    gpu.set_frame(W, H)
    gpu.init_rng(1234)
    cam = camera_get_copy(scenes.camera_for(W, H))
    for idx in (2, 3, 4):
        gpu.render(cam, 1, 8, aux=True, sync=True)
        out = gpu.denoise_mix(idx)
    np.testing.assert_array_equal(out, z["bgra"])


def _headless():
    from cpppathtracer_amd import build
    return build.build_examples()


@pytest.mark.parametrize("scene,W,H,spp,depth", [("s4", 64, 36, 2, 8), ("s3", 48, 32, 3, 4), ("s1000", 64, 36, 2, 16),
                                                  ("s1000", 32, 18, 64, 8)])
def test_cpp_api_render_matches_oracle(oracle_mod, sky, tmp_path, scene, W, H, spp, depth):
    out = tmp_path / "rad.bin"
    r = subprocess.run([_headless(), "--scene", scene, "--width", str(W), "--height", str(H), "--spp", str(spp),
                        "--depth", str(depth), "--seed", "1234", "--out", str(out)],
                       cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rgb = np.fromfile(out, dtype=np.float32).reshape(H * W, 3)
    cam = oracle_mod.camera_get_copy(scenes.camera_for(W, H))
    rows = np.arange(H, dtype=np.int32)
    rng = oracle_mod.init_rng(1234, W, rows)
    acc, _, _, _ = oracle_mod.render(scenes.SCENES[scene](), cam, sky, rows, spp, depth, rng, threads=8)
    want = acc[:, :3] / acc[:, 3:4]
    np.testing.assert_array_equal(rgb.view(np.uint32), want.astype(np.float32).view(np.uint32))


@pytest.mark.parametrize("devices", [1, 2])
def test_cpp_api_animated_refit(oracle_mod, sky, tmp_path, devices):
    """A dynamic scene through the C++ API: after the first frame, every 10th object moves by
    +0.75 in x before each of 3 more frames (SceneBVH::UpdateObject -> device refit, in every
    context of PathTracer::SetDevices).  The last frame equals the oracle's render of the refit
    BVH (bvh.cu:122-157) with the RNG streams carried across the frames."""
    W, H, spp, depth, K = 48, 27, 2, 16, 3
    out = tmp_path / "rad.bin"
    r = subprocess.run([_headless(), "--scene", "s1000", "--width", str(W), "--height", str(H), "--spp", str(spp),
                        "--depth", str(depth), "--seed", "1234", "--animate", str(K), "--out", str(out),
                        "--devices", str(devices)],
                       cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert f"frame {K}:" in r.stdout, r.stdout
    objs = scenes.scene_s1000()
    cam = oracle_mod.camera_get_copy(scenes.camera_for(W, H))
    rows = np.arange(H, dtype=np.int32)
    rng = oracle_mod.init_rng(1234, W, rows)
    acc, _, _, _ = oracle_mod.render(objs, cam, sky, rows, spp, depth, rng, threads=8)
    moved = np.arange(1, len(objs), 10)
    x = objs["center"][moved, 0].astype(np.float32).copy()
    for _ in range(K):
        x = (x + np.float32(0.75)).astype(np.float32)
        edits = []
        for i, xi in zip(moved, x):
            o = objs[int(i)].copy()
            o["center"][0] = xi
            edits.append((int(i), o))
        acc, _ = oracle_mod.render_edited(objs, edits, cam, sky, rows, spp, depth, rng, threads=8)
    want = acc[:, :3] / acc[:, 3:4]
    rgb = np.fromfile(out, dtype=np.float32).reshape(H * W, 3)
    np.testing.assert_array_equal(rgb.view(np.uint32), want.astype(np.float32).view(np.uint32))


def test_cpp_api_dispatch_pipeline(oracle_mod, sky, tmp_path):
    """InitPipeline + DispatchRay x3: GetCopy at thread start (idx 1), then 1 spp + denoise +
    mix per dispatch with idx 2, 3, 4 (path_tracer.cu:256-306) — same bytes as the oracle."""
    out = tmp_path / "frame.bin"
    r = subprocess.run([_headless(), "--scene", "s4", "--width", "64", "--height", "48", "--depth", "8",
                        "--dispatch", "3", "--bgra", str(out)], cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "cur_sample_idx 4" in r.stdout
    z = np.load(os.path.join(GOLDEN, "display_s4_64x48_3frames.npz"))
    np.testing.assert_array_equal(np.fromfile(out, dtype=np.uint8).reshape(48, 64, 4), z["bgra"])


def test_cpp_api_textured_materials(oracle_mod, sky, tmp_path):
    """PocaTextureUtils::AddTexByFile + Material::have_tex_/tex_ through the C++ API: the
    floor, Glass and Metal sphere of s4 sample a PPM texture (W/4 upload quirk included)."""
    W, H, spp, depth = 48, 32, 2, 8
    rgb = np.random.default_rng(77).integers(0, 256, size=(12, 32, 3), dtype=np.uint8)
    ppm = tmp_path / "tex.ppm"
    with open(ppm, "wb") as f:
        f.write(b"P6\n32 12\n255\n" + rgb.tobytes())
    out = tmp_path / "rad.bin"
    r = subprocess.run([_headless(), "--scene", "s4", "--width", str(W), "--height", str(H), "--spp", str(spp),
                        "--depth", str(depth), "--seed", "1234", "--out", str(out), "--texture", str(ppm)],
                       cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    handle = int(r.stdout.split("texture handle ")[1].split()[0])
    from cpppathtracer_amd import texture_io, types
    rgba = np.concatenate([rgb, np.full((12, 32, 1), 255, np.uint8)], axis=2)
    objs = scenes.scene_s4()
    for i in (0, 1, 2):
        m = objs[i]["material"].copy()
        objs[i]["material"] = types.set_material_texture(m, handle)
    oracle_mod.bind_texture(handle, texture_io.from_full_rgba(rgba))
    try:
        cam = oracle_mod.camera_get_copy(scenes.camera_for(W, H))
        rows = np.arange(H, dtype=np.int32)
        rng = oracle_mod.init_rng(1234, W, rows)
        acc, _, _, _ = oracle_mod.render(objs, cam, sky, rows, spp, depth, rng)
    finally:
        oracle_mod.clear_textures()
    want = acc[:, :3] / acc[:, 3:4]
    got = np.fromfile(out, dtype=np.float32).reshape(H * W, 3)
    np.testing.assert_array_equal(got.view(np.uint32), want.astype(np.float32).view(np.uint32))
