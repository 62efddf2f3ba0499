"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

The reference has no tests, fixtures or golden images and cannot be
built here, so the goldens are the oracle's own outputs at fixed seeds: they pin the oracle
against regressions (tests/test_goldens.py) and are the target the HIP path must reproduce
bit for bit (tests/test_gpu_goldens.py).  Re-run only on a deliberate oracle change:

    python tools/make_goldens.py
"""
import hashlib
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import oracle  # noqa: E402
from cpppathtracer_amd import scenes, texture_io  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")

# name: (scene, W, H, spp, depth, seed, store_full)
CASES = {
    "c1_s3_256x256_4spp_d4": ("s3", 256, 256, 4, 4, 1234, False),
    "s3_64x64_4spp_d8": ("s3", 64, 64, 4, 8, 1234, True),
    "s4_64x48_4spp_d16": ("s4", 64, 48, 4, 16, 1234, True),
    "s4_48x32_2spp_d32_seed7": ("s4", 48, 32, 2, 32, 7, True),
    "s1000_64x36_2spp_d16": ("s1000", 64, 36, 2, 16, 1234, True),
}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def render_case(scene, W, H, spp, depth, seed, sky):
    objs = scenes.SCENES[scene]()
    cam = oracle.camera_get_copy(scenes.camera_for(W, H))
    rows = np.arange(H, dtype=np.int32)
    rng = oracle.init_rng(seed, W, rows, threads=8)
    acc, st, nrm, dep = oracle.render(objs, cam, sky, rows, spp, depth, rng, want_aux=True, threads=8)
    return acc, rng, st, nrm


def main():
    sky = texture_io.load_cptex()
    os.makedirs(OUT, exist_ok=True)
    for name, (scene, W, H, spp, depth, seed, full) in CASES.items():
        acc, rng, st, nrm = render_case(scene, W, H, spp, depth, seed, sky)
        meta = dict(scene=scene, width=W, height=H, spp=spp, depth=depth, seed=seed)
        arrays = dict(
            stats=np.array([st[k] for k in ("segments", "nodes", "prims", "hits", "misses")], dtype=np.uint64),
            accum_sha256=np.array(sha(acc)), rng_sha256=np.array(sha(rng)), normal_sha256=np.array(sha(nrm)),
            row_sums=acc.reshape(H, W, 4).sum(axis=1, dtype=np.float64),
            meta=np.array(repr(meta)),
        )
        if full:
            arrays.update(accum=acc, rng=rng)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **arrays)
        print(name, st, "mean", acc[:, :3].sum() / (W * H * spp * 3))
    # display path: 3 DispatchRay-style frames (1 spp, denoise, mix with idx 2, 3, 4)
    W, H = 64, 48
    objs = scenes.scene_s4()
    cam = oracle.camera_get_copy(scenes.camera_for(W, H))
    rows = np.arange(H, dtype=np.int32)
    rng = oracle.init_rng(1234, W, rows, threads=8)
    mix = np.zeros((W * H, 3), np.float32)
    out = np.zeros((H, W, 4), np.uint8)
    for idx in (2, 3, 4):
        acc, _, nrm, dep = oracle.render(objs, cam, sky, rows, 1, 8, rng, want_aux=True, threads=8)
        oracle.denoise_mix(acc, nrm, dep, mix, out, W, H, idx)
    np.savez_compressed(os.path.join(OUT, "display_s4_64x48_3frames.npz"), bgra=out, mix=mix)
    print("display", out[..., :3].mean())


if __name__ == "__main__":
    main()
