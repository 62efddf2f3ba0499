"""How far does FMA contraction move the integrator's output?  (DIAGNOSTIC, DESIGN.md §Oracle and parity status)

The reference was compiled by nvcc without --use_fast_math, so a*b+c was contracted into FMA
(SURVEY.md 8(a) numeric semantics).  The shipped oracle and libcpt.so are both built with
-ffp-contract=off and agree bit for bit.  This script renders the same pixels with the
shipped oracle and with its contraction-on build (`make -C oracle fma`: g++ -mfma
-ffp-contract=fast), and reports per-pixel differences at several pass counts:

  * identical_pixels: accumulator sums equal bit for bit
  * identical_rng:    XORWOW end states equal (the pixel's stream has not diverged)
  * rmse:             RMS over pixels and channels of the per-pixel mean radiance difference
  * max_abs:          its maximum
  * mean_radiance:    the image's mean per-pixel radiance (for scale)

    python tools/fp_contract_rmse.py [--out profiles/fp_contract_rmse.json] [--threads 8]

One ulp anywhere changes which side of a surface a bounce starts from or flips a hit, the
pass draws a different number of randoms, and the rest of that pixel's passes follow another
stream: the two images then differ by Monte-Carlo noise, not by rounding.  So this bounds
what "bit-exact vs the oracle" says about the nvcc-built reference: nothing per pixel once a
stream diverges; the images agree only as estimators of the same integral.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import oracle  # noqa: E402  (test infrastructure: this is a diagnostic, not the product)
from cpppathtracer_amd import camera_get_copy, scenes, texture_io  # noqa: E402

CASES = {
    # config: (scene, W, H, depth, row step, spp)
    "c3": ("s4", 1920, 1080, 16, 68, 1024),
    "c4": ("s1000", 1920, 1080, 16, 135, 1024),
}
CHECKPOINTS = (1, 4, 16, 64, 256, 1024)


def render_checkpoints(lib_path, objs, cam, sky, rows, spp, depth, seed, threads):
    oracle.use_library(lib_path)
    W = int(np.asarray(cam["width"]).reshape(-1)[0])
    rng = oracle.init_rng(seed, W, rows, threads=threads)
    acc = np.zeros((rows.size * W, 4), dtype=np.float32)
    out, done = {}, 0
    for c in (c for c in CHECKPOINTS if c <= spp):
        acc, _, _, _ = oracle.render(objs, cam, sky, rows, c - done, depth, rng, accum=acc, accumulate=True,
                                     threads=threads)
        done = c
        out[c] = (acc.copy(), rng.copy())
    return out


def compare(a, b):
    (acc_a, rng_a), (acc_b, rng_b) = a, b
    same_px = np.all(acc_a.view(np.uint32) == acc_b.view(np.uint32), axis=1)
    same_rng = np.all(rng_a == rng_b, axis=0)
    ma = acc_a[:, :3] / acc_a[:, 3:4]
    mb = acc_b[:, :3] / acc_b[:, 3:4]
    d = (ma - mb).astype(np.float64)
    return {
        "identical_pixels": round(float(same_px.mean()), 6),
        "identical_rng": round(float(same_rng.mean()), 6),
        "rmse": float(np.sqrt(np.mean(d * d))),
        "max_abs": float(np.abs(d).max()),
        "mean_radiance": float(ma.mean()),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "fp_contract_rmse.json"))
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--seed", type=int, default=scenes.DEFAULT_SEED)
    ap.add_argument("--configs", default="c3,c4")
    args = ap.parse_args()
    oracle.build()
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "fma"], check=True)
    shipped = oracle.LIB_PATH
    fma = os.path.join(os.path.dirname(shipped), "libcpt_oracle_fma.so")
    sky = texture_io.load_cptex()
    res = {"seed": args.seed, "shipped": "oracle -O2 -ffp-contract=off",
           "variant": "oracle -O2 -mfma -ffp-contract=fast (g++ contraction; nvcc's choices differ)",
           "configs": {}}
    for name in args.configs.split(","):
        scene, W, H, depth, step, spp = CASES[name]
        objs = scenes.SCENES[scene]()
        cam = camera_get_copy(scenes.camera_for(W, H))
        rows = np.arange(0, H, step, dtype=np.int32)
        t = time.time()
        a = render_checkpoints(shipped, objs, cam, sky, rows, spp, depth, args.seed, args.threads)
        b = render_checkpoints(fma, objs, cam, sky, rows, spp, depth, args.seed, args.threads)
        res["configs"][name] = {
            "sample": f"{scene} {W}x{H}, rows 0..{H - 1} step {step} ({rows.size} rows x {W} px), depth {depth}",
            "by_spp": {str(c): compare(a[c], b[c]) for c in a},
            "seconds": round(time.time() - t, 1),
        }
        print(name, json.dumps(res["configs"][name]), flush=True)
    oracle.use_library(None)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
