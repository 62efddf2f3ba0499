"""Diagnostic: C5's frame (3840x2160, S1000) at 2 spp rendered monolithically and as the 8-way
row partition (one process, partitions rendered one after another), with tail consolidation
forced on and off.  Prints, for each variant, the pixels whose pass count is not spp and the
pixels that differ from the monolithic render, and checks a few rows against the oracle.

    python tools/debug_c5_partition.py [--world 8] [--spp 2] [--lib path]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--spp", type=int, default=2)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--oracle-rows", default="0,7,8,1079,1080,2151,2159")
    args = ap.parse_args()
    import torch  # noqa: F401
    import oracle
    from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io, tiling
    W, H, SPP, DEPTH = args.width, args.height, args.spp, 16
    objs = scenes.scene_s1000()
    sky = texture_io.load_cptex()
    cam = camera_get_copy(scenes.camera_for(W, H))

    def render(rows, consolidate):
        with Renderer(0) as r:
            r.set_scene(objs)
            r.set_env(sky)
            r.set_frame(W, H, rows)
            r.init_rng(scenes.DEFAULT_SEED)
            r.render(cam, SPP, DEPTH, ordered=True, schedule="cost", sync=True, consolidate=consolidate)
            return r.read_accum()

    mono = render(None, None).reshape(H, W, 4)
    print(f"mono: pixels with passes != spp: {(mono[..., 3] != SPP).sum()}", flush=True)
    orows = np.array([int(x) for x in args.oracle_rows.split(",")], np.int32)
    orng = oracle.init_rng(scenes.DEFAULT_SEED, W, orows, threads=8)
    oacc, _, _, _ = oracle.render(objs, cam, sky, orows, SPP, DEPTH, orng, threads=8)
    d = (mono[orows].reshape(-1, 4).view(np.uint32) != oacc.view(np.uint32)).any(axis=1)
    print(f"mono vs oracle on rows {orows.tolist()}: differing pixels {d.sum()}", flush=True)
    for cons in (True, False, None):
        fb = np.zeros((H, W, 4), np.float32)
        for rank in range(args.world):
            rows = tiling.partition_rows(H, args.world, rank)
            fb[rows] = render(rows, cons).reshape(rows.size, W, 4)
        bad = fb[..., 3] != SPP
        diff = (fb.view(np.uint32) != mono.view(np.uint32)).any(axis=2)
        ys = np.flatnonzero(diff.any(axis=1))
        print(f"partition x{args.world} consolidate={cons}: passes != spp: {bad.sum()}, differ from mono: "
              f"{diff.sum()} px in {ys.size} rows {ys[:12].tolist()}", flush=True)
        if diff.any():
            y, x = np.argwhere(diff)[0]
            print(f"   first differing pixel ({x},{y}): part {fb[y, x].tolist()} mono {mono[y, x].tolist()}", flush=True)


if __name__ == "__main__":
    main()
