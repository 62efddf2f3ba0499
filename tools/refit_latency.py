"""Latency of cpt_update_objects (device refit) vs cpt_update_objects_rebuild (host SAH rebuild,
re-linearisation of the nine orders, full upload) on S1000-generator scenes, then a render of
the edited scene through both, checked equal.

    python tools/refit_latency.py [--sizes 1000,30000] [--batches 1,16,256]

Prints one line per (scene size, batch size): median host wall ms of each call (the call
returns after the device copies are updated).
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1000,30000")
    ap.add_argument("--batches", default="1,16,256")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    r = Renderer(0)
    sky = texture_io.load_cptex()
    rng = np.random.default_rng(0)
    out = []
    for n in (int(x) for x in args.sizes.split(",")):
        objs = scenes.scene_s1000(n=n)
        r.set_scene(objs)
        info = r.walk_info()
        bounded = np.flatnonzero(objs["type"] != 1)
        for b in (int(x) for x in args.batches.split(",")):
            t = {False: [], True: []}
            for rep in range(args.reps):
                idx = rng.choice(bounded, size=min(b, bounded.size), replace=False).astype(np.int32)
                new = objs[idx].copy()
                new["center"][:, 0] += rng.uniform(-5, 5, idx.size).astype(np.float32)
                for rebuild in (False, True):
                    r.update_objects(idx, new, rebuild=rebuild)
                    t[rebuild].append(r.last_update_ms())
                    r.update_objects(idx, objs[idx], rebuild=rebuild)   # back
            row = dict(objects=n + 1, n_wide=info["n_wide"], batch=int(b),
                       device_refit_ms=float(np.median(t[False])), host_rebuild_ms=float(np.median(t[True])))
            print(json.dumps(row), flush=True)
            out.append(row)
        # the edited scene renders the same through both paths
        idx = bounded[:64].astype(np.int32)
        new = objs[idx].copy()
        new["center"][:, 2] += np.float32(3.0)
        imgs = []
        for rebuild in (False, True):
            r.set_scene(objs)
            r.update_objects(idx, new, rebuild=rebuild)
            r.set_env(sky)
            r.set_frame(256, 144)
            r.init_rng(7)
            r.render(camera_get_copy(scenes.camera_for(256, 144)), 4, 16, ordered=True, sync=True)
            imgs.append(r.read_accum())
        assert np.array_equal(imgs[0].view(np.uint32), imgs[1].view(np.uint32))
        print(json.dumps(dict(objects=n + 1, render_refit_equals_rebuild=True)), flush=True)
    r.close()


if __name__ == "__main__":
    main()
