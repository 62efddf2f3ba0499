"""Full-frame parity sweep (GPU box): render a configuration with the reference-order walk and
the ordered walk, run the oracle on the same pixels, and report the pixels whose RNG end state
or radiance differ.  Usage: python tools/walk_parity.py [--config c4] [--spp 2] [--rows N]"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--spp", type=int, default=2)
    ap.add_argument("--rows", type=int, default=0, help="0 = all rows")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default="gpurun_out/walk_parity.json")
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime first)
    import oracle
    from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io
    cfg = scenes.CONFIGS[a.config]
    W, H, depth = cfg["width"], cfg["height"], cfg["depth"]
    rows = np.arange(H, dtype=np.int32) if not a.rows else np.linspace(0, H - 1, a.rows).astype(np.int32)
    objs = scenes.SCENES[cfg["scene"]]()
    sky = texture_io.load_cptex()
    cam = camera_get_copy(scenes.camera_for(W, H))
    out = {"config": a.config, "spp": a.spp, "rows": int(rows.size), "width": W}
    res = {}
    with Renderer(0) as r:
        r.set_scene(objs)
        r.set_env(sky)
        r.set_frame(W, H, rows)
        for walk in ("reference", "ordered"):
            r.init_rng(1234)
            r.reset_stats()
            r.render(cam, a.spp, depth, stats=True, sync=True, ordered=(walk == "ordered"))
            res[walk] = (r.read_accum(), r.read_rng(), r.stats())
    rng = oracle.init_rng(1234, W, rows, threads=a.threads)
    acc, st, _, _ = oracle.render(objs, cam, sky, rows, a.spp, depth, rng, threads=a.threads)
    res["oracle"] = (acc, rng, st)
    for walk in ("reference", "ordered"):
        ga, gr, gs = res[walk]
        bad = np.flatnonzero((gr != rng).any(axis=0) | (ga.view(np.uint32) != acc.view(np.uint32)).any(axis=1))
        out[walk] = {"stats": gs, "diverging_pixels": int(bad.size),
                     "first": [[int(rows[i // W]), int(i % W)] for i in bad[:32]]}
    out["oracle"] = {"stats": st}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: (v if not isinstance(v, dict) else {kk: vv for kk, vv in v.items() if kk != "first"})
                      for k, v in out.items()}))


if __name__ == "__main__":
    main()
