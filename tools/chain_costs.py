"""Distribution of pixel chain lengths (path segments over all `spp` passes) from the oracle
(DIAGNOSTIC): the makespan of a strong-scaled render cannot drop below
its longest chain, while the N = 1 time follows the sum.

    python tools/chain_costs.py [--config c4] [--row-step 16] [--spp 1024] [--out profiles/chain_costs_c4.json]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import oracle  # noqa: E402  (test infrastructure: a diagnostic, not the product)
from cpppathtracer_amd import camera_get_copy, scenes, texture_io  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--row-step", type=int, default=16)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cfg = scenes.CONFIGS[a.config]
    W, H, depth = cfg["width"], cfg["height"], cfg["depth"]
    spp = a.spp or cfg["spp"]
    objs = scenes.SCENES[cfg["scene"]]()
    cam = camera_get_copy(scenes.camera_for(W, H))
    rows = np.arange(0, H, a.row_step, dtype=np.int32)
    seg = oracle.pixel_segments(objs, cam, texture_io.load_cptex(), rows, spp, depth, scenes.DEFAULT_SEED,
                                threads=a.threads).astype(np.float64)
    q = {f"p{p}": float(np.percentile(seg, p)) for p in (50, 90, 99, 99.9, 99.99)}
    per_row = seg.reshape(rows.size, W)
    res = {
        "config": a.config, "spp": spp, "sample": f"rows 0..{H - 1} step {a.row_step} ({rows.size} rows x {W} px)",
        "segments_per_chain": {"mean": float(seg.mean()), "max": float(seg.max()), **q},
        "max_over_mean": round(float(seg.max() / seg.mean()), 3),
        "row_max": [int(x) for x in per_row.max(axis=1)],
        "row_mean": [round(float(x), 1) for x in per_row.mean(axis=1)],
        "hist_edges": [float(x) for x in np.linspace(0, seg.max(), 21)],
        "hist": [int(x) for x in np.histogram(seg, bins=np.linspace(0, seg.max(), 21))[0]],
    }
    txt = json.dumps(res)
    print(json.dumps({k: v for k, v in res.items() if not k.startswith("row_")}))
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
