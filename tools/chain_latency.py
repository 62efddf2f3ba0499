"""How long does a pixel chain take on an otherwise idle GPU?  (DIAGNOSTIC)

A pixel's `spp` passes are one sequential chain (its XORWOW stream continues from pass to
pass, path_tracer.cu:134-137), so no partition can finish before its slowest chain.  This
renders every 8-row block of the image ALONE (15360 pixels: a fraction of one wave per SIMD,
so each chain runs at the latency-bound speed of a nearly idle SIMD) and reports the
per-block times, next to rank 0 of an N-way partition rendered with the full GPU.

    python tools/chain_latency.py [--config c4] [--spp 128] [--ns 1,8]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--spp", type=int, default=128)
    ap.add_argument("--ns", default="1,8")
    ap.add_argument("--schedule", default="cost")
    a = ap.parse_args()
    import numpy as np
    import torch
    from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io, tiling
    cfg = scenes.CONFIGS[a.config]
    W, H, depth = cfg["width"], cfg["height"], cfg["depth"]
    objs = scenes.SCENES[cfg["scene"]]()
    cam = camera_get_copy(scenes.camera_for(W, H))
    with Renderer(0) as r:
        stream = torch.cuda.Stream()
        torch.cuda.set_stream(stream)
        r.set_stream(stream.cuda_stream)
        r.set_scene(objs)
        r.set_env(texture_io.load_cptex())

        def timed(rows):
            r.set_frame(W, H, rows)
            r.init_rng(scenes.DEFAULT_SEED)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            r.render(cam, a.spp, depth, ordered=True, schedule=a.schedule)
            e1.record(stream)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1)

        timed(np.arange(8, dtype=np.int32))   # warm-up
        blocks = [timed(np.arange(y, min(y + 8, H), dtype=np.int32)) for y in range(0, H, 8)]
        ranks = {n: timed(tiling.partition_rows(H, n, 0)) for n in (int(x) for x in a.ns.split(","))}
    b = np.array(blocks)
    print(json.dumps({
        "config": a.config, "spp": a.spp, "schedule": a.schedule,
        "block_alone_ms": {"max": round(float(b.max()), 3), "argmax_row": int(b.argmax()) * 8,
                           "p90": round(float(np.percentile(b, 90)), 3), "median": round(float(np.median(b)), 3),
                           "min": round(float(b.min()), 3), "all": [round(float(x), 2) for x in b]},
        "rank0_full_gpu_ms": {str(n): round(v, 3) for n, v in ranks.items()},
    }), flush=True)


if __name__ == "__main__":
    main()
