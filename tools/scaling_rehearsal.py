"""1-GPU rehearsal of the row-tiled strong scaling: renders rank 0's rows of
an N-way partition (tiling.partition_rows) and reports the projected efficiency
t(1) / (N * t(N, rank 0)).  The real N-GPU run adds one all-gather of the tiles.
    python tools/scaling_rehearsal.py [--config c4] [--spp 1024] [--block 8] [--ns 1,2,4,8] [--schedule cost]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--schedule", default="cost", choices=["cost", "tiles"])
    ap.add_argument("--block", type=int, default=None)
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--consolidate", default="auto", choices=["auto", "on", "off"],
                    help="megakernel tail consolidation (default: the library's rule)")
    a = ap.parse_args()
    import torch
    from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io, tiling
    cfg = scenes.CONFIGS[a.config]
    W, H, depth = cfg["width"], cfg["height"], cfg["depth"]
    objs = scenes.SCENES[cfg["scene"]]()
    cam = camera_get_copy(scenes.camera_for(W, H))
    block = a.block or tiling.BLOCK_ROWS
    res = {}
    with Renderer(0) as r:
        stream = torch.cuda.Stream()
        torch.cuda.set_stream(stream)
        r.set_stream(stream.cuda_stream)
        r.set_scene(objs)
        r.set_env(texture_io.load_cptex())
        for n in (int(x) for x in a.ns.split(",")):
            times = []
            for rank in range(n) if n <= 8 else (0,):
                rows = tiling.partition_rows(H, n, rank, block)
                r.set_frame(W, H, rows)
                best = None
                for _ in range(a.reps):
                    r.init_rng(1234)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    r.render(cam, a.spp, depth, ordered=True, schedule=a.schedule,
                             consolidate={"auto": None, "on": True, "off": False}[a.consolidate])
                    e1.record(stream)
                    torch.cuda.synchronize()
                    ms = e0.elapsed_time(e1)
                    best = ms if best is None else min(best, ms)
                times.append(best)
            res[n] = {"max_rank_ms": max(times), "mean_rank_ms": sum(times) / len(times), "rows_rank0": int(
                tiling.partition_rows(H, n, 0, block).size)}
    t1 = res[min(res)]["max_rank_ms"]
    for n, v in res.items():
        v["projected_efficiency"] = round(t1 / (n * v["max_rank_ms"]), 4)
    print(json.dumps({"config": a.config, "spp": a.spp, "block_rows": block, "schedule": a.schedule,
                      "consolidate": a.consolidate, "results": res}),
          flush=True)


if __name__ == "__main__":
    main()
