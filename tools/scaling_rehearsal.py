"""1-GPU rehearsal of the row-tiled strong scaling: renders rank 0's rows of
an N-way partition (tiling.partition_rows) and reports the projected efficiency
t(1) / (N * t(N, rank 0)).  The real N-GPU run adds one all-gather of the tiles.
    python tools/scaling_rehearsal.py [--config c4] [--spp 1024] [--block 8] [--ns 1,2,4,8] [--schedule cost]
                                      [--partition interleaved|balanced] [--pilot-passes 1]"""
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
    ap.add_argument("--partition", default="interleaved", choices=["interleaved", "balanced"],
                    help="rows per rank: interleaved 8-row blocks, or blocks dealt by a pilot's cost (tiling.lpt_owner)")
    ap.add_argument("--pilot-passes", type=int, default=1)
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
        pilot_ms = None
        owner_costs = None
        if a.partition == "balanced":
            # the whole frame's pilot, as every rank would run it (deterministic: same costs everywhere)
            r.set_frame(W, H)
            r.init_rng(1234)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            owner_costs = tiling.block_costs_from_tiles(r.tile_costs(cam, a.pilot_passes, depth))
            e1.record(stream)
            torch.cuda.synchronize()
            pilot_ms = e0.elapsed_time(e1)
        for n in (int(x) for x in a.ns.split(",")):
            times = []
            owner = tiling.lpt_owner(owner_costs, n) if owner_costs is not None else None
            for rank in range(n) if n <= 8 else (0,):
                rows = (tiling.partition_rows(H, n, rank, block) if owner is None
                        else tiling.rows_of_owner(H, owner, rank))
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
            res[n] = {"max_rank_ms": max(times), "mean_rank_ms": sum(times) / len(times),
                      "rank_ms": [round(t, 1) for t in times], "rows_rank0": int(
                tiling.partition_rows(H, n, 0, block).size)}
    t1 = res[min(res)]["max_rank_ms"]
    for n, v in res.items():
        v["projected_efficiency"] = round(t1 / (n * v["max_rank_ms"]), 4)
    print(json.dumps({"config": a.config, "spp": a.spp, "block_rows": block, "schedule": a.schedule,
                      "consolidate": a.consolidate, "partition": a.partition, "pilot_passes": a.pilot_passes,
                      "pilot_ms": pilot_ms, "results": res}),
          flush=True)


if __name__ == "__main__":
    main()
