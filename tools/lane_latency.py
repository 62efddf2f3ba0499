"""How fast does ONE pixel chain run when its wave has few lanes and its SIMD few waves?
(DIAGNOSTIC, DESIGN.md §Multi-GPU: the span of a strong-scaled frame is its longest chain.)

Renders the same small pixel set (8 rows of `--width` pixels, camera `--width` wide: 1024
pixels, all in whole 8x8 tiles) with
CPT_LANES_PER_WAVE = k for each k: every wave takes k pixels, so the set occupies
1024 / k waves.  With a 256-lane LDS block build (1 wave per SIMD) every wave then has its
SIMD to itself.  Reports the render time per k and, with the oracle's chain lengths of the
same pixels (`--chains`), the time per segment of the longest chain.

    CPT_LIB_PATH=build/ab/blk256.so python tools/lane_latency.py [--lanes 1,4,16,64]
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def child(a):
    import numpy as np
    import torch
    from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io
    cfg = scenes.CONFIGS["c4"]
    W, H, depth = a.width, cfg["height"], cfg["depth"]
    objs = scenes.SCENES[cfg["scene"]]()
    cam = camera_get_copy(scenes.camera_for(W, H))
    with Renderer(0) as r:
        stream = torch.cuda.Stream()
        torch.cuda.set_stream(stream)
        r.set_stream(stream.cuda_stream)
        r.set_scene(objs)
        r.set_env(texture_io.load_cptex())
        r.set_frame(W, H, np.arange(a.row, a.row + 8, dtype=np.int32))
        best = None
        for _ in range(2):
            r.init_rng(scenes.DEFAULT_SEED)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            r.render(cam, a.spp, depth, ordered=True, schedule="tiles")
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
    print(json.dumps({"ms": best}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", default="1,2,4,8,16,32,64")
    ap.add_argument("--width", type=int, default=128)
    ap.add_argument("--row", type=int, default=600, help="first of 8 rows")
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--max-chain", type=float, default=None, help="oracle: longest chain (segments) of the set")
    ap.add_argument("--replicate", action="store_true",
                    help="k lanes per wave run ONE pixel as k identical copies (CPT_REPLICATE=k): does a lone "
                         "chain run faster on more lanes?")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a)
    res = {}
    for k in (int(x) for x in a.lanes.split(",")):
        env = dict(os.environ, CPT_LANES_PER_WAVE=str(k))
        if a.replicate:
            env["CPT_REPLICATE"] = str(k)
        out = subprocess.run([sys.executable, __file__, "--child", "--width", str(a.width), "--row", str(a.row),
                              "--spp", str(a.spp)], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(out.stderr[-2000:], file=sys.stderr)
            sys.exit(out.returncode)
        ms = json.loads(out.stdout.strip().splitlines()[-1])["ms"]
        res[k] = {"ms": round(ms, 3)}
        if a.max_chain:
            res[k]["us_per_segment_longest_chain"] = round(1000.0 * ms / a.max_chain, 3)
        print(k, res[k], flush=True)
    print(json.dumps({"lib": os.environ.get("CPT_LIB_PATH", "libcpt.so"), "width": a.width, "row": a.row,
                      "spp": a.spp, "replicate": a.replicate, "lanes": res}), flush=True)


if __name__ == "__main__":
    main()
