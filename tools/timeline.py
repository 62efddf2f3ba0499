"""Lane occupancy of the megakernel over time for one rank of a row-tiled render (DIAGNOSTIC:
a CPT_TIMELINE build, cpt_stamps.hpp timeline; never the timed library).  Where a strong-scaled
rank's time goes: the phase while the pixel queue still has work (every lane busy unless a wave
waits on a take) and the tail after it ran dry (chains finish, lanes idle, waves retire into the
keepers of the tail consolidation).

    python tools/timeline.py [--config c5] [--spp 4096] [--n 8] [--rank 0] [--consolidate auto]
        (CPT_LIB_PATH = the timeline build:
         python -c "from cpppathtracer_amd import build as b; b.build(out='build/tl/timeline.so', defines={'CPT_TIMELINE': 1})")
Prints the occupancy per slice of the render, the split of the lane-time, and one JSON line.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

TICK_MS = 1e-5            # s_memrealtime: 100 MHz
BIN_TICKS = 1 << 17


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--spp", type=int, default=4096)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--consolidate", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--slices", type=int, default=24)
    a = ap.parse_args()
    import numpy as np
    import torch
    from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io, tiling
    cfg = scenes.CONFIGS[a.config]
    W, H, depth = cfg["width"], cfg["height"], cfg["depth"]
    cam = camera_get_copy(scenes.camera_for(W, H))
    lanes = torch.cuda.get_device_properties(0).multi_processor_count * 1024
    with Renderer(0) as r:
        r.set_scene(scenes.SCENES[cfg["scene"]]())
        r.set_env(texture_io.load_cptex())
        rows = tiling.partition_rows(H, a.n, a.rank)
        r.set_frame(W, H, rows)
        r.init_rng(1234)
        r.debug_timeline()   # clear (and arm the queue-dry minimum)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r.render(cam, a.spp, depth, ordered=True, schedule="cost", sync=True,
                 consolidate={"auto": None, "on": True, "off": False}[a.consolidate])
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        bins, dry = r.debug_timeline()
    nz = np.nonzero(bins[:, 1])[0]
    # the render spans less than the ring: its bins are one circular run; start after the gap
    gap = np.argmax(np.diff(np.concatenate([nz, [nz[0] + len(bins)]])))
    order = np.roll(np.arange(len(bins)), -int((nz[gap + 1] if gap + 1 < len(nz) else nz[0])))
    b = bins[order].astype(np.float64)
    last = np.nonzero(b[:, 1])[0][-1]
    b = b[: last + 1]
    t0_bin = int(order[0])
    busy, alive, busy_dry, busy_l0 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]   # lane x ticks
    cap = lanes * BIN_TICKS
    occ = busy / cap
    dry_ms = None
    if dry != 0xFFFFFFFFFFFFFFFF and dry:
        dry_bin = ((dry >> 17) - t0_bin) % len(bins)
        dry_ms = dry_bin * BIN_TICKS * TICK_MS
    n = len(b)
    print(f"{a.config} rank {a.rank} of {a.n}: {rows.size} rows x {W} px x {a.spp} spp, {ms:.1f} ms (events); "
          f"{n} bins of {BIN_TICKS * TICK_MS:.2f} ms; queue dry at {dry_ms} ms")
    print(" slice_ms   busy_lanes%  waves_alive%  busy_after_dry%  busy_in_level0%")
    per = max(1, n // a.slices)
    for i in range(0, n, per):
        s = slice(i, min(n, i + per))
        c = cap * (s.stop - s.start)
        print(f"{i * BIN_TICKS * TICK_MS:8.1f}   {100 * busy[s].sum() / c:10.1f}  {100 * alive[s].sum() / c:11.1f}  "
              f"{100 * busy_dry[s].sum() / c:14.1f}  {100 * busy_l0[s].sum() / c:14.1f}")
    span = n * BIN_TICKS
    total_busy = busy.sum()
    full = (dry_ms / (BIN_TICKS * TICK_MS)) if dry_ms is not None else n
    k = int(full)
    out = {"config": a.config, "n": a.n, "rank": a.rank, "spp": a.spp, "rows": int(rows.size), "ms": round(ms, 1),
           "queue_dry_ms": None if dry_ms is None else round(dry_ms, 1),
           "mean_busy_lanes_frac": round(total_busy / (lanes * span), 4),
           "busy_frac_before_dry": round(busy[:k].sum() / max(1, cap * k), 4),
           "busy_frac_after_dry": round(busy[k:].sum() / max(1, cap * (n - k)), 4),
           "lane_time_after_dry_frac": round(busy[k:].sum() / total_busy, 4),
           "time_after_dry_frac": round((n - k) / n, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
