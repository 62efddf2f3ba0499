"""Can a pixel chain be split?  (DIAGNOSTIC)

A pixel's passes are one sequential chain because each pass starts where the previous pass
left the pixel's XORWOW stream (path_tracer.cu:134-137); the next pass's start is known only
once the current pass has drawn all its numbers.  This records every pass's draw count and
segment count with the oracle (oracle.pass_trace) and asks how predictable the draw count is
on the longest chains, and what a speculative scheme would save: while the main lane runs
pass k from its known state, m helper lanes run passes k+1..k+m from the state advanced by
j times the last pass's draw count; the chain advances past every pass whose guess was right.

    python tools/pass_trace.py [--row-step 64] [--spp 1024] [--top 200]
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


def speculative_span(draws, segs, m):
    """Span in segments of one chain under m-lane last-value speculation: each step costs
    the longest of the m + 1 passes run side by side, and commits the passes up to the first
    wrong guess."""
    k, n, t, prev = 0, len(draws), 0, draws[0]
    while k < n:
        j = 1
        while j <= m and k + j < n and draws[k + j - 1] == prev:
            j += 1
        t += int(segs[k:min(n, k + m + 1)].max())
        prev = draws[k + j - 1]
        k += j
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--row-step", type=int, default=64)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--top", type=int, default=200)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    a = ap.parse_args()
    cfg = scenes.CONFIGS[a.config]
    W, H, depth = cfg["width"], cfg["height"], cfg["depth"]
    spp = a.spp or cfg["spp"]
    objs = scenes.SCENES[cfg["scene"]]()
    cam = camera_get_copy(scenes.camera_for(W, H))
    rows = np.arange(a.row_step // 2, H, a.row_step, dtype=np.int32)
    draws, segs = oracle.pass_trace(objs, cam, texture_io.load_cptex(), rows, spp, depth, scenes.DEFAULT_SEED,
                                    threads=a.threads)
    d, s = draws.astype(np.int32), segs.astype(np.int32)
    total = s.sum(axis=1)
    top = np.argsort(-total)[:a.top]
    same = d[:, 1:] == d[:, :-1]
    vals, cnt = np.unique(d[top], return_counts=True)
    order = np.argsort(-cnt)
    res = {
        "config": a.config, "spp": spp, "sample": f"rows {rows[0]}..{H - 1} step {a.row_step} ({rows.size} x {W} px)",
        "chain_segments": {"mean": float(total.mean()), "max": int(total.max())},
        "top_chains": int(top.size),
        "top_passes_at_max_depth": round(float((s[top] == depth).mean()), 4),
        "top_draw_counts": {int(v): int(c) for v, c in zip(vals[order][:12], cnt[order][:12])},
        "last_value_hit_rate": {"all": round(float(same.mean()), 4), "top": round(float(same[top].mean()), 4)},
        "speculative_span_over_serial_top50": {
            str(m): round(float(np.mean([speculative_span(d[i], s[i], m) / total[i] for i in top[:50]])), 4)
            for m in (1, 3, 7, 15)},
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
