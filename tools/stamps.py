"""Wave-time breakdown of the megakernel from a CPT_STAMPS diagnostic build (cpt_stamps.hpp;
never the timed library).

    python tools/stamps.py [config] [spp] [--rows=a:b] [--width=W] [--schedule=cost|tiles|previous] [--consolidate=on|off]   (CPT_LIB_PATH = the stamped build)

Build the diagnostic library with
    python -c "from cpppathtracer_amd import build as b; b.build(out='build/diag/stamps.so', defines={'CPT_STAMPS': 1})"
Prints each section's share of the waves' time and the per-round / per-iteration cycles.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: F401,E402
from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io  # noqa: E402

NAMES = ["refill", "walk_nodes", "walk_leaf_rounds", "certificate_attrs", "hit_shading", "rest", "ray_setup",
         "platforms"]
args = [a for a in sys.argv[1:] if not a.startswith("--")]
cfg = scenes.CONFIGS[args[0] if args else "c4"]
spp = int(args[1]) if len(args) > 1 else 8
rows = None
width = cfg["width"]
schedule = "cost"
consolidate = None
for a in sys.argv[1:]:
    if a.startswith("--consolidate="):
        consolidate = {"on": True, "off": False}[a[14:]]
    if a.startswith("--schedule="):
        schedule = a[11:]
    if a.startswith("--width="):
        width = int(a[8:])
    if a.startswith("--rows="):
        lo, hi = (int(x) for x in a[7:].split(":"))
        rows = np.arange(lo, hi, dtype=np.int32)
r = Renderer(0)
r.set_scene(scenes.SCENES[cfg["scene"]]())
r.set_env(texture_io.load_cptex())
r.set_frame(width, cfg["height"], rows)
r.init_rng(1234)
cam = camera_get_copy(scenes.camera_for(width, cfg["height"]))
r.render(cam, 1, cfg["depth"], sync=True, ordered=True)   # warm-up
r.init_rng(1234)
r.reset_stats()
if schedule == "previous":   # the DispatchRay loop's order: from a previous render's draws
    r.render(cam, spp, cfg["depth"], sync=True, ordered=True, schedule="previous")
    r.init_rng(1234)
    r.reset_stats()
r.render(cam, spp, cfg["depth"], stats=True, sync=True, ordered=True, schedule=schedule, consolidate=consolidate)
c = r.diag_counters()
st = dict(zip(["segments", "nodes", "prims", "hits", "misses"], r.raw_counters()[:5]))
tot = sum(c[:8]) + c[11] + c[12]
rounds, iters, leaf_rounds = c[8], c[9], c[10]
out = {
    "config": cfg, "spp": spp, "counts": st,
    "share": {n: round(c[i] / tot, 4) for i, n in enumerate(NAMES)},
    "wave_cycles": tot, "wave_rounds": rounds, "walk_iterations": iters, "leaf_rounds": leaf_rounds,
    "cycles_per_round": round(tot / max(1, rounds), 1),
    "walk_iterations_per_round": round(iters / max(1, rounds), 2),
    "leaf_rounds_per_round": round(leaf_rounds / max(1, rounds), 2),
    "cycles_per_walk_iteration": round((c[1] + c[2] + c[11] + c[12]) / max(1, iters), 1),
    "cycles_per_leaf_round": round((c[2] + c[12]) / max(1, leaf_rounds), 1),
    "tail_share": round((c[11] + c[12]) / tot, 4),
    "tail_iterations_per_round": round(c[13] / max(1, rounds), 2),
    "lanes_per_round": round(st["segments"] / max(1, rounds), 2),
    "lanes_per_walk_iteration": round(st["nodes"] / max(1, iters), 2),
}
print(json.dumps(out))
