"""Exec-mask census of the megakernel from a CPT_EXECDIAG diagnostic build (cpt_stamps.hpp
execdiag; never the timed library): for each code region, how often a wave enters it and with
how many active lanes.  A VALU instruction with <= 16 active lanes costs ~3x the cycles of a
fuller one when several waves share a CU (tools/exec_count_probe.hip), so thinly entered
regions are the candidates for predication.

    python tools/execdiag.py [config] [spp]        (CPT_LIB_PATH = the CPT_EXECDIAG build)

Build: python -c "from cpppathtracer_amd import build as b; b.build(out='build/diag/execdiag.so', defines={'CPT_EXECDIAG': 1})"
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io  # noqa: E402

REGIONS = ["refill_take", "walk_node_visit", "leaf_round", "certificate_attrs", "eval_material", "glass_block",
           "sky_fetch", "sky_second_fetch", "sky_defer_store", "start_pass_tail", "start_pass_take",
           "pixel_writeback", "segment_start", "shade_entry", "hand_over", "mirror_enum_draw"]
args = [a for a in sys.argv[1:] if not a.startswith("--")]
name = args[0] if args else "c4"
cfg = scenes.CONFIGS[name]
spp = int(args[1]) if len(args) > 1 else 8
r = Renderer(0)
r.set_scene(scenes.SCENES[cfg["scene"]]())
r.set_env(texture_io.load_cptex())
r.set_frame(cfg["width"], cfg["height"])
r.init_rng(1234)
cam = camera_get_copy(scenes.camera_for(cfg["width"], cfg["height"]))
r.reset_stats()
r.render(cam, spp, cfg["depth"], sync=True, ordered=True, schedule="cost")
c = r.execdiag_counters()
rounds = int(c[0][13]) or 1
out = {"config": name, "spp": spp, "regions": {}}
for i, n in enumerate(REGIONS):
    e = int(c[0][i])
    if not e:
        continue
    out["regions"][n] = {"entries": e, "per_shade_round": round(e / rounds, 3),
                         "mean_lanes": round(int(c[3][i]) / e, 2),
                         "frac_le16": round(int(c[1][i]) / e, 4), "frac_le8": round(int(c[2][i]) / e, 4)}
print(json.dumps(out, indent=1))
