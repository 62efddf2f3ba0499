"""Supply / demand of a cross-wave walk pool in the megakernel, from a CPT_POOLDIAG diagnostic
build (cpt_stamps.hpp pooldiag; never the timed library).  For every node-visit iteration of the
wide walk: the lanes of the wave whose walk has already ended (they idle until the wave's walk
phase ends: the demand a pool of walks could fill) and the walks other waves of the workgroup hold
suspended at that moment (the supply such a pool would have).  sum min(idle, supply) / sum idle
bounds the share of idle lane-iterations a zero-cost pool could fill (DESIGN.md §Lane use).

    python tools/pooldiag.py [config] [spp]        (CPT_LIB_PATH = the CPT_POOLDIAG build)
Build: python tools/build_variants.py pooldiag:CPT_POOLDIAG=1
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
name = args[0] if args else "c4"
cfg = scenes.CONFIGS[name]
spp = int(args[1]) if len(args) > 1 else 16
r = Renderer(0)
r.set_scene(scenes.SCENES[cfg["scene"]]())
r.set_env(texture_io.load_cptex())
r.set_frame(cfg["width"], cfg["height"])
r.init_rng(1234)
cam = camera_get_copy(scenes.camera_for(cfg["width"], cfg["height"]))
r.reset_stats()
r.render(cam, spp, cfg["depth"], sync=True, ordered=True, schedule="cost")
c = r.execdiag_counters()[0]
it, idle, fill, work, sup, nsusp, calls = (int(x) for x in c[:7])
out = {"config": name, "spp": spp, "node_iterations": it, "walk_calls": calls, "walks_suspended": nsusp,
       "mean_working_lanes": round(work / max(it, 1), 2), "mean_idle_lanes": round(idle / max(it, 1), 2),
       "mean_supply": round(sup / max(it, 1), 2), "fillable_idle_frac": round(fill / max(idle, 1), 4),
       "lanes_if_filled": round((work + fill) / max(it, 1), 2)}
print(json.dumps(out, indent=1))
