"""Per-phase cycle shares of k_megakernel from a CPT_STAMPS diagnostic build (never timed)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401
from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io
cfg = scenes.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4"]
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 8
r = Renderer(0)
r.set_scene(scenes.SCENES[cfg["scene"]]())
r.set_env(texture_io.load_cptex())
r.set_frame(cfg["width"], cfg["height"])
r.init_rng(1234)
cam = camera_get_copy(scenes.camera_for(cfg["width"], cfg["height"]))
r.reset_stats()
r.render(cam, spp, cfg["depth"], stats=True, sync=True)
c = r.raw_counters()
tot = sum(c[5:8])
print("counts", dict(zip(["segments", "nodes", "prims", "hits", "misses"], c[:5])))
print("refill %.1f%%  trace %.1f%%  shade+rest %.1f%%  (wave-cycles %d)" % (100 * c[5] / tot, 100 * c[6] / tot, 100 * c[7] / tot, tot))
