"""Per-phase cycle shares from CPT_STAMPS diagnostic builds (never timed).
  CPT_STAMPS=1: megakernel refill / trace / shade;  CPT_STAMPS=2: BVH walk leaf / slab / whole iteration."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io  # noqa: E402

cfg = scenes.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4"]
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 8
mode = int(sys.argv[3]) if len(sys.argv) > 3 else 1
r = Renderer(0)
r.set_scene(scenes.SCENES[cfg["scene"]]())
r.set_env(texture_io.load_cptex())
r.set_frame(cfg["width"], cfg["height"])
r.init_rng(1234)
cam = camera_get_copy(scenes.camera_for(cfg["width"], cfg["height"]))
r.reset_stats()
r.render(cam, spp, cfg["depth"], stats=True, sync=True, ordered=os.environ.get("CPT_WALK", "ordered") == "ordered")
c = r.raw_counters()
print("counts", dict(zip(["segments", "nodes", "prims", "hits", "misses"], c[:5])))
if mode == 1:
    tot = sum(c[5:8])
    print("refill %.1f%%  trace %.1f%%  shade+rest %.1f%%  (wave-cycles %d)" % (100 * c[5] / tot, 100 * c[6] / tot,
                                                                              100 * c[7] / tot, tot))
else:
    # per-iteration wave-cycles, normalised by lane-level node visits / 64 (the ideal iteration count)
    it = c[7]
    print("walk iterations: leaf %.1f%%  slab %.1f%%  rest %.1f%%  (iteration wave-cycles %d)" % (
        100 * c[5] / it, 100 * c[6] / it, 100 * (it - c[5] - c[6]) / it, it))
    print("wave-cycles per lane node visit x64: %.1f" % (it / (c[1] / 64.0)))
