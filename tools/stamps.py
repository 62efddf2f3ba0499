"""Per-phase cycle shares from CPT_STAMPS diagnostic builds (never timed).
  CPT_STAMPS=1: megakernel refill / trace / shade;  CPT_STAMPS=2: BVH walk leaf / slab / whole iteration;
  CPT_STAMPS=4: hit shading / miss shading / rest of the megakernel loop;
  CPT_STAMPS=3: wave-level counts (walk iterations, iterations with a lane at a leaf / at an inner
  node, segment rounds) for the lane-efficiency breakdown.
Build a diagnostic library with build.build(out=..., defines={"CPT_STAMPS": m}) and point
CPT_LIB_PATH at it."""
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
elif mode == 4:
    tot = c[7]
    print("hit shading %.1f%%  miss shading %.1f%%  rest %.1f%%  (wave-cycles %d)" % (
        100 * c[5] / tot, 100 * c[6] / tot, 100 * (tot - c[5] - c[6]) / tot, tot))
elif mode == 3:
    seg, nodes, hits = c[0], c[1], c[3]
    w_seg = c[4] - (seg - hits)          # stats[4] = misses + segment rounds
    w_leaf, w_inner, w_it = c[5], c[6], c[7]
    print("segment rounds %d: %.1f of 64 lanes trace per round" % (w_seg, seg / w_seg))
    print("walk iterations %d: %.1f of 64 lanes step per iteration (%.1f walk iterations per round, "
          "%.1f node visits per segment)" % (w_it, nodes / w_it, w_it / w_seg, nodes / seg))
    print("iterations with a lane at a leaf %.1f%%, at an inner node %.1f%%, both %.1f%%" % (
        100 * w_leaf / w_it, 100 * w_inner / w_it, 100 * (w_leaf + w_inner - w_it) / w_it))
else:
    # per-iteration wave-cycles, normalised by lane-level node visits / 64 (the ideal iteration count)
    it = c[7]
    print("walk iterations: leaf %.1f%%  slab %.1f%%  rest %.1f%%  (iteration wave-cycles %d)" % (
        100 * c[5] / it, 100 * c[6] / it, 100 * (it - c[5] - c[6]) / it, it))
    print("wave-cycles per lane node visit x64: %.1f" % (it / (c[1] / 64.0)))
