"""Run one tail-consolidation render (tests/test_gpu_consolidation.py's partly filled last
workgroup) with a short keeper spin limit, so a lost hand-over ends as CPT_ERR_DEVICE instead
of a long wait.  Prints ok / error / mismatch.  CPT_LIB_PATH selects the library.
    python tools/debug_cons_case.py W H schedule"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: F401,E402
import oracle  # noqa: E402
from cpppathtracer_amd import CptError, Renderer, camera_get_copy, scenes, texture_io  # noqa: E402

W, H, schedule = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
objs = scenes.scene_s1000(n=200)
spp, depth, seed = 24, 8, 77
sky = texture_io.load_cptex()
with Renderer(0) as r:
    r.set_scene(objs)
    r.set_env(sky)
    r.set_frame(W, H)
    r.init_rng(seed)
    r.set_debug_consolidation(0, 18, 14)
    cam = camera_get_copy(scenes.camera_for(W, H))
    try:
        r.render(cam, spp, depth, ordered=True, schedule=schedule, consolidate=True, sync=True)
    except CptError as e:
        print("error", e)
        sys.exit(0)
    acc = r.read_accum()
rows = np.arange(H, dtype=np.int32)
rng = oracle.init_rng(seed, W, rows, threads=8)
oacc, _, _, _ = oracle.render(objs, camera_get_copy(scenes.camera_for(W, H)), sky, rows, spp, depth, rng, threads=8)
bad = (acc.view(np.uint32) != oacc.view(np.uint32)).any(axis=1)
print("ok" if not bad.any() else f"mismatch {int(bad.sum())} pixels, passes {np.unique(acc[:, 3])}")
