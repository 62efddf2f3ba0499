"""Multi-rank display path rehearsal (SURVEY.md §8(e) next tier): DispatchRay-style frames
(1 spp + Denoising + Mix) rendered as row bands, one rank per GPU, gathered into full frames,
and checked on rank 0 against the single-GPU display path on the same seed.

    torchrun --nproc-per-node N --master-addr 127.0.0.1 tools/display_ranks.py [W H frames]

Backend: nccl (RCCL) when every rank has its own GPU; CPT_DISPLAY_BACKEND=gloo lets N ranks
share one GPU (bands then travel through host memory).  Prints one JSON line on rank 0.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io  # noqa: E402
from cpppathtracer_amd.display import BandedDisplay  # noqa: E402


def main():
    W, H, frames = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (1920, 1080, 8)))
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    backend = os.environ.get("CPT_DISPLAY_BACKEND", "nccl")
    dev = local if backend == "nccl" else 0
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group(backend, rank=rank, world_size=world)
    sky = texture_io.load_cptex()
    objs = scenes.scene_s1000()
    cam = camera_get_copy(scenes.camera_for(W, H))
    with Renderer(dev) as r:
        r.set_scene(objs)
        r.set_env(sky)
        disp = BandedDisplay(r, W, H, 1234, rank, world)
        times = []
        for i in range(frames):
            t = time.perf_counter()
            band = disp.dispatch(cam, i + 2, 16, ordered=True)
            frame = disp.gather(band)
            times.append(time.perf_counter() - t)
    ok = None
    if rank == 0:
        with Renderer(dev) as ref:
            ref.set_scene(objs)
            ref.set_env(sky)
            ref.set_frame(W, H)
            ref.init_rng(1234)
            for i in range(frames):
                ref.render(cam, 1, 16, aux=True, sync=True, ordered=True)
                want = ref.denoise_mix(i + 2)
        ok = bool(np.array_equal(frame, want))
        print(json.dumps({"tool": "display_ranks", "world": world, "backend": backend if world > 1 else None,
                          "width": W, "height": H, "frames": frames, "identical_to_single_gpu": ok,
                          "ms_per_frame_after_first": round(1e3 * float(np.mean(times[1:] or times)), 3)}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
