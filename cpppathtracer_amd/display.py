"""Row-banded multi-GPU display path (SURVEY.md §8(e), next tier).

The reference's interactive loop renders 1 spp per dispatch, then runs Denoising + Mix and
hands a BGRA8 frame to the callback (path_tracer.cu:256-306).  Across N GPUs (one process per
GPU) each rank owns a contiguous band of output rows (tiling.display_band), renders the band
plus a 3-row halo (tiling.display_rows), denoises and mixes its band on its own GPU
(cpt_denoise_mix_band), and one all-gather of the BGRA8 bands (RCCL over xGMI) assembles the
frame.  The frame is byte-identical to the single-GPU display path (tests/test_display_bands.py
on the oracle with gloo ranks, tests/test_gpu_display_bands.py on the GPU).
"""
import numpy as np

from . import tiling


class BandedDisplay:
    """One rank's share of the display path.

    renderer: a Renderer with scene and environment set; the frame is set here (band + halo
    rows).  rank/world: this process's place in the display group (world 1 = the whole frame).
    """

    def __init__(self, renderer, width, height, seed, rank=0, world=1):
        self.r = renderer
        self.width, self.height, self.rank, self.world = width, height, rank, world
        self.y0, self.y1 = tiling.display_band(height, world, rank)
        self.rows = tiling.display_rows(height, world, rank)
        self.band_rows = tiling.max_band_rows(height, world)
        renderer.set_frame(width, height, self.rows)
        renderer.init_rng(seed)

    def dispatch(self, cam, cur_sample_idx, max_depth, **render_kw):
        """One DispatchRay task on this rank: 1 spp (not accumulated) with the first-hit
        normal/depth, then Denoising + Mix of the band.  Returns the band's BGRA8 rows."""
        if self.y1 <= self.y0:
            return np.zeros((0, self.width, 4), dtype=np.uint8)
        self.r.render(cam, 1, max_depth, aux=True, sync=True, **render_kw)
        return self.r.denoise_mix_band(cur_sample_idx, self.y0, self.y1)

    def gather(self, band, group=None):
        """All-gather of the ranks' BGRA8 bands (padded to the largest band) into the full
        (height, width, 4) frame on every rank.  On GPU ranks the bands travel as device
        tensors (RCCL); with the gloo backend as host tensors."""
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return tiling.stitch_bands(band[None], self.height, self.width, 1)
        backend = dist.get_backend(group)
        dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        send = torch.zeros((self.band_rows, self.width, 4), dtype=torch.uint8, device=dev)
        if band.shape[0]:
            send[: band.shape[0]] = torch.from_numpy(np.ascontiguousarray(band)).to(dev)
        out = torch.empty((self.world * self.band_rows, self.width, 4), dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(out, send, group=group)
        g = out.view(self.world, self.band_rows, self.width, 4).cpu().numpy()
        return tiling.stitch_bands(g, self.height, self.width, self.world)
