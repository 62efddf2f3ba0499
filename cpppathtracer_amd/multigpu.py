"""Row-tiled multi-GPU frame assembly: one process per GPU renders the rows
of its interleaved 8-row blocks (tiling.partition_rows), then one all-gather of the fp32
accumulator tiles (RCCL over xGMI; gloo host copies for CPU/shared-GPU rehearsals) and an
on-device row stitch give every rank the full framebuffer.  bench.py's N > 1 step.

A pixel's stream depends only on (seed, x, y) (path_tracer.cu:36-42), so the stitched frame is
bit-identical to a monolithic render (tests/test_multi_gpu_cpu.py on the oracle,
tests/test_gpu_multirank.py through libcpt.so).
"""
import numpy as np
import torch
import torch.distributed as dist

from . import tiling


class TileGather:
    """Buffers and the collective for one rank's share of a row-tiled frame."""

    def __init__(self, width, height, world, rank, device, backend="nccl", parts=None):
        """parts: every rank's rows (a partition of the frame's rows, the same list on every
        rank); default: the interleaved 8-row blocks (tiling.partition_rows)."""
        self.width, self.height, self.world, self.rank = width, height, world, rank
        self.backend = backend
        if parts is None:
            parts = [tiling.partition_rows(height, world, r) for r in range(world)]
        self.rows = np.asarray(parts[rank], dtype=np.int32)
        self.max_rows = max(int(p.size) for p in parts)
        self.send = torch.zeros((self.max_rows * width, 4), dtype=torch.float32, device=device)
        self.gathered = torch.zeros((world * self.max_rows * width, 4), dtype=torch.float32, device=device)
        self.stitch_idx = torch.from_numpy(tiling.parts_stitch_index(parts, height)).to(device)
        self.device = torch.device(device)

    def __call__(self, renderer):
        """The full (height, width, 4) fp32 framebuffer (rgb sums + pass count) after this
        rank's render: device copy of the local tile, all-gather, row stitch.

        The copy is ordered against torch's current stream on the device, with no host wait
        (cpt_copy_accum_device): it starts after the work queued there so far -- the zero fills
        above, the previous frame's collective still reading `send` -- and the all-gather queued
        next reads the copied tile.  Device errors of the render surface at the next
        synchronising call (the renderer's, or torch.cuda.synchronize for the frame)."""
        stream = torch.cuda.current_stream(self.device).cuda_stream if self.device.type == "cuda" else 0
        renderer.copy_accum_device(self.send.data_ptr(), self.rows.size * self.width * 16, stream)
        if self.world == 1 and not dist.is_initialized():
            return self.send.view(self.max_rows, self.width, 4)[: self.height]
        # with a process group the collective runs at any world size, 1 included (bench.py under
        # torch.distributed.run with one rank, tests/test_gpu_rccl.py): the RCCL branch below is
        # then exercised on a one-GPU box
        if self.backend == "nccl":
            dist.all_gather_into_tensor(self.gathered, self.send)
        else:   # gloo: host copies (rehearsal with ranks sharing a GPU)
            g_host = self.gathered.cpu()
            dist.all_gather_into_tensor(g_host, self.send.cpu())
            self.gathered.copy_(g_host)
        return self.gathered.view(self.world * self.max_rows, self.width, 4).index_select(0, self.stitch_idx)
