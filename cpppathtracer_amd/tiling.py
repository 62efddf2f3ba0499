"""Row tiling of the image across GPUs.

Each rank renders the global rows of its interleaved 8-row blocks (block b -> rank
b % world): the sky-heavy top rows and the object-heavy bottom rows are dealt evenly, so the
ranks' work is balanced without a pilot pass.  A pixel's XORWOW stream depends only on
(seed, x, y) (path_tracer.cu:36-42), so any row partition gives results bit-identical to a
monolithic render.  After the render, the fp32 accumulator tiles are gathered into one
framebuffer with a single all-gather (RCCL over xGMI on MI355X; gloo in the CPU tests).
"""
import numpy as np

BLOCK_ROWS = 8   # one row of the megakernel's 8x8 pixel tiles


def weak_scaled_size(width: int, height: int, world: int) -> tuple:
    """Weak scaling (bench.py --scaling weak): N times the pixels at the same aspect, i.e. each
    axis scaled by sqrt(N) and rounded to whole 8x8 tiles (N = 4: 1920x1080 -> 3840x2160)."""
    if world <= 1:
        return width, height
    f = world ** 0.5
    return int(round(width * f / 8)) * 8, int(round(height * f / 8)) * 8


def partition_rows(height: int, world: int, rank: int, block: int = BLOCK_ROWS) -> np.ndarray:
    ys = np.arange(height, dtype=np.int32)
    return ys[(ys // block) % world == rank]


def max_rows(height: int, world: int, block: int = BLOCK_ROWS) -> int:
    return max(int(partition_rows(height, world, r, block).size) for r in range(world))


def stitch(gathered: np.ndarray, height: int, width: int, world: int, block: int = BLOCK_ROWS) -> np.ndarray:
    """gathered: [world * max_rows * width, C] (each rank's tile padded to max_rows rows)
    -> framebuffer [height * width, C] in global row order."""
    mr = max_rows(height, world, block)
    c = gathered.shape[-1]
    g = gathered.reshape(world, mr, width, c)
    out = np.empty((height, width, c), dtype=gathered.dtype)
    for r in range(world):
        rows = partition_rows(height, world, r, block)
        out[rows] = g[r, : rows.size]
    return out.reshape(height * width, c)


def stitch_index(height: int, width: int, world: int, block: int = BLOCK_ROWS) -> np.ndarray:
    """Row gather index for an on-device stitch: framebuffer row y = gathered row idx[y]."""
    mr = max_rows(height, world, block)
    idx = np.empty(height, dtype=np.int64)
    for r in range(world):
        rows = partition_rows(height, world, r, block)
        idx[rows] = r * mr + np.arange(rows.size)
    return idx
