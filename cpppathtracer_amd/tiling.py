"""Row tiling of the image across GPUs.

Each rank renders the global rows of its interleaved 8-row blocks (block b -> rank
b % world): the sky-heavy top rows and the object-heavy bottom rows are dealt evenly, so the
ranks' work is balanced without a pilot pass.  Or (lpt_owner) the blocks are dealt by the work a
short pilot of the whole frame measures, heaviest first to the least-loaded rank.  A pixel's XORWOW stream depends only on
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


def lpt_owner(block_costs, world: int) -> np.ndarray:
    """Cost-balanced partition of row blocks (longest processing time first): blocks heaviest
    first (ties by block index), each to the rank with the least cost so far (ties to the lowest
    rank).  A pure function of the costs, so every rank computes the same partition from the same
    pilot without exchanging anything.  Returns the owning rank of each block."""
    costs = np.asarray(block_costs, dtype=np.int64)
    order = sorted(range(costs.size), key=lambda b: (-int(costs[b]), b))
    load = [0] * world
    owner = np.empty(costs.size, dtype=np.int32)
    for b in order:
        r = min(range(world), key=lambda k: (load[k], k))
        owner[b] = r
        load[r] += int(costs[b])
    return owner


def rows_of_owner(height: int, owner, rank: int, block: int = BLOCK_ROWS) -> np.ndarray:
    """The rows of the blocks `owner` gives to `rank` (ascending)."""
    ys = np.arange(height, dtype=np.int32)
    return ys[np.asarray(owner)[ys // block] == rank]


def block_costs_from_tiles(tile_costs, block: int = BLOCK_ROWS) -> np.ndarray:
    """Per row block cost from the pilot's per 8x8 tile costs (Renderer.tile_costs of the whole
    frame): a block of 8 rows is one row of tiles."""
    assert block == 8, "the pilot's tiles are 8 rows high"
    return np.asarray(tile_costs, dtype=np.int64).sum(axis=1)


def parts_stitch_index(parts, height: int) -> np.ndarray:
    """Row gather index for any partition (parts[r] = rank r's rows, each rank's tile padded to
    the largest): framebuffer row y = gathered row idx[y]."""
    mr = max(int(p.size) for p in parts)
    idx = np.full(height, -1, dtype=np.int64)
    for r, rows in enumerate(parts):
        idx[rows] = r * mr + np.arange(rows.size)
    assert (idx >= 0).all(), "the partition must cover every row"
    return idx


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


# ---- display path (Denoising + Mix, path_tracer.cu:177-254) across ranks ------------------
# The denoiser reads a 5x5 neighbourhood by LINEAR offset over the W' x H' launch
# (W' = 16 floor(W/16), H' likewise), so x +- 2 wraps into the adjacent row: a pixel of row y
# reads rows y - 3 .. y + 3.  Each rank owns a contiguous band of output rows and renders the
# band plus a 3-row halo (the halo rows' streams depend only on (seed, x, y), so both ranks
# that render a halo row compute it identically); no per-pass exchange is needed, and one
# all-gather of the BGRA8 bands assembles the frame.
HALO_ROWS = 3


def display_band(height: int, world: int, rank: int) -> tuple:
    """Output rows [y0, y1) of the display launch owned by `rank` (contiguous, near-equal)."""
    he = 16 * (height // 16)
    return rank * he // world, (rank + 1) * he // world


def display_rows(height: int, world: int, rank: int) -> np.ndarray:
    """The rows a display rank renders: its band and the halo, clipped to [0, H')."""
    he = 16 * (height // 16)
    y0, y1 = display_band(height, world, rank)
    if y1 <= y0:
        return np.zeros(0, dtype=np.int32)
    return np.arange(max(0, y0 - HALO_ROWS), min(he, y1 + HALO_ROWS), dtype=np.int32)


def max_band_rows(height: int, world: int) -> int:
    return max(b - a for a, b in (display_band(height, world, r) for r in range(world)))


def stitch_bands(gathered: np.ndarray, height: int, width: int, world: int) -> np.ndarray:
    """gathered: [world, max_band_rows, width, 4] BGRA8 bands -> the (height, width, 4) frame
    (rows past H' stay 0, as in the single-GPU display path)."""
    out = np.zeros((height, width, 4), dtype=gathered.dtype)
    for r in range(world):
        y0, y1 = display_band(height, world, r)
        out[y0:y1] = gathered[r, : y1 - y0]
    return out


def stitch_index(height: int, width: int, world: int, block: int = BLOCK_ROWS) -> np.ndarray:
    """Row gather index for an on-device stitch: framebuffer row y = gathered row idx[y]."""
    mr = max_rows(height, world, block)
    idx = np.empty(height, dtype=np.int64)
    for r in range(world):
        rows = partition_rows(height, world, r, block)
        idx[rows] = r * mr + np.arange(rows.size)
    return idx
