"""Environment-texture fixture I/O (``.cptex``).

Format (little endian): ``b"CPTTEX01"``, uint32 logical_width, uint32 height,
uint32 valid_cols, uint32 reserved, then ``valid_cols * height`` RGBA8 texels row-major.
``valid_cols`` < logical_width encodes the reference upload quirk (textures.cu:32-33:
only width/4 texels per row reach the cudaArray); texels at x >= valid_cols read as 0.
"""
import os
import struct
from dataclasses import dataclass

import numpy as np

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")
SKY_PATH = os.path.join(ASSET_DIR, "sky.cptex")


@dataclass
class EnvTexture:
    rgba: np.ndarray     # (height, valid_cols, 4) uint8, C-contiguous
    width: int           # logical width (addressing / filtering use this)
    height: int

    @property
    def valid_cols(self) -> int:
        return int(self.rgba.shape[1])


def load_cptex(path: str = SKY_PATH) -> EnvTexture:
    with open(path, "rb") as f:
        hdr = f.read(24)
        if len(hdr) != 24 or hdr[:8] != b"CPTTEX01":
            raise ValueError(f"{path}: not a CPTTEX01 file")
        w, h, cols, _ = struct.unpack("<IIII", hdr[8:])
        data = np.frombuffer(f.read(), dtype=np.uint8)
    if data.size != cols * h * 4:
        raise ValueError(f"{path}: payload {data.size} B, expected {cols * h * 4}")
    return EnvTexture(np.ascontiguousarray(data.reshape(h, cols, 4)), int(w), int(h))


def from_full_rgba(rgba: np.ndarray) -> EnvTexture:
    """Apply the reference upload quirk to a full (H, W, 4) image: keep W/4 columns."""
    h, w, _ = rgba.shape
    return EnvTexture(np.ascontiguousarray(rgba[:, : w // 4, :].astype(np.uint8)), int(w), int(h))
