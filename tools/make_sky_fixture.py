"""Decode the reference's sky environment map into the raw texture fixture.

Run once in the build container (it reads /root/reference, which does not exist on
the GPU box):  python tools/make_sky_fixture.py

What it reproduces (reference behaviour, not a fix):
  * textures.cu:15-17   cv::imread (BGR) + cvtColor(BGR2RGBA)  -> RGBA8, alpha = 255.
                        PIL decodes the 8-bit RGB PNG losslessly to the same bytes.
  * textures.cu:32-33   cudaMemcpy2DToArray(..., width*sizeof(uint8_t), height, ...)
                        copies only `width` BYTES per row = width/4 texels, so only
                        columns [0, width/4) of the cudaArray hold image data.  We keep
                        exactly those columns; the renderer treats the rest as zero.

Output: assets/sky.cptex  (format: see cpppathtracer_amd/texture_io.py / include/cpt.h)
"""
import os
import struct
import sys

import numpy as np

REF_PNG = "/root/reference/textures/sky.png"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets", "sky.cptex")


def fixture_bytes(png_path: str = REF_PNG) -> bytes:
    """The .cptex file's bytes for the PNG at `png_path` (header + the W/4 valid columns as
    RGBA8).  tests/test_sky_fixture.py re-runs this on the reference's PNG and compares it with
    the committed assets/sky.cptex byte for byte."""
    from PIL import Image

    img = Image.open(png_path)
    assert img.mode == "RGB", img.mode
    rgb = np.asarray(img, dtype=np.uint8)  # (H, W, 3)
    h, w, _ = rgb.shape
    valid_cols = w // 4  # textures.cu:32-33 quirk: width bytes, not width texels
    rgba = np.empty((h, valid_cols, 4), dtype=np.uint8)
    rgba[..., :3] = rgb[:, :valid_cols, :]
    rgba[..., 3] = 255
    # header: magic, logical width, height, stored (valid) columns, reserved
    hdr = b"CPTTEX01" + struct.pack("<IIII", w, h, valid_cols, 0)
    return hdr + np.ascontiguousarray(rgba).tobytes()


def main() -> int:
    data = fixture_bytes(REF_PNG)
    with open(OUT, "wb") as f:
        f.write(data)
    print(f"wrote {OUT}: {len(data)} bytes")
    return 0


if __name__ == "__main__":
    sys.exit(main())
