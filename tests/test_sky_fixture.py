"""The one reference-held input, textures/sky.png, is pinned (round-5 verdict item 6).

assets/sky.cptex is the PNG decoded once, offline, by tools/make_sky_fixture.py with the
reference's W/4-valid-column upload (cuSrc/textures.cu:14-33: cv::imread + BGR2RGBA, then a
cudaMemcpy2DToArray of `width` bytes per row).  Every golden and every sky-lit parity case reads
that file, so a regenerated or hand-edited fixture would move them all silently:
  * test_fixture_sha256 (every box, CPU and GPU) pins the committed bytes to a hash;
  * test_fixture_matches_reference_png (this container only: /root/reference does not exist on
    the GPU box) re-decodes the reference's PNG with PIL and compares byte for byte.
"""
import hashlib
import importlib.util
import os

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(REPO, "assets", "sky.cptex")
REF_PNG = "/root/reference/textures/sky.png"
SKY_SHA256 = "0d19217d1883675c5d30e72e457ffcf3be1c7189381de65dacd7ca296a838fea"


def test_fixture_sha256():
    with open(FIXTURE, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == SKY_SHA256


def test_fixture_header_and_columns():
    from cpppathtracer_amd import texture_io
    t = texture_io.load_cptex(FIXTURE)
    # sky.png is 1280 x 1280 RGB; only width/4 = 320 columns hold image data (textures.cu:32-33)
    assert (t.width, t.height) == (1280, 1280)
    assert t.rgba.shape == (1280, 320, 4)
    assert (t.rgba[..., 3] == 255).all()


@pytest.mark.skipif(not os.path.exists(REF_PNG), reason="reference PNG absent (GPU box)")
def test_fixture_matches_reference_png():
    pytest.importorskip("PIL")
    spec = importlib.util.spec_from_file_location("make_sky_fixture", os.path.join(REPO, "tools", "make_sky_fixture.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    with open(FIXTURE, "rb") as f:
        committed = f.read()
    assert mod.fixture_bytes(REF_PNG) == committed
