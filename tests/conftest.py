import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libcpt.so's HIP kernels)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def sky():
    from cpppathtracer_amd import texture_io
    return texture_io.load_cptex()


@pytest.fixture(scope="session")
def gpu():
    """A Renderer on cuda:0.  GPU tests fail (never skip) when the HIP path is unavailable,
    so a box without the native library can't pass them silently."""
    import torch  # noqa: F401  (load torch's HIP runtime first: one runtime per process)
    from cpppathtracer_amd import Renderer
    r = Renderer(0)
    yield r
    r.close()


def frame_rows(h, rows=None):
    return np.arange(h, dtype=np.int32) if rows is None else np.asarray(rows, dtype=np.int32)


def lobe_exponents(oracle_mod, scene):
    """The inv_alpha of every non-Diffuse material of a scene: 1.0 / (double)powf(1000, smoothness)
    (material.cu:43-45, cpt_kernels.hip k_prepare_materials; Diffuse's exponent is 1/2)."""
    from cpppathtracer_amd import scenes, types
    objs = scenes.SCENES[scene]()
    sm = sorted({float(o["material"]["smoothness"]) for o in objs if int(o["material"]["type"]) != types.DIFFUSE})
    return [1.0 / float(oracle_mod.lib().or_powf(np.float32(1000.0), np.float32(s))) for s in sm]
