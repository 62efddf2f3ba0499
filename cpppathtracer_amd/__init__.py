"""MI355X-native path-tracing integrator (DearPoca/CppPathTracer's hot path on gfx950).

The compute path is libcpt.so (hand-written HIP kernels behind the C-ABI in include/cpt.h).
This package is the host-side mirror used by tests and the benchmark.
"""
from . import scenes, texture_io, types  # noqa: F401
from ._lib import CptError, lib_path, load  # noqa: F401
from .renderer import Renderer, camera_get_copy, device_count  # noqa: F401

__all__ = ["Renderer", "camera_get_copy", "device_count", "CptError", "load", "lib_path", "scenes",
           "texture_io", "types"]
