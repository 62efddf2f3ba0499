"""CPU-side checks of the C-ABI library and the host logic (no GPU needed).

* libcpt.so loads and exports every symbol include/cpt.h declares;
* without a GPU, cpt_create fails loudly with CPT_ERR_NO_DEVICE (no CPU fallback exists);
* the product's host BVH build equals the oracle's restatement of SceneBVH::Divide
  (bvh.cu:31-90), node for node;
* the product's MotionalCamera::GetCopy equals the oracle's (motional_camera.cu:177-200);
* the POD layouts match the reference's structs byte for byte.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from cpppathtracer_amd import _lib, scenes, types

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "cpt.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(cpt_\w+)\s*\(", text, re.M)))


def test_header_symbols_exported():
    L = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.PROTOTYPES), set(syms) ^ set(_lib.PROTOTYPES)


def test_abi_version_and_status_strings():
    L = _lib.load()
    assert L.cpt_abi_version() == 1
    assert L.cpt_status_string(0) == b"ok"
    assert L.cpt_status_string(2) == b"no HIP device"


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible; covered by the gpu tests")
    L = _lib.load()
    h = ctypes.c_void_p()
    st = L.cpt_create(0, ctypes.byref(h))
    assert st == 2 and not h.value
    assert b"no HIP device" in L.cpt_last_error(None)
    with pytest.raises(_lib.CptError):
        from cpppathtracer_amd import Renderer
        Renderer(0)


def test_layouts(oracle_mod):
    L = oracle_mod.lib()
    assert (L.or_sizeof(0), L.or_sizeof(1), L.or_sizeof(2)) == (40, 72, 136)
    assert types.MATERIAL_DTYPE.itemsize == 40
    assert types.OBJECT_DTYPE.fields["center"][1] == 48
    assert types.OBJECT_DTYPE.fields["height"][1] == 68
    assert types.CAMERA_DTYPE.fields["vertical"][1] == 124


def _product_bvh(objs):
    L = _lib.load()
    objs = np.ascontiguousarray(objs)
    n = ctypes.c_int(0)
    cap = max(1, 2 * len(objs))
    boxes = np.zeros((cap, 6), np.float32)
    links = np.zeros((cap, 4), np.int32)
    st = L.cpt_bvh_build_host(ctypes.c_void_p(objs.ctypes.data) if len(objs) else None, len(objs),
                              ctypes.c_void_p(boxes.ctypes.data), ctypes.c_void_p(links.ctypes.data), cap,
                              ctypes.byref(n))
    assert st == 0
    return boxes[:n.value], links[:n.value]


@pytest.mark.parametrize("name", ["s3", "s4", "s1000"])
def test_bvh_matches_oracle(oracle_mod, name):
    objs = scenes.SCENES[name]()
    b1, l1 = _product_bvh(objs)
    b2, l2 = oracle_mod.build_bvh(objs)
    assert len(b1) == 2 * len(objs) - 1
    np.testing.assert_array_equal(l1, l2)
    np.testing.assert_array_equal(b1.view(np.uint32), b2.view(np.uint32))


def test_bvh_edge_cases(oracle_mod):
    assert len(_product_bvh(np.zeros(0, dtype=types.OBJECT_DTYPE))[0]) == 0
    one = scenes.scene_s3()[:1]
    b, l = _product_bvh(one)
    assert l.tolist() == [[1, -1, -1, 0]]
    # negative radius (the reference's inner glass sphere, video_renderer.cpp:96-99): |r| box
    o = scenes.scene_s3()[:2].copy()
    o[1]["radius"] = -5.0
    b1, l1 = _product_bvh(o)
    b2, l2 = oracle_mod.build_bvh(o)
    np.testing.assert_array_equal(b1, b2)
    np.testing.assert_array_equal(l1, l2)


def test_bvh_is_balanced_median_split():
    objs = scenes.scene_s1000()
    _, links = _product_bvh(objs)
    depth = np.zeros(len(links), np.int32)
    for i, (leaf, l, r, _) in enumerate(links):
        if not leaf:
            depth[l] = depth[i] + 1
            depth[r] = depth[i] + 1
    assert depth.max() == int(np.ceil(np.log2(len(objs))))
    leaves = links[links[:, 0] == 1][:, 3]
    assert sorted(leaves.tolist()) == list(range(len(objs)))


@pytest.mark.parametrize("wh", [(256, 256), (1280, 720), (1920, 1080), (3840, 2160), (333, 77)])
def test_camera_get_copy_matches_oracle(oracle_mod, wh):
    from cpppathtracer_amd import camera_get_copy
    cam = scenes.camera_for(*wh)
    a = camera_get_copy(cam)
    b = oracle_mod.camera_get_copy(cam)
    assert a.tobytes() == b.tobytes()
    assert int(a["cur_sample_idx"]) == 1
    assert np.allclose(np.linalg.norm(a["w"]), 1.0, atol=1e-6)


@pytest.mark.parametrize("scene", ["s3", "s4", "s1000"])
def test_cpp_driver_scenes_equal_python_scenes(tmp_path, scene):
    """The C++ headless driver builds S3/S4/S1000 through the drop-in API (AddObject +
    BuildBVH); the objects BuildBVH copied equal scenes.py's byte for byte, so the C++ API
    parity tests on the GPU render exactly the oracle's scenes."""
    import subprocess
    from cpppathtracer_amd import build
    out = tmp_path / "objs.bin"
    r = subprocess.run([build.build_examples(), "--scene", scene, "--dump-scene", str(out)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(out, dtype=np.uint8)
    want = np.ascontiguousarray(scenes.SCENES[scene]()).view(np.uint8).ravel()
    np.testing.assert_array_equal(got, want)


def test_denoise_mix_rejects_bad_host_buffers():
    """Advisor r04: the display call checks the caller's frame with exceptions (not asserts, which
    `python -O` strips): the C-ABI would write H*W*4 bytes into it."""
    import numpy as np
    import pytest
    from cpppathtracer_amd import Renderer
    r = object.__new__(Renderer)   # no context: the checks run before any C-ABI call
    r.height, r.width = 4, 8
    for bad in (np.zeros((4, 8, 4), dtype=np.float32), np.zeros((4, 8, 3), dtype=np.uint8),
                np.zeros((8, 8, 4), dtype=np.uint8)[::2], bytearray(128)):
        with pytest.raises(ValueError):
            r.denoise_mix(1, out=bad)
    ro = np.zeros((4, 8, 4), dtype=np.uint8)
    ro.flags.writeable = False
    with pytest.raises(ValueError):
        r.denoise_mix(1, out=ro)
