"""ctypes wrapper over oracle/build/libcpt_oracle.so — TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference integrator (oracle/cpt_oracle.cpp).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product package (cpppathtracer_amd) never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libcpt_oracle.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (g++ is in the image and on the GPU box)."""
    if force or not os.path.exists(LIB_PATH) or (
        os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "cpt_oracle.cpp"))
    ):
        subprocess.run(["make", "-s", "-C", _HERE, "-B" if force else "all"], check=True)
    return LIB_PATH


def use_library(path=None):
    """DIAGNOSTIC: bind the module to another build of the oracle (e.g. the FMA-contraction
    variant, `make -C oracle fma`); None returns to the default build."""
    global _lib, _lib_path
    _lib = None
    _lib_path = path


_lib_path = None


def lib():
    global _lib
    if _lib is None:
        if _lib_path is None:
            build()
        L = ctypes.CDLL(_lib_path or LIB_PATH)
        P = ctypes.c_void_p
        i32, u64, f32, f64 = ctypes.c_int, ctypes.c_uint64, ctypes.c_float, ctypes.c_double
        L.or_abi_version.restype = i32
        L.or_sizeof.argtypes = [i32]
        L.or_sizeof.restype = i32
        for n in ("or_pow",):
            getattr(L, n).argtypes = [f64, f64]
            getattr(L, n).restype = f64
        for n in ("or_log", "or_exp", "or_atan"):
            getattr(L, n).argtypes = [f64]
            getattr(L, n).restype = f64
        L.or_powf.argtypes = [f32, f32]
        L.or_powf.restype = f32
        for n in ("or_sinf", "or_cosf", "or_asinf", "or_atanf"):
            getattr(L, n).argtypes = [f32]
            getattr(L, n).restype = f32
        L.or_math_batch.argtypes = [i32, P, P, P, ctypes.c_long]
        L.or_math_batch.restype = None
        L.or_curand_init.argtypes = [u64, u64, P]
        L.or_curand_init.restype = None
        L.or_xorwow_next.argtypes = [P]
        L.or_xorwow_next.restype = ctypes.c_uint32
        L.or_uniform.argtypes = [P]
        L.or_uniform.restype = f32
        L.or_seq_jump_matrix_pow4.argtypes = [i32, P]
        L.or_seq_jump_matrix_pow4.restype = None
        L.or_jump_matrix_pow4.argtypes = [i32, P]
        L.or_jump_matrix_pow4.restype = None
        L.or_init_rng.argtypes = [u64, i32, P, i32, P, i32]
        L.or_init_rng.restype = None
        L.or_camera_get_copy.argtypes = [P]
        L.or_camera_get_copy.restype = None
        L.or_build_bvh.argtypes = [P, i32, P, P, i32]
        L.or_build_bvh.restype = i32
        L.or_denoise_mix.argtypes = [P, P, P, P, P, i32, i32, ctypes.c_uint32]
        L.or_denoise_mix.restype = None
        L.or_denoise_mix_band.argtypes = [P, P, P, P, P, i32, i32, i32, i32, i32, ctypes.c_uint32]
        L.or_denoise_mix_band.restype = None
        L.or_render.argtypes = [P, i32, P, P, i32, i32, i32, P, i32, i32, i32, P, P, P, P, P, i32, i32]
        L.or_render.restype = i32
        L.or_render_edited.argtypes = [P, i32, P, P, i32, P, P, i32, i32, i32, P, i32, i32, i32, P, P, P, i32]
        L.or_render_edited.restype = i32
        L.or_render_edited_ex.argtypes = [P, i32, P, P, i32, P, P, i32, i32, i32, P, i32, i32, i32, P, P, P, i32, i32]
        L.or_render_edited_ex.restype = i32
        L.or_bind_texture.argtypes = [u64, P, i32, i32, i32, i32, i32]
        L.or_bind_texture.restype = None
        L.or_clear_textures.argtypes = []
        L.or_clear_textures.restype = None
        L.or_last_fallbacks.argtypes = []
        L.or_last_fallbacks.restype = u64
        L.or_set_pixel_segments.argtypes = [P]
        L.or_set_pixel_segments.restype = None
        L.or_set_pass_trace.argtypes = [P, P]
        L.or_set_pass_trace.restype = None
        L.or_set_walk.argtypes = [i32]
        L.or_set_walk.restype = None
        _lib = L
    return _lib


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def math_batch(op: int, a, b=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b if b is not None else np.zeros_like(a), dtype=np.float32)
    out = np.empty_like(a)
    lib().or_math_batch(op, _ptr(a), _ptr(b), _ptr(out), a.size)
    return out


def curand_init(seed: int, subsequence: int) -> np.ndarray:
    out = np.zeros(6, dtype=np.uint32)
    lib().or_curand_init(seed, subsequence, _ptr(out))
    return out


def seq_jump_matrix_pow4(t: int) -> np.ndarray:
    out = np.zeros(800, dtype=np.uint32)
    lib().or_seq_jump_matrix_pow4(t, _ptr(out))
    return out


def jump_matrix_pow4(t: int) -> np.ndarray:
    out = np.zeros(800, dtype=np.uint32)
    lib().or_jump_matrix_pow4(t, _ptr(out))
    return out


def init_rng(seed: int, width: int, rows, threads: int = 1) -> np.ndarray:
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    out = np.zeros((6, rows.size * width), dtype=np.uint32)
    lib().or_init_rng(seed, width, _ptr(rows), rows.size, _ptr(out), threads)
    return out


def camera_get_copy(cam):
    """MotionalCamera::GetCopy on a CAMERA_DTYPE scalar/0-d array; returns the updated copy."""
    c = np.array(cam, copy=True)
    lib().or_camera_get_copy(_ptr(c))
    return c


def build_bvh(objs):
    objs = np.ascontiguousarray(objs)
    cap = max(1, 2 * len(objs))
    box = np.zeros((cap, 6), dtype=np.float32)
    link = np.zeros((cap, 4), dtype=np.int32)
    m = lib().or_build_bvh(_ptr(objs), len(objs), _ptr(box), _ptr(link), cap)
    return box[:m], link[:m]


def render(objs, cam, env, rows, spp, max_depth, rng, accum=None, want_aux=False, accumulate=False,
           threads=1):
    """Run `spp` passes of the reference integrator over `rows` (global row indices).

    rng: uint32 [6, n_rows*W] planar XORWOW state, advanced in place.
    Returns (accum [n_rows*W, 4] float32, stats dict, normal or None, depth or None).
    """
    objs = np.ascontiguousarray(objs)
    cam = np.ascontiguousarray(cam)
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    W = int(np.asarray(cam["width"]).reshape(-1)[0])
    npix = rows.size * W
    assert rng.dtype == np.uint32 and rng.shape == (6, npix) and rng.flags.c_contiguous
    if accum is None:
        accum = np.zeros((npix, 4), dtype=np.float32)
    normal = np.zeros((npix, 3), dtype=np.float32) if want_aux else None
    depth = np.zeros(npix, dtype=np.float32) if want_aux else None
    stats = np.zeros(5, dtype=np.uint64)
    env_ptr = _ptr(env.rgba) if env is not None else None
    ew, eh, ec = (env.width, env.height, env.valid_cols) if env is not None else (1, 1, 0)
    rc = lib().or_render(_ptr(objs), len(objs), _ptr(cam), env_ptr, ew, eh, ec, _ptr(rows), rows.size, spp,
                         max_depth, _ptr(rng), _ptr(accum), _ptr(normal), _ptr(depth), _ptr(stats),
                         1 if accumulate else 0, threads)
    if rc != 0:
        raise ValueError(f"or_render failed: {rc}")
    st = dict(zip(("segments", "nodes", "prims", "hits", "misses"), (int(x) for x in stats)))
    return accum, st, normal, depth


def bind_texture(handle, tex, address_mode=2, filter_mode=1):
    """Bind texels (texture_io.EnvTexture) to a material texture handle (process-wide)."""
    rgba = np.ascontiguousarray(tex.rgba, dtype=np.uint8)
    lib().or_bind_texture(handle, _ptr(rgba), tex.width, tex.height, tex.valid_cols, address_mode, filter_mode)


def clear_textures():
    lib().or_clear_textures()


def last_fallbacks() -> int:
    """DIAGNOSTIC: certificate fallbacks of the last render() in the ordered walk."""
    return int(lib().or_last_fallbacks())


def pixel_segments(objs, cam, env, rows, spp, max_depth, seed, threads=1):
    """DIAGNOSTIC: each pixel's number of path segments over `spp` passes (the length of its
    sequential chain) -> uint32 [n_rows * W]."""
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    W = int(np.asarray(cam["width"]).reshape(-1)[0])
    out = np.zeros(rows.size * W, dtype=np.uint32)
    rng = init_rng(seed, W, rows, threads=threads)
    lib().or_set_pixel_segments(_ptr(out))
    try:
        render(objs, cam, env, rows, spp, max_depth, rng, threads=threads)
    finally:
        lib().or_set_pixel_segments(None)
    return out


def pass_trace(objs, cam, env, rows, spp, max_depth, seed, threads=1):
    """DIAGNOSTIC: per pixel and pass, the pass's RNG draws and path segments -> two uint8
    arrays [n_rows * W, spp]."""
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    W = int(np.asarray(cam["width"]).reshape(-1)[0])
    draws = np.zeros((rows.size * W, spp), dtype=np.uint8)
    segs = np.zeros((rows.size * W, spp), dtype=np.uint8)
    rng = init_rng(seed, W, rows, threads=threads)
    lib().or_set_pass_trace(_ptr(draws), _ptr(segs))
    try:
        render(objs, cam, env, rows, spp, max_depth, rng, threads=threads)
    finally:
        lib().or_set_pass_trace(None, None)
    return draws, segs


def set_walk(ordered: bool):
    """DIAGNOSTIC: make render() walk the BVH the way CPT_TRAVERSAL_ORDERED does (near child
    first, reference-rank tie rule) instead of the reference's right-first DFS.  Process-wide."""
    lib().or_set_walk(1 if ordered else 0)


def render_edited(objs, edits, cam, env, rows, spp, max_depth, rng, threads=1, walk_rebuild=False):
    """render() on the BVH of `objs` after SceneBVH::UpdateObject edits [(index, new_object), ...]
    (refit, same topology, bvh.cu:122-157).  The diagnostic ordered walk's own tree is refit the
    same way (cpt_update_objects), or rebuilt from the edited objects with walk_rebuild
    (cpt_update_objects_rebuild).  Returns (accum, stats)."""
    objs = np.ascontiguousarray(objs)
    cam = np.ascontiguousarray(cam)
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    idx = np.ascontiguousarray([i for i, _ in edits], dtype=np.int32)
    new = np.ascontiguousarray(np.array([o for _, o in edits], dtype=objs.dtype))
    npix = rows.size * int(np.asarray(cam["width"]).reshape(-1)[0])
    assert rng.dtype == np.uint32 and rng.shape == (6, npix) and rng.flags.c_contiguous
    accum = np.zeros((npix, 4), dtype=np.float32)
    stats = np.zeros(5, dtype=np.uint64)
    env_ptr = _ptr(env.rgba) if env is not None else None
    ew, eh, ec = (env.width, env.height, env.valid_cols) if env is not None else (1, 1, 0)
    rc = lib().or_render_edited_ex(_ptr(objs), len(objs), _ptr(idx), _ptr(new), idx.size, _ptr(cam), env_ptr, ew, eh,
                                   ec, _ptr(rows), rows.size, spp, max_depth, _ptr(rng), _ptr(accum), _ptr(stats),
                                   threads, int(bool(walk_rebuild)))
    if rc != 0:
        raise ValueError(f"or_render_edited failed: {rc}")
    return accum, dict(zip(("segments", "nodes", "prims", "hits", "misses"), (int(x) for x in stats)))


def denoise_mix(accum, normal, depth, mix, out, width, height, cur_sample_idx):
    """Denoising + Mix on host arrays (mix [W*H,3] float32 and out [H,W,4] uint8 in/out)."""
    for a, dt in ((accum, np.float32), (normal, np.float32), (depth, np.float32), (mix, np.float32), (out, np.uint8)):
        assert a.dtype == dt and a.flags.c_contiguous
    lib().or_denoise_mix(_ptr(accum), _ptr(normal), _ptr(depth), _ptr(mix), _ptr(out), width, height, cur_sample_idx)


def denoise_mix_band(accum, normal, depth, mix, out, width, height, row0, y0, y1, cur_sample_idx):
    """Denoising + Mix for output rows [y0, y1): accum [n,4] / normal [n,3] / depth [n] hold the
    rendered rows row0, row0+1, ... (band + 3-row halo); mix [(y1-y0)*W,3] and out [y1-y0,W,4]
    hold the band's rows (in/out)."""
    for a, dt in ((accum, np.float32), (normal, np.float32), (depth, np.float32), (mix, np.float32), (out, np.uint8)):
        assert a.dtype == dt and a.flags.c_contiguous
    n_rows = accum.reshape(-1, 4).shape[0] // width
    he = 16 * (height // 16)
    assert 0 <= y0 < y1 <= he and row0 <= max(0, y0 - 3) and row0 + n_rows >= min(he, y1 + 3)
    assert mix.size >= (y1 - y0) * width * 3 and out.size >= (y1 - y0) * width * 4
    lib().or_denoise_mix_band(_ptr(accum), _ptr(normal), _ptr(depth), _ptr(mix), _ptr(out), width, height, row0, y0,
                              y1, cur_sample_idx)
