"""Host-side driver over the C-ABI: one ``Renderer`` = one ``cpt_ctx`` on one GPU.

This is the Python view of the reference's PathTracer pipeline (path_tracer.cu:44-115,
256-319) for tests, the benchmark and multi-GPU tiling; C++ users get the same through
include/cpppathtracer/path_tracer.h.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import (CPT_PATH_WAVEFRONT, CPT_RENDER_ACCUMULATE, CPT_RENDER_AUX, CPT_RENDER_STATS, CPT_RENDER_SYNC,
                   CPT_SCHEDULE_CONSOLIDATE, CPT_SCHEDULE_COST, CPT_SCHEDULE_NO_CONSOLIDATE, CPT_SCHEDULE_PREVIOUS,
                   CPT_TRAVERSAL_ORDERED,
                   CPT_TRAVERSAL_PLAIN_LEAVES, CptError, check)

PATHS = ("megakernel", "wavefront")
from .types import CAMERA_DTYPE, OBJECT_DTYPE


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def device_count() -> int:
    L = _lib.load()
    n = ctypes.c_int(0)
    check(L.cpt_get_device_count(ctypes.byref(n)))
    return n.value


def camera_get_copy(cam):
    """MotionalCamera::GetCopy on a CAMERA_DTYPE value (returns the updated copy)."""
    L = _lib.load()
    c = np.array(cam, dtype=CAMERA_DTYPE, copy=True)
    check(L.cpt_camera_get_copy(_p(c)))
    return c


class Renderer:
    def __init__(self, device: int = 0):
        self._L = _lib.load()
        h = ctypes.c_void_p()
        st = self._L.cpt_create(device, ctypes.byref(h))
        if st != 0:
            raise CptError(st, (self._L.cpt_last_error(None) or b"").decode())
        self._ctx = h
        self.device = device
        self.width = self.height = self.n_rows = 0
        self.rows = None

    # -- lifecycle -------------------------------------------------------------------
    def close(self):
        if getattr(self, "_ctx", None):
            self._L.cpt_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, st):
        return check(st, self._ctx)

    # -- setup -----------------------------------------------------------------------
    def set_stream(self, hip_stream_handle):
        self._check(self._L.cpt_set_stream(self._ctx, ctypes.c_void_p(hip_stream_handle or 0)))

    def set_scene(self, objs):
        objs = np.ascontiguousarray(objs, dtype=OBJECT_DTYPE)
        self._check(self._L.cpt_set_scene(self._ctx, _p(objs) if len(objs) else None, len(objs)))

    def update_object(self, index, obj):
        o = np.array(obj, dtype=OBJECT_DTYPE, copy=True)
        self._check(self._L.cpt_update_object(self._ctx, index, _p(o)))

    def update_objects(self, indices, objs, rebuild=False):
        """SceneBVH::UpdateObject for a batch: refit on the device (cpt_update_objects), or with
        the ordered walk's tree rebuilt on the host (rebuild=True, cpt_update_objects_rebuild)."""
        idx = np.ascontiguousarray(indices, dtype=np.int32)
        o = np.ascontiguousarray(objs, dtype=OBJECT_DTYPE)
        if o.shape != idx.shape:
            raise ValueError(f"update_objects: {o.shape[0] if o.ndim else 1} objects for {idx.size} indices")
        fn = self._L.cpt_update_objects_rebuild if rebuild else self._L.cpt_update_objects
        self._check(fn(self._ctx, int(idx.size), _p(idx), _p(o)))

    def material_count(self) -> int:
        """Material slots the scene holds (cpt_get_material_count)."""
        n = ctypes.c_int(0)
        self._check(self._L.cpt_get_material_count(self._ctx, ctypes.byref(n)))
        return n.value

    def last_update_ms(self) -> float:
        ms = ctypes.c_float(0)
        self._check(self._L.cpt_last_update_ms(self._ctx, ctypes.byref(ms)))
        return float(ms.value)

    def bvh_export(self):
        n = ctypes.c_int(0)
        self._check(self._L.cpt_scene_bvh_export(self._ctx, None, None, 0, ctypes.byref(n)))
        m = n.value
        boxes = np.zeros((max(m, 1), 6), dtype=np.float32)
        links = np.zeros((max(m, 1), 4), dtype=np.int32)
        self._check(self._L.cpt_scene_bvh_export(self._ctx, _p(boxes), _p(links), m, ctypes.byref(n)))
        return boxes[:m], links[:m]

    def set_env(self, env):
        """env: texture_io.EnvTexture (or None for a black environment)."""
        if env is None:
            self._check(self._L.cpt_set_env_texture(self._ctx, None, 1, 1, 0))
            return
        rgba = np.ascontiguousarray(env.rgba, dtype=np.uint8)
        self._check(self._L.cpt_set_env_texture(self._ctx, _p(rgba), env.width, env.height, env.valid_cols))

    def bind_texture(self, handle, tex, address_mode=2, filter_mode=1):
        """Bind texels (texture_io.EnvTexture) to a material texture handle (cpt_bind_texture);
        defaults = AddTexByFile's mirror + linear."""
        rgba = np.ascontiguousarray(tex.rgba, dtype=np.uint8)
        self._check(self._L.cpt_bind_texture(self._ctx, handle, _p(rgba), tex.width, tex.height, tex.valid_cols,
                                             address_mode, filter_mode))

    def set_frame(self, width, height, rows=None):
        if rows is None:
            self._check(self._L.cpt_set_frame(self._ctx, width, height, None, 0))
            self.rows = np.arange(height, dtype=np.int32)
        else:
            r = np.ascontiguousarray(rows, dtype=np.int32)
            self._check(self._L.cpt_set_frame(self._ctx, width, height, _p(r), r.size))
            self.rows = r
        self.width, self.height, self.n_rows = width, height, int(self.rows.size)

    def init_rng(self, seed):
        self._check(self._L.cpt_init_rng(self._ctx, ctypes.c_uint64(seed)))

    # -- render ----------------------------------------------------------------------
    def render(self, cam, spp, max_depth, accumulate=False, aux=False, stats=False, sync=False, flags=0,
               path="megakernel", ordered=False, schedule="tiles", consolidate=None):
        """path: "megakernel" (per-lane regeneration, state in VGPRs) or "wavefront" (SoA state in
        HBM, extend/shade kernels with ballot compaction).  Both give identical results.
        ordered: near-first BVH walk per direction octant (CPT_TRAVERSAL_ORDERED); same closest
        hits as the reference order up to box/primitive rounding (DESIGN.md §Ordered walk).
        ordered="plain": the same walk testing each leaf where it meets it (per-ray node/prim
        counts, CPT_TRAVERSAL_PLAIN_LEAVES) instead of parking leaves for wave-wide rounds.
        schedule: "tiles" (8x8 tiles dequeued in row-major order) or "cost" (CPT_SCHEDULE_COST: a
        short pilot render measures each tile's work and the megakernel dequeues the tiles
        heaviest first; same results, DESIGN.md §Cost schedule) or "previous"
        (CPT_SCHEDULE_PREVIOUS: heaviest first by the previous such render's per-tile RNG draws,
        no pilot; for repeated renders of few passes, the DispatchRay loop).
        consolidate: None (the library's default: on for frames of more than 1 and at most 4
        pixels per lane and spp >= 512), True or
        False (CPT_SCHEDULE_[NO_]CONSOLIDATE): the megakernel's tail consolidation, same results."""
        if path not in PATHS:
            raise ValueError(f"path must be one of {PATHS}")
        if schedule not in ("tiles", "cost", "previous"):
            raise ValueError("schedule must be 'tiles', 'cost' or 'previous'")
        c = np.ascontiguousarray(np.array(cam, dtype=CAMERA_DTYPE))
        f = flags | (CPT_PATH_WAVEFRONT if path == "wavefront" else 0)
        f |= CPT_TRAVERSAL_ORDERED if ordered else 0
        f |= CPT_TRAVERSAL_PLAIN_LEAVES if ordered == "plain" else 0
        f |= CPT_RENDER_ACCUMULATE if accumulate else 0
        f |= CPT_RENDER_AUX if aux else 0
        f |= CPT_RENDER_STATS if stats else 0
        f |= CPT_RENDER_SYNC if sync else 0
        f |= CPT_SCHEDULE_COST if schedule == "cost" else 0
        f |= CPT_SCHEDULE_PREVIOUS if schedule == "previous" else 0
        if consolidate is not None:
            f |= CPT_SCHEDULE_CONSOLIDATE if consolidate else CPT_SCHEDULE_NO_CONSOLIDATE
        self._check(self._L.cpt_render(self._ctx, _p(c), spp, max_depth, f))

    def tile_costs(self, cam, passes, max_depth, ordered=True):
        """The cost schedule's pilot alone (cpt_tile_costs): each 8x8 tile's work over `passes`
        passes from the current RNG states (nothing written back), [tiles_y, tiles_x] uint32."""
        c = np.ascontiguousarray(np.array(cam, dtype=CAMERA_DTYPE))
        ty, tx = (self.n_rows + 7) // 8, (self.width + 7) // 8
        out = np.zeros((ty, tx), dtype=np.uint32)
        f = CPT_TRAVERSAL_ORDERED if ordered else 0
        f |= CPT_TRAVERSAL_PLAIN_LEAVES if ordered == "plain" else 0
        self._check(self._L.cpt_tile_costs(self._ctx, _p(c), int(passes), int(max_depth), f, _p(out), out.size))
        return out

    def synchronize(self):
        self._check(self._L.cpt_synchronize(self._ctx))

    def last_render_ms(self) -> float:
        ms = ctypes.c_float(0)
        self._check(self._L.cpt_last_render_ms(self._ctx, ctypes.byref(ms)))
        return float(ms.value)

    def last_kernel_stats(self):
        """(average ms per launch, launches) of the last render's dominant kernel, without the
        cost schedule's pilot (HIP events on the launch stream; waits for the render)."""
        ms, n = ctypes.c_float(0), ctypes.c_int(0)
        self._check(self._L.cpt_last_kernel_stats(self._ctx, ctypes.byref(ms), ctypes.byref(n)))
        return float(ms.value), int(n.value)

    # -- readback --------------------------------------------------------------------
    @property
    def npix(self):
        return self.n_rows * self.width

    def read_accum(self):
        out = np.zeros((self.npix, 4), dtype=np.float32)
        self._check(self._L.cpt_read_accum(self._ctx, _p(out)))
        return out

    def clear_accum(self):
        self._check(self._L.cpt_clear_accum(self._ctx))

    def read_rng(self):
        out = np.zeros((6, self.npix), dtype=np.uint32)
        self._check(self._L.cpt_read_rng(self._ctx, _p(out)))
        return out

    def write_rng(self, planar6):
        a = np.ascontiguousarray(planar6, dtype=np.uint32)
        if a.shape != (6, self.npix):
            raise ValueError(f"write_rng: expected shape (6, {self.npix}), got {a.shape}")
        self._check(self._L.cpt_write_rng(self._ctx, _p(a)))

    def read_aux(self):
        n = np.zeros((self.npix, 3), dtype=np.float32)
        d = np.zeros(self.npix, dtype=np.float32)
        self._check(self._L.cpt_read_aux(self._ctx, _p(n), _p(d)))
        return n, d

    def write_accum(self, rgba):
        """Restore the accumulator ([npix, 4] float32) from a host copy (checkpoint / resume)."""
        a = np.ascontiguousarray(rgba, dtype=np.float32).reshape(self.npix, 4)
        self._check(self._L.cpt_write_accum(self._ctx, _p(a)))

    def write_aux(self, normal3, depth):
        """Restore the first-hit normal ([npix, 3]) and depth ([npix]) buffers from host copies."""
        n = np.ascontiguousarray(normal3, dtype=np.float32).reshape(self.npix, 3)
        d = np.ascontiguousarray(depth, dtype=np.float32).reshape(self.npix)
        self._check(self._L.cpt_write_aux(self._ctx, _p(n), _p(d)))

    def copy_accum_device(self, device_ptr, nbytes, stream):
        """Device copy of the accumulator, ordered against the caller's HIP stream (a handle,
        e.g. torch.cuda.current_stream().cuda_stream; 0 = the null stream) with no host wait:
        it starts after the work queued there so far and that stream's next work sees it."""
        self._check(self._L.cpt_copy_accum_device(self._ctx, ctypes.c_void_p(device_ptr), nbytes,
                                                  ctypes.c_void_p(stream or None)))

    def gather_rows(self, src):
        """cpt_gather_rows: place the rows Renderer `src` rendered into this frame (row tiling)."""
        self._check(self._L.cpt_gather_rows(self._ctx, src._ctx))

    GATHER_MODES = {-1: None, 0: "same_device", 1: "peer", 2: "staged"}

    def last_gather_mode(self, src):
        """How the last gather_rows(src) reached src's buffers: "same_device", "peer" (xGMI
        reads with peer access), "staged" (a peer copy first), or None (no gather yet)."""
        m = ctypes.c_int(-1)
        self._check(self._L.cpt_last_gather_mode(self._ctx, src._ctx, ctypes.byref(m)))
        return self.GATHER_MODES[m.value]

    def set_debug_gather(self, force_staged):
        """Test hook: route this context's gathers through the staged peer copy."""
        self._check(self._L.cpt_set_debug_gather(self._ctx, int(bool(force_staged))))

    def stats(self):
        s = (ctypes.c_uint64 * 5)()
        self._check(self._L.cpt_get_stats(self._ctx, s))
        return dict(zip(("segments", "nodes", "prims", "hits", "misses"), (int(x) for x in s)))

    def raw_counters(self):
        out = np.zeros(8, dtype=np.uint64)
        self._check(self._L.cpt_get_raw_counters(self._ctx, _p(out)))
        return [int(x) for x in out]

    def debug_timeline(self):
        """DIAGNOSTIC: the lane-occupancy timeline of a CPT_TIMELINE build (cpt_debug_timeline):
        ([4096, 4] uint64 bins, first tick the queue ran dry); clears it."""
        out = np.zeros(4 * 4096 + 4, dtype=np.uint64)
        self._check(self._L.cpt_debug_timeline(self._ctx, _p(out), out.size))
        return out[: 4 * 4096].reshape(4096, 4), int(out[4 * 4096])

    def diag_counters(self):
        """DIAGNOSTIC: the 16 stamp slots of a CPT_STAMPS build (cpt_stamps.hpp)."""
        out = np.zeros(16, dtype=np.uint64)
        self._check(self._L.cpt_get_diag_counters(self._ctx, _p(out)))
        return [int(x) for x in out]

    def execdiag_counters(self):
        """DIAGNOSTIC: the exec-mask census of a CPT_EXECDIAG build (cpt_stamps.hpp execdiag)."""
        out = np.zeros(64, dtype=np.uint64)
        self._check(self._L.cpt_get_execdiag_counters(self._ctx, _p(out)))
        return out.reshape(4, 16)

    def walk_info(self):
        """[reference-order nodes, binary octant-order nodes, 4-wide nodes per octant, platforms]."""
        out = np.zeros(4, dtype=np.int32)
        self._check(self._L.cpt_get_walk_info(self._ctx, _p(out)))
        return dict(zip(("n_bvh", "n_walk", "n_wide", "n_unb"), (int(x) for x in out)))

    def measure_read_pattern(self, bytes_per_lane, nbytes=1 << 30, iters=1):
        """DIAGNOSTIC: GB/s of a streaming read in one of the display kernel's access shapes
        (cpt_measure_read_pattern: 4, 12 or 16 bytes per lane)."""
        out = ctypes.c_float(0.0)
        self._check(self._L.cpt_measure_read_pattern(self._ctx, int(bytes_per_lane), int(nbytes), int(iters),
                                                     ctypes.byref(out)))
        return out.value

    def measure_read_bandwidth(self, nbytes=4 << 30, iters=10):
        """HBM streaming-read ceiling in GB/s (cpt_measure_read_bandwidth)."""
        out = ctypes.c_float(0.0)
        self._check(self._L.cpt_measure_read_bandwidth(self._ctx, int(nbytes), int(iters), ctypes.byref(out)))
        return float(out.value)

    def set_debug_consolidation(self, flags=0, keeper_spin_log2=0, publish_wait_log2=0):
        """TEST HOOK (cpt_set_debug_consolidation): provoke the tail consolidation's error paths."""
        self._check(self._L.cpt_set_debug_consolidation(self._ctx, flags, keeper_spin_log2, publish_wait_log2))

    def reset_stats(self):
        self._check(self._L.cpt_reset_stats(self._ctx))

    def selftest_qdiv(self, which, n, seed=1, examples=16):
        """Returns (mismatch count, [(a, d) float32 pairs of some mismatches])."""
        out = np.zeros(examples + 1, dtype=np.uint64)
        self._check(self._L.cpt_selftest_qdiv(self._ctx, which, n, seed, _p(out), out.size))
        cnt = int(out[0])
        pairs = [(np.uint32(int(v) >> 32).view(np.float32), np.uint32(int(v) & 0xFFFFFFFF).view(np.float32))
                 for v in out[1:1 + min(cnt, examples)]]
        return cnt, pairs

    def denoise_mix(self, cur_sample_idx, out=None, host=True):
        """Denoising + Mix display pass; returns the BGRA8 frame (height, width, 4), into `out`
        when given (a preallocated, e.g. pinned, host array of that shape).  host=False keeps the
        frame on the device (no host write; returns None): the display kernel's device-only time."""
        if not host:
            self._check(self._L.cpt_denoise_mix(self._ctx, cur_sample_idx, None))
            return None
        if out is None:
            out = np.zeros((self.height, self.width, 4), dtype=np.uint8)
        # explicit checks, not asserts: the C-ABI writes a full H*W*4 frame into `out` (a kernel
        # store through a pinned alias or a hipMemcpyAsync), so a bad buffer must raise, also
        # under `python -O`
        if not isinstance(out, np.ndarray) or out.dtype != np.uint8:
            raise ValueError("denoise_mix: `out` must be a numpy uint8 array")
        if out.size != self.height * self.width * 4:
            raise ValueError(f"denoise_mix: `out` holds {out.size} bytes, the frame needs "
                             f"{self.height * self.width * 4}")
        if not out.flags["C_CONTIGUOUS"] or not out.flags["WRITEABLE"]:
            raise ValueError("denoise_mix: `out` must be C-contiguous and writeable")
        self._check(self._L.cpt_denoise_mix(self._ctx, cur_sample_idx, _p(out)))
        return out

    def display_band(self):
        """The output rows (y0, y1) the display buffers hold (cpt_display_band)."""
        y0, y1 = ctypes.c_int(0), ctypes.c_int(0)
        self._check(self._L.cpt_display_band(self._ctx, ctypes.byref(y0), ctypes.byref(y1)))
        return y0.value, y1.value

    def read_mix(self):
        """The Mix running mean of the display band: [(y1 - y0) * width, 3] float32, sized from
        the library's own band (a failed band switch cannot leave it stale)."""
        y0, y1 = self.display_band()
        out = np.zeros(((y1 - y0) * self.width, 3), dtype=np.float32)
        self._check(self._L.cpt_read_mix(self._ctx, _p(out), out.size))
        return out

    def last_display_ms(self) -> float:
        """Device time of the last display kernel (Denoising + Mix), HIP events."""
        ms = ctypes.c_float()
        self._check(self._L.cpt_last_display_ms(self._ctx, ctypes.byref(ms)))
        return ms.value

    def denoise_mix_band(self, cur_sample_idx, y0, y1, host=True):
        """Display path for output rows [y0, y1) (cpt_denoise_mix_band): the frame's rows must be
        one ascending run covering the band and its 3-row halo.  Returns the band's BGRA8 rows
        (y1 - y0, width, 4), or None with host=False (then copy_bgra_device moves them)."""
        out = np.zeros((y1 - y0, self.width, 4), dtype=np.uint8) if host else None
        self._check(self._L.cpt_denoise_mix_band(self._ctx, cur_sample_idx, int(y0), int(y1),
                                                 _p(out) if host else None))
        return out

    def copy_bgra_device(self, device_ptr, nbytes, stream):
        """Device copy of the display band's BGRA8 rows, ordered against `stream` as
        copy_accum_device."""
        self._check(self._L.cpt_copy_bgra_device(self._ctx, ctypes.c_void_p(device_ptr), nbytes,
                                                 ctypes.c_void_p(stream or None)))

    def reset_display(self):
        self._check(self._L.cpt_reset_display(self._ctx))

    def math_batch(self, op, a, b=None):
        a = np.ascontiguousarray(a, dtype=np.float32)
        b = np.ascontiguousarray(b if b is not None else np.zeros_like(a), dtype=np.float32)
        out = np.empty_like(a)
        self._check(self._L.cpt_math_batch(self._ctx, op, _p(a), _p(b), _p(out), a.size))
        return out
