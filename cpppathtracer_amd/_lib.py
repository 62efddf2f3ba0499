"""ctypes binding of libcpt.so (include/cpt.h).

The product path has exactly one implementation: the HIP kernels in libcpt.so.  If the
library is missing or fails to load, every entry point raises — there is no CPU fallback.
"""
import ctypes
import os

from . import build as _build

_lib = None

# Every symbol include/cpt.h declares, with its ctypes prototype.
_P = ctypes.c_void_p
_I = ctypes.c_int
_U32 = ctypes.c_uint32
_U64 = ctypes.c_uint64
_SZ = ctypes.c_size_t
PROTOTYPES = {
    "cpt_abi_version": (_I, []),
    "cpt_status_string": (ctypes.c_char_p, [_I]),
    "cpt_get_device_count": (_I, [_P]),
    "cpt_create": (_I, [_I, _P]),
    "cpt_destroy": (_I, [_P]),
    "cpt_last_error": (ctypes.c_char_p, [_P]),
    "cpt_set_stream": (_I, [_P, _P]),
    "cpt_camera_get_copy": (_I, [_P]),
    "cpt_set_scene": (_I, [_P, _P, _I]),
    "cpt_update_object": (_I, [_P, _I, _P]),
    "cpt_update_objects": (_I, [_P, _I, _P, _P]),
    "cpt_update_objects_rebuild": (_I, [_P, _I, _P, _P]),
    "cpt_last_update_ms": (_I, [_P, _P]),
    "cpt_get_material_count": (_I, [_P, _P]),
    "cpt_scene_bvh_export": (_I, [_P, _P, _P, _I, _P]),
    "cpt_bvh_build_host": (_I, [_P, _I, _P, _P, _I, _P]),
    "cpt_set_env_texture": (_I, [_P, _P, _I, _I, _I]),
    "cpt_bind_texture": (_I, [_P, _U64, _P, _I, _I, _I, _I, _I]),
    "cpt_set_frame": (_I, [_P, _I, _I, _P, _I]),
    "cpt_init_rng": (_I, [_P, _U64]),
    "cpt_read_rng": (_I, [_P, _P]),
    "cpt_write_rng": (_I, [_P, _P]),
    "cpt_render": (_I, [_P, _P, _I, _I, _U32]),
    "cpt_synchronize": (_I, [_P]),
    "cpt_read_accum": (_I, [_P, _P]),
    "cpt_clear_accum": (_I, [_P]),
    "cpt_read_aux": (_I, [_P, _P, _P]),
    "cpt_write_accum": (_I, [_P, _P]),
    "cpt_write_aux": (_I, [_P, _P, _P]),
    "cpt_copy_accum_device": (_I, [_P, _P, _SZ, _P]),
    "cpt_gather_rows": (_I, [_P, _P]),
    "cpt_last_gather_mode": (_I, [_P, _P, _P]),
    "cpt_set_debug_gather": (_I, [_P, _I]),
    "cpt_get_stats": (_I, [_P, _P]),
    "cpt_reset_stats": (_I, [_P]),
    "cpt_get_raw_counters": (_I, [_P, _P]),
    "cpt_get_walk_info": (_I, [_P, _P]),
    "cpt_measure_read_bandwidth": (_I, [_P, _SZ, _I, _P]),
    "cpt_measure_read_pattern": (_I, [_P, _I, _SZ, _I, _P]),
    "cpt_cap_disk_bound": (_I, [ctypes.c_float, _P]),
    "cpt_last_render_ms": (_I, [_P, _P]),
    "cpt_get_diag_counters": (_I, [_P, _P]),
    "cpt_get_execdiag_counters": (_I, [_P, _P]),
    "cpt_last_kernel_stats": (_I, [_P, _P, _P]),
    "cpt_denoise_mix": (_I, [_P, _U32, _P]),
    "cpt_host_register": (_I, [_P, _SZ]),
    "cpt_host_unregister": (_I, [_P]),
    "cpt_denoise_mix_band": (_I, [_P, _U32, _I, _I, _P]),
    "cpt_copy_bgra_device": (_I, [_P, _P, _SZ, _P]),
    "cpt_last_display_ms": (_I, [_P, _P]),
    "cpt_reset_display": (_I, [_P]),
    "cpt_display_band": (_I, [_P, _P, _P]),
    "cpt_debug_timeline": (_I, [_P, _P, _I]),
    "cpt_tile_costs": (_I, [_P, _P, _I, _I, ctypes.c_uint32, _P, _SZ]),
    "cpt_read_mix": (_I, [_P, _P, _SZ]),
    "cpt_math_batch": (_I, [_P, _I, _P, _P, _P, _SZ]),
    "cpt_selftest_qdiv": (_I, [_P, _I, _U64, _U64, _P, _I]),
    "cpt_set_debug_consolidation": (_I, [_P, _U32, _I, _I]),
}

CPT_RENDER_ACCUMULATE = 0x1
CPT_RENDER_AUX = 0x2
CPT_RENDER_STATS = 0x4
CPT_RENDER_SYNC = 0x8
CPT_PATH_MEGAKERNEL = 0x000
CPT_PATH_WAVEFRONT = 0x100
CPT_TRAVERSAL_ORDERED = 0x200
CPT_TRAVERSAL_PLAIN_LEAVES = 0x400
CPT_SCHEDULE_COST = 0x800
CPT_SCHEDULE_CONSOLIDATE = 0x1000
CPT_SCHEDULE_NO_CONSOLIDATE = 0x2000
CPT_SCHEDULE_PREVIOUS = 0x4000
CPT_ERR_STATE = 5
CPT_ERR_DEVICE = 7   # a kernel abandoned work (reported at the next synchronising call)


class CptError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"[cpt status {status}] {msg}")
        self.status = status


def lib_path() -> str:
    return _build.LIB_PATH


def load(build_if_missing: bool = True):
    """Load libcpt.so; build it first (hipcc) when absent and allowed."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("CPT_LIB_PATH") or _build.LIB_PATH   # CPT_LIB_PATH: A/B builds only
    if not os.path.exists(path):
        if not build_if_missing:
            raise CptError(-1, f"{path} missing: run __graft_entry__.build() (hipcc) first")
        _build.build()
    L = ctypes.CDLL(path)
    ab_variant = "CPT_LIB_PATH" in os.environ
    for name, (res, args) in PROTOTYPES.items():
        if ab_variant and not hasattr(L, name):
            continue   # an older A/B build may predate an entry point; the shipped library has all
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.cpt_abi_version() != 1:
        raise CptError(-1, f"libcpt ABI {L.cpt_abi_version()} != 1")
    _lib = L
    return L


def check(status, ctx=None):
    if status != 0:
        L = load()
        msg = L.cpt_last_error(ctx)
        raise CptError(status, (msg or b"").decode() or L.cpt_status_string(status).decode())
    return status
