"""ctypes binding of libcbev.so (the HIP C-ABI declared in include/cbev.h).

The library is built in-tree (`__graft_entry__.build()` or `python -m
carlabev_env_amd.build`). There is no CPU fallback: if the library is missing
or cannot be loaded, `lib()` raises.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# CBEV_LIB overrides the path (performance-experiment builds only)
LIB_PATH = os.environ.get("CBEV_LIB") or os.path.join(HERE, "libcbev.so")

_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64

_lib = None


class CbevError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CbevError(f"{LIB_PATH} not built; run `python -m carlabev_env_amd.build` (hipcc, gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    L.cbev_abi_version.restype = _I
    L.cbev_params_size.restype = _I
    L.cbev_layout_of.argtypes = [_P, _P]
    L.cbev_layout_of.restype = _I
    L.cbev_field_names.argtypes = [_I]
    L.cbev_field_names.restype = ctypes.c_char_p
    L.cbev_last_error.restype = ctypes.c_char_p
    L.cbev_create.argtypes = [_P, _P, _I, ctypes.POINTER(_P)]
    L.cbev_create.restype = _I
    L.cbev_destroy.argtypes = [_P]
    L.cbev_destroy.restype = None
    L.cbev_set_map.argtypes = [_P, _P, _I64]
    L.cbev_set_map.restype = _I
    L.cbev_step.argtypes = [_P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P]
    L.cbev_step.restype = _I
    L.cbev_reset.argtypes = [_P, _P, _I, _P, _I, _P, _P, _I, _P, _I, _P]
    L.cbev_reset.restype = _I
    L.cbev_bank_frames.argtypes = [_P, _P, _I, _P, _P]
    L.cbev_bank_frames.restype = _I
    L.cbev_reset_frames.argtypes = [_P, _P, _I, _P, _I, _P, _P, _I, _P, _P, _I, _P]
    L.cbev_reset_frames.restype = _I
    L.cbev_reset_masked.argtypes = [_P, _P, _I, _P, _P, _I, _P, _P, _I, _P]
    L.cbev_reset_masked.restype = _I
    L.cbev_reset_terminated.argtypes = [_P, _P, _I, _P, _I, _P, _P, _I, _P]
    L.cbev_reset_terminated.restype = _I
    L.cbev_bank_cursor.argtypes = [_P, _P]
    L.cbev_bank_cursor.restype = _I
    L.cbev_reset_counts.argtypes = [_P, _P, _I]
    L.cbev_reset_counts.restype = _I
    L.cbev_bank_stride.argtypes = [_I]
    L.cbev_bank_stride.restype = _I
    L.cbev_set_deferred_reset.argtypes = [_P, _I]
    L.cbev_set_deferred_reset.restype = _I
    L.cbev_reset_pending.argtypes = [_P]
    L.cbev_reset_pending.restype = _I
    L.cbev_flush.argtypes = [_P]
    L.cbev_flush.restype = _I
    L.cbev_expand_obs.argtypes = [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P]
    L.cbev_expand_obs.restype = _I
    L.cbev_pack_frames.argtypes = [_P, _P, _I, _P, _P]
    L.cbev_pack_frames.restype = _I
    L.cbev_unpack_frames.argtypes = [_P, _P, _I, _P, _P]
    L.cbev_unpack_frames.restype = _I
    L.cbev_vector_obs.argtypes = [_P, _P, _I, _P, _P]
    L.cbev_vector_obs.restype = _I
    L.cbev_set_fov_mask.argtypes = [_P, _P]
    L.cbev_set_fov_mask.restype = _I
    L.cbev_set_obs_size.argtypes = [_P, _I, _I]
    L.cbev_set_obs_size.restype = _I
    L.cbev_resize_obs.argtypes = [_P, _P, _I, _P, _I, _P, _I, _I64, _P]
    L.cbev_resize_obs.restype = _I
    L.cbev_set_episode_stats.argtypes = [_P, _P, _I, _P, _P, _I]
    L.cbev_set_episode_stats.restype = _I
    L.cbev_episode_slot.argtypes = [_P, _P]
    L.cbev_episode_slot.restype = _I
    L.cbev_wall_clock_hz.argtypes = [_P, _P]
    L.cbev_wall_clock_hz.restype = _I
    L.cbev_termination_count.argtypes = [_P, _P]
    L.cbev_termination_count.restype = _I
    L.cbev_error_flags.argtypes = [_P, _P, _I]
    L.cbev_error_flags.restype = _I
    L.cbev_profile.argtypes = [_P, _I]
    L.cbev_profile.restype = _I
    L.cbev_profile_read.argtypes = [_P, _P, _P]
    L.cbev_profile_read.restype = _I
    L.cbev_profile_raster.argtypes = [_P, _P, _I, _P, _I, _P, _P]
    L.cbev_profile_raster.restype = _I
    _lib = L
    return L


def check(rc: int, what: str = "cbev call"):
    if rc != 0:
        msg = lib().cbev_last_error().decode("utf-8", "replace")
        raise CbevError(f"{what} failed ({rc}): {msg}")


EXPORTED_SYMBOLS = ("cbev_abi_version", "cbev_params_size", "cbev_layout_of", "cbev_field_names", "cbev_last_error",
                    "cbev_create", "cbev_destroy", "cbev_set_map", "cbev_step", "cbev_reset", "cbev_bank_frames",
                    "cbev_reset_frames", "cbev_reset_masked", "cbev_reset_terminated", "cbev_bank_cursor",
                    "cbev_reset_counts", "cbev_bank_stride",
                    "cbev_set_deferred_reset", "cbev_reset_pending", "cbev_flush",
                    "cbev_expand_obs", "cbev_vector_obs", "cbev_set_fov_mask", "cbev_set_obs_size", "cbev_resize_obs", "cbev_profile", "cbev_profile_read",
                    "cbev_profile_raster", "cbev_error_flags", "cbev_set_episode_stats", "cbev_episode_slot",
                    "cbev_wall_clock_hz", "cbev_termination_count", "cbev_pack_frames", "cbev_unpack_frames")

ERR_ACTION_INDEX = 1  # CBEV_ERR_ACTION_INDEX (include/cbev.h)
ERR_RASTER_WINDOW = 2  # CBEV_ERR_RASTER_WINDOW (include/cbev.h)
ERR_RETREAT_ROUTE = 4  # CBEV_ERR_RETREAT_ROUTE (include/cbev.h)
