"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY — importable by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg. The product package never imports this module.
Build with `make -C oracle` (also done by __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_D = ctypes.c_double
_I = ctypes.c_int32
_P = ctypes.c_void_p


class OrcInfo(ctypes.Structure):
    _fields_ = [("state", _D * 4), ("last_state", _D * 4), ("dist2wp", _D), ("set_point", _D * 3),
                ("n_wps", _I), ("wps_x", _D * 5), ("wps_y", _D * 5), ("comfort", _D * 6),
                ("dist2goal", _D), ("dist2goal_t1", _D), ("speed_limit", _D),
                ("tile_class", _I), ("collided", _I), ("actor_id", _I), ("n_actors", _I),
                ("actors", (_D * 4) * 64)]


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(
            os.path.join(HERE, "cbev_oracle.c")):
        subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_angle_mod.restype = _D
        L.orc_angle_mod.argtypes = [_D]
        L.orc_state_update.argtypes = [_P, _D, _D, _D]
        L.orc_calc_target_index.restype = _I
        L.orc_calc_target_index.argtypes = [_D, _D, _D, _P, _P, _I, _P]
        L.orc_stanley_control.restype = _D
        L.orc_stanley_control.argtypes = [_D, _D, _D, _D, _P, _P, _P, _I, _I, _P]
        L.orc_comfort.argtypes = [_D, _D, _D, _D, _I, _D, _D, _D, _P]
        L.orc_comfort_violations.restype = _I
        L.orc_comfort_violations.argtypes = [_D] * 6
        L.orc_hero_physics_vec.argtypes = [_P, _P, _P, _P, _P, ctypes.c_float, ctypes.c_float, ctypes.c_float, _I, _P]
        L.orc_smooth_and_compute.restype = _I
        L.orc_smooth_and_compute.argtypes = [_P, _P, _I, _I, _I, _P, _P, _P]
        L.orc_route_progress.restype = _D
        L.orc_route_progress.argtypes = [_D, _D, _P, _P, _P, _I]
        L.orc_cumulative_lengths.argtypes = [_P, _P, _I, _P]
        L.orc_lateral_error.restype = _D
        L.orc_lateral_error.argtypes = [_D, _D, _P, _P, _I]
        L.orc_carl_step_vec.restype = _D
        L.orc_carl_step_vec.argtypes = [_P, _P, _P, _P, _P, _P, _P, _I, _P, _P]
        L.orc_shaping_step_vec.restype = _D
        L.orc_shaping_step_vec.argtypes = [_P, _P, _P, _P, _P, _P]
        L.orc_info_size.restype = _I
        L.orc_step.restype = _I
        L.orc_step.argtypes = [_P, _P, _P, _P, _P, _P, _P]
        L.orc_reset_obs.argtypes = [_P, _P, _P, _P, _P, _P]
        L.orc_step_batch.restype = _I
        L.orc_step_batch.argtypes = [_P, _P, _P, _P, ctypes.c_int64, _I, _P, _I, _P, _P]
        L.orc_actor_step_rec.argtypes = [_P, _P, _I, _D, _D]
        L.orc_crop_origin.argtypes = [_P, _D, _D, _P]
        if L.orc_info_size() != ctypes.sizeof(OrcInfo):
            raise RuntimeError("OrcInfo layout mismatch")
        _lib = L
    return _lib


def ptr(a: np.ndarray):
    return a.ctypes.data_as(_P)


def f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


# ------------------------------------------------------------------ helpers
def angle_mod(x: float) -> float:
    return lib().orc_angle_mod(float(x))


def state_update(st: np.ndarray, acc: float, delta: float, target_speed: float) -> None:
    assert st.dtype == np.float64 and st.size == 8
    lib().orc_state_update(ptr(st), float(acc), float(delta), float(target_speed))


def calc_target_index(x, y, yaw, cx, cy):
    cx, cy = f64(cx), f64(cy)
    err = np.zeros(1)
    idx = lib().orc_calc_target_index(float(x), float(y), float(yaw), ptr(cx), ptr(cy), len(cx), ptr(err))
    return idx, float(err[0])


def stanley_control(x, y, yaw, v, cx, cy, cyaw, target_idx):
    cx, cy, cyaw = f64(cx), f64(cy), f64(cyaw)
    idx = np.zeros(1, np.int32)
    d = lib().orc_stanley_control(float(x), float(y), float(yaw), float(v), ptr(cx), ptr(cy), ptr(cyaw), len(cx),
                                  int(target_idx), ptr(idx))
    return d, int(idx[0])


def comfort(speed, prev_speed, yaw, prev_yaw, has_prev, pal, palat, pyr):
    out = np.zeros(7)
    lib().orc_comfort(speed, prev_speed, yaw, prev_yaw, int(has_prev), pal, palat, pyr, ptr(out))
    return out


def smooth_and_compute(ax, ay, window=11, poly=3):
    ax, ay = f64(ax), f64(ay)
    n = max(len(ax), 2)
    cx, cy, cyaw = np.zeros(n), np.zeros(n), np.zeros(n)
    m = lib().orc_smooth_and_compute(ptr(ax), ptr(ay), len(ax), window, poly, ptr(cx), ptr(cy), ptr(cyaw))
    return cx[:m], cy[:m], cyaw[:m]


def cumulative_lengths(rx, ry):
    rx, ry = i32(rx), i32(ry)
    out = np.zeros(max(len(rx), 1))
    lib().orc_cumulative_lengths(ptr(rx), ptr(ry), len(rx), ptr(out))
    return out[:len(rx)]


def route_progress(px, py, rx, ry, cum):
    rx, ry, cum = i32(rx), i32(ry), f64(cum)
    return lib().orc_route_progress(float(px), float(py), ptr(rx), ptr(ry), ptr(cum), len(rx))


def lateral_error(px, py, wx, wy):
    wx, wy = f64(wx), f64(wy)
    return lib().orc_lateral_error(float(px), float(py), ptr(wx), ptr(wy), len(wx))


class Oracle:
    """Batched reference-semantics stepper over host records (numpy)."""

    def __init__(self, params, padded_map: np.ndarray, caps_c, record_bytes: int):
        self.P = params
        self.map = np.ascontiguousarray(padded_map)
        self.caps = caps_c
        self.rb = int(record_bytes)
        self.scratch = np.zeros(params.render_w * params.render_h, np.uint8)
        self.L = lib()

    def step(self, recs: np.ndarray, n: int, actions: np.ndarray, frames: np.ndarray | None):
        a = np.ascontiguousarray(actions)
        stride = a.strides[0] if a.ndim > 0 else a.itemsize
        self.L.orc_step_batch(ctypes.byref(self.P), ptr(self.map), ctypes.byref(self.caps), ptr(recs), self.rb, n,
                              ptr(a), int(stride), ptr(frames) if frames is not None else None, ptr(self.scratch))

    def step_one(self, rec: np.ndarray, action: np.ndarray, frame: np.ndarray | None):
        a = np.ascontiguousarray(action)
        return self.L.orc_step(ctypes.byref(self.P), ptr(self.map), ctypes.byref(self.caps), ptr(rec), ptr(a),
                               ptr(frame) if frame is not None else None, ptr(self.scratch))

    def reset_obs(self, rec: np.ndarray, frame: np.ndarray):
        self.L.orc_reset_obs(ctypes.byref(self.P), ptr(self.map), ctypes.byref(self.caps), ptr(rec), ptr(frame),
                             ptr(self.scratch))

    def crop_origin(self, x, y):
        out = np.zeros(2, np.int32)
        self.L.orc_crop_origin(ctypes.byref(self.P), float(x), float(y), ptr(out))
        return int(out[0]), int(out[1])
