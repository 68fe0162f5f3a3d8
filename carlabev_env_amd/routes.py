"""Reset-time route preparation on the host (NumPy/SciPy).

Scene construction stays on the host (`src/managers/` is out of
scope for the device path). What the device needs from a reset is the
realised controller state, so the packer runs the reference's reset-time
arithmetic here, with the same libraries the reference uses:

  smooth_and_compute     src/control/utils.py:200-269 (scipy savgol_filter)
  Controller.set_route   src/control/stanley_controller.py:34-49 (±1 px jitter)
  calc_target_index      src/control/stanley_controller.py:100-123
  stanley_control        src/control/stanley_controller.py:64-89
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
from scipy.ndimage import convolve1d
from scipy.signal import savgol_coeffs, savgol_filter  # noqa: F401 (savgol_filter: the tests' cross-check)

L_WHEELBASE = 2.9
K_GAIN = 2.0
MAX_STEER = np.radians(30.0)


_SG_CACHE: dict = {}


def _sg_tables(window: int, poly: int):
    """What scipy.signal.savgol_filter(x, window, poly) recomputes on every call
    (scipy 1.15 signal/_savitzky_golay.py:230-360, numpy polyfit): the
    convolution coefficients and polyfit's scaled Vandermonde matrix, its column
    scale and rcond for the edge fits. Deterministic, so computed once."""
    key = (window, poly)
    if key not in _SG_CACHE:
        coeffs = savgol_coeffs(window, poly, deriv=0, delta=1.0)
        t = np.arange(0, window) + 0.0
        lhs = np.vander(t, poly + 1)
        scale = np.sqrt((lhs * lhs).sum(axis=0))
        lhs /= scale
        _SG_CACHE[key] = (coeffs, lhs, scale, len(t) * np.finfo(t.dtype).eps)
    return _SG_CACHE[key]


def savgol_interp(x: np.ndarray, window: int, poly: int) -> np.ndarray:
    """scipy.signal.savgol_filter(x, window, poly) (mode "interp", deriv 0) of a
    1-D float64 array, bit for bit: the same convolve1d of the same
    coefficients, then each edge refit with the same lstsq call np.polyfit makes
    (savgol_filter -> _fit_edges_polyfit -> _fit_edge) and np.polyval -- without
    recomputing the coefficients and polyfit's matrix on every call."""
    coeffs, lhs, scale, rcond = _sg_tables(window, poly)
    y = convolve1d(x, coeffs, axis=-1, mode="constant")
    n, half = x.shape[0], window // 2
    for ws, is_, ie in ((0, 0, half), (n - window, n - half, n)):
        rhs = x[ws:ws + window].reshape(window, 1) + 0.0  # polyfit's `y + 0.0`
        c = np.linalg.lstsq(lhs, rhs, rcond)[0]
        c = (c.T / scale).T
        i = np.arange(is_ - ws, ie - ws)
        y[is_:ie] = np.polyval(c, i.reshape(-1, 1)).reshape(ie - is_)  # / (delta ** 0) = / 1.0: exact
    return y


_SMOOTH_MEMO: "OrderedDict[tuple, tuple]" = OrderedDict()
_SMOOTH_MEMO_CAP = 64  # recent routes: a scene smooths its ego route for the profile check and again at packing


def smooth_and_compute(ax, ay, window: int = 9, poly: int = 3):
    """utils.py:200-269, memoised on the exact input bytes (a pure function:
    a repeated route returns copies of the same arrays)."""
    ax = np.asarray(ax, dtype=float)
    ay = np.asarray(ay, dtype=float)
    key = (ax.tobytes(), ay.tobytes(), int(window), int(poly))
    hit = _SMOOTH_MEMO.get(key)
    if hit is None:
        hit = _smooth_and_compute(ax, ay, window, poly)
        _SMOOTH_MEMO[key] = hit
        if len(_SMOOTH_MEMO) > _SMOOTH_MEMO_CAP:
            _SMOOTH_MEMO.popitem(last=False)
    else:
        _SMOOTH_MEMO.move_to_end(key)
    return tuple(a.copy() for a in hit)


def _smooth_and_compute(ax, ay, window: int, poly: int):
    if ax.size != ay.size:
        raise ValueError("ax and ay must have same length")
    d = np.hypot(np.diff(ax), np.diff(ay))
    keep = np.concatenate(([True], d > 1e-9))
    ax, ay = ax[keep], ay[keep]
    if len(ax) < 2:
        x0, y0 = ax[0], ay[0]
        ax = np.array([x0, x0 + 1e-3])
        ay = np.array([y0, y0])
    if window % 2 == 0:
        window += 1
    if window > len(ax):
        window = len(ax) if len(ax) % 2 == 1 else len(ax) - 1
    if window < 3:
        window = 3
    poly = min(poly, window - 1)
    if len(ax) >= window:
        cx = savgol_interp(ax, window, poly)
        cy = savgol_interp(ay, window, poly)
    else:
        cx, cy = ax.copy(), ay.copy()
    seg = np.hypot(np.diff(cx), np.diff(cy))
    s = np.concatenate(([0.0], np.cumsum(seg)))
    if s[-1] <= 1e-9:
        z = np.zeros_like(cx)
        return cx, cy, z.copy(), z.copy(), s
    dx_ds = np.gradient(cx, s)
    dy_ds = np.gradient(cy, s)
    cyaw = np.unwrap(np.arctan2(dy_ds, dx_ds))
    d2x = np.gradient(dx_ds, s)
    d2y = np.gradient(dy_ds, s)
    denom = dx_ds ** 2 + dy_ds ** 2
    small = denom < 1e-9
    denom_safe = np.where(small, 1.0, denom)
    ck = (dx_ds * d2y - dy_ds * d2x) / (denom_safe ** 1.5)
    ck[small] = 0.0
    return cx, cy, cyaw, ck, s


def angle_mod(x):
    return ((np.asarray(x, dtype=float).flatten() + np.pi) % (2 * np.pi) - np.pi).item()


def calc_target_index(x, y, yaw, cx, cy):
    fx = x + L_WHEELBASE * np.cos(yaw)
    fy = y + L_WHEELBASE * np.sin(yaw)
    dx = [fx - icx for icx in cx]
    dy = [fy - icy for icy in cy]
    d = np.hypot(dx, dy)
    idx = int(np.argmin(d))
    fav = [-np.cos(yaw + np.pi / 2), -np.sin(yaw + np.pi / 2)]
    err = np.dot([dx[idx], dy[idx]], fav)
    return idx, err


def stanley_target(x, y, yaw, v, cx, cy, cyaw, target_idx):
    cur, err = calc_target_index(x, y, yaw, cx, cy)
    if target_idx >= cur:
        cur = target_idx
    return cur


class ControllerInit:
    """Realised controller state after `Controller.set_route` (+ hero's initial
    stanley_control, hero.py:83-86)."""

    __slots__ = ("x", "y", "yaw", "v", "cx", "cy", "cyaw", "target_idx")

    def __init__(self, ax, ay, v0: float, *, jitter_start: bool = True, np_rng=None, yaw0: float = 0.0,
                 hero: bool = False):
        cx, cy, cyaw, _, _ = smooth_and_compute(ax, ay, window=11, poly=3)
        if jitter_start:
            if np_rng is None:
                np_rng = np.random.default_rng()
            x = cx[0] + int(np_rng.integers(-1, 2))
            y = cy[0] + int(np_rng.integers(-1, 2))
        else:
            x, y = cx[0], cy[0]
        # State.__init__ leaves yaw = 0.0 until set_route assigns it
        tidx, _ = calc_target_index(x, y, yaw0, cx, cy)
        yaw = cyaw[tidx]
        if hero:
            tidx = stanley_target(x, y, yaw, v0, cx, cy, cyaw, tidx)
        self.x, self.y, self.yaw, self.v = float(x), float(y), float(yaw), float(v0)
        self.cx, self.cy, self.cyaw = cx, cy, cyaw
        self.target_idx = int(tidx)


def cumulative_lengths_int(rx, ry):
    """CaRL cumulative route lengths over the int32 raw route (carl_reward_fn.py:20-26)."""
    route = list(zip(np.asarray(rx, np.int32), np.asarray(ry, np.int32)))
    lengths = [0.0]
    for i in range(1, len(route)):
        dx = route[i][0] - route[i - 1][0]
        dy = route[i][1] - route[i - 1][1]
        lengths.append(lengths[-1] + np.hypot(dx, dy))
    return np.asarray(lengths, dtype=np.float64)
