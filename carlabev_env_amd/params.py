"""Resolve an EnvConfig into the numeric constants the HIP step consumes.

`CbevParams` mirrors `struct cbev_params` of include/cbev_layout.h byte for
byte (checked against the library's `cbev_params_size()` in the CPU tests).
Geometry follows the reference's renderer set-up:
  anchor       envs/fov.py:30-36
  crop size    envs/fov.py:38-44
  padding      envs/world.py:_build_render_layers (padding = crop size)
  hero size    src/actors/hero.py:13-18 (scale = int(1024/S), w = int(32/scale))
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np

from .config import (ASSET_DIR, EnvConfig, get_action_profile_spec, get_reward_profile_spec)

_I32 = ctypes.c_int32
_F64 = ctypes.c_double


class CbevParams(ctypes.Structure):
    _fields_ = [(n, _I32) for n in (
        "size", "crop", "pad", "anchor_x", "anchor_y", "map_w", "map_h", "render_w", "render_h",
        "map_pitch", "hero_w", "scale", "action_kind", "n_discrete", "reward_kind", "max_actions",
        "collide_min_dist", "pad0")] + [
        ("action_table", (ctypes.c_float * 3) * 16)] + [(n, _F64) for n in (
            "lane_center_exponent", "lane_center_floor", "off_lane_penalty", "speed_penalty_scale",
            "speed_penalty_floor", "ttc_threshold", "ttc_penalty_floor", "sidewalk_step_penalty",
            "sidewalk_penalty_scale")] + [(n, _I32) for n in (
                "offroad_terminate_after", "zero_speed_reward_offroad", "zero_progress_reward_offroad",
                "pad1")] + [(n, _F64) for n in (
                    "k_lat_quadratic", "k_progress", "k_flow", "k_align_bonus", "k_reverse", "k_ttc", "alive_bias",
                    "k_smooth", "k_steer_smooth", "k_steer_jerk", "k_route_dev", "route_dev_start",
                    "max_speed_for_flow", "lat_clip", "yaw_small", "lat_small")]


# CaRLRewardFn.__init__ defaults (src/deeprl/carl_reward_fn.py:74-88)
CARL_DEFAULTS = dict(lane_center_exponent=1.0, lane_center_floor=0.2, off_lane_penalty=0.0, speed_penalty_scale=6.0,
                     speed_penalty_floor=0.1, ttc_threshold=4.0, ttc_penalty_floor=0.1)
# RewardFn.__init__ defaults (src/deeprl/reward.py:14-42)
SHAPING_DEFAULTS = dict(max_actions=5000, sidewalk_step_penalty=-0.12, sidewalk_penalty_scale=-0.006,
                        offroad_terminate_after=40, zero_speed_reward_offroad=True, zero_progress_reward_offroad=True,
                        k_lat_quadratic=0.004, k_progress=0.06, k_flow=0.010, k_align_bonus=0.02, k_reverse=0.03,
                        k_ttc=0.03, alive_bias=0.0025, k_smooth=0.0006, k_steer_smooth=0.003, k_steer_jerk=0.01,
                        k_route_dev=0.006, route_dev_start=8.0, max_speed_for_flow=6.0, lat_clip=4.0, yaw_small=0.12,
                        lat_small=0.8)

MAP_PITCH_ALIGN = 64


def fov_geometry(size: int, ax_frac: float = 0.5, ay_frac: float = 0.5):
    """(anchor_x, anchor_y, crop) exactly as FovRenderer computes them."""
    max_idx = size - 1
    ax = int(round(max_idx * ax_frac))
    ay = int(round(max_idx * ay_frac))
    ax = max(0, min(max_idx, ax))
    ay = max(0, min(max_idx, ay))
    mx = max(ax, (size - 1) - ax)
    my = max(ay, (size - 1) - ay)
    crop = int(math.ceil(2.0 * math.hypot(mx, my)))
    return ax, ay, max(size, crop)


def load_class_map(map_name: str, size: int) -> np.ndarray:
    path = os.path.join(ASSET_DIR, f"{map_name}-{size}-class.npz")
    with np.load(path, allow_pickle=False) as z:
        return np.ascontiguousarray(z["classes"])


def padded_map(classes: np.ndarray, pad: int) -> tuple[np.ndarray, int]:
    """Render surface of world.py:_build_padded_render_map as class ids:
    NON_DRIVABLE fill, map blitted at (pad, pad). Rows padded to a 64-byte pitch."""
    h, w = classes.shape
    rw, rh = w + 2 * pad, h + 2 * pad
    pitch = (rw + MAP_PITCH_ALIGN - 1) // MAP_PITCH_ALIGN * MAP_PITCH_ALIGN
    out = np.zeros((rh, pitch), dtype=np.uint8)
    out[pad:pad + h, pad:pad + w] = classes
    return out, pitch


def build_params(cfg: EnvConfig, classes: np.ndarray) -> CbevParams:
    P = CbevParams()
    S = int(cfg.size)
    ax, ay, crop = fov_geometry(S, cfg.ego_anchor_x_frac, cfg.ego_anchor_y_frac)
    h, w = classes.shape
    P.size, P.crop, P.pad = S, crop, crop
    P.anchor_x, P.anchor_y = ax, ay
    P.map_w, P.map_h = w, h
    P.render_w, P.render_h = w + 2 * crop, h + 2 * crop
    P.map_pitch = (P.render_w + MAP_PITCH_ALIGN - 1) // MAP_PITCH_ALIGN * MAP_PITCH_ALIGN
    P.scale = int(1024 / S)
    P.hero_w = int(32 / P.scale)
    aspec = get_action_profile_spec(cfg.action_profile_id)
    if aspec["action_mode"] == "discrete":
        acts = np.asarray(aspec["discrete_actions"], dtype=np.float32)
        if len(acts) > 16:
            raise ValueError("at most 16 discrete actions are supported")
        P.action_kind, P.n_discrete = 0, len(acts)
        for i, a in enumerate(acts):
            for j in range(3):
                P.action_table[i][j] = float(a[j])
    else:
        P.action_kind, P.n_discrete = 1, 0
    rspec = get_reward_profile_spec(cfg.reward_profile_id)
    params = dict(rspec["parameters"])
    if rspec["family"] == "carl":
        P.reward_kind = 0
        merged = dict(CARL_DEFAULTS)
        merged.update({k: v for k, v in params.items() if k in CARL_DEFAULTS})
        sh = dict(SHAPING_DEFAULTS)
    else:
        P.reward_kind = 1
        merged = dict(CARL_DEFAULTS)
        sh = dict(SHAPING_DEFAULTS)
        sh.update(params)
    for k, v in merged.items():
        setattr(P, k, float(v))
    P.max_actions = int(sh["max_actions"])
    for k, v in sh.items():
        if k == "max_actions":
            continue
        if k in ("offroad_terminate_after",):
            setattr(P, k, int(v))
        elif k in ("zero_speed_reward_offroad", "zero_progress_reward_offroad"):
            setattr(P, k, 1 if v else 0)
        else:
            setattr(P, k, float(v))
    P.collide_min_dist = 35  # CarlaBEV._compute_outcome: collision_check(min_dist=35) (carlabev.py:173)
    return P


def params_dict(P: CbevParams) -> dict:
    out = {}
    for name, _ in P._fields_:
        val = getattr(P, name)
        if name == "action_table":
            val = [[val[i][j] for j in range(3)] for i in range(16)]
        out[name] = val
    return out
