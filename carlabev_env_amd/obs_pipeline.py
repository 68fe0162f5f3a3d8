"""Host side of the device wrapper stack (wrap_env, CarlaBEV/envs/__init__.py:62-83).

Maps an EnvConfig onto the `cbev_expand_obs` / `cbev_resize_obs` kinds of
include/cbev.h and derives the wrapped observation spaces:

  ResizeObservation(obs_size)          cbev_resize_obs   (only when obs_size != (size, size))
  SemanticMaskWrapper | Grayscale      the expansion LUT (palette id -> channels / gray)
  FrameStackObservation(frame_stack)   the device frame ring
  Flatten | VehicleTemporalFusion | WeightedVehicleHistory
                                       expansion kind 0 / 3 / 4

`area_table` and `match_palette` document the resize encoding; the device builds
its own tables (cbev.hip `area_tab`) with the same double-precision arithmetic.
"""
from __future__ import annotations

import math

import numpy as np

from .semantics import PALETTE, semantic_mask_channels

KIND_FLAT, KIND_GRAY, KIND_RGB, KIND_TEMPORAL, KIND_WEIGHTED, KIND_GRAY_RAW = 0, 1, 2, 3, 4, 5
OFF_PALETTE = 15  # CBEV_PX_OFF_PALETTE
FUSION_KIND = {"stack": KIND_FLAT, "vehicle_temporal": KIND_TEMPORAL, "vehicle_weighted": KIND_WEIGHTED}
HISTORY_FRAMES = 3  # VehicleTemporalFusionWrapper history_frames / len(weights) (rgb_to_semantic.py:281,310)


def fused_channels(mode: str, fusion: str, frame_stack: int = 4) -> int:
    """Channel count of the wrapped semantic observation (rgb_to_semantic.py:236-332)."""
    chans = semantic_mask_channels(mode)
    C = len(chans)
    if fusion == "stack":
        return frame_stack * C
    if "vehicle" not in chans:
        raise ValueError(f"semantic_mask_ch={mode!r} does not expose a vehicle channel, "
                         "so vehicle history fusion is unsupported.")
    if frame_stack < HISTORY_FRAMES:
        raise ValueError(f"{fusion} requires frame_stack >= {HISTORY_FRAMES}, got {frame_stack}")
    if fusion == "vehicle_temporal":
        return C - 1 + HISTORY_FRAMES
    if fusion == "vehicle_weighted":
        return C
    raise ValueError(f"unknown temporal_fusion_mode {fusion!r}")


def area_table(ssize: int, dsize: int):
    """computeResizeAreaTab (opencv 4.11 resize.cpp) for scale = 1 / (dsize / ssize),
    grouped per destination index: (off[dsize + 1], src index, float32 alpha)."""
    scale = 1.0 / (dsize / ssize)
    off = np.zeros(dsize + 1, np.int32)
    idx, alpha = [], []
    for dx in range(dsize):
        off[dx] = len(idx)
        f1 = dx * scale
        f2 = f1 + scale
        cell = min(scale, ssize - f1)
        s1, s2 = math.ceil(f1), math.floor(f2)
        s2 = min(s2, ssize - 1)
        s1 = min(s1, s2)
        if s1 - f1 > 1e-3:
            idx.append(s1 - 1)
            alpha.append((s1 - f1) / cell)
        for sx in range(s1, s2):
            idx.append(sx)
            alpha.append(1.0 / cell)
        if f2 - s2 > 1e-3:
            idx.append(s2)
            alpha.append(min(min(f2 - s2, 1.0), cell) / cell)
    off[dsize] = len(idx)
    return off, np.asarray(idx, np.int32), np.asarray(alpha, np.float32)


def match_palette(rgb: np.ndarray) -> np.ndarray:
    """Byte code of a resized RGB frame for the semantic path: the palette id whose
    colour equals the pixel exactly, else OFF_PALETTE."""
    rgb = np.asarray(rgb, np.uint8)
    code = np.full(rgb.shape[:-1], OFF_PALETTE, np.uint8)
    for pid in range(len(PALETTE) - 1, -1, -1):
        code[np.all(rgb == PALETTE[pid], axis=-1)] = pid
    return code
