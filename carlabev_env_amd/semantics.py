"""Palette ids of the device frame and the lookup tables of the wrapper stack.

Device frames store one palette id per pixel (include/cbev_layout.h
CBEV_PX_*); every colour the reference can draw into the observation surface
has exactly one id, so the id frame is a lossless encoding of `render()`
(`CarlaBEV/envs/carlabev.py:233-249`). Colours: `CarlaBEV/semantics.py:19-28`,
traffic-light colours `src/actors/traffic_light.py:46-54`, hero colour (0,0,0)
`src/managers/actor_manager.py:45,55`.
"""
from __future__ import annotations

import numpy as np

NON_DRIVABLE, DRIVABLE, SIDEWALK, VEHICLE, PEDESTRIAN, ROUTE, TL_RED, YELLOW, BLACK, TL_UNKNOWN = range(10)

PALETTE = np.array([
    (150, 150, 150),  # NON_DRIVABLE
    (255, 255, 255),  # DRIVABLE
    (220, 220, 220),  # SIDEWALK
    (0, 7, 175),      # VEHICLE
    (255, 0, 0),      # PEDESTRIAN
    (0, 255, 0),      # ROUTE (targets, green traffic light)
    (255, 64, 64),    # TRAFFIC_LIGHT_RED
    (255, 255, 0),    # yellow traffic light (== EGO colour in semantics.py)
    (0, 0, 0),        # hero overlay / compose background
    (100, 100, 100),  # traffic light in an unknown state
], dtype=np.uint8)

# channel predicates of rgb_to_semantic_mask (wrappers/rgb_to_semantic.py:65-142),
# expressed on palette ids
_CH = {
    "non_drivable": {NON_DRIVABLE},
    "drivable": {DRIVABLE, ROUTE},   # white OR green
    "sidewalk": {SIDEWALK},
    "vehicle": {VEHICLE},
    "pedestrian": {PEDESTRIAN},
    "route": {ROUTE},
    "traffic_light_red": {TL_RED},
}
SEMANTIC_MASK_CHANNELS = {
    "binary": ("drivable",),
    "2-class": ("drivable", "route"),
    "4-class": ("drivable", "vehicle", "pedestrian", "route"),
    "5-class": ("drivable", "sidewalk", "vehicle", "pedestrian", "route"),
    "6-class": ("non_drivable", "drivable", "sidewalk", "vehicle", "pedestrian", "route"),
    "7-class": ("non_drivable", "drivable", "sidewalk", "vehicle", "pedestrian", "route", "traffic_light_red"),
}


def semantic_mask_channels(mode: str):
    if mode not in SEMANTIC_MASK_CHANNELS:
        raise ValueError(f"Unsupported semantic_mask_ch={mode!r}. Expected one of: "
                         f"{', '.join(sorted(SEMANTIC_MASK_CHANNELS))}")
    return SEMANTIC_MASK_CHANNELS[mode]


def semantic_lut(mode: str) -> np.ndarray:
    """lut[id] = bitmask of the channels set for palette id `id`."""
    chans = semantic_mask_channels(mode)
    lut = np.zeros(16, dtype=np.uint32)
    for c, name in enumerate(chans):
        for pid in _CH[name]:
            lut[pid] |= np.uint32(1 << c)
    return lut


def gray_lut() -> np.ndarray:
    """gymnasium 1.x GrayscaleObservation on each palette colour:
    sum(obs * [0.2125, 0.7154, 0.0721], axis=-1).astype(uint8). Parity unpinned:
    gymnasium is not installed here."""
    lut = np.zeros(16, dtype=np.uint32)
    g = np.sum(np.multiply(PALETTE, np.array([0.2125, 0.7154, 0.0721])), axis=-1).astype(np.uint8)
    lut[:len(g)] = g
    return lut


def rgb_lut() -> np.ndarray:
    lut = np.zeros(16, dtype=np.uint32)
    p = PALETTE.astype(np.uint32)
    lut[:len(p)] = (p[:, 0] << 16) | (p[:, 1] << 8) | p[:, 2]
    return lut


def ids_to_rgb(frames: np.ndarray) -> np.ndarray:
    return PALETTE[np.asarray(frames)]


def rgb_to_semantic_mask_ids(ids: np.ndarray, mode: str = "6-class") -> np.ndarray:
    """Host one-hot of an id frame, (C, H, W) float32 — used by tests."""
    lut = semantic_lut(mode)
    m = lut[np.asarray(ids)]
    chans = semantic_mask_channels(mode)
    return np.stack([((m >> c) & 1).astype(np.float32) for c in range(len(chans))])
