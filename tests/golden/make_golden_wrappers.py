"""Golden vectors for the observation-wrapper stack, from the reference's own code.

Runs ONLY in the build container (needs /root/reference); writes
tests/golden/wrappers.npz, which tests/test_oracle_golden.py pins the wrapper
oracle (oracle/wrappers.py) against. Captured reference functions
(CarlaBEV/wrappers/rgb_to_semantic.py):
  rgb_to_semantic_mask            :65-142   every semantic_mask_ch
  flatten_stacked_frames          :145-149
  fuse_vehicle_temporal_channels  :152-166
  fuse_weighted_vehicle_history   :169-191

`rgb_to_semantic.py:1` imports gymnasium for its wrapper classes only; a
test-only stand-in (`ObservationWrapper`, `spaces.Box`) lets the module import.
None of the captured numbers flows through the stand-in: the functions above
are NumPy on the arrays passed in.

Inputs are palette-id frames (the device frame format) expanded to RGB with
the reference palette (`CarlaBEV/semantics.py:19-28`, traffic-light colours
`src/actors/traffic_light.py:46-54`), plus a set of off-palette colours (the
blends a resize produces), so the exact-colour matching is exercised too.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refimport  # noqa: E402


def _install_gymnasium_stub() -> None:
    if "gymnasium" in sys.modules:
        return
    gym = types.ModuleType("gymnasium")
    spaces = types.ModuleType("gymnasium.spaces")

    class Box:  # shape holder only
        def __init__(self, low=None, high=None, shape=None, dtype=None):
            self.low, self.high, self.shape, self.dtype = low, high, shape, dtype

    class ObservationWrapper:
        def __init__(self, env):
            self.env = env
            self.observation_space = getattr(env, "observation_space", None)

    spaces.Box = Box
    gym.spaces = spaces
    gym.ObservationWrapper = ObservationWrapper
    gym.Wrapper = ObservationWrapper
    sys.modules.update({"gymnasium": gym, "gymnasium.spaces": spaces})


refimport.setup()
_install_gymnasium_stub()
refimport._bare_pkg("CarlaBEV.wrappers", f"{refimport.REF}/CarlaBEV/wrappers")

from CarlaBEV.wrappers.rgb_to_semantic import (  # noqa: E402
    SEMANTIC_MASK_CHANNELS,
    flatten_stacked_frames,
    fuse_vehicle_temporal_channels,
    fuse_weighted_vehicle_history,
    rgb_to_semantic_mask,
)

# palette ids -> RGB (include/cbev_layout.h CBEV_PX_*), incl. the off-palette
# blend colours at ids 10..15 (never produced by the device raster)
PALETTE16 = np.array([
    (150, 150, 150), (255, 255, 255), (220, 220, 220), (0, 7, 175), (255, 0, 0), (0, 255, 0),
    (255, 64, 64), (255, 255, 0), (0, 0, 0), (100, 100, 100),
    (202, 202, 202), (128, 131, 215), (255, 128, 128), (0, 254, 0), (185, 185, 185), (254, 255, 255),
], dtype=np.uint8)


def main():
    rng = np.random.default_rng(2024)
    F, H, W = 4, 12, 20
    n = 6
    ids = rng.integers(0, 16, size=(n, F, H, W)).astype(np.uint8)
    ids[0] = rng.integers(0, 10, size=(F, H, W))  # on-palette only
    ids[1, :, :, :] = 3  # all vehicle
    out = {"ids": ids, "palette": PALETTE16}
    for mode in SEMANTIC_MASK_CHANNELS:
        masks = np.stack([np.stack([rgb_to_semantic_mask(PALETTE16[ids[e, f]], mode=mode) for f in range(F)])
                          for e in range(n)])  # (n, F, C, H, W)
        key = mode.replace("-", "_")
        out[f"mask_{key}"] = masks.astype(np.float32)
        out[f"flat_{key}"] = np.stack([flatten_stacked_frames(masks[e]) for e in range(n)])
        if "vehicle" in SEMANTIC_MASK_CHANNELS[mode]:
            out[f"temporal_{key}"] = np.stack([fuse_vehicle_temporal_channels(masks[e], mode=mode)
                                               for e in range(n)])
            out[f"weighted_{key}"] = np.stack([fuse_weighted_vehicle_history(masks[e], mode=mode)
                                               for e in range(n)])
    path = os.path.join(HERE, "wrappers.npz")
    np.savez_compressed(path, **out)
    print(f"wrappers.npz: {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
