"""Convert the reference's Town01 semantic PNG maps into 1-byte class maps.

Runs in the build container only (it reads /root/reference). Output goes to
carlabev_env_amd/assets/<map>-<size>-class.npz and is committed, so the GPU
box never needs the reference tree.

Why a 1-byte class map is lossless: the reference loads two images per size
(`CarlaBEV/envs/utils.py:49-62`): the `-sem.png` label image (values
{0,127,255}) is turned into RGB with the semantic palette for tile queries,
and the `-rgb.png` image is what gets blitted into the render surface. This
script checks that the RGB image equals palette(sem) pixel for pixel, so one
uint8 class id per texel carries both. Class ids follow
`CarlaBEV/semantics.py:8-18,34-38`: label 0 -> NON_DRIVABLE(0),
127 -> DRIVABLE(1), 255 -> SIDEWALK(2).
"""
from __future__ import annotations

import argparse
import os

import numpy as np
from PIL import Image

REF_ASSETS = "/root/reference/CarlaBEV/assets"
OUT_DIR = os.path.join(os.path.dirname(__file__), "..", "carlabev_env_amd", "assets")

LABEL_TO_CLASS = {0: 0, 127: 1, 255: 2}
CLASS_RGB = {0: (150, 150, 150), 1: (255, 255, 255), 2: (220, 220, 220)}


def convert(map_name: str, size: int) -> str:
    sem = np.array(Image.open(os.path.join(REF_ASSETS, map_name, f"{map_name}-{size}-sem.png")))
    rgb = np.array(Image.open(os.path.join(REF_ASSETS, map_name, f"{map_name}-{size}-rgb.png")).convert("RGB"))
    cls = np.full(sem.shape, 255, dtype=np.uint8)
    for label, c in LABEL_TO_CLASS.items():
        cls[sem == label] = c
    if (cls == 255).any():
        raise ValueError("unexpected label value in semantic map")
    pal = np.zeros(sem.shape + (3,), np.uint8)
    for c, col in CLASS_RGB.items():
        pal[cls == c] = col
    if not np.array_equal(pal, rgb):
        raise ValueError(f"{map_name}-{size}: rgb image is not palette(sem); 1-byte map would be lossy")
    out = os.path.join(OUT_DIR, f"{map_name}-{size}-class.npz")
    np.savez_compressed(out, classes=cls)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--map", default="Town01")
    ap.add_argument("--sizes", default="64,128,256")
    args = ap.parse_args()
    os.makedirs(OUT_DIR, exist_ok=True)
    for s in args.sizes.split(","):
        print(convert(args.map, int(s)))


if __name__ == "__main__":
    main()
