"""Static FOV corner mask (EnvConfig.fov_masked) for the device raster.

`FovRenderer._build_mask_surface` (CarlaBEV/envs/fov.py:46-68) fills four corner
triangles with leg m = int(size * mask_frac) (mask_frac 0.5, fov.py:15) into an
SRCALPHA surface with `pygame.draw.polygon`; `apply_mask` (fov.py:96-99) blits
it over the composed observation, so those pixels become black (alpha 255
blends to the source colour exactly). It runs before the ego is drawn
(world.py:137-157); the ego is black too, so the order does not show.

The pixel set follows pygame 2.6.1's scanline polygon fill (src_c/draw.c
draw_fillpoly), restated here; pygame is not installed, so the exact boundary
pixels are parity unpinned. The device applies the mask as a
byte mask (0xff = black) inside k_raster's output stores (`cbev_set_fov_mask`).
"""
from __future__ import annotations

import math

import numpy as np


def _scan_fill(mask: np.ndarray, xs, ys) -> None:
    H, W = mask.shape

    def span(xa, y, xb):
        lo, hi = max(min(xa, xb), 0), min(max(xa, xb), W - 1)
        if 0 <= y < H and lo <= hi:
            mask[y, lo:hi + 1] = True

    n = len(xs)
    y_lo, y_hi = min(ys), max(ys)
    if y_lo == y_hi:
        span(min(xs), y_lo, max(xs))
        return
    edges = []  # non-horizontal edges, top end first
    for i in range(n):
        j = (i - 1) % n
        if ys[j] == ys[i]:
            continue
        (xt, yt), (xb, yb) = sorted(((xs[j], ys[j]), (xs[i], ys[i])), key=lambda p: p[1])
        edges.append((xt, yt, xb, yb))
    for y in range(y_lo, y_hi + 1):
        cuts = []
        for xt, yt, xb, yb in edges:
            if yt <= y < yb or (y == y_hi and yb == y_hi):
                f = np.float32((y - yt) * (xb - xt) / np.float32(yb - yt))
                f = math.floor(f) if len(cuts) % 2 == 0 else math.ceil(f)
                cuts.append(int(f) + xt)
        cuts.sort()
        for k in range(0, len(cuts) - 1, 2):
            span(cuts[k], y, cuts[k + 1])
    for i in range(n):  # horizontal border edges strictly inside the y range
        j = (i - 1) % n
        if y_lo < ys[i] < y_hi and ys[j] == ys[i]:
            span(xs[i], ys[i], xs[j])


def fov_corner_mask(size: int, mask_frac: float = 0.5) -> np.ndarray:
    """(size, size) uint8, 0xff where the FOV mask blacks the observation out."""
    S, m = int(size), int(size * mask_frac)
    mask = np.zeros((S, S), bool)
    corners = (((0, 0), (m, 0), (0, m)), ((S, 0), (S - m, 0), (S, m)), ((0, S), (0, S - m), (m, S)),
               ((S, S), (S - m, S), (S, S - m)))
    for tri in corners:
        _scan_fill(mask, [p[0] for p in tri], [p[1] for p in tri])
    return np.where(mask, np.uint8(0xFF), np.uint8(0))
