"""Vectorised NumPy restatement of the FOV raster (test-only cross-check).

A third, independent statement of the reference's render path, used to
cross-check the C oracle's raster in CPU tests: scene surface = padded map +
rects painted in draw order (actor_manager.py:121-132), crop
(world.py:105-111), pygame transform.rotate / rotate90 (fixed-point inverse
map), get_rect(center=anchor) + blit onto a black surface (fov.py:84-94),
hero overlay (hero.py:26-32).
"""
from __future__ import annotations

import math

import numpy as np

BLACK = 8


def paint(scene: np.ndarray, x: int, y: int, w: int, h: int, col: int):
    H, W = scene.shape
    x0, y0, x1, y1 = max(x, 0), max(y, 0), min(x + w, W), min(y + h, H)
    if x1 > x0 and y1 > y0:
        scene[y0:y1, x0:x1] = col


def crop_origin(P, x: float, y: float):
    C = float(P.crop)
    offx = math.trunc((P.pad + x) + (-C / 2))
    offy = math.trunc((P.pad + y) + (-C / 2))
    xm = int(round(offx + C / 2.0)) - P.crop // 2
    ym = int(round(offy + C / 2.0)) - P.crop // 2
    xm = max(0, min(max(0, P.render_w - P.crop), xm))
    ym = max(0, min(max(0, P.render_h - P.crop), ym))
    return xm, ym


def rotate_compose(P, crop: np.ndarray, yaw: float, reset: bool) -> np.ndarray:
    C, S = P.crop, P.size
    angle = np.float32(90.0) if reset else np.float32(math.degrees(yaw) + 90)
    out = np.full((S, S), BLACK, dtype=np.uint8)
    bg = crop[0, 0]
    if math.fmod(float(angle), 90.0) == 0.0:
        # C semantics of (int)angle / 90 % 4: truncating division and remainder
        k = int(math.fmod(math.trunc(int(angle) / 90), 4))
        if k < 0:
            k += 4
        rot = np.rot90(crop, k)  # counter-clockwise, as pygame rotate90
        nx = ny = C
    else:
        rad = float(angle) * .01745329251994329
        s, c = math.sin(rad), math.cos(rad)
        cx, cy, sx, sy = c * C, c * C, s * C, s * C
        nx = int(max(abs(cx + sy), abs(cx - sy), abs(-cx + sy), abs(-cx - sy)))
        ny = int(max(abs(sx + cy), abs(sx - cy), abs(-sx + cy), abs(-sx - cy)))
        icy = ny // 2
        xd, yd = (C - nx) * 32768, (C - ny) * 32768
        isin, icos = int(s * 65536), int(c * 65536)
        ax = (nx << 15) - int(c * ((nx - 1) << 15))
        ay = (ny << 15) - int(s * ((nx - 1) << 15))
        yy, xx = np.meshgrid(np.arange(ny, dtype=np.int64), np.arange(nx, dtype=np.int64), indexing="ij")
        dx = (ax + isin * (icy - yy)) + xd + xx * icos
        dy = (ay - icos * (icy - yy)) + yd + xx * isin
        ok = (dx >= 0) & (dy >= 0) & (dx <= (C << 16) - 1) & (dy <= (C << 16) - 1)
        rot = np.full((ny, nx), bg, dtype=np.uint8)
        rot[ok] = crop[dy[ok] >> 16, dx[ok] >> 16]
    rx, ry = P.anchor_x - nx // 2, P.anchor_y - ny // 2
    for v in range(S):
        j = v - ry
        if 0 <= j < ny:
            u = np.arange(S)
            i = u - rx
            m = (i >= 0) & (i < nx)
            out[v, u[m]] = rot[j, i[m]]
    return out


def render(P, padded: np.ndarray, view, reset: bool = False) -> np.ndarray:
    from carlabev_env_amd import layout as LY
    scene = padded[:, :P.render_w].copy()
    if not reset:
        for a in range(view.i("NACT")):
            sz = int(view.ai[LY.AI["SIZE"], a])
            x = round(P.pad + view.ad[LY.AD["X"], a]) - sz // 2
            y = round(P.pad + view.ad[LY.AD["Y"], a]) - sz // 2
            paint(scene, x, y, sz, sz, 3 if view.ai[LY.AI["KIND"], a] == 1 else 4)
        nt = view.i("NROUTE")
        for i in range(nt):
            if (int(view.vis[i >> 5]) >> (i & 31)) & 1:
                sz = 2 if i < nt - 1 else 4
                paint(scene, round(P.pad + view.cx[i]) - sz // 2, round(P.pad + view.cy[i]) - sz // 2, sz, sz, 5)
        for k in range(view.i("NTL")):
            t = view.ti[:, k]
            paint(scene, int(t[LY.TI["RX"]]), int(t[LY.TI["RY"]]), int(t[LY.TI["RW"]]), int(t[LY.TI["RH"]]),
                  int(t[LY.TI["COLOR"]]))
    xm, ym = crop_origin(P, view.h("X"), view.h("Y"))
    crop = scene[ym:ym + P.crop, xm:xm + P.crop]
    out = rotate_compose(P, crop, view.h("YAW"), reset)
    hx, hy = P.anchor_x - P.hero_w // 2, P.anchor_y - P.hero_w // 2
    paint(out, hx, hy, P.hero_w, P.hero_w, BLACK)
    return out
