"""CPU restatement of the reference's observation-wrapper stack (NumPy).

TEST INFRASTRUCTURE ONLY — importable by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg; the product package never imports it. It is the
checker for the device expansion/resize kernels (`cbev_expand_obs`,
`cbev_resize_obs`, include/cbev.h).

The wrapper order is `wrap_env` (CarlaBEV/envs/__init__.py:62-83):
  ResizeObservation(obs_size) -> SemanticMaskWrapper | GrayscaleObservation
  -> FrameStackObservation(frame_stack) -> Flatten | VehicleTemporalFusion
  | WeightedVehicleHistory.

Pinning:
  * rgb_to_semantic_mask / flatten / both fusions follow
    CarlaBEV/wrappers/rgb_to_semantic.py and are pinned against vectors captured
    from the reference itself (tests/golden/wrappers.npz,
    tests/golden/make_golden_wrappers.py).
  * grayscale (gymnasium 1.2.2 GrayscaleObservation) and resize (gymnasium
    ResizeObservation -> cv2.resize INTER_AREA, opencv 4.11) live in third-party
    packages that are not installed here; they are restated
    from those packages' published algorithms: **parity unpinned**.
"""
from __future__ import annotations

import math

import numpy as np

# CarlaBEV/semantics.py:19-28 (semantic colours) and the palette ids of
# include/cbev_layout.h CBEV_PX_* (NON_DRIVABLE .. TL_UNKNOWN)
PALETTE = np.array([
    (150, 150, 150), (255, 255, 255), (220, 220, 220), (0, 7, 175), (255, 0, 0), (0, 255, 0),
    (255, 64, 64), (255, 255, 0), (0, 0, 0), (100, 100, 100),
], dtype=np.uint8)

WHITE, RED, RED_LIGHT, BLUE, GREEN, GRAY, GRAYS = (
    (255, 255, 255), (255, 0, 0), (255, 64, 64), (0, 7, 175), (0, 255, 0), (150, 150, 150), (220, 220, 220))

SEMANTIC_MASK_CHANNELS = {  # rgb_to_semantic.py:5-41
    "binary": ("drivable",),
    "2-class": ("drivable", "route"),
    "4-class": ("drivable", "vehicle", "pedestrian", "route"),
    "5-class": ("drivable", "sidewalk", "vehicle", "pedestrian", "route"),
    "6-class": ("non_drivable", "drivable", "sidewalk", "vehicle", "pedestrian", "route"),
    "7-class": ("non_drivable", "drivable", "sidewalk", "vehicle", "pedestrian", "route", "traffic_light_red"),
}


def vehicle_channel_index(mode: str) -> int:
    """rgb_to_semantic.py:55-62."""
    return SEMANTIC_MASK_CHANNELS[mode].index("vehicle")


def rgb_to_semantic_mask(rgb: np.ndarray, mode: str = "6-class") -> np.ndarray:
    """rgb_to_semantic.py:65-142: exact colour matches, (C, H, W) float32."""
    rgb = np.asarray(rgb, dtype=np.uint8)

    def eq(c):
        return np.all(rgb == np.array(c, np.uint8), axis=-1)

    is_white, is_red, is_red_light, is_blue = eq(WHITE), eq(RED), eq(RED_LIGHT), eq(BLUE)
    is_green, is_gray, is_grays = eq(GREEN), eq(GRAY), eq(GRAYS)
    drivable = is_white | is_green
    planes = {"non_drivable": is_gray, "drivable": drivable, "sidewalk": is_grays, "vehicle": is_blue,
              "pedestrian": is_red, "route": is_green, "traffic_light_red": is_red_light}
    return np.stack([planes[c] for c in SEMANTIC_MASK_CHANNELS[mode]]).astype(np.float32)


def flatten_stacked_frames(obs: np.ndarray) -> np.ndarray:
    """rgb_to_semantic.py:145-149: (F, C, H, W) -> (F*C, H, W)."""
    s = np.asarray(obs, np.float32)
    return s.reshape(-1, *s.shape[2:])


def fuse_vehicle_temporal(obs: np.ndarray, mode: str, history_frames: int = 3) -> np.ndarray:
    """rgb_to_semantic.py:152-166: current frame without the vehicle channel, then
    vehicle_t, vehicle_t-1, vehicle_t-2."""
    s = np.asarray(obs, np.float32)
    v = vehicle_channel_index(mode)
    hist = s[-history_frames:]
    static = np.delete(hist[-1], v, axis=0)
    return np.concatenate([static, hist[::-1, v]], axis=0).astype(np.float32)


def fuse_weighted_vehicle(obs: np.ndarray, mode: str, weights=(1.0, 0.5, 0.25)) -> np.ndarray:
    """rgb_to_semantic.py:169-191: static channels of the current frame, then
    clip(sum_k w_k * vehicle_{t-k}, 0, 1) accumulated in float32 in that order."""
    s = np.asarray(obs, np.float32)
    v = vehicle_channel_index(mode)
    hist = s[-len(weights):][::-1]
    static = np.delete(hist[0], v, axis=0)
    acc = np.zeros_like(hist[0][v], dtype=np.float32)
    for frame, w in zip(hist, weights):
        acc += np.float32(w) * frame[v]
    acc = np.clip(acc, 0.0, 1.0)
    return np.concatenate([static, acc[None]], axis=0).astype(np.float32)


def grayscale(rgb: np.ndarray) -> np.ndarray:
    """gymnasium 1.2.2 GrayscaleObservation.observation (keep_dim=False):
    sum(obs * [0.2125, 0.7154, 0.0721], axis=-1).astype(uint8) — float64, truncating
    cast. Parity unpinned (gymnasium is not installed)."""
    return np.sum(np.multiply(rgb, np.array([0.2125, 0.7154, 0.0721])), axis=-1).astype(np.uint8)


# ---------------------------------------------------------------- cv2.resize(INTER_AREA)
def area_tab(ssize: int, dsize: int, scale: float):
    """opencv 4.11 imgproc/src/resize.cpp computeResizeAreaTab (double arithmetic,
    float32 weights): list of (dst index, src index, alpha)."""
    tab = []
    for dx in range(dsize):
        fsx1 = dx * scale
        fsx2 = fsx1 + scale
        cell = min(scale, ssize - fsx1)
        sx1, sx2 = math.ceil(fsx1), math.floor(fsx2)
        sx2 = min(sx2, ssize - 1)
        sx1 = min(sx1, sx2)
        if sx1 - fsx1 > 1e-3:
            tab.append((dx, sx1 - 1, np.float32((sx1 - fsx1) / cell)))
        for sx in range(sx1, sx2):
            tab.append((dx, sx, np.float32(1.0 / cell)))
        if fsx2 - sx2 > 1e-3:
            tab.append((dx, sx2, np.float32(min(min(fsx2 - sx2, 1.0), cell) / cell)))
    return tab


def _round_u8(v: np.ndarray) -> np.ndarray:
    """saturate_cast<uchar>(float): cvRound (nearest, ties to even) then clamp."""
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def resize_area(img: np.ndarray, out_hw) -> np.ndarray:
    """cv2.resize(img, (w, h), interpolation=INTER_AREA) for a downscale
    (gymnasium ResizeObservation.observation). Restated from opencv 4.11
    resize.cpp (hal::resize: area-fast path for integer scales, otherwise
    ResizeArea_Invoker with float32 accumulation). Parity unpinned."""
    img = np.asarray(img, np.uint8)
    H, W = img.shape[:2]
    h, w = int(out_hw[0]), int(out_hw[1])
    if (h, w) == (H, W):
        return img.copy()
    inv_x, inv_y = w / W, h / H
    sx, sy = 1.0 / inv_x, 1.0 / inv_y
    if sx < 1 or sy < 1:
        raise NotImplementedError("INTER_AREA upscaling falls back to bilinear in OpenCV")
    ix, iy = int(round(sx)), int(round(sy))
    if abs(sx - ix) < np.finfo(float).eps and abs(sy - iy) < np.finfo(float).eps:
        # resizeAreaFast: integer cell averages. scale 2 (the SIMD op's path):
        # (a+b+c+d+2)>>2; other integer scales: saturate_cast(sum * (1.f/area)).
        blocks = img[:h * iy, :w * ix].reshape(h, iy, w, ix, -1).astype(np.int64).sum(axis=(1, 3))
        if ix == 2 and iy == 2:
            out = (blocks + 2) >> 2
        else:
            out = _round_u8(blocks.astype(np.float32) * np.float32(1.0 / (ix * iy)))
        return out.reshape(h, w, *img.shape[2:]).astype(np.uint8)
    xt, yt = area_tab(W, w, sx), area_tab(H, h, sy)
    src = img.astype(np.float32).reshape(H, W, -1)
    out = np.zeros((h, w, src.shape[2]), np.uint8)
    acc = np.zeros((w, src.shape[2]), np.float32)
    prev = yt[0][0]
    for dy, syi, beta in yt:
        buf = np.zeros((w, src.shape[2]), np.float32)
        row = src[syi]
        for dxi, sxi, alpha in xt:
            buf[dxi] = buf[dxi] + row[sxi] * alpha
        if dy != prev:
            out[prev] = _round_u8(acc)
            acc = beta * buf
            prev = dy
        else:
            acc = acc + beta * buf
    out[prev] = _round_u8(acc)
    return out.reshape(h, w, *img.shape[2:])


def wrap_obs_stack(id_frames: np.ndarray, obs_mode: str, mode: str = "6-class", obs_size=None,
                   fusion: str = "stack") -> np.ndarray:
    """The wrapped observation of one env from its F newest id frames (oldest
    first), exactly as wrap_env composes the wrappers (envs/__init__.py:62-83)."""
    frames = []
    for ids in id_frames:
        rgb = PALETTE[ids]
        if obs_size is not None:
            rgb = resize_area(rgb, obs_size)
        frames.append(rgb_to_semantic_mask(rgb, mode) if obs_mode == "bev_semantic" else grayscale(rgb))
    stacked = np.stack(frames)
    if obs_mode != "bev_semantic":
        return stacked
    if fusion == "vehicle_temporal":
        return fuse_vehicle_temporal(stacked, mode)
    if fusion == "vehicle_weighted":
        return fuse_weighted_vehicle(stacked, mode)
    return flatten_stacked_frames(stacked)


# ---------------------------------------------------------------- FOV corner mask
def _fillpoly(mask: np.ndarray, px, py) -> None:
    """pygame 2.6.1 src_c/draw.c draw_fillpoly (scanline fill, clipped to the surface):
    per scanline, intersections with the non-horizontal edges (y1 <= y < y2, or the
    last line), floor for even / ceil for odd intersection counts, sorted, filled in
    pairs; then horizontal border edges strictly between miny and maxy."""
    H, Wd = mask.shape
    n = len(px)

    def hline(x1, y, x2):
        if not 0 <= y < H:
            return
        a, b = max(min(x1, x2), 0), min(max(x1, x2), Wd - 1)
        if a <= b:
            mask[y, a:b + 1] = True

    miny, maxy = min(py), max(py)
    if miny == maxy:  # one pixel high: a line from the leftmost to the rightmost point
        hline(min(px), miny, max(px))
        return
    for y in range(miny, maxy + 1):
        xs = []
        for i in range(n):
            ip = i - 1 if i else n - 1
            y1, y2 = py[ip], py[i]
            if y1 < y2:
                x1, x2 = px[ip], px[i]
            elif y1 > y2:
                y2, y1 = py[ip], py[i]
                x2, x1 = px[ip], px[i]
            else:
                continue
            if (y1 <= y < y2) or (y == maxy and y2 == maxy):
                t = np.float32((y - y1) * (x2 - x1) / np.float32(y2 - y1))
                t = np.float32(math.floor(t)) if len(xs) % 2 == 0 else np.float32(math.ceil(t))
                xs.append(int(t) + x1)
        xs.sort()
        for k in range(0, len(xs) - 1, 2):
            hline(xs[k], y, xs[k + 1])
    for i in range(n):
        ip = i - 1 if i else n - 1
        y = py[i]
        if miny < y < maxy and py[ip] == y:
            hline(px[i], y, px[ip])


def fov_mask(size: int, mask_frac: float = 0.5) -> np.ndarray:
    """FovRenderer._build_mask_surface (envs/fov.py:46-68): four opaque corner
    triangles of leg m = int(size * mask_frac); apply_mask (fov.py:96-99) blits
    them black onto the composed output before the ego is drawn (world.py:137-157).
    Returns the (size, size) bool mask. Parity unpinned (pygame is not installed)."""
    S, m = size, int(size * mask_frac)
    mask = np.zeros((S, S), bool)
    for pts in ([(0, 0), (m, 0), (0, m)], [(S, 0), (S - m, 0), (S, m)], [(0, S), (0, S - m), (m, S)],
                [(S, S), (S - m, S), (S, S - m)]):
        _fillpoly(mask, [p[0] for p in pts], [p[1] for p in pts])
    return mask
