"""Worst-case LDS bytes of one k_raster tile window over every heading
(carlabev_env_amd/csrc/cbev.hip, Tiles::lds_bytes).

A tile of TC x TR output pixels samples the crop at an affine map of its
pixels: the corners' samples are (TC - 1, TR - 1) steps of the rotated unit
vectors apart, so the window (in the orientation k_raster picks: rows along
the axis the output rows run closer to) spans at most floor(extent) + 2 texels
each way. A row of the window is the 16-texel chunks covering its texels at
any start offset (the staging reads the nibble map from 8-texel boundaries),
16 bytes each in LDS, plus 4 bytes (an odd dword count per row).
"""
import math


def bound(tc: int, tr: int, step_deg: float = 0.01):
    best, arg = 0, None
    for i in range(int(round(90 / step_deg)) + 1):
        th = math.radians(i * step_deg)
        c, s = abs(math.cos(th)), abs(math.sin(th))
        if s > c:  # the transposed orientation: the same extents with the axes swapped
            c, s = s, c
        eu, ev = (tc - 1) * c + (tr - 1) * s, (tc - 1) * s + (tr - 1) * c
        nu, nv = math.floor(eu) + 2, math.floor(ev) + 2
        nc = (nu + 14) // 16 + 1  # 16-texel chunks over nu texels, at any start offset within a chunk
        b = nv * (16 * nc + 4)
        if b > best:
            best, arg = b, (i * step_deg, nu, nv, nc)
    return best, arg


if __name__ == "__main__":
    for tc, tr in ((64, 64), (128, 64), (128, 128)):
        b, arg = bound(tc, tr)
        print(f"{tc} x {tr}: {b} bytes (heading {arg[0]:.2f} deg, {arg[1]} x {arg[2]} texels, {arg[3]} chunks),"
              f" {163840 // b} workgroups per CU by LDS")
