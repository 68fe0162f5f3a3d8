"""Offline model of k_raster's LDS bank conflicts (csrc/cbev.hip tile_out):
for a heading, the window layout and a lane -> pixel mapping, the extra LDS
cycles of the 16 byte gathers of every wave chunk, by the ds_read_b32 rule of
MI355X_MICROARCH.md §LDS (two 32-lane groups, bank = dword mod 32, one cycle
per extra distinct dword on a bank; lanes reading the same dword share it).
ds_read_u8 is assumed to bank like ds_read_b32 (SQ_LDS_BANK_CONFLICT on the
GPU is the check). Usage: python tools/lds_conflict_sim.py
"""
from __future__ import annotations

import math

import numpy as np

TC, TR = 128, 128


def rot(theta_deg, C=182, S=128, anchor=64):
    """pygame rotozoom constants (cbev.hip rot_setup) for the crop C."""
    rad = theta_deg * 0.017453292519943295
    sn, cs = math.sin(rad), math.cos(rad)
    m1 = max(abs(cs * C + sn * C), abs(cs * C - sn * C))
    m2 = max(abs(sn * C + cs * C), abs(sn * C - cs * C))
    nx, ny = int(m1), int(m2)
    isin, icos = int(sn * 65536), int(cs * 65536)
    xd, yd = (C - nx) * 32768, (C - ny) * 32768
    axf = (nx << 15) - int(cs * ((nx - 1) << 15))
    ayf = (ny << 15) - int(sn * ((nx - 1) << 15))
    icy = ny // 2
    dx00 = axf + isin * icy + xd
    dy00 = ayf - icos * icy + yd
    return dict(isin=isin, icos=icos, dx00=dx00, dy00=dy00, rx0=anchor - nx // 2, ry0=anchor - ny // 2)


def samples(R, X, Y):
    xx, yy = X - R["rx0"], Y - R["ry0"]
    sx = R["dx00"] + xx * R["icos"] - yy * R["isin"]
    sy = R["dy00"] + xx * R["isin"] + yy * R["icos"]
    return sx >> 16, sy >> 16


def conflicts(theta, mapping="rows", pad=4, transpose=True, xmin=37):
    R = rot(theta)
    tr = transpose and abs(R["isin"]) > abs(R["icos"])
    lane = np.arange(64)
    if mapping == "rows":
        lrow, lcol = lane // 8, 16 * (lane % 8)
    elif mapping == "across":
        lrow, lcol = (lane & 31) >> 2, 16 * ((lane & 3) + 4 * (lane >> 5))
    elif mapping == "stagger":  # row r of a half-wave starts its 8 groups at group (2 r) mod 8
        r = lane // 8
        lrow, lcol = r, 16 * ((lane % 8 + 2 * r) % 8)
    elif mapping == "c32":  # a half-wave = 32 rows of one column group (wave 0: groups 0, 1)
        lrow, lcol = lane & 31, 16 * (lane >> 5)
    elif mapping.startswith("col"):  # "colW": a half-wave = 16 rows x column groups {w, w + 4} (wave w)
        w = int(mapping[3:] or 0)
        k = lane & 31
        lrow, lcol = 16 * (lane >> 5) + (k & 15), 16 * (w + 4 * (k >> 4))
    else:
        raise ValueError(mapping)
    # window: bounding box of the tile (one tile = the whole 128 x 128 output)
    cx, cy = samples(R, np.array([0, TC - 1, 0, TC - 1]), np.array([0, 0, TR - 1, TR - 1]))
    u_lo, v_lo = (cy.min(), cx.min()) if tr else (cx.min(), cy.min())
    u_hi = cy.max() if tr else cx.max()
    ushift = xmin & 3
    c0 = (ushift + u_lo) >> 4
    nc = ((ushift + u_hi) >> 4) - c0 + 1
    sb = 16 * nc + pad
    ou = ushift - 16 * c0
    extra = 0
    n_instr = 0
    rows_per_chunk = 32 if mapping.startswith("col") or mapping == "c32" else 8
    for chunk in range(TR // rows_per_chunk):
        Y = chunk * rows_per_chunk + lrow
        for b in range(16):
            X = lcol + b
            sx, sy = samples(R, X, Y)
            u, v = (sy, sx) if tr else (sx, sy)
            addr = (v - v_lo) * sb + ou + u
            dw = addr // 4
            for half in (slice(0, 32), slice(32, 64)):
                d = np.unique(dw[half])
                banks = np.bincount(d % 32, minlength=32)
                extra += banks.max() - 1
            n_instr += 1
    return extra / n_instr  # extra cycles per gather instruction (2 halves; conflict-free = 0)


if __name__ == "__main__":
    thetas = np.arange(0.0, 360.0, 2.5)
    for mapping in ("rows", "across", "stagger"):
        for pad in (4, 12, 20, 36):
            for transpose in (False, True):
                e = np.array([conflicts(t, mapping, pad, transpose) for t in thetas])
                print(f"{mapping:8s} pad {pad:2d} transposed {int(transpose)}: extra cycles per gather mean "
                      f"{e.mean():5.2f} (0 deg {e[0]:.1f}, 5 deg {e[2]:.1f}, 45 deg {e[18]:.1f}, 90 deg {e[36]:.1f})")


def best_per_heading(thetas, pads=(4, 12, 20, 28, 36, 44, 52, 60), mappings=("rows", "across")):
    """Per heading the (mapping, pad) with the fewest modelled extra cycles."""
    out = []
    for t in thetas:
        best = min((conflicts(t, m, p, True), m, p) for m in mappings for p in pads)
        out.append(best)
    return out
