"""Per-env state record layout (host mirror of include/cbev_layout.h).

The C header is the single source of truth: field names are parsed from its
`CBEV_*_FIELDS` lists, and the group offsets are recomputed with the same
arithmetic as `cbev_make_layout` (tests/test_layout.py checks both against the
values the built C-ABI library exports).
"""
from __future__ import annotations

import ctypes
import os
import re
from dataclasses import dataclass

import numpy as np

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(_REPO, "include", "cbev_layout.h")


def _parse_fields(text: str, group: str) -> list[str]:
    lines = text.split("\n")
    start = next((i for i, ln in enumerate(lines) if ln.startswith(f"#define CBEV_{group}_FIELDS(F_)")), None)
    if start is None:
        raise RuntimeError(f"cannot find CBEV_{group}_FIELDS in {HEADER}")
    body = []
    for ln in lines[start:]:
        body.append(ln.split("#define", 1)[-1] if ln is lines[start] else ln)
        if not ln.rstrip().endswith("\\"):
            break
    joined = re.sub(r"/\*.*?\*/", " ", "\n".join(body), flags=re.S)
    joined = joined.replace(f"CBEV_{group}_FIELDS(F_)", "")
    return re.findall(r"F_\((\w+)\)", joined)


def _load_names():
    with open(HEADER, "r", encoding="utf-8") as f:
        text = f.read()
    return {g: _parse_fields(text, g) for g in ("HD", "HI", "AD", "AI", "TI", "EP")}


NAMES = _load_names()
HD = {n: i for i, n in enumerate(NAMES["HD"])}
HI = {n: i for i, n in enumerate(NAMES["HI"])}
AD = {n: i for i, n in enumerate(NAMES["AD"])}
AI = {n: i for i, n in enumerate(NAMES["AI"])}
TI = {n: i for i, n in enumerate(NAMES["TI"])}
EP = {n: i for i, n in enumerate(NAMES["EP"])}  # episode summary row columns (CBEV_EP_FIELDS)
STATS_BYTES = 1856                              # sizeof(cbev_episode_stats)
ACB_PTS = int(re.search(r"#define CBEV_ACB_PTS (\d+)", open(HEADER).read()).group(1))  # points per pruning circle

# enums mirrored from the header (values are part of the C-ABI)
BEH = {"none": 0, "timed_brake": 1, "cross": 2, "stop_mid": 3, "yield_return": 4}
BSTATE = {"idle": 0, "waiting": 1, "entering": 2, "yielding": 3, "stalled": 4, "crossing": 5,
          "cleared": 6, "retreating": 7, "retreated": 8}
CAUSE = {None: 0, "collision": 1, "success": 2, "ckpt": 3, "out_of_bounds": 4, "max_actions": 5,
         "off_road": 6, "unknown": 7}
CAUSE_NAME = {v: k for k, v in CAUSE.items()}
COLL = {None: 0, "vehicle": 1, "pedestrian": 2, "target": 3}
COLL_NAME = {v: k for k, v in COLL.items()}


class CbevCaps(ctypes.Structure):
    _fields_ = [("route_cap", ctypes.c_int32), ("actor_cap", ctypes.c_int32),
                ("actor_route_cap", ctypes.c_int32), ("tl_cap", ctypes.c_int32)]


class CbevLayout(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in (
        "hd", "hi", "cx", "cy", "cyaw", "raw_x", "raw_y", "raw_cum", "vis", "ad", "ai",
        "acx", "acy", "acyaw", "aix", "aiy", "arx", "ary", "ti", "acf", "acb", "record_bytes")] + [
        ("vis_words", ctypes.c_int32), ("pad", ctypes.c_int32)]


def _align(v: int, a: int) -> int:
    return (v + a - 1) // a * a


@dataclass(frozen=True)
class Caps:
    route_cap: int
    actor_cap: int
    actor_route_cap: int
    tl_cap: int

    def c(self) -> CbevCaps:
        return CbevCaps(self.route_cap, self.actor_cap, self.actor_route_cap, self.tl_cap)


@dataclass(frozen=True)
class Layout:
    caps: Caps
    off: dict
    record_bytes: int
    vis_words: int

    @staticmethod
    def make(caps: Caps) -> "Layout":
        R, A, RA, T = caps.route_cap, caps.actor_cap, caps.actor_route_cap, caps.tl_cap
        off = {}
        o = 0

        def put(name, nbytes):
            nonlocal o
            off[name] = o
            o = _align(o + nbytes, 64)

        put("hd", 8 * len(HD))
        put("hi", 4 * len(HI))
        put("cx", 8 * R)
        put("cy", 8 * R)
        put("cyaw", 8 * R)
        put("raw_x", 4 * R)
        put("raw_y", 4 * R)
        put("raw_cum", 8 * R)
        vis_words = (R + 31) // 32
        put("vis", 8 * vis_words)  # vis, then vis_draw
        put("ad", 8 * len(AD) * A)
        put("ai", 4 * len(AI) * A)
        for n in ("acx", "acy", "acyaw", "aix", "aiy", "arx", "ary"):
            put(n, 8 * A * RA)
        put("ti", 4 * len(TI) * T)
        put("acf", 8 * A * RA)  # acx / acy as float32 pairs (the actor target search's first pass)
        put("acb", 8 * A * ((RA + ACB_PTS - 1) // ACB_PTS))  # pruning circles of acf's point blocks
        return Layout(caps, off, _align(o, 256), vis_words)


def check_library_layout(L, caps: Caps) -> "Layout":
    """This header's layout for `caps`, refused unless the loaded library (L, the
    ctypes handle) computes the same one: a library built from another version of
    include/cbev_layout.h would read records of a different shape."""
    py = Layout.make(caps)
    out = CbevLayout()
    rc = L.cbev_layout_of(ctypes.byref(caps.c()), ctypes.byref(out))
    bad = [n for n, o in py.off.items() if getattr(out, n) != o]
    if rc != 0 or bad or out.record_bytes != py.record_bytes or out.vis_words != py.vis_words:
        raise RuntimeError(f"the loaded libcbev.so lays records out differently from {HEADER} "
                           f"({', '.join(bad) or 'record_bytes'}): rebuild it (python -m carlabev_env_amd.build)")
    return py


class RecordView:
    """Named numpy views into one record (a writable uint8 buffer)."""

    def __init__(self, buf: np.ndarray, layout: Layout):
        assert buf.dtype == np.uint8 and buf.size >= layout.record_bytes
        c, o = layout.caps, layout.off
        R, A, RA, T = c.route_cap, c.actor_cap, c.actor_route_cap, c.tl_cap

        def v(name, dtype, shape):
            n = int(np.prod(shape)) * np.dtype(dtype).itemsize
            return buf[o[name]:o[name] + n].view(dtype).reshape(shape)

        self.hd = v("hd", np.float64, (len(HD),))
        self.hi = v("hi", np.int32, (len(HI),))
        self.cx = v("cx", np.float64, (R,))
        self.cy = v("cy", np.float64, (R,))
        self.cyaw = v("cyaw", np.float64, (R,))
        self.raw_x = v("raw_x", np.int32, (R,))
        self.raw_y = v("raw_y", np.int32, (R,))
        self.raw_cum = v("raw_cum", np.float64, (R,))
        self.vis = v("vis", np.uint32, (layout.vis_words,))
        self.vis_draw = buf[o["vis"] + 4 * layout.vis_words:o["vis"] + 8 * layout.vis_words].view(np.uint32)
        self.ad = v("ad", np.float64, (len(AD), A))
        self.ai = v("ai", np.int32, (len(AI), A))
        self.acx = v("acx", np.float64, (A, RA))
        self.acy = v("acy", np.float64, (A, RA))
        self.acyaw = v("acyaw", np.float64, (A, RA))
        self.aix = v("aix", np.float64, (A, RA))
        self.aiy = v("aiy", np.float64, (A, RA))
        self.arx = v("arx", np.float64, (A, RA))
        self.ary = v("ary", np.float64, (A, RA))
        self.ti = v("ti", np.int32, (len(TI), T))
        self.acf = v("acf", np.float32, (A, RA, 2))
        self.acb = v("acb", np.uint32, (A, (RA + ACB_PTS - 1) // ACB_PTS, 2))

    def h(self, name):
        return self.hd[HD[name]]

    def i(self, name):
        return int(self.hi[HI[name]])


def batch_views(buf: np.ndarray, layout: Layout, n: int) -> dict:
    """Strided numpy views of the same field across n consecutive records."""
    rb = layout.record_bytes
    assert buf.size >= n * rb
    base = buf[: n * rb].reshape(n, rb)
    out = {}
    o = layout.off
    out["hd"] = base[:, o["hd"]:o["hd"] + 8 * len(HD)].view(np.float64)
    out["hi"] = base[:, o["hi"]:o["hi"] + 4 * len(HI)].view(np.int32)
    return out


def retreat_route_violations(hi: np.ndarray, ai: np.ndarray, caps: Caps) -> np.ndarray:
    """Records whose StopReturn (yield_return) actor would rebuild a retreat
    route longer than the narrow k_actors rebuilds (64 points, one per lane;
    contexts of at most 64 actor slots): hi = int32[n][HI_COUNT], ai =
    int32[n][AI_COUNT][A] of n records. scene_pack refuses such actors when it
    packs a scene; this check covers records written any other way (the kernel
    would only flag CBEV_ERR_RETREAT_ROUTE and keep the actor's old route)."""
    if caps.actor_cap == 0 or caps.actor_cap > 64:
        return np.zeros(hi.shape[0], bool)
    nact = hi[:, HI["NACT"]]
    live = np.arange(caps.actor_cap)[None, :] < nact[:, None]
    bad = (ai[:, AI["BEH"], :] == BEH["yield_return"]) & (ai[:, AI["NRX"], :] + 1 > min(caps.actor_route_cap, 64))
    return (bad & live).any(axis=1)


def acb_circles(pts: np.ndarray) -> np.ndarray:
    """The pruning circles (acb) of an actor's float32 route points pts[n][2]:
    per block of ACB_PTS points, the bounding box's centre in 1/8 px fixed point
    and the largest distance of a point from that (quantised) centre, rounded up
    to 1/8 px plus 1/8 px. uint32[ceil(n / ACB_PTS)][2] (cbev_layout.h acb)."""
    n = len(pts)
    out = np.zeros(((n + ACB_PTS - 1) // ACB_PTS, 2), np.uint32)
    p = pts.astype(np.float64)
    for b in range(len(out)):
        q = p[ACB_PTS * b: ACB_PTS * (b + 1)]
        cq = np.clip(np.rint((q.min(0) + q.max(0)) * 0.5 * 8.0) + 32768, 0, 65535).astype(np.int64)
        c = (cq - 32768) / 8.0
        r = float(np.max(np.hypot(q[:, 0] - c[0], q[:, 1] - c[1])))
        out[b, 0] = int(cq[0]) | (int(cq[1]) << 16)
        out[b, 1] = int(np.ceil(r * 8.0)) + 1
    return out
