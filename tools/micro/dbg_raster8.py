"""Debug aid: one config-2 step on the GPU, per-env frame mismatches against the
oracle with the sampled texel of each bad pixel (from the record's RS_* set-up)."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "oracle")
import oracle as O  # noqa: E402
from carlabev_env_amd import layout as LY  # noqa: E402
from carlabev_env_amd._lib import check, lib  # noqa: E402
from helpers import action_stream, bench_caps, build_records, world  # noqa: E402

P_ = ctypes.c_void_p


def ptr(t):
    return P_(t.data_ptr())


def main():
    n = 48
    caps = bench_caps(2)
    cfg, P, padded, layout, builder = world(128, caps=caps)
    recs, _ = build_records(builder, n, ["rt_no_traffic_v1"], seed0=10_000)
    L = lib()
    ctx = P_()
    check(L.cbev_create(ctypes.byref(P), ctypes.byref(caps.c()), 0, ctypes.byref(ctx)), "create")
    check(L.cbev_set_map(ctx, padded.ctypes.data_as(P_), padded.nbytes), "map")
    S = P.size
    d_recs = torch.from_numpy(recs.copy()).cuda()
    d_frames = torch.zeros((n, S, S), dtype=torch.uint8, device="cuda")
    check(L.cbev_reset(ctx, ptr(d_recs), n, None, 0, None, None, 0, ptr(d_frames), 1, None), "reset")
    orc = O.Oracle(P, padded, caps.c(), layout.record_bytes)
    h = np.zeros((n, S, S), np.uint8)
    for e in range(n):
        orc.reset_obs(recs[e], h[e])
    acts = action_stream(P, n, 1, seed=1234)
    a = torch.from_numpy(np.ascontiguousarray(acts[0])).cuda()
    z = [torch.zeros(n, dtype=dt, device="cuda") for dt in (torch.float64, torch.uint8, torch.uint8, torch.int32)]
    info = torch.zeros((n, 16), dtype=torch.float32, device="cuda")
    check(L.cbev_step(ctx, ptr(d_recs), n, ptr(a), ptr(d_frames), *[ptr(t) for t in z], ptr(info), None), "step")
    for e in range(n):
        orc.step_one(recs[e], np.ascontiguousarray(acts[0, e]), h[e])
    torch.cuda.synchronize()
    df = d_frames.cpu().numpy()
    dr = d_recs.cpu().numpy()
    pitch = padded.shape[1] if padded.ndim == 2 else P.map_pitch
    pm = padded.reshape(-1, pitch) if padded.ndim == 1 else padded
    C = P.crop
    for e in range(n):
        v = LY.RecordView(dr[e], layout)
        R = {k: v.i("RS_" + k) for k in ("XMIN", "YMIN", "R90", "NX", "NY", "ISIN", "ICOS", "DX00", "DY00", "RX0", "RY0",
                                          "FAST")}
        bad = np.argwhere(df[e] != h[e])
        line = f"env {e:2d} bad {len(bad):6d} r90 {R['R90']} fast {R['FAST']} icos {R['ICOS']} isin {R['ISIN']}"
        if len(bad) and not R["R90"]:
            yy, xx = bad[:, 0] - R["RY0"], bad[:, 1] - R["RX0"]
            dx = R["DX00"] + xx * R["ICOS"] - yy * R["ISIN"]
            dy = R["DY00"] + xx * R["ISIN"] + yy * R["ICOS"]
            tx, ty = dx >> 16, dy >> 16
            # bbox of the whole output's samples
            oy, ox = np.mgrid[0:S, 0:S]
            ax = (R["DX00"] + (ox - R["RX0"]) * R["ICOS"] - (oy - R["RY0"]) * R["ISIN"]) >> 16
            ay = (R["DY00"] + (ox - R["RX0"]) * R["ISIN"] + (oy - R["RY0"]) * R["ICOS"]) >> 16
            line += f" win x[{ax.min()},{ax.max()}] y[{ay.min()},{ay.max()}] C {C} xmin {R['XMIN']}"
            dv = df[e][bad[:, 0], bad[:, 1]]
            hv = h[e][bad[:, 0], bad[:, 1]]
            mv = pm[R["YMIN"] + ty, R["XMIN"] + tx]
            line += f" | host==map {np.mean(hv == mv):.2f}"
            hits = {}
            for oyy in range(-2, 3):
                for oxx in range(-3, 4):
                    m = pm[R["YMIN"] + ty + oyy, R["XMIN"] + tx + oxx]
                    hits[(oyy, oxx)] = float(np.mean(m == dv))
            best = sorted(hits.items(), key=lambda kv: -kv[1])[:3]
            line += f" | dev==map at offsets {best}"
            line += f" | bad rows {np.unique(bad[:, 0])[:6]} cols {np.unique(bad[:, 1])[:6]} dv {np.unique(dv)[:6]}"
        print(line, flush=True)
    L.cbev_destroy(ctx)


if __name__ == "__main__":
    main()
