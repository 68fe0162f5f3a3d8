"""k_reset_copy in isolation: launch time against the number of envs reset.

Config 3 shapes (4096 envs, caps 64/25/64/0, a 4-frame ring, 512-entry bank
whose actor routes hold 29 of 64 points), masks with 0 / 41 / 183 / 410 / 4096
envs selected, HIP events around 200 back-to-back launches each.
Run: python tools/micro/reset_copy_bench.py  (GPU)
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from carlabev_env_amd import layout as LY  # noqa: E402
from carlabev_env_amd._lib import check, lib  # noqa: E402
from helpers import world  # noqa: E402

P_ = ctypes.c_void_p


def ptr(t):
    return P_(t.data_ptr())


def main():
    caps = LY.Caps(64, 25, 64, 0)
    cfg, P, padded, layout, builder = world(caps=caps)
    L = lib()
    ctx = P_()
    check(L.cbev_create(ctypes.byref(P), ctypes.byref(caps.c()), 0, ctypes.byref(ctx)), "create")
    check(L.cbev_set_map(ctx, padded.ctypes.data_as(P_), padded.nbytes), "set_map")
    n, B, F, S = 4096, 512, 4, P.size
    rb = layout.record_bytes
    bank = np.random.default_rng(0).integers(0, 255, (B, rb), dtype=np.uint8)
    for b in range(B):
        v = LY.RecordView(bank[b], layout)
        for row in ("NROUTE", "NINIT", "NRX"):
            v.ai[LY.AI[row], :] = 29
    d_bank = torch.from_numpy(bank).cuda()
    d_recs = torch.zeros((n, rb), dtype=torch.uint8, device="cuda")
    bf = torch.randint(0, 10, (B, S, S), dtype=torch.uint8, device="cuda")
    ring = torch.zeros((F, n, S, S), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    for k in (0, 41, 183, 410, 4096):
        m = np.zeros(n, np.uint8)
        m[np.random.default_rng(k).choice(n, k, replace=False)] = 1
        mask = torch.from_numpy(m).cuda()
        for _ in range(10):
            check(L.cbev_reset_frames(ctx, ptr(d_recs), n, ptr(d_bank), B, ptr(mask), None, 3, ptr(bf), ptr(ring), F,
                                      P_(s.cuda_stream)), "reset_frames")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(200):
            check(L.cbev_reset_frames(ctx, ptr(d_recs), n, ptr(d_bank), B, ptr(mask), None, 3, ptr(bf), ptr(ring), F,
                                      P_(s.cuda_stream)), "reset_frames")
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1000 / 200
        print(f"resets {k:5d}: {us:7.2f} us per launch", flush=True)
    L.cbev_destroy(ctx)


if __name__ == "__main__":
    main()
