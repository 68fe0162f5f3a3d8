"""Phase timing of k_ego (and k_raster / k_actors) from
in-kernel s_memtime stamps. Builds a -DCBEV_TIMING variant of libcbev.so into
gpurun_out/, runs config-2 steps through bench.build_env and prints, per
kernel, the mean cycles of stage-in / compute / write-back over workgroups and
the launch span. Usage (GPU box): python tools/micro/step_phases.py [--config 2]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np


def main():
    REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--defs", default="")
    ap.add_argument("--reset", action="store_true", help="canonical loop: reset the terminated envs from the bank each step")
    ap.add_argument("--src", default=None, help="a variant of csrc/cbev.hip (same directory) instead of the product source")
    a = ap.parse_args()
    so = os.path.join(REPO, "gpurun_out", "libcbev_timing.so")
    os.makedirs(os.path.dirname(so), exist_ok=True)
    sys.path.insert(0, REPO)
    from carlabev_env_amd import build as B  # noqa: E402

    subprocess.run([B.HIPCC, *B.FLAGS, "-DCBEV_TIMING", *a.defs.split(), "-o", so, a.src or B.SRC], check=True)
    os.environ["CBEV_LIB"] = so
    sys.path.insert(0, REPO)
    import torch  # noqa: E402

    import bench  # noqa: E402
    from carlabev_env_amd._lib import lib  # noqa: E402

    cfgd = bench.CONFIGS[a.config]
    n = cfgd["envs"]
    env, host, start = bench.build_env(cfgd, n, 0, torch.device("cuda", 0))
    acts = torch.from_numpy(bench.make_actions(env.params, n, a.steps, cfgd["act_seed"], 0)).cuda()
    L = lib()
    L.cbev_debug_times.argtypes = [ctypes.c_void_p]
    L.cbev_debug_occupancy.argtypes = [ctypes.c_int, ctypes.c_int]
    for b in (10560, 22688, 24576, 38384):
        print(f"raster occupancy API (size {cfgd['size']}, {b} B LDS): {L.cbev_debug_occupancy(cfgd['size'], b)} WGs/CU")
    env.auto_obs = False
    for t in range(a.steps):
        env.step_async_only(acts[t])
        if a.reset:
            env.reset_terminated()
    torch.cuda.synchronize()
    NS = 7
    buf = np.zeros(2 * NS * 4096 * 4 + NS * 4096, np.uint64)
    assert L.cbev_debug_times(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    xcc = buf[2 * NS * 4096 * 4:].reshape(NS, 4096).astype(np.int64)
    hwid = xcc >> 32
    xcc = xcc & 0xFFFFFFFF
    buf = buf[:2 * NS * 4096 * 4].reshape(2, NS, 4096, 4)
    for k, name in enumerate(("k_ego A: stage-in / S1+S2 search / S3 chain + S4", "k_ego B: S5 collision pre-pass / S6 collide chain / stage-out", "k_raster", "k_ego wave 0: DMA issued / S1 done / S2 min / S2 done", "collide_env(thread0)", "k_ego S5 (wave 0): segs / lateral / reduce / targets", "k_actors: behaviour / search / stanley+update (per wave)")):
        if not (buf[0, k, :, 0] > 0).any():
            continue
        st = buf[0, k].astype(np.int64)
        rt = buf[1, k].astype(np.int64)
        used = st[:, 0] > 0
        st, rt = st[used], rt[used]
        print(f"{name}: realtime (100 MHz) launch span {(rt[:, 3].max() - rt[:, 0].min()) / 100:.2f} us, "
              f"WG mean {(rt[:, 3] - rt[:, 0]).mean() / 100:.2f} us, first start->last start "
              f"{(rt[:, 0].max() - rt[:, 0].min()) / 100:.2f} us; clock {((st[:, 3] - st[:, 0]).sum() / max((rt[:, 3] - rt[:, 0]).sum(), 1)) / 100:.2f} GHz")
        d = np.diff(st, axis=1)
        if k in (3, 5):  # cycles since the start of k_ego A (3) / B (5) in the same workgroup
            ref = buf[0, 0 if k == 3 else 1].astype(np.int64)[used][:, 0]
            print(f"{name}: cycles since the phase start: {[round(float((st[:, j] - ref).mean())) for j in range(4)]}")
            print(f"   p50 {[round(float(np.percentile(st[:, j] - ref, 50))) for j in range(4)]} "
                  f"p90 {[round(float(np.percentile(st[:, j] - ref, 90))) for j in range(4)]} "
                  f"max {[round(float((st[:, j] - ref).max())) for j in range(4)]}")
            continue
        print(f"{name}: {used.sum()} WGs; cycles mean phase1 {d[:, 0].mean():.0f} (max {d[:, 0].max():.0f})  phase2 {d[:, 1].mean():.0f} "
              f"(max {d[:, 1].max():.0f})  phase3 {d[:, 2].mean():.0f}; WG total mean {(st[:, 3] - st[:, 0]).mean():.0f}; "
              )
        tot = st[:, 3] - st[:, 0]
        ends = (rt[:, 3] - rt[:, 0].min()) / 100
        print(f"   WG cycles p10/p50/p90/p99/max {np.percentile(tot, [10, 50, 90, 99]).round().tolist()} {tot.max()}; "
              f"end time (us after the first start) p50 {np.percentile(ends, 50):.2f} p90 {np.percentile(ends, 90):.2f} "
              f"p99 {np.percentile(ends, 99):.2f} max {ends.max():.2f}")
        idx = np.flatnonzero(used)
        xs = xcc[k][used] & 0xF
        print(f"   XCC id: workgroups with xcc == w % 8: {(xs == (idx % 8)).mean() * 100:.1f}%; first 16: {list(xs[:16])}")
        # residency: workgroups live at once on one CU (XCC, SE, SH, CU from HW_ID), from the realtime stamps
        hw = hwid[k][used]
        cu = (xs << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
        peak = []
        for c in np.unique(cu):
            m = cu == c
            ev = sorted([(t, 1) for t in rt[m, 0]] + [(t, -1) for t in rt[m, 3]], key=lambda z: (z[0], z[1]))
            live = best = 0
            for _, dlt in ev:
                live += dlt
                best = max(best, live)
            peak.append((best, m.sum()))
        peak = np.array(peak)
        print(f"   CUs used {len(peak)}; WGs per CU mean {peak[:, 1].mean():.1f} (max {peak[:, 1].max()}); "
              f"peak resident WGs per CU mean {peak[:, 0].mean():.2f} (min {peak[:, 0].min()}, max {peak[:, 0].max()})")
        for x in range(8):  # s_memtime is per XCD: spans within one XCD (workgroup w runs on XCD w % 8)
            m = (idx % 8) == x
            if m.any():
                sx = st[m]
                print(f"   xcd {x}: WGs {m.sum()} span {sx[:, 3].max() - sx[:, 0].min()} start-spread {sx[:, 0].max() - sx[:, 0].min()}")



if __name__ == "__main__":
    main()
