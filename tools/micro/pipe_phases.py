"""Phase timing of k_raster_pipe from in-kernel s_memtime stamps (timing build,
-DCBEV_TIMING): per item of every workgroup, the cycles of the DMA wait +
barrier, the paint, the next item's set-up + DMA issue and the output, and the
launch span. Usage (GPU box): python tools/micro/pipe_phases.py [--config 2] [--defs ...]
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
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--defs", default="")
    ap.add_argument("--so", default=None, help="prebuilt timing library")
    a = ap.parse_args()
    sys.path.insert(0, REPO)
    so = a.so
    if so is None:
        so = os.path.join(REPO, "gpurun_out", "libcbev_ptiming.so")
        os.makedirs(os.path.dirname(so), exist_ok=True)
        from carlabev_env_amd import build as B  # noqa: E402
        subprocess.run([B.HIPCC, *B.FLAGS, "-DCBEV_TIMING", *a.defs.split(), "-o", so, B.SRC], check=True)
    os.environ["CBEV_LIB"] = so
    import torch  # noqa: E402

    import bench  # noqa: E402
    from carlabev_env_amd._lib import lib  # noqa: E402

    cfgd = bench.CONFIGS[a.config]
    n = cfgd["envs"]
    env, host, start = bench.build_env(cfgd, n, 0, torch.device("cuda", 0))
    acts = torch.from_numpy(bench.make_actions(env.params, n, a.steps, cfgd["act_seed"], 0)).cuda()
    L = lib()
    L.cbev_debug_pipe_times.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    env.auto_obs = False
    for t in range(a.steps):
        env.step_async_only(acts[t])
        env.reset_terminated()
    torch.cuda.synchronize()
    st = np.zeros((1024, 32, 5), np.uint64)
    hw = np.zeros(1024, np.uint32)
    assert L.cbev_debug_pipe_times(st.ctypes.data, hw.ctypes.data) == 0
    st = st.astype(np.int64)
    used = st[:, :31, 1] > 0
    nwg = int((st[:, 31, 4] > 0).sum())
    t0 = st[:nwg, 31, 4].min()
    items = used[:nwg].sum(1)
    print(f"config {a.config}: {nwg} workgroups, items per workgroup {items.min()}..{items.max()}")
    ph = ["wait+barrier", "paint", "issue next", "output"]
    for k, name in enumerate(ph):
        d = st[:nwg, :31, k + 1] - st[:nwg, :31, k]
        v = d[used[:nwg]]
        print(f"  {name:14s} mean {v.mean():8.0f}  p50 {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f} cycles")
    first = st[:nwg, 0, 1] - st[:nwg, 31, 4]
    print(f"  prologue (start -> first item ready) mean {first.mean():.0f} cycles")
    ends = np.array([st[w, items[w] - 1, 4] for w in range(nwg)])
    starts = st[:nwg, 31, 4]
    print(f"  workgroup start spread {np.ptp(starts)} cycles; end spread {np.ptp(ends)}; span {ends.max() - t0} cycles")
    per = (ends - starts) / np.maximum(items, 1)
    print(f"  cycles per item (workgroup lifetime / items): mean {per.mean():.0f}")
    cu = (hw[:nwg] >> 8) & 0xF
    se = (hw[:nwg] >> 13) & 0x7
    print("  HW_ID of the first 8 workgroups:", [hex(x) for x in hw[:8]])


if __name__ == "__main__":
    main()
