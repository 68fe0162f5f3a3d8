"""Phase timing of the staged thread-per-env kernels (k_hero, k_collide) from
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

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=2)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--defs", default="")
a = ap.parse_args()
so = os.path.join(REPO, "gpurun_out", "libcbev_timing.so")
os.makedirs(os.path.dirname(so), exist_ok=True)
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
                "-ffp-contract=off", "-fno-fast-math", f"-I{REPO}/include", "-DCBEV_TIMING", *a.defs.split(),
                "-o", so, f"{REPO}/carlabev_env_amd/csrc/cbev.hip"], check=True)
os.environ["CBEV_LIB"] = so
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from carlabev_env_amd._lib import lib  # noqa: E402

cfgd = bench.CONFIGS[a.config]
n = cfgd["envs"]
env, host = bench.build_env(cfgd, n, 0, torch.device("cuda", 0))
acts = torch.from_numpy(bench.make_actions(env.params, n, a.steps, cfgd["act_seed"], 0)).cuda()
L = lib()
L.cbev_debug_times.argtypes = [ctypes.c_void_p]
for t in range(a.steps):
    env.step_async_only(acts[t])
torch.cuda.synchronize()
buf = np.zeros((2, 4096, 4), np.uint64)
assert L.cbev_debug_times(buf.ctypes.data_as(ctypes.c_void_p)) == 0
for k, name in enumerate(("k_hero", "k_collide")):
    st = buf[k].astype(np.int64)
    used = st[:, 0] > 0
    st = st[used]
    d = np.diff(st, axis=1)
    print(f"{name}: {used.sum()} WGs; cycles mean stage_in {d[:, 0].mean():.0f}  compute {d[:, 1].mean():.0f} "
          f"(max {d[:, 1].max():.0f})  write_back {d[:, 2].mean():.0f}; WG total mean {(st[:, 3] - st[:, 0]).mean():.0f}; "
          f"launch span {st[:, 3].max() - st[:, 0].min()} cycles; start spread {st[:, 0].max() - st[:, 0].min()}")
