"""k_raster time against the ego heading: the config's bench scenes with every
ego yaw set to one angle, one cbev_step (render set-up for that heading), then
cbev_profile_raster over --reps back-to-back launches. Shows how the gathers'
LDS bank conflicts depend on the orientation (rows vs columns of the image).
Usage (GPU box): python tools/micro/raster_orient.py [--config 2]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import numpy as np


def main():
    REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, REPO)

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--angles", default="0,3,10,30,45,60,80,87,90")
    ap.add_argument("--burn", type=int, default=200, help="canonical-loop steps before the sweep (envs spread over the map)")
    a = ap.parse_args()

    import torch  # noqa: E402

    import bench  # noqa: E402
    from carlabev_env_amd import layout as LY  # noqa: E402
    from carlabev_env_amd._lib import check, lib  # noqa: E402

    L0 = lib()
    cfgd = bench.CONFIGS[a.config]
    n = cfgd["envs"]
    dev = torch.device("cuda", 0)
    # a stream of its own: launches on HIP's legacy default stream carry an
    # implicit synchronisation of several us each (bench.py does the same)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    env, host, _start = bench.build_env(cfgd, n, 0, dev)
    acts = torch.zeros((n,), dtype=torch.int32, device=dev) if env.params.action_kind == 0 else \
        torch.zeros((n, 3), dtype=torch.float32, device=dev)
    env.auto_obs = False
    if a.burn:
        ra = torch.from_numpy(bench.make_actions(env.params, n, a.burn, cfgd["act_seed"], 0)).to(dev)
        for t in range(a.burn):
            env.step_async_only(ra[t])
            env.reset_terminated()
        torch.cuda.synchronize()
    base = env.records.clone()
    for _ in range(20):  # ~0.5 s of launches: the GPU at its steady clocks before anything is timed
        check(L0.cbev_profile_raster(env._ctx, env.records.data_ptr(), n, env.frames().data_ptr(), 1000,
                                     env._stream(), ctypes.byref(ctypes.c_double())), "profile_raster")
    ms0 = ctypes.c_double()
    check(L0.cbev_profile_raster(env._ctx, env.records.data_ptr(), n, env.frames().data_ptr(), a.reps, env._stream(),
                                 ctypes.byref(ms0)), "profile_raster")
    print(f"after the burn-in, headings as they are: raster {ms0.value * 1e3:6.2f} us/launch", flush=True)
    L = lib()
    yaw_off = env.layout.off["hd"] + 8 * LY.HD["YAW"]
    ms = ctypes.c_double()
    for deg in [float(x) for x in a.angles.split(",")]:
        env.records.copy_(base)
        r = env.records.view(n, -1)
        yaw = torch.full((n,), np.radians(deg), dtype=torch.float64, device=dev)
        r[:, yaw_off:yaw_off + 8] = yaw.view(torch.uint8).view(n, 8)
        env.step_async_only(acts)
        torch.cuda.synchronize()
        times = []
        for _ in range(3):
            check(L.cbev_profile_raster(env._ctx, env.records.data_ptr(), n, env.frames().data_ptr(), a.reps, env._stream(),
                                        ctypes.byref(ms)), "profile_raster")
            times.append(ms.value * 1e3)  # ms per launch
        print(f"heading {deg:5.1f} deg: raster {np.median(times):6.2f} us/launch", flush=True)



if __name__ == "__main__":
    main()
