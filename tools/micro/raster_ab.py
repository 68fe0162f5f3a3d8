"""A/B timing of k_raster builds: every library given is loaded side by side
(ctypes), gets its own context on the same seeded bench scenes (bench.build_env
for --config), takes one cbev_step from the same records and actions, then
cbev_profile_raster times --reps back-to-back raster launches (HIP events).
Frames of every build are compared with the first one's (bit-exact). Prints
us per launch, repeated --rounds times, interleaved across builds.
Usage (GPU box): python tools/micro/raster_ab.py --config 2 --libs a.so b.so ...
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
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--burn", type=int, default=40, help="canonical-loop steps before timing (varied headings)")
    a = ap.parse_args()

    import torch  # noqa: E402

    import bench  # noqa: E402
    from carlabev_env_amd import _lib  # noqa: E402

    cfgd = bench.CONFIGS[a.config]
    n = cfgd["envs"]
    dev = torch.device("cuda", 0)
    env, host, _start = bench.build_env(cfgd, n, 0, dev)
    acts = torch.from_numpy(bench.make_actions(env.params, n, a.burn + 1, cfgd["act_seed"], 0)).to(dev)
    env.auto_obs = False
    for t in range(a.burn):
        env.step_async_only(acts[t])
        env.reset_terminated()
    torch.cuda.synchronize()
    recs0 = env.records.clone()
    P = env.params
    S = P.size
    libs = []
    for spec in a.libs:  # path[:VAR=value,...]: environment set while the library's context is created
        path, _, envs = spec.partition(":")
        saved = {}
        for kv in filter(None, envs.split(",")):
            k_, v_ = kv.split("=")
            saved[k_] = os.environ.get(k_)
            os.environ[k_] = v_
        L = ctypes.CDLL(os.path.abspath(path))
        for name in ("cbev_create", "cbev_set_map", "cbev_step", "cbev_profile_raster"):
            getattr(L, name).restype = ctypes.c_int
        L.cbev_destroy.restype = None
        ctx = ctypes.c_void_p()
        rc = L.cbev_create(ctypes.byref(P), ctypes.byref(env.caps.c()), 0, ctypes.byref(ctx))
        assert rc == 0, (path, rc)
        assert L.cbev_set_map(ctx, env.map_host.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(env.map_host.nbytes)) == 0
        for k_, v_ in saved.items():
            if v_ is None:
                os.environ.pop(k_, None)
            else:
                os.environ[k_] = v_
        libs.append((os.path.basename(path) + (":" + envs if envs else ""), L, ctx))
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    res = {name: [] for name, _, _ in libs}
    ref = None
    outs = {}
    for name, L, ctx in libs:
        recs = recs0.clone()
        fr = torch.zeros((n, S, S), dtype=torch.uint8, device=dev)
        rew = torch.zeros(n, dtype=torch.float64, device=dev)
        te = torch.zeros(n, dtype=torch.uint8, device=dev)
        tr = torch.zeros_like(te)
        ca = torch.zeros(n, dtype=torch.int32, device=dev)
        assert L.cbev_step(ctx, p(recs), n, p(acts[a.burn]), p(fr), p(rew), p(te), p(tr), p(ca), None, None) == 0
        torch.cuda.synchronize()
        outs[name] = (recs, fr)
        if ref is None:
            ref = fr.clone()
        else:
            bad = int((fr != ref).sum())
            print(f"{name}: frames differing from {libs[0][0]}: {bad}")
    for r in range(a.rounds):
        for name, L, ctx in libs:
            recs, fr = outs[name]
            ms = ctypes.c_double()
            assert L.cbev_profile_raster(ctx, p(recs), n, p(fr), a.reps, None, ctypes.byref(ms)) == 0
            res[name].append(ms.value * 1e3)
    for name, v in res.items():
        v = np.array(v)
        print(f"{name:28s} raster us/launch: median {np.median(v):7.2f}  min {v.min():7.2f}  max {v.max():7.2f}")



if __name__ == "__main__":
    main()
