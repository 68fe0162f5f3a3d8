"""Does a captured HIP graph of the step (k_hero, k_raster, k_collide, k_reset)
shrink the inter-kernel gaps? Times config 2 with plain launches and with one
graph replay per step (actions copied into a fixed buffer first)."""
from __future__ import annotations

import os
import sys
import time


def main():
    REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, REPO)
    import torch  # noqa: E402

    import bench  # noqa: E402

    cfgd = bench.CONFIGS[2]
    n = cfgd["envs"]
    env, host, _start = bench.build_env(cfgd, n, 0, torch.device("cuda", 0))
    steps = 200
    acts = torch.from_numpy(bench.make_actions(env.params, n, steps + 20, cfgd["act_seed"], 0)).cuda()
    abuf = acts[0].clone()
    env.auto_obs = False


    def one(a):
        env.step_async_only(a)
        env.reset_terminated()


    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for t in range(10):
            one(acts[t])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(steps):
            one(acts[t])
        torch.cuda.synchronize()
        plain = (time.perf_counter() - t0) / steps
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            one(abuf)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(steps):
            abuf.copy_(acts[t])
            g.replay()
        torch.cuda.synchronize()
        graph = (time.perf_counter() - t0) / steps
    print(f"plain {plain * 1e6:.1f} us/step  graph {graph * 1e6:.1f} us/step")



if __name__ == "__main__":
    main()
