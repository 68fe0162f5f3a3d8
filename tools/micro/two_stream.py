"""Feasibility timing (not a product path): the step's kernels over the env
batch cut into K parts, each part's cbev_step on its own stream, against one
cbev_step over the whole batch. The parts are independent env ranges, so a
part's steps depend only on its own earlier steps (stream order); statistics
off, no resets (timing only). Usage (GPU box):
python tools/micro/two_stream.py [--config 2] [--steps 200]"""
from __future__ import annotations

import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    import torch
    import bench
    from carlabev_env_amd._lib import lib
    cfgd = bench.CONFIGS[a.config]
    n = cfgd["envs"]
    env, host, start = bench.build_env(cfgd, n, 0, torch.device("cuda", 0), info_mode="none", defer_reset=False)
    acts = torch.from_numpy(bench.make_actions(env.params, n, a.steps, cfgd["act_seed"], 0)).cuda()
    L = lib()
    rec, rew, term, trunc, cause, info = env._p_step
    rb, SS = env.rb, env._slot_bytes // n
    for t in range(50):
        env.step_async_only(acts[t % a.steps])
    torch.cuda.synchronize()
    ring0 = env._p_ring
    asz = acts.element_size() * (acts[0].numel() // n)

    def run(parts, streams):
        cut = [n * k // parts for k in range(parts + 1)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(a.steps):
            head = t % env.F
            for k in range(parts):
                o, m = cut[k], cut[k + 1] - cut[k]
                s = streams[k % len(streams)]
                rc = L.cbev_step(env._ctx, rec + o * rb, m, acts[t].data_ptr() + o * asz,
                                 ring0 + head * env._slot_bytes + o * SS, rew + 8 * o, term + o, trunc + o,
                                 cause + 4 * o, info + 64 * o, s.cuda_stream)
                assert rc == 0
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e6

    def run_fj(home, sa, sb):
        """per step: fork from `home` (event), part A on sa, part B on sb, join back to home"""
        half = n // 2
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(a.steps):
            head = t % env.F
            ef = torch.cuda.Event()
            ef.record(home)
            for st in (sa, sb):
                if st is not home:
                    st.wait_event(ef)
            for k, (o, m, st) in enumerate(((0, half, sa), (half, n - half, sb))):
                rc = L.cbev_step(env._ctx, rec + o * rb, m, acts[t].data_ptr() + o * asz,
                                 ring0 + head * env._slot_bytes + o * SS, rew + 8 * o, term + o, trunc + o,
                                 cause + 4 * o, info + 64 * o, st.cuda_stream)
                assert rc == 0
            for st in (sa, sb):
                if st is not home:
                    ej = torch.cuda.Event()
                    ej.record(st)
                    home.wait_event(ej)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e6

    s0 = torch.cuda.current_stream()
    ss = [torch.cuda.Stream() for _ in range(4)]
    hp = torch.cuda.Stream(priority=-1)
    for name, parts, streams in (("1 part, 1 stream", 1, [s0]), ("2 parts, 1 stream", 2, [s0]),
                                 ("2 parts, 2 streams", 2, ss[:2]), ("4 parts, 2 streams", 4, ss[:2]),
                                 ("1 part, 1 stream (again)", 1, [s0])):
        run(parts, streams)  # warm
        us = run(parts, streams)
        print(f"config {a.config} {name}: {us:.1f} us per step, {n / us:.1f} M env-steps/s", flush=True)
    for name, home, sa, sb in (("fork/join: A on home (default), B on a stream", s0, s0, ss[0]),
                               ("fork/join: A on home (default), B on a high-priority stream", s0, s0, hp),
                               ("fork/join: A, B on two streams, home default", s0, ss[0], ss[1]),
                               ("fork/join: A on home (a stream), B on another", ss[2], ss[2], ss[3])):
        run_fj(home, sa, sb)
        us = run_fj(home, sa, sb)
        print(f"config {a.config} {name}: {us:.1f} us per step, {n / us:.1f} M env-steps/s", flush=True)


if __name__ == "__main__":
    main()
