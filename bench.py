"""Benchmark: env-steps/sec of the batched CarlaBEV step on MI355X.

Workload (BASELINE.json configs; default = configs[1], the metric's config):
  --config 2  4096 envs/GPU, 128x128 semantic obs, ego-only (rt_no_traffic_v1),
              discrete9, scene_seed = 10000 + global_env_id, actions default_rng(1234 + env_id)
  --config 3  4096 envs/GPU, bev_rgb (grayscale 4-stack), rt_hard_v1 traffic, actions default_rng(7 + id)
  --config 4  8192 envs/GPU, semantic, continuous, rt_medium_v1, RCCL gather of frames to rank 0 every step
  --config 5  2048 envs/GPU, 256x256 semantic, lead_brake/jaywalk/red_light_runner mix, comfort export

One timed "step" = `step()` for every env (ego + actors + raster + collision/reward
+ termination) followed by the reference's canonical loop reset of the envs that
terminated (reset_mask = terminated | truncated, served on the device from a
pre-built scene bank). Inputs are resident in HBM before the timed region.
`value` = env-steps/s summed over ranks (weak scaling: envs per GPU fixed).
The wire-format observation (float32 one-hot 4-stack / gray stack) is timed
in a second pass and reported as `with_wire_obs`.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

CONFIGS = {
    2: dict(envs=4096, size=128, obs_mode="bev_semantic", difficulty="rt_no_traffic_v1", action="discrete9_v1",
            seed0=10_000, act_seed=1234, caps=dict(route_cap=64, actor_cap=0, actor_route_cap=2, tl_cap=0),
            workload="ego-only empty scene (rt_no_traffic_v1), 4096 envs/GPU, 128x128 semantic 6-class"),
    3: dict(envs=4096, size=128, obs_mode="bev_rgb", difficulty="rt_hard_v1", action="discrete9_v1",
            seed0=20_000, act_seed=7, caps=dict(route_cap=64, actor_cap=25, actor_route_cap=288, tl_cap=0),
            workload="random traffic (rt_hard_v1, 25 vehicles), 4096 envs/GPU, 128x128 RGB->gray 4-stack"),
    4: dict(envs=8192, size=128, obs_mode="bev_semantic", difficulty="rt_medium_v1", action="continuous_gsb_v1",
            seed0=40_000, act_seed=99, caps=dict(route_cap=64, actor_cap=16, actor_route_cap=288, tl_cap=0),
            gather=True, workload="rt_medium_v1, continuous, 8192 envs/GPU, RCCL frame gather to rank 0",
            workload_n1="rt_medium_v1, continuous, 8192 envs/GPU (one shard; no gather at N=1)"),
    5: dict(envs=2048, size=256, obs_mode="bev_semantic", difficulty="mix3", action="discrete9_v1",
            seed0=30_000, act_seed=1234, caps=dict(route_cap=64, actor_cap=4, actor_route_cap=64, tl_cap=4),
            workload="lead_brake/jaywalk/red_light_runner mix, 2048 envs/GPU, 256x256 semantic, comfort export"),
}

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip-level parameters (spec)
BANK_MIN = 4096  # reset-bank rows at least; the bank holds max(BANK_MIN, 2 n) scenes
BANK_GID0 = 1_000_000  # bank scenes: global ids 1e6 + rank * B + i, distinct from every start scene (id < 1e6)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def scene_options(cfgd, env_id):
    from carlabev_env_amd.config import RandomNavigationReset, build_random_navigation_options
    if cfgd["difficulty"] == "mix3":
        return {"scene": ("lead_brake", "jaywalk", "red_light_runner")[env_id % 3]}
    return build_random_navigation_options(RandomNavigationReset(difficulty_id=cfgd["difficulty"]))


def make_actions(P, n, steps, seed0, offset):
    out = np.zeros((steps, n), np.int32) if P.action_kind == 0 else np.zeros((steps, n, 3), np.float32)
    for e in range(n):
        rng = np.random.default_rng(seed0 + offset + e)
        if P.action_kind == 0:
            out[:, e] = rng.integers(0, P.n_discrete, size=steps)
        else:
            out[:, e] = rng.uniform([0, -1, 0], [1, 1, 1], size=(steps, 3)).astype(np.float32)
    return out


def env_config(cfgd):
    from carlabev_env_amd.config import EnvConfig
    S = cfgd["size"]
    action_mode = "continuous" if cfgd["action"].startswith("continuous") else "discrete"
    return EnvConfig(size=S, obs_size=(S, S), obs_mode=cfgd["obs_mode"], render_mode="rgb_array",
                     action_mode=action_mode, action_profile_id=cfgd["action"])


def build_scene_sets(cfgd, n, rank, cache=None):
    """The n seeded start scenes (global ids rank*n + i, scene_seed = seed0 + id)
    and the reset bank of B = max(BANK_MIN, 2 n) further seeded scenes (global ids
    BANK_GID0 + rank*B + j: no bank scene is a start scene), built by host worker
    processes before the GPU is touched (scene generation stays on the host,
    SURVEY §8). Scenes are a pure function of (config, n, rank): `cache` keeps them
    across runs on one box."""
    from carlabev_env_amd import layout as LY
    from carlabev_env_amd.scene_pool import build_scenes
    rb = LY.Layout.make(LY.Caps(**cfgd["caps"])).record_bytes
    B = max(BANK_MIN, 2 * n)
    key = None
    if cache:
        os.makedirs(cache, exist_ok=True)
        key = os.path.join(cache, f"v4_cfg{cfgd['seed0']}_{cfgd['difficulty']}_{n}_{B}_{rank}_{rb}")
    if key and os.path.exists(key + "_bank.npy"):
        log(f"[rank {rank}] loaded {n} start scenes + {B} bank scenes from {cache}")
        return np.load(key + "_recs.npy"), np.load(key + "_bank.npy")
    t0 = time.time()
    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    args = (env_config(cfgd).model_dump(), cfgd["caps"], cfgd["difficulty"], cfgd["seed0"], rb)
    host = build_scenes(*args, [rank * n + i for i in range(n)], workers=workers)
    bank = build_scenes(*args, [BANK_GID0 + rank * B + j for j in range(B)], workers=workers)
    log(f"[rank {rank}] built {n} start scenes + {B} bank scenes on {workers} workers in {time.time() - t0:.1f}s")
    if key:
        np.save(key + "_recs.npy", host)
        np.save(key + "_bank.npy", bank)
    return host, bank


def build_env(cfgd, n, rank, device, info_mode="full", scenes=None, defer_reset=True):
    """Vector env with every env reset to its seeded start scene and the reset
    bank attached (terminated envs take its rows in order)."""
    from carlabev_env_amd.vector_env import CarlaBEVVectorEnv
    import torch
    host, bank = scenes if scenes is not None else build_scene_sets(cfgd, n, rank)
    env = CarlaBEVVectorEnv({"env": env_config(cfgd), "num_envs": n}, device=device, caps=cfgd["caps"],
                            info_mode=info_mode, defer_reset=defer_reset)
    env.attach_bank(torch.from_numpy(bank).to(device))
    env.auto_obs = False
    start = torch.from_numpy(host).to(device)
    env.load_scenes(start)
    return env, host, start


def cpu_baseline(cfgd, host_recs, env, seconds):
    """Reference-semantics CPU oracle on a bounded sample of the same workload
    (same scenes, same action streams), timed two ways as SURVEY.md §8(d) asks:
    (i) one thread stepping 64 envs (the reference's SyncVectorEnv model) and
    (ii) one thread per usable host core (os.sched_getaffinity, capped at 16 =
    the GPU box's CPU share), each stepping its own 64-env block. ctypes drops
    the GIL inside orc_step_batch, so the threads run in parallel. `value` is
    leg (ii); leg (i) is reported beside it."""
    import threading
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    P = env.params
    blk = min(64, host_recs.shape[0])
    acts_all = None

    def leg(threads, secs):
        nonlocal acts_all
        n_tot = min(blk * threads, host_recs.shape[0])
        per = n_tot // threads
        if acts_all is None or acts_all.shape[1] < n_tot:
            acts_all = make_actions(P, n_tot, 4000, cfgd["act_seed"], 0)
        counts = [0] * threads
        stop = time.perf_counter() + secs

        def work(k):
            lo, hi = k * per, (k + 1) * per
            recs = host_recs[lo:hi].copy()
            orc = O.Oracle(P, env.map_host, env.caps.c(), env.rb)
            frames = np.zeros((hi - lo, P.size, P.size), np.uint8)
            t = 0
            while time.perf_counter() < stop and t < acts_all.shape[0]:
                orc.step(recs, hi - lo, np.ascontiguousarray(acts_all[t, lo:hi]), frames)
                t += 1
            counts[k] = t * (hi - lo)

        t0 = time.perf_counter()
        ths = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t0
        return sum(counts) / dt, sum(counts), dt, per

    v1, s1, d1, _ = leg(1, seconds / 3)
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    vm, sm, dm, per = leg(cores, 2 * seconds / 3) if cores > 1 else (v1, s1, d1, blk)
    return {"value": vm, "unit": "env-steps/s", "cores": cores, "kind": "port",
            "single_thread_value": v1,
            "sample": f"{cores} threads x {per} envs of the same workload ({sm} env-steps in {dm:.1f}s); "
                      f"single thread: {blk} envs ({s1} env-steps in {d1:.1f}s). oracle/cbev_oracle.c, "
                      "per-step full padded-map restore as in scene.py:93"}


def measure_peaks(env, device, reps=20):
    """Bandwidth this box reaches on plain streams the size of one step's frames
    (HIP events on the current stream): a write-only fill (the raster's output
    floor) and a device-to-device copy (read + write bytes)."""
    import torch
    nbytes = int(env.frames().numel())
    a = torch.empty(nbytes, dtype=torch.uint8, device=device)
    b = torch.empty_like(a)
    out = {}
    for name, fn, traffic in (("write", lambda: a.fill_(7), nbytes), ("copy", lambda: b.copy_(a), 2 * nbytes)):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        out[f"{name}_gbs"] = round(traffic * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
    out["bytes"] = nbytes
    out["how"] = f"torch fill_ / copy_ of one step's frame bytes, {reps} back-to-back, HIP events"
    del a, b
    return out


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` run by hand (no torch.distributed.run around it): start
    N rank processes of this same script, one per GPU, with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set, and wait for them. The parent never touches the
    GPU (it has not imported torch); rank 0 prints the JSON line. If any rank
    fails, the others are terminated (by PID) so none waits in a barrier."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                log(f"[launcher] rank {procs.index(p)} exited with {code}; stopping the others")
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def gather_budget(config: int, ranks: int = 8, link_gbs: float = 153.0, links: int = 7) -> dict:
    """Per-rank gather payload of `config` at its bench size, nibble-packed (as
    FrameGather sends it) and unpacked, and rank 0's ingress time for `ranks`
    ranks over `links` point-to-point xGMI links of `link_gbs` GB/s."""
    from carlabev_env_amd.sharding import payload_bytes
    cfgd = CONFIGS[config]
    packed, plain = payload_bytes(cfgd["envs"], cfgd["size"]), payload_bytes(cfgd["envs"], cfgd["size"], packed=False)
    ingress = lambda b: round((ranks - 1) * b / (links * link_gbs * 1e9) * 1e3, 3)  # noqa: E731
    return {"envs_per_rank": cfgd["envs"], "bytes_packed": packed, "bytes_unpacked": plain, "ranks": ranks,
            "rank0_ingress_ms_packed": ingress(packed), "rank0_ingress_ms_unpacked": ingress(plain)}


def dry_run(args, world, rank):
    """CPU rehearsal of the N-rank path (gloo): rendezvous, the packed frame
    gather of config 4 (FrameGather on CPU tensors), barrier-bracketed timing and
    the max over ranks. No GPU and no env: `value` stays null."""
    import torch
    import torch.distributed as dist
    from carlabev_env_amd.sharding import FrameGather
    if world > 1:
        dist.init_process_group("gloo")
    n, S = args.envs or 8, CONFIGS[args.config]["size"]
    g = FrameGather(n, S, "cpu") if world > 1 else None
    frames = torch.full((n, S, S), rank, dtype=torch.uint8)
    rew = torch.arange(n, dtype=torch.float64) + 1000 * rank
    term = torch.zeros(n, dtype=torch.uint8)
    ok = True
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if g is not None:
            g.gather(frames, rew, term)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
        if rank == 0:
            f, r, _c, _t, _tr = g.gathered()
            ok = all(bool((f[k * n:(k + 1) * n] == k).all()) and bool((r[k * n:(k + 1) * n] == rew - 1000 * rank + 1000 * k).all())
                     for k in range(world))
    if rank == 0:
        print(json.dumps({"metric": "env-steps/sec (whole node) at N_envs x 128x128 semantic obs", "value": None,
                          "unit": "env-steps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(el / max(args.steps, 1) * 1e3, 4), "dry_run": True,
                          "gather_ok": ok, "gather_bytes_per_step": None if g is None else g.bytes_per_step,
                          "at_config_size": gather_budget(args.config),
                          "config": {"config_id": args.config, "envs_per_gpu": n, "global_envs": n * world}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def start_scene_pool(cfgd, workers, rank, world):
    """Host workers building fresh seeded scenes (global ids 2_000_000 + rank,
    + world, ...) for the bank, started before the GPU is touched."""
    from carlabev_env_amd import layout as LY
    from carlabev_env_amd.config import EnvConfig
    from carlabev_env_amd.scene_pool import ScenePool
    S = cfgd["size"]
    action_mode = "continuous" if cfgd["action"].startswith("continuous") else "discrete"
    cfg = EnvConfig(size=S, obs_size=(S, S), obs_mode=cfgd["obs_mode"], render_mode="rgb_array",
                    action_mode=action_mode, action_profile_id=cfgd["action"])
    rb = LY.Layout.make(LY.Caps(**cfgd["caps"])).record_bytes
    return ScenePool(cfg.model_dump(), cfgd["caps"], cfgd["difficulty"], cfgd["seed0"], rb, workers=workers,
                     first_gid=2_000_000 + rank, stride=world, batch=16 if cfgd["difficulty"] == "rt_no_traffic_v1" else 4)


def fresh_pass(env, pool, one_step, args, world, n, device, seconds=2.0):
    """The canonical loop with the bank refreshed from the host ScenePool while it
    runs (at least `seconds` of wall time, so the host rates are measurable):
    every 8 steps the finished scenes replace the oldest bank rows (and their
    cached reset frames are rendered). Reports the pool's scene rate, the
    device's reset rate and the share of resets a fresh scene can have served."""
    import torch
    pool.request(4 * pool.batch * pool.workers)
    pool.poll(timeout=60.0)  # workers up and producing
    total = args.warmup + args.steps
    for t in range(args.warmup):
        one_step(t, False)
    torch.cuda.synchronize()
    term0 = env.termination_count()
    d0 = pool.delivered
    slot = 0
    steps = 0
    t0 = time.perf_counter()
    while steps < args.steps or time.perf_counter() - t0 < seconds:
        t = args.warmup + steps % args.steps
        one_step(t, False)
        steps += 1
        if steps % 8 == 0:
            gids, recs, ctxs = pool.poll(max_scenes=env.bank.shape[0], contexts=True)
            if len(gids):
                slot = env.refresh_bank(slot, recs, ctxs)
                pool.request(len(gids))
            if steps % 64 == 0:  # keep the host no more than ~64 steps ahead of the device
                torch.cuda.current_stream().synchronize()
    env.flush()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    resets = env.termination_count() - term0
    fresh_scenes = pool.delivered - d0
    return {"workers": pool.workers, "steps": steps, "seconds": round(el, 3), "value": round(world * n * steps / el, 1),
            "scenes_per_s": round(fresh_scenes / el, 1), "resets_per_s": round(resets / el, 1),
            "fresh_reset_frac": round(min(1.0, fresh_scenes / resets), 4) if resets else 1.0,
            "note": "per rank; resets beyond the fresh scenes reuse bank scenes (recycled)"}


def surface_loop(cfgd, n, device, acts, pool, steps, warmup, fresh):
    """INTEGRATION.md §1's loop verbatim on the reference surface (make_env,
    step, reset(options={"reset_mask": done, **opts}); tools/debug_env.py:56-132):
    obs is the fresh float32 wire observation of every step, `done` goes to the
    host each step, the masked envs are rebuilt by the host (CarlaBEV.reset,
    carlabev.py:96-148). fresh=False: no seeds, as the reference's loop resets, so
    every reset is the scene of the config's seed (carlabev.py:84) and is served
    from the builder's memo after its first build; fresh=True: each reset call
    passes a new seed per env (reset(seed=[...], options)), so every reset
    builds a scene nobody built before (on the BuildPool's workers)."""
    import torch
    from carlabev_env_amd.vector_env import make_env
    opts = scene_options(cfgd, 0)
    env = make_env({"env": env_config(cfgd), "num_envs": n}, device=device, caps=cfgd["caps"], reset_pool=pool)
    t0 = time.perf_counter()
    obs, _ = env.reset(seed=0, options=opts)
    torch.cuda.synchronize()
    init_s = time.perf_counter() - t0
    calls = [0]

    def run(k, t_off):
        resets = 0
        for t in range(k):
            obs, rew, term, trunc, infos = env.step(acts[(t_off + t) % acts.shape[0]])
            done = term | trunc
            if done.any():
                m = done.cpu().numpy()
                resets += int(m.sum())
                if fresh:
                    calls[0] += 1
                    seeds = [10_000_000 + calls[0] * n + i for i in range(n)]
                    obs, _ = env.reset(seed=seeds, options={"reset_mask": m, **opts})
                else:
                    obs, _ = env.reset(options={"reset_mask": m, **opts})
        return resets

    run(warmup, 0)
    torch.cuda.synchronize()
    b0, h0, p0 = env.builder.builds, env.builder.memo_hits, env.pool_builds
    t0 = time.perf_counter()
    resets = run(steps, warmup)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    built = env.builder.builds - b0 + env.pool_builds - p0
    out = {"value": round(n * steps / el, 1), "unit": "env-steps/s", "steps": steps, "warmup": warmup,
           "ms_per_step": round(el / steps * 1e3, 3), "resets_per_step": round(resets / steps, 2),
           "scenes_built": built, "memo_copies": env.builder.memo_hits - h0 - (env.pool_builds - p0),
           "fresh_reset_frac": round(built / resets, 4) if resets else None,
           "pool_workers": 0 if pool is None else pool.workers, "initial_reset_s": round(init_s, 2),
           "loop": ("step(a) -> done = term | trunc -> reset(seed=[fresh per env], options={'reset_mask': done, **opts})"
                    if fresh else "step(a) -> done = term | trunc -> reset(options={'reset_mask': done, **opts})")}
    env.close()
    del env, obs
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-wire", action="store_true")
    ap.add_argument("--raster-reps", type=int, default=50, help="back-to-back k_raster launches timed for the roofline")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo rehearsal of the N-rank path (no GPU, value null)")
    ap.add_argument("--scene-cache", default=None, help="directory to keep built scenes in across runs (one box)")
    ap.add_argument("--fresh-workers", type=int, default=4,
                    help="host processes feeding fresh seeded scenes into the reset bank in a last timed pass (0: off)")
    ap.add_argument("--burn-in", type=int, default=200,
                    help="canonical-loop steps before the timed passes, which all start from the state they leave")
    ap.add_argument("--repeats", type=int, default=5,
                    help="timed passes of exactly --steps steps each (re-seeded between); value = their median")
    ap.add_argument("--no-defer-reset", action="store_true",
                    help="launch every canonical reset at once (k_reset_mask) instead of folding it into the next step")
    ap.add_argument("--surface-steps", type=int, default=None,
                    help="timed steps of the reference-surface loop legs (surface_loop, surface_loop_fresh; "
                         "0: off; default 100 at config 2, off elsewhere)")
    ap.add_argument("--surface-warmup", type=int, default=300,
                    help="untimed steps before them (from the initial reset to a steady reset rate)")
    ap.add_argument("--surface-workers", type=int, default=16, help="BuildPool workers for the surface-loop resets")
    ap.add_argument("--info-mode", default="full", choices=("none", "full"),
                    help="full (default, as the reference's step() always runs Stats.step, carlabev.py:226-227): "
                         "device episode statistics + a StepInfos per step (not read); none: statistics off")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        log(f"[bench] WORLD_SIZE={world} overrides --gpus {args.gpus}")
    if args.dry_run:
        return dry_run(args, world, rank)

    cfgd = CONFIGS[args.config]
    if args.surface_steps is None:
        args.surface_steps = 100 if args.config == 2 else 0
    n = args.envs or cfgd["envs"]
    scenes = build_scene_sets(cfgd, n, rank, args.scene_cache)  # host workers, before the GPU is touched
    pool = None
    if args.fresh_workers > 0:  # spawned before this process touches the GPU
        pool = start_scene_pool(cfgd, args.fresh_workers, rank, world)
    bpool = None
    if args.surface_steps > 0 and args.surface_workers > 0:  # likewise
        from carlabev_env_amd.scene_pool import BuildPool
        bpool = BuildPool(env_config(cfgd).model_dump(), cfgd["caps"], workers=args.surface_workers, chunk=1)

    import torch
    import torch.distributed as dist
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    from carlabev_env_amd._lib import check, lib
    env, host_recs, start_recs = build_env(cfgd, n, rank, device, args.info_mode, scenes,
                                           defer_reset=not args.no_defer_reset)
    del scenes
    P = env.params
    total_steps = args.warmup + args.steps
    burn = max(0, args.burn_in)
    # one action stream per env: the burn-in's steps, then the warmup + timed steps of every pass
    acts_all = torch.from_numpy(make_actions(P, n, burn + total_steps, cfgd["act_seed"], rank * n)).to(device)
    acts = acts_all[burn:]
    gather = cfgd.get("gather", False) and world > 1
    gatherer = None
    if gather:
        from carlabev_env_amd.sharding import FrameGather
        gatherer = FrameGather(n, cfgd["size"], device, dst=0, ctx=env._ctx, stream_fn=env._stream)

    env.auto_obs = False

    def one_step(t, wire):
        env.step_async_only(acts[t])
        env.step_infos()
        if gatherer is not None:  # config 4: frames + reward/cause/flags of every rank to rank 0, one RCCL gather
            gatherer.gather(env.frames(), env.reward, env.term, env.trunc, env.cause)
        env.reset_terminated()  # canonical loop: reset(reset_mask=terminated), next bank rows
        if wire:
            env._obs()

    def timed(wire, profile):
        for t in range(args.warmup):
            one_step(t, wire)
        if profile:
            check(lib().cbev_profile(env._ctx, 1), "profile")
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for t in range(args.warmup, total_steps):
            one_step(t, wire)
        # the last step's reset is folded into no next step here: it runs now, in the
        # timed region (k_reset_mask), like every other step's reset
        env.flush()
        host_enqueue = time.perf_counter() - t0
        if gatherer is not None:
            gatherer.wait()  # the last steps' gathers are part of the timed region
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device=device)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        ms3 = None
        if profile:
            buf = (ctypes.c_double * 3)()
            cnt = ctypes.c_int64()
            check(lib().cbev_profile_read(env._ctx, buf, ctypes.byref(cnt)), "profile_read")
            check(lib().cbev_profile(env._ctx, 0), "profile")
            ms3 = [buf[i] / max(cnt.value, 1) for i in range(3)]
        return el, ms3, host_enqueue

    snap = {}

    def reseed():  # back to the steady-state snapshot, so every pass replays a comparable workload
        if not snap:  # before the burn-in: the seeded start scenes
            env.load_scenes(start_recs)
            return
        env.records.copy_(snap["records"])
        env.ring.copy_(snap["ring"])
        env.head = snap["head"]

    def burn_in():
        """The canonical loop from the seeded start scenes for `burn` steps, then a
        snapshot of every env's state and frame stack: the timed passes start from
        episodes of mixed ages (the steady-state termination and reset rate of the
        loop) instead of all envs at step 0 of their first episode."""
        env.load_scenes(start_recs)
        term0 = env.termination_count()
        for t in range(burn):
            env.step_async_only(acts_all[t])
            env.reset_terminated()
        env.flush()
        torch.cuda.synchronize()
        snap["records"] = env.records.clone()
        snap["ring"] = env.ring.clone()
        snap["head"] = env.head
        return env.termination_count() - term0

    # The step runs on a stream of its own: launches on HIP's legacy default
    # stream carry implicit synchronisation that costs several us per kernel.
    stream = torch.cuda.Stream(device)
    with torch.cuda.stream(stream):
        # bring the GPU to its steady clocks before any timed pass (a fresh box's first
        # few ms of kernels run measurably slower); the state is re-seeded afterwards
        t_end = time.perf_counter() + 0.5
        while time.perf_counter() < t_end:
            for t in range(min(20, total_steps)):
                one_step(t, False)
            torch.cuda.synchronize()
        burn_resets = burn_in() if burn else 0
        passes = []
        term0 = env.termination_count()
        rows0 = env.bank_rows_used()
        counts0 = env.reset_counts()
        for _ in range(max(1, args.repeats)):  # headline passes, no instrumentation
            reseed()
            passes.append(timed(False, False))
        pass_resets = env.termination_count() - term0
        pass_rows = env.bank_rows_used() - rows0
        distinct_rows = int(np.unique(env.bank_rows_between(counts0, env.reset_counts(), env.bank.shape[0])).size)
        els = sorted(p[0] for p in passes)
        el = els[len(els) // 2]
        host_enq = sorted(p[2] for p in passes)[len(els) // 2]
        peak = measure_peaks(env, device)
        reseed()
        el_prof, ms3, _ = timed(False, True)  # same workload with HIP events around each kernel (roofline)
        value = world * n * args.steps / el
        burst_ms = None
        # k_raster's own launch duration: one more step (no reset, so every
        # record holds this step's render set-up), then a burst of raster
        # launches over it between two events (cbev_profile_raster); the
        # per-kernel events above also count each launch's dispatch gap
        env.step_async_only(acts[total_steps - 1])
        bm = ctypes.c_double()
        check(lib().cbev_profile_raster(env._ctx, env.records.data_ptr(), n, env.frames().data_ptr(),
                                        args.raster_reps, env._stream(), ctypes.byref(bm)), "profile_raster")
        burst_ms = bm.value
        wire_value = None
        if not args.no_wire:
            reseed()
            el_w, _, _ = timed(True, False)
            wire_value = world * n * args.steps / el_w
        fresh = None
        if pool is not None:
            reseed()
            fresh = fresh_pass(env, pool, one_step, args, world, n, device)
    surf = surf_fresh = None
    if args.surface_steps > 0:
        surf = surface_loop(cfgd, n, device, acts_all, bpool, args.surface_steps, args.surface_warmup, fresh=False)
        surf_fresh = surface_loop(cfgd, n, device, acts_all, bpool, args.surface_steps, args.surface_warmup,
                                  fresh=True)

    S = P.size
    # per env: S^2 texels sampled + S^2 frame bytes + ego state
    algo_bytes = 2 * S * S + 64
    raster_ms = burst_ms if burst_ms is not None else ms3[2]
    achieved = n * algo_bytes / (raster_ms * 1e-3) / 1e9
    traffic = write_bytes = None
    pmc_path = os.path.join(REPO, "profiles", f"pmc_raster_config{args.config}.json")
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        if pmc.get("envs") == n:
            traffic = pmc.get("hbm_bytes_per_launch")
            write_bytes = pmc.get("write_kb", 0.0) * 1024
    t_s = raster_ms * 1e-3
    frame_bytes = n * S * S
    counter_fields = {
        # counter-measured DRAM rates of the same launch time (profiles/pmc_raster_config*.json)
        "write_frac_measured": None if write_bytes is None else round(write_bytes / t_s / 1e9 / peak["write_gbs"], 4),
        "hbm_counter_frac": None if traffic is None else round(traffic / t_s / 1e9 / HBM_PEAK_GBS, 4),
        # kernel time over the time this box's fill_ needs for the frame bytes alone
        "write_floor_ratio": round(t_s / (frame_bytes / (peak["write_gbs"] * 1e9)), 3),
    }
    cpu = None
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline(cfgd, host_recs, env, args.cpu_seconds)
    if rank == 0:
        out = {
            "metric": "env-steps/sec (whole node) at N_envs x 128x128 semantic obs",
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64 state / u8 frames",
            "data": "synthetic seeded scenes (the reference's scene generator restated on its Town01 lane graphs), seeded action streams",
            "info_mode": args.info_mode,
            "reset": ("folded into the next step's k_ego (cbev_set_deferred_reset)"
                      if bool(lib().cbev_reset_pending is not None) and not args.no_defer_reset
                      and cfgd["caps"]["actor_cap"] == 0 else "k_reset_mask launch per step"),
            "config": {"workload": cfgd["workload"] if gather or "workload_n1" not in cfgd else cfgd["workload_n1"],
                       "config_id": args.config, "envs_per_gpu": n,
                       "global_envs": n * world, "obs_size": S, "obs_mode": cfgd["obs_mode"],
                       "parallelism": f"env-sharded x{world}" + (" + RCCL gather" if gather else "")},
            "repeats": len(els),
            "ms_per_step_min_max": [round(els[0] / args.steps * 1e3, 4), round(els[-1] / args.steps * 1e3, 4)],
            "value_min_max": [round(world * n * args.steps / els[-1], 1), round(world * n * args.steps / els[0], 1)],
            "burn_in_steps": burn,
            "resets_per_step": round(pass_resets / (max(1, args.repeats) * total_steps), 2),
            "resets_per_step_note": (f"canonical-loop resets (reset_mask=terminated) per step over the headline "
                                     f"passes (warmup + timed steps), from a snapshot taken after {burn} burn-in "
                                     f"steps ({burn_resets} resets)"),
            "bank_scenes": int(env.bank.shape[0]),
            "bank_scene_ids": (f"{BANK_GID0} + rank*{int(env.bank.shape[0])} + j: seeded scenes distinct from the "
                               f"{n} start scenes (ids rank*{n} + i)"),
            # the resets of the headline passes (env e's j-th reset: bank row (e + j * stride) % B)
            "bank_rows_handed_out": pass_rows,
            "distinct_bank_rows_handed_out": distinct_rows,
            "host_enqueue_ms_per_step": round(host_enq / args.steps * 1e3, 4),
            "ms_per_step_with_kernel_events": round(el_prof / args.steps * 1e3, 4),
            # per-step HIP-event spans; with no actor slots (config 2) k_actors is not launched and
            # its span is only the two back-to-back event records
            "kernel_ms": {"k_actors": (round(ms3[0], 5) if cfgd["caps"]["actor_cap"] > 0 else None),
                          "k_ego": round(ms3[1], 5), "k_raster": round(ms3[2], 5)},
            "raster_ms_per_launch": None if burst_ms is None else round(burst_ms, 5),
            "roofline": {"bound": "hbm", "kernel": "k_raster", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "peak_measured": peak, **counter_fields,
                         "traffic": traffic, "algorithmic_bytes_per_env": algo_bytes,
                         "timing": (f"HIP events around {args.raster_reps} back-to-back launches on the step stream"
                                    if burst_ms is not None else "HIP events around each launch in the timed steps"),
                         # the same bytes over the per-step event time (includes each launch's dispatch gap)
                         "achieved_step_events": round(n * algo_bytes / (ms3[2] * 1e-3) / 1e9, 1)},
            "with_wire_obs": None if wire_value is None else round(wire_value, 1),
            "fresh_resets": fresh,
            # the reference surface's own loop, host scene builds included
            "surface_loop": surf,
            "surface_loop_fresh": surf_fresh,
            "gather_bytes_per_step": None if gatherer is None else gatherer.bytes_per_step,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    env.close()
    if pool is not None:
        pool.close()
    if bpool is not None:
        bpool.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
