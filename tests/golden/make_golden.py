"""Generate golden input/output vectors from the reference's own Python code.

Runs ONLY in the build container (needs /root/reference); the outputs are
committed under tests/golden/*.npz and are what the oracle is pinned against
(tests/test_oracle_golden.py). Nothing here travels to the GPU box as code that
runs there; only the .npz data files are read by tests.

Every vector set names the reference function it captures:
  state_update.npz   Controller/State.update         src/control/state.py:29-51
  smooth_route.npz   smooth_and_compute               src/control/utils.py:200-269
  stanley.npz        calc_target_index/stanley/pid    src/control/stanley_controller.py:64-123
  hero.npz           Discrete/ContinuousAgent.step    src/actors/hero.py:88-187
  actors.npz         Vehicle/Pedestrian.step + behaviours
                                                      src/actors/actor.py:86-124, behavior/*.py
  carl_reward.npz    CaRLRewardFn.step                src/deeprl/carl_reward_fn.py:149-341
  shaping_reward.npz RewardFn.step                    src/deeprl/reward.py:80-278
  comfort.npz        compute_comfort_kinematics       src/deeprl/comfort.py:17-70
  route_geom.npz     compute_route_progress / cumulative_lengths / lateral_error
                                                      carl_reward_fn.py:20-58, control/utils.py:165-197
  seeds.json         derive_seed / build_rng_bundle   src/randomness.py:13-65
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refimport  # noqa: E402

refimport.setup()

from CarlaBEV.src.control.stanley_controller import Controller  # noqa: E402
from CarlaBEV.src.control.utils import smooth_and_compute, lateral_error  # noqa: E402
from CarlaBEV.src.actors.hero import DiscreteAgent, ContinuousAgent  # noqa: E402
from CarlaBEV.src.actors.vehicle import Vehicle  # noqa: E402
from CarlaBEV.src.actors.pedestrian import Pedestrian  # noqa: E402
from CarlaBEV.src.actors.behavior.registry import build_behavior  # noqa: E402
from CarlaBEV.src.deeprl.carl_reward_fn import (  # noqa: E402
    CaRLRewardFn,
    compute_route_progress,
    cumulative_lengths,
)
from CarlaBEV.src.deeprl.reward import RewardFn  # noqa: E402
from CarlaBEV.src.deeprl.comfort import compute_comfort_kinematics, count_comfort_violations  # noqa: E402
from CarlaBEV.src.randomness import build_rng_bundle, derive_seed  # noqa: E402
from CarlaBEV.config.action_profiles import ACTION_PROFILE_PRESETS  # noqa: E402
from CarlaBEV.config.reward_profiles import REWARD_PROFILE_PRESETS  # noqa: E402

OUT = HERE


def save(name, **arrays):
    path = os.path.join(OUT, name)
    np.savez_compressed(path, **arrays)
    print(f"{name}: {os.path.getsize(path)} bytes")


def rand_route(rng, n_pts, spacing=12.5, noise=0.6, turn_p=0.15, origin=None):
    """Manhattan-ish random route in surface px (int32, like agent_route)."""
    if origin is None:
        origin = rng.uniform(100, 900, size=2)
    p = np.array(origin, dtype=float)
    d = rng.integers(0, 4)
    dirs = np.array([[1, 0], [0, 1], [-1, 0], [0, -1]], dtype=float)
    pts = []
    for _ in range(n_pts):
        pts.append(p.copy())
        if rng.random() < turn_p:
            d = (d + (1 if rng.random() < 0.5 else 3)) % 4
        p = p + dirs[d] * spacing + rng.normal(0, noise, 2)
    pts = np.array(pts)
    return pts[:, 0].astype(np.int32), pts[:, 1].astype(np.int32)


def ragged(list_of_arrays, dtype=float):
    lens = np.array([len(a) for a in list_of_arrays], dtype=np.int64)
    off = np.concatenate([[0], np.cumsum(lens)])
    flat = np.concatenate([np.asarray(a, dtype=dtype) for a in list_of_arrays]) if len(list_of_arrays) else np.zeros(0, dtype)
    return flat, off


# ---------------------------------------------------------------- G1 State.update
def gen_state_update(rng):
    M, K = 256, 24
    init = np.zeros((M, 5))
    acc = rng.normal(0, 6, (M, K))
    delta = rng.uniform(-1.0, 1.0, (M, K))
    out = np.zeros((M, K, 8))
    for m in range(M):
        ts = float(rng.choice([5.0, 38.4, 12.0]))
        c = Controller(target_speed=ts)
        c.x, c.y = float(rng.uniform(0, 1000)), float(rng.uniform(0, 1200))
        c.yaw = float(rng.uniform(-3.3, 3.3))
        c.v = float(rng.uniform(-ts, ts))
        init[m] = (c.x, c.y, c.yaw, c.v, ts)
        for k in range(K):
            c.update(float(acc[m, k]), float(delta[m, k]))
            out[m, k] = (c.x, c.y, c.yaw, c.v, c.x_1, c.y_1, c.yaw_1, c.v_1)
    save("state_update.npz", init=init, acc=acc, delta=delta, out=out)


# ---------------------------------------------------------------- G2 smooth_and_compute
def gen_smooth(rng):
    ins_x, ins_y, outs_x, outs_y, outs_yaw = [], [], [], [], []
    lengths = list(range(1, 70)) + list(rng.integers(2, 200, 60))
    for n in lengths:
        rx, ry = rand_route(rng, int(n))
        if rng.random() < 0.2 and n > 3:  # consecutive duplicates
            k = int(rng.integers(1, n))
            rx = np.insert(rx, k, rx[k - 1])
            ry = np.insert(ry, k, ry[k - 1])
        cx, cy, cyaw, _, _ = smooth_and_compute(rx, ry, window=11, poly=3)
        ins_x.append(rx); ins_y.append(ry)
        outs_x.append(cx); outs_y.append(cy); outs_yaw.append(cyaw)
    ix, ioff = ragged(ins_x, np.int32)
    iy, _ = ragged(ins_y, np.int32)
    ox, ooff = ragged(outs_x)
    oy, _ = ragged(outs_y)
    oyaw, _ = ragged(outs_yaw)
    save("smooth_route.npz", in_x=ix, in_y=iy, in_off=ioff, cx=ox, cy=oy, cyaw=oyaw, out_off=ooff)


# ---------------------------------------------------------------- G3 Stanley
def gen_stanley(rng):
    rows = []
    routes_x, routes_y, routes_yaw = [], [], []
    for r in range(120):
        rx, ry = rand_route(rng, int(rng.integers(2, 90)))
        cx, cy, cyaw, _, _ = smooth_and_compute(rx, ry, window=11, poly=3)
        routes_x.append(cx); routes_y.append(cy); routes_yaw.append(cyaw)
        c = Controller(target_speed=38.4)
        c.cx, c.cy, c.cyaw = cx, cy, cyaw
        for q in range(8):
            i = int(rng.integers(0, len(cx)))
            c.x = float(cx[i] + rng.normal(0, 6))
            c.y = float(cy[i] + rng.normal(0, 6))
            c.yaw = float(cyaw[i] + rng.normal(0, 0.6))
            c.v = float(rng.choice([0.0, 1e-4, rng.uniform(-5, 40)]))
            c.target_idx = int(rng.integers(0, len(cx)))
            c._target_speed = float(rng.uniform(0, 40))
            idx0, err = c.calc_target_index()
            delta, idx1 = c.stanley_control()
            pid = c.pid_control()
            rows.append((r, c.x, c.y, c.yaw, c.v, c.target_idx, c._target_speed, idx0, err, delta, idx1, pid))
    rx_, off = ragged(routes_x)
    ry_, _ = ragged(routes_y)
    ryaw, _ = ragged(routes_yaw)
    save("stanley.npz", cx=rx_, cy=ry_, cyaw=ryaw, off=off, rows=np.array(rows, dtype=float))


# ---------------------------------------------------------------- G4 hero physics
def gen_hero(rng):
    eps = []
    modes = [("discrete9_v1", 128), ("discrete13_v1", 128), ("continuous_gsb_v1", 128), ("discrete9_v1", 256),
             ("continuous_gsb_v1", 256)]
    routes_x, routes_y, acts, init_rows, traj = [], [], [], [], []
    smx, smy, smyaw = [], [], []
    meta = []
    E, K = 40, 200
    for e in range(E):
        profile, win = modes[e % len(modes)]
        spec = ACTION_PROFILE_PRESETS[profile]
        rx, ry = rand_route(rng, int(rng.integers(2, 60)))
        v0_mps = float(rng.choice([0.0, 0.0, 3.0]))
        vt_mps = float(rng.choice([12.0, 8.0]))
        seed = int(rng.integers(0, 2**31 - 1))
        Agent = ContinuousAgent if spec.action_mode == "continuous" else DiscreteAgent
        agent = Agent(route=(rx, ry), window_size=win, target_speed=vt_mps / 0.3125,
                      initial_speed=v0_mps / 0.3125, color=(0, 0, 0), np_rng=np.random.default_rng(seed))
        routes_x.append(rx); routes_y.append(ry)
        smx.append(agent.cx); smy.append(agent.cy); smyaw.append(agent.cyaw)
        init_rows.append((agent.x, agent.y, agent.yaw, agent.v, agent.target_idx, seed, win, v0_mps, vt_mps))
        if spec.action_mode == "continuous":
            a = rng.uniform([-0.2, -1.3, -0.2], [1.2, 1.3, 1.2], size=(K, 3)).astype(np.float32)
            # mostly gas to move along
            a[:, 0] = np.where(rng.random(K) < 0.7, np.abs(a[:, 0]), a[:, 0])
            act_idx = np.full(K, -1)
        else:
            n = len(spec.discrete_actions)
            p = np.ones(n); p[1] += 4.0; p /= p.sum()
            act_idx = rng.choice(n, size=K, p=p)
            a = np.array([spec.discrete_actions[i] for i in act_idx], dtype=np.float32)
        acts.append(np.concatenate([a.astype(np.float64), act_idx[:, None].astype(np.float64)], axis=1))
        rows = []
        for k in range(K):
            agent.step(a[k] if spec.action_mode == "continuous" else np.asarray(spec.discrete_actions[act_idx[k]], dtype=np.float32))
            lc, lm = agent.last_control, agent.last_comfort
            rows.append((agent.x, agent.y, agent.yaw, agent.v, agent.acc, agent.target_idx,
                         agent.x_1, agent.y_1, agent.yaw_1, agent.v_1,
                         lm["speed_mps"], lm["accel_long"], lm["accel_lat"], lm["jerk_long"], lm["jerk_lat"],
                         lm["yaw_rate"], lm["yaw_acc"],
                         lc["cmd_gas"], lc["cmd_steer"], lc["cmd_brake"], lc["applied_delta"]))
        traj.append(rows)
        meta.append(profile)
    rx_, roff = ragged(routes_x, np.int32)
    ry_, _ = ragged(routes_y, np.int32)
    sx, soff = ragged(smx)
    sy, _ = ragged(smy)
    syaw, _ = ragged(smyaw)
    save("hero.npz", route_x=rx_, route_y=ry_, route_off=roff, cx=sx, cy=sy, cyaw=syaw, cx_off=soff,
         init=np.array(init_rows, dtype=float), actions=np.array(acts), traj=np.array(traj, dtype=float),
         profiles=np.array(meta))


# ---------------------------------------------------------------- G5 actors + behaviours
BEHAVIOURS = [
    ("vehicle", None),
    ("vehicle", {"type": "timed_brake", "params": {"start_brake_t": 1.5, "decel_mps2": 2.5}}),
    ("vehicle", {"type": "timed_brake", "params": {"start_brake_t": 0.3, "decel_mps2": 8.0}}),
    ("pedestrian", {"type": "cross", "params": {"start_delay": 0.5}}),
    ("pedestrian", {"type": "stop_mid", "params": {"start_delay": 0.2}}),
    ("pedestrian", {"type": "yield_return", "params": {"start_delay": 0.0, "yield_duration": 1.0}}),
    ("pedestrian", {"type": "yield_return", "params": {"start_delay": 0.4, "yield_duration": 0.3}}),
    ("pedestrian", None),
]
BEH_ID = {None: 0, "timed_brake": 1, "cross": 2, "stop_mid": 3, "yield_return": 4}
STATE_ID = {"idle": 0, "waiting": 1, "entering": 2, "yielding": 3, "stalled": 4, "crossing": 5,
            "cleared": 6, "retreating": 7, "retreated": 8}


def gen_actors(rng):
    routes_x, routes_y, init_rows, traj, meta = [], [], [], [], []
    E, K = 48, 160
    for e in range(E):
        kind, beh = BEHAVIOURS[e % len(BEHAVIOURS)]
        n = int(rng.integers(3, 40)) if kind == "vehicle" else int(rng.integers(3, 12))
        spacing = 12.5 if kind == "vehicle" else 3.0
        pts_x, pts_y = rand_route(rng, n, spacing=spacing, noise=0.3)
        rx = [float(x) for x in pts_x]
        ry = [float(y) for y in pts_y]
        seed = int(rng.integers(0, 2**31 - 1))
        speed = float(rng.choice([12.0, 6.0])) if kind == "vehicle" else float(rng.choice([1.5, 2.5]))
        behavior, _ = build_behavior(kind, beh) if beh is not None else (None, None)
        Cls = Vehicle if kind == "vehicle" else Pedestrian
        act = Cls(map_size=128, routeX=rx, routeY=ry, behavior=behavior, target_speed=speed,
                  np_rng=np.random.default_rng(seed))
        act.reset()
        c = act._controller
        bparams = (list(beh["params"].values()) + [0.0, 0.0])[:2] if beh else [0.0, 0.0]
        init_rows.append((c.x, c.y, c.yaw, c.v, c.target_idx, seed, speed, 0 if kind == "vehicle" else 1,
                          BEH_ID[None if beh is None else beh["type"]], *bparams))
        routes_x.append(rx); routes_y.append(ry)
        rows = []
        t = 0.0
        for k in range(K):
            t += 0.1
            act.step(t, 0.1)
            c = act._controller
            rows.append((c.x, c.y, c.yaw, c.v, c.target_idx, act.target_speed, c._target_speed,
                         STATE_ID.get(act.behavior_state, -1), len(c.cx), len(act.rx)))
        traj.append(rows)
    rx_, roff = ragged(routes_x)
    ry_, _ = ragged(routes_y)
    save("actors.npz", route_x=rx_, route_y=ry_, route_off=roff, init=np.array(init_rows, dtype=float),
         traj=np.array(traj, dtype=float))


# ---------------------------------------------------------------- G6/G7 rewards
COLL = {None: 0, "vehicle": 1, "pedestrian": 2, "target": 3}
CAUSE = {None: 0, "collision": 1, "success": 2, "ckpt": 3, "out_of_bounds": 4, "max_actions": 5,
         "off_road": 6, "unknown": 7}
MAXA = 4  # actors_state entries per step in the fixture


def _synthetic_info(rng, cx, cy, cyaw, i, force=None):
    n = len(cx)
    idx = int(min(i, n - 1))
    x = float(cx[idx] + rng.normal(0, 3))
    y = float(cy[idx] + rng.normal(0, 3))
    yaw = float(cyaw[idx] + rng.normal(0, 0.2))
    v = float(rng.uniform(-2, 45))
    if idx + 5 <= n:
        wps = (cx[idx:idx + 5], cy[idx:idx + 5], cyaw[idx:idx + 5])
    else:
        wps = (cx[idx:-1], cy[idx:-1], cyaw[idx:-1])
    set_point = np.array([cx[idx], cy[idx], cyaw[idx]])
    dist2wp = float(np.linalg.norm(np.array([x, y]) - set_point[:-1]))
    if rng.random() < 0.05:
        dist2wp = float(rng.uniform(50, 80))
    tile = int(rng.choice([1, 1, 1, 1, 1, 2, 0], p=None)) if force != "safe" else 1
    coll = None
    aid = None
    r = rng.random()
    if force != "safe":
        if r < 0.04:
            coll, aid = "vehicle", 0
        elif r < 0.06:
            coll, aid = "pedestrian", 1
        elif r < 0.14:
            coll, aid = "target", int(rng.integers(0, 20))
        elif r < 0.16:
            coll, aid = "target", "goal"
    nact = int(rng.integers(0, MAXA + 1))
    actors = []
    for _ in range(nact):
        actors.append({"pos": (x + rng.normal(0, 15), y + rng.normal(0, 15)),
                       "vel": (rng.normal(0, 20), rng.normal(0, 20)), "type": "vehicle"})
    comfort = {k: float(rng.normal(0, s)) for k, s in
               (("accel_long", 2.0), ("accel_lat", 2.0), ("yaw_rate", 15), ("jerk_long", 3), ("jerk_lat", 3),
                ("yaw_acc", 90))}
    info = {
        "hero": {"state": [x, y, yaw, v], "last_state": [x - 1, y, yaw - float(rng.normal(0, 0.05)),
                                                           v - float(rng.normal(0, 0.5))],
                 "dist2wp": dist2wp, "set_point": set_point, "next_wps": wps, **comfort},
        "scene": {"dist2goal": float(rng.uniform(0, 200)), "dist2goal_t_1": float(rng.uniform(0, 200)),
                  "num_vehicles": 0, "route_length": 0.0, "speed_limit": 35},
        "collision": {"tile": None, "tile_class": tile, "collided": coll, "actor_id": aid,
                      "actors_state": actors},
    }
    return info


def _info_row(info):
    h = info["hero"]
    xs, ys, yaws = h["next_wps"]
    wps = np.full((5, 3), np.nan)
    wps[:len(xs), 0], wps[:len(xs), 1], wps[:len(xs), 2] = xs, ys, yaws
    act = np.full((MAXA, 4), np.nan)
    for j, a in enumerate(info["collision"]["actors_state"]):
        act[j] = (*a["pos"], *a["vel"])
    aid = info["collision"]["actor_id"]
    aid_code = -1 if aid is None else (-2 if aid == "goal" else int(aid))
    head = [*h["state"], *h["last_state"], h["dist2wp"], *h["set_point"], len(xs),
            h["accel_long"], h["accel_lat"], h["yaw_rate"], h["jerk_long"], h["jerk_lat"], h["yaw_acc"],
            info["scene"]["dist2goal"], info["scene"]["dist2goal_t_1"], info["scene"]["speed_limit"],
            info["collision"]["tile_class"], COLL[info["collision"]["collided"]], aid_code,
            len(info["collision"]["actors_state"])]
    return np.concatenate([np.array(head, dtype=float), wps.ravel(), act.ravel()])


def gen_carl(rng):
    seqs = []
    routes_x, routes_y = [], []
    profiles = []
    for s in range(60):
        prof = "carl_base_v1" if s % 3 else "carl_safety_v1"
        rx, ry = rand_route(rng, int(rng.integers(2, 40)))
        cx, cy, cyaw, _, _ = smooth_and_compute(rx, ry, window=11, poly=3)
        fn = CaRLRewardFn(**REWARD_PROFILE_PRESETS[prof].parameters)
        fn.reset(np.array(rx, np.int32), np.array(ry, np.int32))
        rows = []
        for i in range(40):
            info = _synthetic_info(rng, cx, cy, cyaw, i // 2, force="safe" if i < 2 else None)
            row = _info_row(info)
            rew, term, cause, info = fn.step(info)
            pen = info["reward"]["penalties"]
            extra = [rew, float(term), CAUSE[cause], info["reward"]["RC_t"],
                     pen.get("lane_center", np.nan), pen.get("off_lane", np.nan), pen.get("speed", np.nan),
                     pen.get("ttc", np.nan), pen.get("comfort", np.nan),
                     np.nan if fn._s_prev is None else fn._s_prev]
            rows.append(np.concatenate([row, np.array(extra, dtype=float)]))
        seqs.append(rows)
        routes_x.append(rx); routes_y.append(ry)
        profiles.append(prof)
    rx_, roff = ragged(routes_x, np.int32)
    ry_, _ = ragged(routes_y, np.int32)
    save("carl_reward.npz", route_x=rx_, route_y=ry_, route_off=roff, rows=np.array(seqs),
         profiles=np.array(profiles))


def gen_shaping(rng):
    seqs = []
    for s in range(40):
        rx, ry = rand_route(rng, int(rng.integers(2, 40)))
        cx, cy, cyaw, _, _ = smooth_and_compute(rx, ry, window=11, poly=3)
        fn = RewardFn(max_actions=int(rng.choice([5000, 30])))
        fn.reset()
        rows = []
        for i in range(40):
            info = _synthetic_info(rng, cx, cy, cyaw, i // 2)
            row = _info_row(info)
            rew, term, cause, info = fn.step(info)
            rows.append(np.concatenate([row, np.array([rew, float(term), CAUSE[cause], fn._consecutive_offroad,
                                                       fn._last_delta_yaw, fn.max_actions], dtype=float)]))
        seqs.append(rows)
    save("shaping_reward.npz", rows=np.array(seqs))


# ---------------------------------------------------------------- G8 comfort
def gen_comfort(rng):
    rows = []
    for i in range(2000):
        sp, psp = rng.uniform(-5, 45, 2)
        yaw, pyaw = rng.uniform(-4, 4, 2)
        prevs = rng.normal(0, 3, 3)
        has_prev = float(rng.random() < 0.8)
        out = compute_comfort_kinematics(
            speed_px_s=sp, prev_speed_px_s=psp, yaw_rad=yaw, prev_yaw_rad=pyaw, dt=0.1, meters_per_pixel=0.3125,
            prev_accel_long=prevs[0] if has_prev else None, prev_accel_lat=prevs[1] if has_prev else None,
            prev_yaw_rate_deg=prevs[2] if has_prev else None)
        nv, _ = count_comfort_violations(out)
        rows.append((sp, psp, yaw, pyaw, *prevs, has_prev, out["speed_mps"], out["accel_long"], out["accel_lat"],
                     out["jerk_long"], out["jerk_lat"], out["yaw_rate"], out["yaw_acc"], nv))
    save("comfort.npz", rows=np.array(rows, dtype=float))


# ---------------------------------------------------------------- G9 route geometry
def gen_route_geom(rng):
    rows, rxs, rys = [], [], []
    for r in range(150):
        rx, ry = rand_route(rng, int(rng.integers(1, 50)))
        route = list(zip(np.array(rx, np.int32), np.array(ry, np.int32)))
        lengths = cumulative_lengths(route)
        for q in range(6):
            i = int(rng.integers(0, len(rx)))
            px, py = float(rx[i] + rng.normal(0, 8)), float(ry[i] + rng.normal(0, 8))
            s = compute_route_progress(px, py, route, lengths)
            k = int(rng.integers(0, len(rx)))
            wps = np.array([np.array(rx[k:k + 5], float), np.array(ry[k:k + 5], float)]).T
            le = lateral_error(px, py, wps, signed=True)
            rows.append((r, px, py, s, lengths[-1], k, min(5, len(rx) - k), le))
        rxs.append(rx); rys.append(ry)
    rx_, off = ragged(rxs, np.int32)
    ry_, _ = ragged(rys, np.int32)
    save("route_geom.npz", route_x=rx_, route_y=ry_, off=off, rows=np.array(rows, dtype=float))


# ---------------------------------------------------------------- G10 seeds
def gen_seeds():
    out = {"derive_seed": [], "bundle": []}
    for base in (0, 1, 7, 11, 10000, 20000, 40001, 2**31 - 2):
        for part in ("route", "traffic", "scenario"):
            out["derive_seed"].append([base, part, derive_seed(base, part)])
        b = build_rng_bundle(scene_seed=base)
        out["bundle"].append({
            "scene_seed": base, "route_seed": b.route_seed, "traffic_seed": b.traffic_seed,
            "scenario_seed": b.scenario_seed,
            "route_rng_random": [b.route_rng.random() for _ in range(3)],
            "route_np_integers": [int(b.route_np_rng.integers(-1, 2)) for _ in range(4)],
        })
    with open(os.path.join(OUT, "seeds.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("seeds.json written")


def main():
    rng = np.random.default_rng(20261015)
    gen_state_update(rng)
    gen_smooth(rng)
    gen_stanley(rng)
    gen_hero(rng)
    gen_actors(rng)
    gen_carl(rng)
    gen_shaping(rng)
    gen_comfort(rng)
    gen_route_geom(rng)
    gen_seeds()


if __name__ == "__main__":
    main()
