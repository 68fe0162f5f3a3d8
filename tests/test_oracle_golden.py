"""Pin the CPU oracle (and the host reset-time arithmetic) to the reference.

Every fixture under tests/golden/ was captured by running the reference's own
Python functions (tests/golden/make_golden.py). Tolerances: the oracle
restates float64 NumPy/libm arithmetic in C with the same operation order, so
the kinematics match to ~1e-12 relative; index/branch outputs (argmin
indices, causes, termination, behaviour states) must match exactly. The
Savitzky–Golay route smoother is re-derived in C by normal equations instead of
SciPy's SVD lstsq, so it is compared at 1e-8 absolute.
"""
from __future__ import annotations

import ctypes
import json
import os

import numpy as np
import pytest

import oracle as O
from carlabev_env_amd import layout as LY
from carlabev_env_amd.routes import ControllerInit, smooth_and_compute as host_smooth, cumulative_lengths_int
from carlabev_env_amd.scene_pack import ActorSpec, init_actor_slot
from carlabev_env_amd.params import CbevParams, CARL_DEFAULTS, SHAPING_DEFAULTS
from carlabev_env_amd.config import REWARD_PROFILES

G = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def ragged_get(flat, off, i):
    return flat[off[i]:off[i + 1]]


def close(a, b, rtol=1e-12, atol=1e-12):
    return np.allclose(a, b, rtol=rtol, atol=atol, equal_nan=True)


# ------------------------------------------------------------- kinematics
def test_state_update_matches_reference():
    z = load("state_update.npz")
    init, acc, delta, out = z["init"], z["acc"], z["delta"], z["out"]
    for m in range(init.shape[0]):
        st = np.zeros(8)
        st[:4] = init[m, :4]
        for k in range(acc.shape[1]):
            O.state_update(st, acc[m, k], delta[m, k], init[m, 4])
            assert close(st, out[m, k], rtol=1e-13, atol=1e-12), (m, k, st, out[m, k])


def test_host_smoothing_is_bit_exact_with_reference():
    z = load("smooth_route.npz")
    for i in range(len(z["in_off"]) - 1):
        rx = ragged_get(z["in_x"], z["in_off"], i)
        ry = ragged_get(z["in_y"], z["in_off"], i)
        cx, cy, cyaw, _, _ = host_smooth(rx, ry, window=11, poly=3)
        assert np.array_equal(cx, ragged_get(z["cx"], z["out_off"], i))
        assert np.array_equal(cy, ragged_get(z["cy"], z["out_off"], i))
        assert np.array_equal(cyaw, ragged_get(z["cyaw"], z["out_off"], i))


def test_oracle_smoothing_matches_reference():
    z = load("smooth_route.npz")
    for i in range(len(z["in_off"]) - 1):
        rx = ragged_get(z["in_x"], z["in_off"], i)
        ry = ragged_get(z["in_y"], z["in_off"], i)
        cx, cy, cyaw = O.smooth_and_compute(rx, ry, 11, 3)
        gx = ragged_get(z["cx"], z["out_off"], i)
        gyaw = ragged_get(z["cyaw"], z["out_off"], i)
        assert len(cx) == len(gx), i
        assert np.allclose(cx, gx, atol=1e-8, rtol=0), (i, np.abs(cx - gx).max())
        assert np.allclose(cy, ragged_get(z["cy"], z["out_off"], i), atol=1e-8, rtol=0)
        # headings compared modulo 2*pi: a route running exactly west can come out as
        # +pi or -pi depending on the sign of a ~1e-16 gradient (np.unwrap then
        # carries that branch along the whole route)
        dyaw = (cyaw - gyaw + np.pi) % (2 * np.pi) - np.pi
        assert np.allclose(dyaw, 0.0, atol=1e-7), (i, np.abs(dyaw).max())


def test_stanley_matches_reference():
    z = load("stanley.npz")
    for row in z["rows"]:
        r, x, y, yaw, v, tidx, ts, idx0, err, delta, idx1, pid = row
        r = int(r)
        cx, cy, cyaw = (ragged_get(z[k], z["off"], r) for k in ("cx", "cy", "cyaw"))
        i0, e = O.calc_target_index(x, y, yaw, cx, cy)
        assert i0 == int(idx0)
        assert close(e, err, rtol=1e-12, atol=1e-12)
        d, i1 = O.stanley_control(x, y, yaw, v, cx, cy, cyaw, int(tidx))
        assert i1 == int(idx1)
        assert close(d, delta, rtol=1e-12, atol=1e-13), (d, delta)
        assert close(1.0 * (ts - v), pid)


def test_comfort_matches_reference():
    z = load("comfort.npz")
    for row in z["rows"]:
        sp, psp, yaw, pyaw, p0, p1, p2, has_prev = row[:8]
        out = O.comfort(sp, psp, yaw, pyaw, int(has_prev), p0, p1, p2)
        assert close(out, row[8:15], rtol=1e-12, atol=1e-9)
        nv = O.lib().orc_comfort_violations(out[1], out[2], out[5], out[3], out[4], out[6])
        assert nv == int(row[15])


def test_route_geometry_matches_reference():
    z = load("route_geom.npz")
    for row in z["rows"]:
        r, px, py, s, total, k, nw, le = row
        r, k, nw = int(r), int(k), int(nw)
        rx = ragged_get(z["route_x"], z["off"], r)
        ry = ragged_get(z["route_y"], z["off"], r)
        cum = O.cumulative_lengths(rx, ry)
        assert close(cum[-1], total)
        assert np.array_equal(cum, cumulative_lengths_int(rx, ry))
        assert close(O.route_progress(px, py, rx, ry, cum), s, rtol=1e-12, atol=1e-9)
        e = O.lateral_error(px, py, rx[k:k + nw].astype(float), ry[k:k + nw].astype(float))
        assert close(e, le, rtol=1e-12, atol=1e-12) or (np.isinf(e) and np.isinf(le))


# ------------------------------------------------------------- hero
def test_hero_reset_and_physics_match_reference():
    z = load("hero.npz")
    init, acts, traj, profiles = z["init"], z["actions"], z["traj"], z["profiles"]
    for e in range(init.shape[0]):
        x, y, yaw, v, tidx, seed, win, v0, vt = init[e]
        rx = ragged_get(z["route_x"], z["route_off"], e)
        ry = ragged_get(z["route_y"], z["route_off"], e)
        ci = ControllerInit(rx, ry, v0 / 0.3125, jitter_start=True, np_rng=np.random.default_rng(int(seed)),
                            hero=True)
        assert (ci.x, ci.y, ci.yaw, ci.v, ci.target_idx) == (x, y, yaw, v, int(tidx)), e
        assert np.array_equal(ci.cx, ragged_get(z["cx"], z["cx_off"], e))
        st = np.zeros(13)
        st[:4] = (x, y, yaw, v)
        st[9] = vt / 0.3125
        it = np.array([int(tidx), len(ci.cx), 0], dtype=np.int32)
        cx, cy, cyaw = np.ascontiguousarray(ci.cx), np.ascontiguousarray(ci.cy), np.ascontiguousarray(ci.cyaw)
        out = np.zeros(11)
        scale = int(1024 / int(win))
        cont = str(profiles[e]).startswith("continuous")
        for k in range(traj.shape[1]):
            g, s, b = (np.float32(a) for a in acts[e, k, :3])
            if cont:
                g, s, b = np.clip(g, 0.0, 1.0), np.clip(s, -1.0, 1.0), np.clip(b, 0.0, 1.0)
            O.lib().orc_hero_physics_vec(O.ptr(st), O.ptr(it), O.ptr(cx), O.ptr(cy), O.ptr(cyaw), float(g),
                                         float(s), float(b), scale, O.ptr(out))
            ref = traj[e, k]
            got = np.concatenate([st[:5], [it[0]], st[4:8], out])
            got[4] = st[8]
            assert it[0] == int(ref[5]), (e, k)
            assert close(got, ref, rtol=1e-11, atol=1e-9), (e, k, np.abs(got - ref).max(), got - ref)


# ------------------------------------------------------------- actors
BEH_TYPES = {0: None, 1: "timed_brake", 2: "cross", 3: "stop_mid", 4: "yield_return"}
BEH_PARAMS = {1: ("start_brake_t", "decel_mps2"), 2: ("start_delay",), 3: ("start_delay",),
              4: ("start_delay", "yield_duration")}


def test_actor_reset_and_step_match_reference():
    z = load("actors.npz")
    init, traj = z["init"], z["traj"]
    caps = LY.Caps(8, 1, 64, 1)
    lay = LY.Layout.make(caps)
    for e in range(init.shape[0]):
        x, y, yaw, v, tidx, seed, speed, kind, beh, p0, p1 = init[e]
        rx = ragged_get(z["route_x"], z["route_off"], e)
        ry = ragged_get(z["route_y"], z["route_off"], e)
        b = int(beh)
        spec_b = None
        if b:
            names = BEH_PARAMS[b]
            spec_b = {"type": BEH_TYPES[b], "params": dict(zip(names, (p0, p1)[:len(names)]))}
        spec = ActorSpec("vehicle" if kind == 0 else "pedestrian", list(rx), list(ry), speed, spec_b)
        buf = np.zeros(lay.record_bytes, np.uint8)
        view = LY.RecordView(buf, lay)
        init_actor_slot(view, 0, spec, np.random.default_rng(int(seed)))
        got0 = (view.ad[LY.AD["X"], 0], view.ad[LY.AD["Y"], 0], view.ad[LY.AD["YAW"], 0], view.ad[LY.AD["V"], 0],
                view.ai[LY.AI["TIDX"], 0])
        assert got0 == (x, y, yaw, v, int(tidx)), e
        t = 0.0
        for k in range(traj.shape[1]):
            t += 0.1
            O.lib().orc_actor_step_rec(ctypes.byref(caps.c()), O.ptr(buf), 0, t, 0.1)
            ref = traj[e, k]
            got = np.array([view.ad[LY.AD["X"], 0], view.ad[LY.AD["Y"], 0], view.ad[LY.AD["YAW"], 0],
                            view.ad[LY.AD["V"], 0], view.ai[LY.AI["TIDX"], 0], view.ad[LY.AD["T_SPEED"], 0],
                            view.ad[LY.AD["CT_SPEED"], 0], view.ai[LY.AI["BSTATE"], 0],
                            view.ai[LY.AI["NROUTE"], 0], view.ai[LY.AI["NRX"], 0]])
            assert np.array_equal(got[[4, 7, 8, 9]], ref[[4, 7, 8, 9]]), (e, k, got, ref)
            assert close(got, ref, rtol=1e-9, atol=1e-7), (e, k, got - ref)


# ------------------------------------------------------------- rewards
def make_params(profile: str) -> CbevParams:
    P = CbevParams()
    spec = REWARD_PROFILES[profile]
    carl = dict(CARL_DEFAULTS)
    sh = dict(SHAPING_DEFAULTS)
    if spec["family"] == "carl":
        carl.update({k: v for k, v in spec["parameters"].items() if k in carl})
    for k, v in carl.items():
        setattr(P, k, float(v))
    for k, v in sh.items():
        if k == "max_actions":
            P.max_actions = int(v)
        elif k == "offroad_terminate_after":
            P.offroad_terminate_after = int(v)
        elif k.startswith("zero_"):
            setattr(P, k, int(bool(v)))
        else:
            setattr(P, k, float(v))
    return P


def row_to_info(row) -> O.OrcInfo:
    info = O.OrcInfo()
    for i in range(4):
        info.state[i] = row[i]
        info.last_state[i] = row[4 + i]
    info.dist2wp = row[8]
    for i in range(3):
        info.set_point[i] = row[9 + i]
    info.n_wps = int(row[12])
    for i in range(6):
        info.comfort[i] = row[13 + i]
    info.dist2goal, info.dist2goal_t1, info.speed_limit = row[19], row[20], row[21]
    info.tile_class, info.collided, info.actor_id, info.n_actors = (int(v) for v in row[22:26])
    wps = row[26:41].reshape(5, 3)
    for i in range(info.n_wps):
        info.wps_x[i], info.wps_y[i] = wps[i, 0], wps[i, 1]
    act = row[41:57].reshape(4, 4)
    for i in range(info.n_actors):
        for j in range(4):
            info.actors[i][j] = act[i, j]
    return info


def test_carl_reward_matches_reference():
    z = load("carl_reward.npz")
    rows, profiles = z["rows"], z["profiles"]
    for s in range(rows.shape[0]):
        P = make_params(str(profiles[s]))
        rx = ragged_get(z["route_x"], z["route_off"], s)
        ry = ragged_get(z["route_y"], z["route_off"], s)
        rx32, ry32 = O.i32(rx), O.i32(ry)
        cum = O.cumulative_lengths(rx, ry)
        spv = np.zeros(1, np.int32)
        sp = np.zeros(1)
        for k in range(rows.shape[1]):
            row = rows[s, k]
            info = row_to_info(row)
            oi = np.zeros(2, np.int32)
            od = np.zeros(6)
            r = O.lib().orc_carl_step_vec(ctypes.byref(P), O.ptr(spv), O.ptr(sp), ctypes.byref(info), O.ptr(rx32),
                                          O.ptr(ry32), O.ptr(cum), len(rx), O.ptr(oi), O.ptr(od))
            ref = row[57:]
            assert oi[0] == int(ref[2]) and oi[1] == int(ref[1]), (s, k, oi, ref[:3])
            assert close(r, ref[0], rtol=1e-12, atol=1e-12), (s, k, r, ref[0])
            assert close(od, ref[3:9], rtol=1e-12, atol=1e-12), (s, k, od, ref[3:9])
            if not np.isnan(ref[9]):
                assert close(sp[0], ref[9], rtol=1e-12, atol=1e-9)


def test_shaping_reward_matches_reference():
    z = load("shaping_reward.npz")
    rows = z["rows"]
    for s in range(rows.shape[0]):
        P = make_params("shaping_base_v1")
        P.max_actions = int(rows[s, 0, -1])
        k_ = np.zeros(1, np.int32)
        off = np.zeros(1, np.int32)
        ldy = np.zeros(1)
        for k in range(rows.shape[1]):
            row = rows[s, k]
            info = row_to_info(row)
            oi = np.zeros(2, np.int32)
            r = O.lib().orc_shaping_step_vec(ctypes.byref(P), O.ptr(k_), O.ptr(off), O.ptr(ldy), ctypes.byref(info),
                                             O.ptr(oi))
            ref = row[57:]
            assert oi[0] == int(ref[2]) and oi[1] == int(ref[1]), (s, k)
            assert close(r, ref[0], rtol=1e-12, atol=1e-12), (s, k, r, ref[0])
            assert off[0] == int(ref[3])
            assert close(ldy[0], ref[4])


# ------------------------------------------------------------- seeds
def test_seed_derivation_matches_reference():
    from carlabev_env_amd.scene_gen import derive_seed, build_rng_bundle
    with open(os.path.join(G, "seeds.json")) as f:
        ref = json.load(f)
    for base, part, val in ref["derive_seed"]:
        assert derive_seed(base, part) == val
    for b in ref["bundle"]:
        bundle = build_rng_bundle(scene_seed=b["scene_seed"])
        assert (bundle.route_seed, bundle.traffic_seed, bundle.scenario_seed) == (
            b["route_seed"], b["traffic_seed"], b["scenario_seed"])
        assert [bundle.route_rng.random() for _ in range(3)] == b["route_rng_random"]
        assert [int(bundle.route_np_rng.integers(-1, 2)) for _ in range(4)] == b["route_np_integers"]
