"""Authored scene files (assets/scenes/*.json) -> SceneSpec, on the host.

Two formats reach `SceneGenerator.build_scene` through `options["config_file"]`
or `options["scene"] = "<path>.json"` (src/managers/scene_generator.py:98-138):

* authored scenes ("actors" list, version 2): `Scenario.load_config`
  (src/scenes/scenarios/__init__.py:210-338) with the optional seeded variation
  (`_resolve_variation_settings` / `_apply_actor_variation`, :87-186), routes
  from waypoints (:12-34), behaviours normalised by `build_behavior`
  (src/actors/behavior/registry.py:94-143) and traffic-light strips
  (src/actors/traffic_light.py:11-43);
* scenario configs (no actors, version 1 or the legacy {"scenario", "kwargs"}
  form): `normalize_scenario_config` + `build_scenario_options_from_config`
  (src/scenes/scenarios/specs.py:185-278), which turn the file into sampler
  options for lead_brake / jaywalk / red_light_runner.

Files are read as JSON only. The realised spec is packed into a device record
like every other scene (scene_pack.pack_scene).
"""
from __future__ import annotations

import json
import random
from copy import deepcopy

import numpy as np

from .scene_pack import ActorSpec, SceneSpec, TrafficLightSpec

# ScenarioSpec fields (specs.py:49-96): key -> (default, cast)
SCENARIO_FIELDS = {
    "jaywalk": {"ego_speed": (12.0, float), "cross_delay": (1.5, float), "pedestrian_speed": (1.6, float),
                "cross_offset": (0.0, float), "yield_duration": (1.2, float), "rear_gap": (5.0, float),
                "rear_speed": (10.0, float)},
    "lead_brake": {"ego_speed": (12.0, float), "lead_gap": (7.5, float), "lead_speed": (12.0, float),
                   "brake_delay": (2.5, float), "brake_strength": (4.0, float), "left_speed": (14.0, float),
                   "rear_gap": (5.0, float), "rear_speed": (10.0, float), "rear_brake_delay": (3.0, float)},
    "red_light_runner": {"ego_speed": (10.0, float), "adv_speed": (16.0, float), "intersection_index": (11, int)},
}

# behaviour library (registry.py:33-76): actor type -> {id: ((field, default), ...)}
BEHAVIOR_LIBRARY = {
    "agent": {"none": ()},
    "vehicle": {"constant_speed": (), "timed_brake": (("start_brake_t", 3.5), ("decel_mps2", 1.0))},
    "pedestrian": {"cross": (("start_delay", 0.0),), "stop_mid": (("start_delay", 0.0),),
                   "yield_return": (("start_delay", 0.0), ("yield_duration", 1.0))},
}
LEGACY_BEHAVIOR_NAMES = {"Normal": "constant_speed", "CrossBehavior": "cross", "StopMidBehavior": "stop_mid",
                         "StopReturnBehavior": "yield_return", "LeadBrakeBehavior": "timed_brake"}
TL_STATES = {"red": "red", "yellow": "yellow", "green": "green"}


def normalize_behavior(actor_type: str, behavior) -> dict:
    """normalize_behavior_spec (registry.py:100-118): unknown ids fall back to the
    actor type's first behaviour; every field parsed with its default."""
    lib = BEHAVIOR_LIBRARY.get(actor_type, {})
    if not lib:
        return {"type": "none", "params": {}}
    if behavior in (None, "", "Normal"):
        return {"type": "none" if "none" in lib else next(iter(lib)), "params": {}}
    if isinstance(behavior, str):
        bid = LEGACY_BEHAVIOR_NAMES.get(behavior, behavior)
        bid = bid if bid in lib else next(iter(lib))
        return {"type": bid, "params": {}}
    bid = LEGACY_BEHAVIOR_NAMES.get(behavior.get("type", ""), behavior.get("type", ""))
    bid = bid if bid in lib else next(iter(lib))
    raw = behavior.get("params", {}) or behavior.get("behavior_kwargs", {}) or {}
    params = {k: float(d if raw.get(k) in (None, "") else raw.get(k)) for k, d in lib[bid]}
    return {"type": bid, "params": params}


def _linear_route(start, end, step_px=8):
    dx, dy = end[0] - start[0], end[1] - start[1]
    n = max(2, int(max(abs(dx), abs(dy)) / max(1, step_px)) + 1)
    rx = np.linspace(start[0], end[0], n).round().astype(int).tolist()
    ry = np.linspace(start[1], end[1], n).round().astype(int).tolist()
    return rx, ry


def route_from_waypoints(waypoints, step_px=8):
    """_build_route_from_waypoints (__init__.py:22-34): 8-px linear segments."""
    if len(waypoints) < 2:
        return [], []
    rx, ry = [], []
    for i in range(len(waypoints) - 1):
        sx, sy = _linear_route(waypoints[i], waypoints[i + 1], step_px)
        if i > 0:
            sx, sy = sx[1:], sy[1:]
        rx.extend(sx)
        ry.extend(sy)
    return rx, ry


def _sample(spec, rng: random.Random, fallback=None):
    """_sample_variation_value (__init__.py:41-62)."""
    if spec is None:
        return fallback
    if not isinstance(spec, dict):
        return spec
    mode = spec.get("mode", "fixed")
    if mode == "fixed":
        return spec.get("value", fallback)
    if mode == "uniform":
        return rng.uniform(float(spec["low"]), float(spec["high"]))
    if mode == "normal":
        v = rng.normalvariate(float(spec["mean"]), float(spec["std"]))
        clip = spec.get("clip")
        if clip is not None and len(clip) == 2:
            v = max(float(clip[0]), min(float(clip[1]), v))
        return v
    if mode == "choice":
        vals = spec.get("values", [])
        return rng.choice(list(vals)) if vals else fallback
    return fallback


def _waypoints(actor: dict) -> list:
    """_normalize_waypoints (__init__.py:65-84)."""
    if actor.get("waypoints"):
        return [[int(round(p[0])), int(round(p[1]))] for p in actor["waypoints"]]
    start, goal = actor.get("start"), actor.get("goal")
    rx, ry = actor.get("rx", []), actor.get("ry", [])
    if start is None and rx and ry:
        start = {"x": rx[0], "y": ry[0]}
    if goal is None and rx and ry:
        goal = {"x": rx[-1], "y": ry[-1]}
    if start is None or goal is None:
        return []
    return [[int(round(start["x"])), int(round(start["y"]))], [int(round(goal["x"])), int(round(goal["y"]))]]


def _variation(data: dict, overrides: dict) -> dict:
    """_resolve_variation_settings (__init__.py:87-109)."""
    var = deepcopy(data.get("variation") or {})
    enabled = overrides.get("variation_enabled")
    enabled = bool(var.get("enabled", False)) if enabled is None else bool(enabled)
    if not enabled:
        return {"enabled": False, "seed": None, "spec": var}
    seed = overrides.get("variation_seed")
    if seed is None:
        seed = var.get("default_seed")
    return {"enabled": True, "seed": int(0 if seed is None else seed), "spec": var}


def _vary_actor(actor_data: dict, scene_var: dict, index: int):
    """_apply_actor_variation (__init__.py:112-186): draws in the reference's order
    (waypoint jitter, global speed scale, speed spec, behaviour params, signal)."""
    actor = deepcopy(actor_data)
    av = deepcopy(actor.get("variation") or {})
    if not scene_var["enabled"] or not av.get("enabled", False):
        return actor, None
    seed = scene_var["seed"] + int(av.get("seed_offset", index))
    rng = random.Random(seed)
    realized = {"type": actor.get("type"), "role": actor.get("role"), "seed": seed}
    glob = scene_var["spec"].get("global", {}) or {}
    wps = _waypoints(actor)
    lock = (av.get("constraints", {}) or {}).get("lock_endpoints", True)
    jitter = av.get("waypoint_jitter_px", glob.get("waypoint_jitter_px"))
    if jitter and wps:
        r = float(jitter)
        out = []
        for i, p in enumerate(wps):
            if lock and i in {0, len(wps) - 1}:
                out.append(list(p))
                continue
            out.append([int(round(p[0] + rng.uniform(-r, r))), int(round(p[1] + rng.uniform(-r, r)))])
        actor["waypoints"] = out
        actor["start"] = {"x": out[0][0], "y": out[0][1]}
        actor["goal"] = {"x": out[-1][0], "y": out[-1][1]}
        realized["waypoint_jitter_px"] = r
        realized["waypoints"] = out
    speed = float(actor.get("cruise_speed", actor.get("initial_speed", actor.get("speed", 0.0))))
    scale = _sample(glob.get("speed_scale"), rng, fallback=1.0)
    if av.get("speed") is not None:
        speed = float(_sample(av.get("speed"), rng, fallback=speed))
    else:
        speed = speed * float(scale)
    speed = max(0.0, speed)
    actor["speed"] = actor["initial_speed"] = actor["cruise_speed"] = speed
    realized["speed"] = round(float(speed), 4)
    beh = deepcopy(actor.get("behavior") or {})
    params = deepcopy(beh.get("params") or {})
    rb = {}
    for key, spec in (av.get("behavior_params", {}) or {}).items():
        if key in params:
            params[key] = _sample(spec, rng, fallback=params[key])
            rb[key] = round(float(params[key]), 4)
    if rb:
        beh["params"] = params
        actor["behavior"] = beh
        realized["behavior_params"] = rb
    if actor.get("type") == "traffic_light" and av.get("signal_state"):
        actor["signal_state"] = _sample(av.get("signal_state"), rng, fallback=actor.get("signal_state", "red"))
        realized["signal_state"] = actor["signal_state"]
    return actor, realized


def load_authored_scene(data: dict, overrides: dict | None = None):
    """Scenario.load_config for the actors format (__init__.py:210-338).
    Returns (SceneSpec, len_route_px, context)."""
    overrides = dict(overrides or {})
    var = _variation(data, overrides)
    realized_all = []
    agent = None
    vehicles, peds, tls = [], [], []
    for idx, actor_data in enumerate(data["actors"]):
        actor, realized = _vary_actor(actor_data, var, idx)
        if realized is not None:
            realized_all.append(realized)
        atype = actor_data["type"]
        rx, ry = actor.get("rx"), actor.get("ry")
        if (not rx or not ry) and actor.get("waypoints"):
            rx, ry = route_from_waypoints(actor["waypoints"])
        rx, ry = rx or [], ry or []
        speed = actor.get("cruise_speed", actor.get("initial_speed", actor.get("speed", 2.0)))
        if atype == "agent":
            agent = (rx, ry, speed, speed)
        elif atype in ("vehicle", "pedestrian"):
            default = "constant_speed" if atype == "vehicle" else "cross"
            beh = normalize_behavior(atype, actor.get("behavior", default))
            (vehicles if atype == "vehicle" else peds).append(
                ActorSpec(atype, [float(v) for v in rx], [float(v) for v in ry], float(speed), beh))
        elif atype == "traffic_light":
            start, goal = actor.get("start"), actor.get("goal")
            if start is None and rx and ry:
                start = {"x": rx[0], "y": ry[0]}
            if goal is None and rx and ry:
                goal = {"x": rx[-1], "y": ry[-1]}
            if start is None or goal is None:
                continue
            dx = float(goal["x"]) - float(start["x"])
            dy = float(goal["y"]) - float(start["y"])
            orient = actor.get("orientation", "horizontal" if abs(dx) >= abs(dy) else "vertical")
            tls.append(TrafficLightSpec(0.5 * (float(start["x"]) + float(goal["x"])),
                                        0.5 * (float(start["y"]) + float(goal["y"])), orient,
                                        TL_STATES.get(actor.get("signal_state", "red"), "red"),
                                        actor.get("width"), actor.get("length")))
    if agent is None:
        raise ValueError(f"authored scene {data.get('scene_id')!r} has no agent")
    rx, ry = agent[0], agent[1]
    # compute_total_dist_px([rx, ry]) (scenes/utils.py:214-221) walks the pair (rx, ry)
    # as two points, so the reference's value is |(ry[0] - rx[0], ry[1] - rx[1])|
    len_route = float(np.hypot(float(ry[0]) - float(rx[0]), float(ry[1]) - float(rx[1])))
    ctx = {"scene_id": data.get("scene_id"), "authored_scene": True, "variation_enabled": var["enabled"],
           "variation_seed": var["seed"], "variation_actor_count": len(realized_all),
           "variation_realized": realized_all}
    spec = SceneSpec([float(v) for v in rx], [float(v) for v in ry], float(agent[3]), float(agent[2]),
                     vehicles=vehicles, pedestrians=peds, traffic_lights=tls)
    return spec, len_route, ctx


def normalize_scenario_config(data: dict) -> dict:
    """normalize_scenario_config + build_scenario_config + coerce_parameters (specs.py:185-241)."""
    if data.get("type") == "scenario_config" or "scenario_id" in data:
        sid = data.get("scenario_id")
        level = int(data.get("level", 1))
        anchor = data.get("anchor", {}) or {}
        params = data.get("parameters", {}) or {}
    elif "scenario" in data and "kwargs" in data:
        kw = dict(data.get("kwargs", {}))
        sid = data.get("scenario")
        level = int(kw.pop("level", 1))
        anchor = {"x": kw.pop("anchor_x", None), "y": kw.pop("anchor_y", None)}
        kw.pop("scene", None)
        params = kw
    else:
        raise ValueError("Unsupported scenario config format.")
    if sid not in SCENARIO_FIELDS:
        raise KeyError(sid)
    coerced = {k: cast(d if params.get(k) in (None, "") else params.get(k))
               for k, (d, cast) in SCENARIO_FIELDS[sid].items()}
    return {"version": 1, "type": "scenario_config", "scene_id": data.get("scene_id", sid), "scenario_id": sid,
            "level": level,
            "anchor": {"x": None if anchor.get("x") is None else int(anchor["x"]),
                       "y": None if anchor.get("y") is None else int(anchor["y"])},
            "parameters": coerced}


def scenario_options_from_config(config: dict, overrides: dict | None = None) -> dict:
    """build_scenario_options_from_config (specs.py:249-273)."""
    opts = dict(config.get("parameters", {}))
    anchor = config.get("anchor", {}) or {}
    if anchor.get("x") is not None:
        opts["anchor_x"] = anchor["x"]
    if anchor.get("y") is not None:
        opts["anchor_y"] = anchor["y"]
    opts["level"] = int(config.get("level", 1))
    opts["scene"] = config["scenario_id"]
    for k, v in (overrides or {}).items():
        if k in {"config_file", "scene", "reset_mask"} or v is None:
            continue
        opts[k] = v
    return opts


def read_scene_file(path: str) -> dict:
    with open(path, "r", encoding="utf-8") as f:
        return json.load(f)
