"""Golden realised scenes for authored scene JSON files, from the reference's loader.

Runs ONLY in the build container (needs /root/reference); writes
tests/golden/authored.json, which tests/test_authored.py pins the host loader
(carlabev_env_amd/authored.py) against. Captured reference code:
  Scenario.load_config (actors format)     src/scenes/scenarios/__init__.py:210-338
    _apply_actor_variation / waypoint routes :12-186
  build_behavior / normalize_behavior_spec src/actors/behavior/registry.py:94-143
  Vehicle / Pedestrian / TrafficLight construction (actor.py:43-77, traffic_light.py:11-75)

Inputs: the reference's authored scene assets (assets/scenes/*.json, scene data
read as JSON), stored with the fixture so the test needs no reference tree.
Captured per scene and variation setting: the ego tuple (route, speeds), each
actor's authored route (`_initial_rx/_initial_ry`), cruise speed and behaviour
parameters, and each traffic light's centre / orientation / state / strip size.
Actor spawn jitter is drawn from fresh entropy in the reference
(stanley_controller.py:39-42) and is not captured.
"""
from __future__ import annotations

import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refimport  # noqa: E402

refimport.setup()
refimport._bare_pkg("CarlaBEV.src.scenes", f"{refimport.REF}/CarlaBEV/src/scenes")

from CarlaBEV.src.scenes.scenarios import Scenario  # noqa: E402

BEHAVIOR_FIELDS = {"CrossBehavior": ("start_delay",), "StopMidBehavior": ("start_delay",),
                   "StopReturnBehavior": ("start_delay", "stop_duration"),
                   "LeadBrakeBehavior": ("start_brake_t", "dec_rate")}


def capture(path, overrides):
    data = json.load(open(path, encoding="utf-8"))
    sc = Scenario(data.get("scenario_id"), map_size=128)
    scene, len_route = sc.load_config(path, **overrides)
    out = {"len_route": float(len_route), "context": sc.last_loaded_context}
    ag = scene["agent"]
    out["agent"] = {"rx": [float(v) for v in ag[0]], "ry": [float(v) for v in ag[1]],
                    "speed": float(ag[2]), "speed2": float(ag[3])}
    for kind in ("vehicle", "pedestrian"):
        acts = []
        for a in scene[kind]:
            b = a.behavior
            beh = None
            if b is not None:
                name = type(b).__name__
                beh = {"class": name, **{k: float(getattr(b, k)) for k in BEHAVIOR_FIELDS[name]}}
            acts.append({"rx": [float(v) for v in a._initial_rx], "ry": [float(v) for v in a._initial_ry],
                         "cruise_mps": float(a.cruise_speed_mps), "behavior": beh})
        out[kind] = acts
    out["traffic_light"] = [{"x": float(t.x), "y": float(t.y), "orientation": t.orientation,
                             "state": int(t.signal_state), "width": float(t.width), "length": float(t.length)}
                            for t in scene["traffic_light"]]
    return out


def main():
    files = sorted(glob.glob(f"{refimport.REF}/CarlaBEV/assets/scenes/*.json"))
    fixture = {"inputs": {}, "cases": []}
    for path in files:
        name = os.path.basename(path)
        fixture["inputs"][name] = json.load(open(path, encoding="utf-8"))
        for overrides in ({}, {"variation_enabled": False}, {"variation_seed": 7}, {"variation_seed": 123456}):
            fixture["cases"].append({"file": name, "overrides": overrides, "scene": capture(path, overrides)})
    dst = os.path.join(HERE, "authored.json")
    with open(dst, "w") as f:
        json.dump(fixture, f, separators=(",", ":"))
    print(f"authored.json: {os.path.getsize(dst)} bytes, {len(fixture['cases'])} cases")


if __name__ == "__main__":
    main()
