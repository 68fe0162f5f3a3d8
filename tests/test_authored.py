"""Authored scene files: the host loader (carlabev_env_amd/authored.py) against
scenes realised by the reference's own loader (tests/golden/authored.json,
made by tests/golden/make_golden_authored.py from the reference's assets).

Compared exactly: ego route and speeds, actor authored routes, cruise speeds,
behaviour types and parameters (after the seeded variation draws), traffic-light
strips, and the realised-variation context. Not compared: actor spawn jitter
(fresh entropy in the reference, stanley_controller.py:39-42).
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from carlabev_env_amd.authored import load_authored_scene, normalize_scenario_config, scenario_options_from_config

G = os.path.join(os.path.dirname(__file__), "golden")
BEH_CLASS = {"cross": "CrossBehavior", "stop_mid": "StopMidBehavior", "yield_return": "StopReturnBehavior",
             "timed_brake": "LeadBrakeBehavior"}
TL_STATE = {"red": 0, "yellow": 1, "green": 2}


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(G, "authored.json")) as f:
        return json.load(f)


def _beh(spec_beh):
    """Our normalised behaviour dict -> the reference object's class and fields."""
    t = spec_beh["type"]
    if t in ("none", "constant_speed"):
        return None
    p = spec_beh["params"]
    out = {"class": BEH_CLASS[t]}
    if t == "timed_brake":
        out.update(start_brake_t=p["start_brake_t"], dec_rate=p["decel_mps2"])
    elif t == "yield_return":
        out.update(start_delay=p["start_delay"], stop_duration=p["yield_duration"])
    else:
        out.update(start_delay=p["start_delay"])
    return out


def test_authored_scenes_match_reference_loader(gold):
    for case in gold["cases"]:
        data = gold["inputs"][case["file"]]
        spec, len_route, ctx = load_authored_scene(data, case["overrides"])
        ref = case["scene"]
        tag = (case["file"], case["overrides"])
        assert spec.agent_rx == ref["agent"]["rx"] and spec.agent_ry == ref["agent"]["ry"], tag
        assert spec.target_speed_mps == ref["agent"]["speed"] and spec.initial_speed_mps == ref["agent"]["speed2"]
        assert len_route == pytest.approx(ref["len_route"], abs=0, rel=0), tag
        for kind, mine in (("vehicle", spec.vehicles), ("pedestrian", spec.pedestrians)):
            assert len(mine) == len(ref[kind]), tag
            for a, r in zip(mine, ref[kind]):
                assert a.rx == r["rx"] and a.ry == r["ry"], tag
                assert a.speed_mps == r["cruise_mps"], tag
                assert _beh(a.behavior) == r["behavior"], tag
        assert len(spec.traffic_lights) == len(ref["traffic_light"])
        for t, r in zip(spec.traffic_lights, ref["traffic_light"]):
            assert (t.x, t.y, t.orientation, TL_STATE[t.state]) == (r["x"], r["y"], r["orientation"], r["state"])
            # strip size: reference defaults when the file has none (traffic_light.py:28-37)
            w = float(t.width) if t.width is not None else max(1.0, 0.45 / (40.0 / 128.0)) + 1.0
            ln = float(t.length) if t.length is not None else max(4.0, 8.5 / (40.0 / 128.0))
            assert (w, ln) == (r["width"], r["length"]), tag
        for k in ("scene_id", "authored_scene", "variation_enabled", "variation_seed", "variation_actor_count",
                  "variation_realized"):
            assert ctx[k] == ref["context"][k], (tag, k)


def test_scenario_config_format_to_sampler_options():
    cfg = normalize_scenario_config({"scenario": "lead_brake", "kwargs": {"level": 2, "anchor_x": 850,
                                                                           "brake_delay": "3.0", "scene": "x"}})
    assert cfg["scenario_id"] == "lead_brake" and cfg["level"] == 2 and cfg["anchor"] == {"x": 850, "y": None}
    assert cfg["parameters"]["brake_delay"] == 3.0 and cfg["parameters"]["lead_gap"] == 7.5
    opts = scenario_options_from_config(cfg, {"scene_seed": 5, "config_file": "f.json", "ego_speed": None})
    assert opts["scene"] == "lead_brake" and opts["anchor_x"] == 850 and "anchor_y" not in opts
    assert opts["scene_seed"] == 5 and "config_file" not in opts and opts["ego_speed"] == 12.0
    with pytest.raises(ValueError):
        normalize_scenario_config({"foo": 1})


def test_authored_scene_files_pack_into_records(gold, tmp_path):
    """config_file / scene=<path>.json through the host reset builder: records pack and
    spawn-validate for every asset."""
    from carlabev_env_amd import EnvConfig
    from carlabev_env_amd import layout as LY
    from helpers import CAPS_FULL, world
    cfg, P, padded, layout, builder = world()
    for name, data in gold["inputs"].items():
        path = tmp_path / name
        path.write_text(json.dumps(data))
        for opts in ({"config_file": str(path)}, {"scene": str(path), "variation_seed": 3}):
            buf = np.zeros(layout.record_bytes, np.uint8)
            info, spec, ctx = builder.build(buf, 0, dict(opts, scene_seed=9))
            v = LY.RecordView(buf, layout)
            assert v.i("NACT") == len(spec.vehicles) + len(spec.pedestrians)
            assert v.i("NTL") == len(spec.traffic_lights)
            assert ctx["authored_scene"] and ctx["scene_id"] == data["scene_id"]
    # a scenario-config file (no actors) goes through the scenario sampler
    sc = tmp_path / "cfg.json"
    sc.write_text(json.dumps({"type": "scenario_config", "scenario_id": "jaywalk", "level": 3,
                              "anchor": {"x": None, "y": None}, "parameters": {"cross_delay": 0.5}}))
    buf = np.zeros(layout.record_bytes, np.uint8)
    info, spec, ctx = builder.build(buf, 0, {"config_file": str(sc), "scene_seed": 4})
    assert ctx["scene"] == "jaywalk" and ctx["level"] == 3
    assert spec.pedestrians[0].behavior["type"] == "yield_return"
