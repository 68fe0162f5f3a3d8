"""Lane-graph planning and planned scenes against the reference's own planners.

Fixture: tests/golden/scenes_graph.json, written by
tests/golden/make_golden_scenes.py, which ran the reference's MapGraph /
GraphPlanner / SceneGenerator / RedLightRunningScenario (networkx 3.4.2) on the
graphs tools/convert_graphs.py extracted from assets/Town01/*.pkl:
  - node classes of every planner           map_graph.py:21-43
  - 200 seeded shortest paths + merged paths graph_planner.py:92-116
  - 52 seeded random-traffic scenes          scene_generator.py:95-327 (all rt_* presets,
    right/left-lane ego graphs, a route profile and an intersection/turn filter)
  - 5 red-light-runner scenes                red_light_running.py:74-245
  - 96 lead_brake / jaywalk scenes           lead_brake.py:18-129, jaywalk.py:29-117, every level
    (8 seeds each), the seeded level draw of build_scene (scene_generator.py:165-191)
    and kwarg overrides (anchors, speeds, gaps, delays)
Everything is compared exactly (the planner's arithmetic is raw/8 and the
same float sums in the same order), including how far each RNG stream was
advanced.
"""
from __future__ import annotations

import json
import os

import numpy as np
import pytest

from carlabev_env_amd import lane_graph
from carlabev_env_amd.scene_gen import SceneGenerator, build_rng_bundle

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "scenes_graph.json")))


@pytest.fixture(scope="module")
def gen():
    return SceneGenerator(None)


def test_node_classes_match_reference():
    graphs = lane_graph.planners("Town01")
    by_file = {stem: graphs[key] for key, stem in lane_graph.PLANNER_FILES.items()}
    for stem, classes in GOLD["node_classes"].items():
        assert by_file[stem].nodes == classes, stem


def test_shortest_and_merged_paths_match_reference():
    graphs = lane_graph.planners("Town01")
    by_file = {stem: graphs[key] for key, stem in lane_graph.PLANNER_FILES.items()}
    n_nopath = 0
    for case in GOLD["paths"]:
        g = by_file[case["graph"]]
        if case["path"] is None:
            n_nopath += 1
            with pytest.raises(lane_graph.NoPath):
                g.shortest_path(case["source"], case["target"])
        else:
            assert g.shortest_path(case["source"], case["target"]) == case["path"], case
        merged, coords = g.find_path(case["source"], case["target"])
        assert merged == case["merged"]
        assert [[float(v) for v in c] for c in coords] == case["coords"]
    assert n_nopath < len(GOLD["paths"])


def test_random_traffic_scenes_match_reference(gen):
    for case in GOLD["random"]:
        bundle = build_rng_bundle(scene_seed=case["seed"])
        spec = gen.build_scene(dict(case["options"]), bundle)
        ag = case["agent"]
        assert [float(v) for v in spec.agent_rx] == ag["rx"] and [float(v) for v in spec.agent_ry] == ag["ry"]
        assert spec.initial_speed_mps == ag["speed"] and spec.target_speed_mps == ag["target_speed"]
        assert spec.len_route_m == case["len_route"]
        assert len(spec.vehicles) == len(case["vehicles"])
        for a, ref in zip(spec.vehicles, case["vehicles"]):
            assert [float(v) for v in a.rx] == ref["rx"] and [float(v) for v in a.ry] == ref["ry"]
            assert a.speed_mps == ref["cruise_mps"]
        for k, v in case["context"].items():
            assert spec.context.get(k) == v, (case["seed"], k)
        # every RNG stream advanced exactly as far as the reference's
        assert bundle.route_rng.random() == case["route_rng_next"]
        assert bundle.traffic_rng.random() == case["traffic_rng_next"]
        assert float(bundle.traffic_np_rng.random()) == case["traffic_np_next"]


def test_red_light_runner_matches_reference(gen):
    for case in GOLD["red_light"]:
        spec = gen.red_light_runner(1, np.random.default_rng(0), dict(case["kwargs"]))
        ag, adv = case["agent"], case["adversary"]
        assert spec.agent_rx == ag["rx"] and spec.agent_ry == ag["ry"]
        assert spec.initial_speed_mps == ag["speed"] and spec.target_speed_mps == ag["target_speed"]
        assert spec.len_route_m == case["len_route"]
        (v,) = spec.vehicles
        assert v.rx == adv["rx"] and v.ry == adv["ry"] and v.speed_mps == adv["cruise_mps"]
        state = {"red": 0, "yellow": 1, "green": 2}
        got = [{"x": t.x, "y": t.y, "orientation": t.orientation, "state": state[t.state], "width": t.width,
                "length": t.length} for t in spec.traffic_lights]
        assert got == case["traffic_light"]


# our behaviour dicts (scene_pack / behavior/registry.py names) <-> the reference's objects
_JAYWALK = {"cross": "CrossBehavior", "stop_mid": "StopMidBehavior", "yield_return": "StopReturnBehavior"}


def _same_behavior(ours, ref):
    if ours is None or ref is None:
        return ours is None and ref is None
    p = ours["params"]
    if ours["type"] == "timed_brake":  # LeadBrakeBehavior(start_brake_t, dec_rate), behavior/lead_brake.py:1-15
        return ref["class"] == "LeadBrakeBehavior" and p["start_brake_t"] == ref["start_brake_t"] and \
            p["decel_mps2"] == ref["dec_rate"]
    if ref["class"] != _JAYWALK.get(ours["type"]) or p["start_delay"] != ref["start_delay"]:
        return False
    return ours["type"] != "yield_return" or p["yield_duration"] == ref["stop_duration"]


def test_lead_brake_and_jaywalk_samplers_match_reference(gen):
    """LeadBrakeScenario.sample / JaywalkScenario.sample through build_scene: the
    level the sampler got (drawn from scenario_rng when not given), ego route and
    speeds, len_route, every actor's route, cruise speed and behaviour, and how
    far scenario_np_rng (the samplers' draws; the actors' spawn jitter is drawn
    from it later, at Actor.reset) and scenario_rng advanced."""
    n = {"lead_brake": 0, "jaywalk": 0}
    for case in GOLD["scenarios"]:
        tag = (case["scene"], case["seed"], case["options"])
        bundle = build_rng_bundle(scene_seed=case["seed"])
        spec = gen.build_scene(dict(case["options"]), bundle)
        assert spec.context["level"] == case["level"], tag
        ag = case["agent"]
        assert [float(v) for v in spec.agent_rx] == ag["rx"] and [float(v) for v in spec.agent_ry] == ag["ry"], tag
        assert spec.initial_speed_mps == ag["speed"] and spec.target_speed_mps == ag["target_speed"], tag
        assert spec.len_route_m == case["len_route"], tag
        for mine, refs in ((spec.vehicles, case["vehicles"]), (spec.pedestrians, case["pedestrians"])):
            assert len(mine) == len(refs), tag
            for a, ref in zip(mine, refs):
                assert [float(v) for v in a.rx] == ref["rx"] and [float(v) for v in a.ry] == ref["ry"], tag
                assert a.speed_mps == ref["cruise_mps"], tag
                assert _same_behavior(a.behavior, ref["behavior"]), (tag, a.behavior, ref["behavior"])
        assert float(bundle.scenario_np_rng.random()) == case["scenario_np_next"], tag
        assert bundle.scenario_rng.random() == case["scenario_rng_next"], tag
        n[case["scene"]] += 1
    assert n["lead_brake"] >= 40 and n["jaywalk"] >= 40


def test_native_search_equals_python_statement():
    """cbevh_shortest_path (libcbev_host.so) = LaneGraph.shortest_path_py on the
    fixture pairs and 400 more seeded pairs per graph (no-path cases included),
    and cbevh_route_length = the reference's loop of np.hypot."""
    from carlabev_env_amd.scene_gen import route_length_meters, route_length_meters_py
    rng = np.random.default_rng(7)
    nopath = 0
    for key, g in lane_graph.planners("Town01").items():
        pairs = [(c["source"], c["target"]) for c in GOLD["paths"] if c["graph"] == lane_graph.PLANNER_FILES[key]]
        pairs += [(g.ids[int(a)], g.ids[int(b)]) for a, b in rng.integers(0, len(g.ids), (400, 2))]
        for s_, t_ in pairs:
            try:
                want = g.shortest_path_py(s_, t_)
            except lane_graph.NoPath:
                nopath += 1
                with pytest.raises(lane_graph.NoPath):
                    g.shortest_path(s_, t_)
                continue
            assert g.shortest_path(s_, t_) == want, (key, s_, t_)
            xs = [g.node_xy_surface(n)[0] for n in want]
            ys = [g.node_xy_surface(n)[1] for n in want]
            assert route_length_meters(xs, ys) == route_length_meters_py(xs, ys)
    assert nopath > 0


def test_shortest_path_edge_cases():
    g = lane_graph.planners("Town01")["vehicle-R"]
    n0 = g.ids[5]
    assert g.shortest_path(n0, n0) == [n0]
    assert g.find_path(n0, n0)[0] == [n0]
    with pytest.raises(KeyError):
        g.shortest_path("no-such-node", n0)


def test_route_profile_metrics_reference_cases():
    """The reference's own route-profile tests (tests/test_route_profile.py:33-54)."""
    from carlabev_env_amd.scene_gen import matches_route_profile, route_profile_metrics
    m = route_profile_metrics([0, 10, 20, 30, 40, 50], [0, 0, 0, 0, 0, 0])
    assert m["route_profile"] == "mostly_straight" and m["turn_count"] == 0 and m["straight_fraction"] > 0.99
    assert matches_route_profile(m, route_profile="mostly_straight")
    assert not matches_route_profile(m, route_profile="single_left")
    m = route_profile_metrics([0, 10, 20, 20, 20, 30, 40], [0, 0, 0, 10, 20, 20, 20])
    assert m["turn_count"] >= 1 and m["route_profile"] in {"single_left", "multi_turn", "mixed"}
    assert matches_route_profile(m, min_turns=1)


def test_route_profile_mix_draws_from_the_route_stream(gen):
    """A route_profile_mix picks the requested profile with route_rng.choices
    (scene_generator.py:79-93,229-234) before the ego route is searched."""
    import random
    opts = {"scene": "rdm", "num_vehicles": 0, "route_dist_range": [30, 130],
            "route_profile_mix": {"mostly_straight": 0.0, "single_right": 1.0}}
    spec = gen.build_scene(dict(opts), build_rng_bundle(scene_seed=77))
    assert spec.context["scenario_param_requested_route_profile"] == "single_right"
    assert spec.context["route_profile"] == "single_right"
    r = random.Random(build_rng_bundle(scene_seed=77).route_seed)
    assert r.choices(["mostly_straight", "single_right"], weights=[0.0, 1.0], k=1)[0] == "single_right"
    with pytest.raises(ValueError):
        gen.build_scene(dict(opts, route_profile_mix={"mostly_straight": -1.0}), build_rng_bundle(scene_seed=1))


def test_savgol_restatement_is_bitwise_scipy():
    """routes.savgol_interp (cached coefficients and polyfit matrix) equals
    scipy.signal.savgol_filter bit for bit (mode "interp", the reference's call in
    control/utils.py:200-269) on every window the routes use and on route-like,
    quantised and noisy inputs; tests/golden/smooth_route.npz pins the whole
    smoothing against the reference itself (test_oracle_golden)."""
    from scipy.signal import savgol_filter
    from carlabev_env_amd.routes import savgol_interp
    rng = np.random.default_rng(11)
    for t in range(1500):
        n = int(rng.integers(3, 300))
        w = (3, 5, 7, 9, 11)[t % 5]
        if w > n:
            continue
        p = min(3, w - 1)
        x = (rng.normal(size=n) * 1000, np.round(rng.uniform(0, 1200, n) * 8) / 8,
             np.cumsum(rng.integers(-3, 4, n)).astype(float) * 0.125 + 500)[t % 3]
        assert np.array_equal(savgol_filter(x, window_length=w, polyorder=p).view(np.int64),
                              savgol_interp(x, w, p).view(np.int64)), (t, n, w)
