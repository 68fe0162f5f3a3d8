"""Golden lane-graph routes and planned scenes, from the reference's planners.

Runs ONLY in the build container (needs /root/reference and networkx); writes
tests/golden/scenes_graph.json, which tests/test_lane_graph.py pins the host
planner (carlabev_env_amd/lane_graph.py) and scene generator
(carlabev_env_amd/scene_gen.py) against. Captured reference code:
  MapGraph node classes / random node / node positions  src/planning/map_graph.py:8-95
  GraphPlanner.find_path (nx.shortest_path + 10 px merge) src/planning/graph_planner.py:92-116
  find_route_in_range / find_route / get_random_node     src/scenes/utils.py:74-211
  compute_route_profile_metrics                          src/control/route_profile.py:55-159
  SceneGenerator.build_scene / generate_random / get_actor src/managers/scene_generator.py:95-344
  RedLightRunningScenario.sample                         src/scenes/scenarios/red_light_running.py:13-245
  LeadBrakeScenario.sample                               src/scenes/scenarios/lead_brake.py:18-129
  JaywalkScenario.sample                                 src/scenes/scenarios/jaywalk.py:29-117
  the scenario level draw of build_scene                 src/managers/scene_generator.py:165-191

The graphs are the JSON that tools/convert_graphs.py extracted from the
reference's assets/Town01/*.pkl without unpickling them. They are handed to the
reference's planners as networkx graph objects (MapGraph accepts a graph in
place of a path, map_graph.py:15-16): no pickle is loaded here, and the two
`pickle` names the planner modules hold are replaced by a stand-in that raises.
The shortest paths come from the container's networkx (3.4.2; the reference
pins 3.6.1, /root/reference/uv.lock:445-446).
"""
from __future__ import annotations

import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
import refimport  # noqa: E402

refimport.setup()
refimport._bare_pkg("CarlaBEV.src.scenes", f"{refimport.REF}/CarlaBEV/src/scenes")
refimport._bare_pkg("CarlaBEV.src.managers", f"{refimport.REF}/CarlaBEV/src/managers")

import networkx as nx  # noqa: E402
import numpy as np  # noqa: E402

from CarlaBEV.src import randomness  # noqa: E402
from CarlaBEV.src.managers import scene_generator as SG  # noqa: E402
from CarlaBEV.src.planning import graph_planner as GP  # noqa: E402
from CarlaBEV.src.planning import map_graph as MG  # noqa: E402
from CarlaBEV.src.scenes.scenarios import red_light_running as RL  # noqa: E402
from CarlaBEV.src.scenes.scenarios import jaywalk as JW  # noqa: E402
from CarlaBEV.src.scenes.scenarios import lead_brake as LB  # noqa: E402

from carlabev_env_amd.config import RandomNavigationReset, build_random_navigation_options  # noqa: E402
from carlabev_env_amd.lane_graph import GRAPH_DIR, PLANNER_FILES  # noqa: E402


def _refuse(*_a, **_k):
    raise RuntimeError("pickle loading is not allowed here")


MG.pickle = types.SimpleNamespace(load=_refuse, loads=_refuse)
RL.pickle = types.SimpleNamespace(load=_refuse, loads=_refuse)


def _attrs(a: dict) -> dict:
    return {k: (np.asarray(v["__ndarray__"], dtype=v["dtype"]).reshape(v["shape"])
                if isinstance(v, dict) and "__ndarray__" in v else (tuple(v) if k == "pos" else v))
            for k, v in a.items()}


def nx_graph(name: str):
    """The networkx graph of one converted JSON file, with the pickled node,
    adjacency and predecessor orders (they decide shortest-path ties)."""
    js = json.load(open(os.path.join(GRAPH_DIR, name + ".json")))
    G = nx.DiGraph() if js["kind"] == "DiGraph" else nx.Graph()
    G.graph.update(js["graph"])
    for n, a in js["nodes"]:
        G.add_node(n, **_attrs(a))
    succ = G._succ if G.is_directed() else G._adj
    for u, nbrs in js["adj"]:
        for v, a in nbrs:
            back = None if G.is_directed() else G._adj[v].get(u)
            succ[u][v] = back if back is not None else _attrs(a)
    if G.is_directed():
        for v, nbrs in js["pred"]:
            for u, _a in nbrs:
                G._pred[v][u] = G._succ[u][v]
    return G


def scene_generator(graphs):
    sg = SG.SceneGenerator.__new__(SG.SceneGenerator)
    sg.cfg = {}
    sg.size, sg.map_name, sg.traffic_enabled = 128, "Town01", True
    pm = SG.PlannerManager.__new__(SG.PlannerManager)
    pm.town_name = "Town01"
    pm.graphs = {key: GP.GraphPlanner(graphs[fn]) for key, fn in PLANNER_FILES.items()}
    sg.planners = pm
    rl = RL.RedLightRunningScenario(map_size=128, map_name="Town01")
    rl._graph = graphs["town01-vehicles-2lanes-100"]
    sg.scenarios = {"red_light_runner": rl, "lead_brake": LB.LeadBrakeScenario(map_size=128),
                    "jaywalk": JW.JaywalkScenario(map_size=128)}
    sg.last_scene_context = {}
    return sg


def _f(v):
    return [float(x) for x in v]


def capture_paths(graphs, n_pairs=40):
    out = []
    rng = np.random.default_rng(2024)
    for fn, G in graphs.items():
        planner = GP.GraphPlanner(G)
        nodes = list(G.nodes)
        for _ in range(n_pairs):
            s, t = (nodes[int(i)] for i in rng.integers(0, len(nodes), 2))
            try:
                path = nx.shortest_path(G, s, t, weight="cost")
            except nx.NetworkXNoPath:
                path = None
            merged, coords = planner.find_path(s, t)
            out.append({"graph": fn, "source": s, "target": t, "path": path, "merged": merged,
                        "coords": [_f(c) for c in coords]})
    return out


def capture_node_classes(graphs):
    out = {}
    for fn, G in graphs.items():
        mgr = MG.MapGraph(G)
        out[fn] = {k: list(v) for k, v in mgr.nodes.items()}
    return out


def capture_random(sg, options, seed):
    bundle = randomness.build_rng_bundle(scene_seed=seed)
    actors, len_route = sg.build_scene(dict(options), rng_bundle=bundle)
    ag = actors["agent"]
    return {"seed": seed, "options": options, "len_route": float(len_route),
            "agent": {"rx": _f(ag[0]), "ry": _f(ag[1]), "speed": float(ag[2]), "target_speed": float(ag[3])},
            "vehicles": [{"rx": _f(v.rx), "ry": _f(v.ry), "cruise_mps": float(v.cruise_speed_mps)}
                         for v in actors["vehicle"]],
            "context": {k: (v if not isinstance(v, (np.floating, np.integer)) else v.item())
                        for k, v in sg.last_scene_context.items()},
            "route_rng_next": bundle.route_rng.random(), "traffic_rng_next": bundle.traffic_rng.random(),
            "traffic_np_next": float(bundle.traffic_np_rng.random())}


def capture_red_light(sg, kwargs):
    actors, len_route = sg.scenarios["red_light_runner"].sample(**kwargs)
    ag = actors["agent"]
    adv = actors["vehicle"][0]
    return {"kwargs": kwargs, "len_route": float(len_route),
            "agent": {"rx": _f(ag[0]), "ry": _f(ag[1]), "speed": float(ag[2]), "target_speed": float(ag[3])},
            "adversary": {"rx": _f(adv.rx), "ry": _f(adv.ry), "cruise_mps": float(adv.cruise_speed_mps)},
            "traffic_light": [{"x": float(t.x), "y": float(t.y), "orientation": t.orientation,
                               "state": int(t.signal_state), "width": float(t.width), "length": float(t.length)}
                              for t in actors["traffic_light"]]}


def _behavior(b):
    """A reference behaviour object as plain data (behavior/lead_brake.py:1-15, behavior/jaywalk.py:4-160)."""
    if b is None:
        return None
    out = {"class": type(b).__name__}
    for k in ("start_brake_t", "dec_rate", "start_delay", "trigger_fraction", "stop_duration", "retreat"):
        if hasattr(b, k):
            v = getattr(b, k)
            out[k] = v if v is None or isinstance(v, bool) else float(v)
    return out


def _actor(a):
    return {"rx": _f(a.rx), "ry": _f(a.ry), "cruise_mps": float(a.cruise_speed_mps), "size": int(a.size),
            "behavior": _behavior(a.behavior)}


def capture_scenario(sg, scene, seed, level=None, kwargs=None):
    """One scenario scene: the sampler called as build_scene calls it (np_rng =
    the bundle's scenario_np_rng; level drawn from scenario_rng when not given),
    recording the level the sampler received and how far both scenario streams
    advanced."""
    bundle = randomness.build_rng_bundle(scene_seed=seed)
    options = {"scene": scene, **(kwargs or {})}
    if level is not None:
        options["level"] = level
    got = {}
    sampler = sg.scenarios[scene].sample

    def recording(**kw):
        got["level"] = kw.get("level")
        return sampler(**kw)

    sg.scenarios[scene].sample = recording
    try:
        actors, len_route = sg.build_scene(dict(options), rng_bundle=bundle)
    finally:
        sg.scenarios[scene].sample = sampler
    ag = actors["agent"]
    return {"scene": scene, "seed": seed, "options": options, "level": int(got["level"]),
            "len_route": float(len_route),
            "agent": {"rx": _f(ag[0]), "ry": _f(ag[1]), "speed": float(ag[2]), "target_speed": float(ag[3])},
            "vehicles": [_actor(v) for v in actors["vehicle"]],
            "pedestrians": [_actor(p) for p in actors["pedestrian"]],
            "scenario_np_next": float(bundle.scenario_np_rng.random()),
            "scenario_rng_next": bundle.scenario_rng.random()}


def scenario_cases():
    """lead_brake / jaywalk: every level with 8 seeds, the seeded level draw
    (no level option), and kwarg overrides of the anchors and speeds."""
    cases = []
    for scene, levels in (("lead_brake", (1, 2, 3, 4)), ("jaywalk", (1, 2, 3, 4))):
        for level in levels:
            for i in range(8):
                cases.append((scene, 50_000 + 97 * i + 1000 * level, level, None))
        for i in range(12):
            cases.append((scene, 70_000 + 31 * i, None, None))
    cases += [("lead_brake", 80_001, 3, {"anchor_x": 300, "anchor_y": 700}),
              ("lead_brake", 80_002, 3, {"ego_speed": 9.5, "rear_gap": 4.25}),
              ("lead_brake", 80_003, 2, {"lead_gap": 6.0, "brake_delay": 2.0, "brake_strength": 3.5}),
              ("lead_brake", 80_004, None, {"anchor_x": 512, "ego_speed": 11.0}),
              ("jaywalk", 80_011, 4, {"anchor_x": 300, "anchor_y": 700}),
              ("jaywalk", 80_012, 4, {"ego_speed": 9.5, "rear_gap": 4.25}),
              ("jaywalk", 80_013, 3, {"cross_offset": 1.0, "cross_delay": 1.5, "pedestrian_speed": 1.8,
                                      "yield_duration": 1.2}),
              ("jaywalk", 80_014, None, {"anchor_y": 950})]
    return cases


def main():
    graphs = {fn: nx_graph(fn) for fn in PLANNER_FILES.values()}
    sg = scene_generator(graphs)
    fixture = {"networkx": nx.__version__, "node_classes": capture_node_classes(graphs),
               "paths": capture_paths(graphs), "random": [], "red_light": [], "scenarios": []}
    seeds = [10_000 + 37 * i for i in range(12)]
    for diff in ("rt_no_traffic_v1", "rt_easy_v1", "rt_medium_v1", "rt_hard_v1"):
        options = build_random_navigation_options(RandomNavigationReset(difficulty_id=diff))
        for seed in seeds:
            fixture["random"].append(capture_random(sg, options, seed))
    extra = [({"ego_route_graph": "right_lane"}, 555), ({"ego_route_graph": "left_lane"}, 556),
             ({"route_profile": "single_left", "route_dist_range": [40, 120]}, 557),
             ({"intersection_required": True, "min_turns": 2}, 558)]
    base = build_random_navigation_options(RandomNavigationReset(difficulty_id="rt_easy_v1"))
    for over, seed in extra:
        fixture["random"].append(capture_random(sg, dict(base, **over), seed))
    for kw in ({}, {"intersection_index": 5}, {"intersection_index": 13}, {"anchor_x": 300.0, "anchor_y": 800.0},
               {"ego_speed": 7.5, "adv_speed": 12.0}):
        fixture["red_light"].append(capture_red_light(sg, kw))
    for scene, seed, level, kw in scenario_cases():
        fixture["scenarios"].append(capture_scenario(sg, scene, seed, level, kw))
    dst = os.path.join(HERE, "scenes_graph.json")
    with open(dst, "w") as f:
        json.dump(fixture, f, separators=(",", ":"))
    print(f"scenes_graph.json: {os.path.getsize(dst)} bytes, {len(fixture['paths'])} paths, "
          f"{len(fixture['random'])} random scenes, {len(fixture['red_light'])} red-light scenes, "
          f"{len(fixture['scenarios'])} lead_brake / jaywalk scenes")


if __name__ == "__main__":
    main()
