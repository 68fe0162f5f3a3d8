"""Host-side seeded scene generation (stays on the host).

What is restated from the reference, same RNG streams and draw order:
  derive_seed / build_rng_bundle       src/randomness.py:13-65
  lead_brake scenario sampler          src/scenes/scenarios/lead_brake.py:18-129
  jaywalk scenario sampler             src/scenes/scenarios/jaywalk.py:28-117
  scenario level draw                  src/managers/scene_generator.py:170-182
      (pinned since round 6: 96 scenes of every level, the seeded level draw and
      kwarg overrides, tests/test_lane_graph.py)

  random traffic (ego route, vehicles)  src/managers/scene_generator.py:196-344,
                                       src/scenes/utils.py:74-211
  route profile metrics                src/control/route_profile.py:55-182
  red_light_runner sampler             src/scenes/scenarios/red_light_running.py:13-245
The routes are planned on the reference's Town01 lane graphs (lane_graph.py,
JSON extracted from `assets/Town01/*.pkl` without unpickling), so a seeded
reset draws the reference's scene; tests/test_lane_graph.py pins the scenes
against tests/golden/scenes_graph.json (the reference's own generator on the
same graphs and seeds).

One deliberate deviation: for S != 128 the scenario samplers get anchors that
are drivable on the size-S map (`scenario_anchors`), since the reference's
literal S=256 semantics (128-scale positions on the 256 map) spawn the ego off
the road; the red-light runner is then placed on synthetic straight routes
through the anchor.

The generator produces `SceneSpec`s; `scene_pack.pack_scene` turns them into
device records. Step parity is defined on realised scenes (the record), which
is also what the GPU and the oracle are compared on.
"""
from __future__ import annotations

import ctypes
import os

import hashlib
import random
from dataclasses import dataclass

import numpy as np

from . import lane_graph
from .authored import load_authored_scene, normalize_scenario_config, read_scene_file, scenario_options_from_config
from .params import load_class_map
from .routes import smooth_and_compute
from .scene_pack import ActorSpec, SceneSpec, TrafficLightSpec

_SEED_MODULUS = 2 ** 31 - 1
MPP = 40.0 / 128.0


def derive_seed(base_seed: int, *parts: object) -> int:
    token = ":".join([str(int(base_seed)), *(str(p) for p in parts)])
    digest = hashlib.sha256(token.encode("utf-8")).hexdigest()
    return int(digest[:16], 16) % _SEED_MODULUS


@dataclass
class RNGBundle:
    scene_seed: int
    route_seed: int
    traffic_seed: int
    scenario_seed: int
    scene_rng: random.Random
    route_rng: random.Random
    traffic_rng: random.Random
    scenario_rng: random.Random
    scene_np_rng: np.random.Generator
    route_np_rng: np.random.Generator
    traffic_np_rng: np.random.Generator
    scenario_np_rng: np.random.Generator


def build_rng_bundle(*, scene_seed: int, route_seed=None, traffic_seed=None, scenario_seed=None) -> RNGBundle:
    scene_seed = int(scene_seed)
    route_seed = derive_seed(scene_seed, "route") if route_seed is None else int(route_seed)
    traffic_seed = derive_seed(scene_seed, "traffic") if traffic_seed is None else int(traffic_seed)
    scenario_seed = derive_seed(scene_seed, "scenario") if scenario_seed is None else int(scenario_seed)
    return RNGBundle(scene_seed, route_seed, traffic_seed, scenario_seed,
                     random.Random(scene_seed), random.Random(route_seed), random.Random(traffic_seed),
                     random.Random(scenario_seed), np.random.default_rng(scene_seed),
                     np.random.default_rng(route_seed), np.random.default_rng(traffic_seed),
                     np.random.default_rng(scenario_seed))


def _rng_state(g: np.random.Generator) -> dict:
    return g.bit_generator.state


def window_128(classes: np.ndarray) -> np.ndarray:
    """The region of a size-S class map addressed by 128-surface coordinates."""
    return classes[:1280, :1024]


def _all_drivable(ii, y0, y1, x0, x1) -> bool:
    return ii[y1, x1] - ii[y0, x1] - ii[y1, x0] + ii[y0, x0] == (y1 - y0) * (x1 - x0)


def scenario_anchors(map_name: str, size: int):
    """Anchors for the authored-geometry scenarios on a size-S map (S != 128).

    The reference samplers place the ego at x = 850, y in [900, 1000) in 128-surface
    coordinates (lead_brake.py:30-41, jaywalk.py:38-53). With the literal S=256
    semantics (256 map queried at 128-scale positions) that spot is NON_DRIVABLE,
    every spawn is rejected and CarlaBEV.reset raises after 10 attempts; the
    samplers accept anchor_x/anchor_y, so the generator passes anchors that are
    drivable on the size-S map: a 120 px northbound road for lead_brake/jaywalk,
    a 250 px one for the red-light runner's ego approach."""
    c = window_128(load_class_map(map_name, size)) == 1
    ii = np.pad(c.astype(np.int64).cumsum(0).cumsum(1), ((1, 0), (1, 0)))
    h, w = c.shape
    north, long_north = [], []
    for y in range(260, h - 20, 10):
        for x in range(20, w - 20, 2):
            if _all_drivable(ii, y - 110, y + 10, x - 4, x + 5):
                north.append((x, y))
                if _all_drivable(ii, y - 250, y + 10, x - 4, x + 5):
                    long_north.append((x, y - 125))
    return north, long_north


def _m2s(m: float) -> float:
    return float(m) / MPP


def route_length_meters(rx, ry) -> float:
    """envs/geometry.py:61-69 (segment lengths hypot(dx, dy) summed in order, then
    scaled), the sum natively (cbevh_route_length: libm hypot as np.hypot,
    float64 additions in the same order)."""
    if len(rx) != len(ry):
        raise ValueError("Route coordinates mismatch.")
    if len(rx) < 2:
        return 0.0
    x = np.asarray(rx, dtype=np.float64)
    y = np.asarray(ry, dtype=np.float64)
    p = ctypes.c_void_p
    total = lane_graph.host_lib().cbevh_route_length(x.ctypes.data_as(p), y.ctypes.data_as(p), len(x))
    return float(total) * MPP


def route_length_meters_py(rx, ry) -> float:
    """route_length_meters as the reference writes it (the tests' cross-check)."""
    if len(rx) != len(ry):
        raise ValueError("Route coordinates mismatch.")
    total = 0.0
    for i in range(1, len(rx)):
        total += np.hypot(float(rx[i]) - float(rx[i - 1]), float(ry[i]) - float(ry[i - 1]))
    return float(total) * MPP


_STRAIGHT = {"straight_fraction": 1.0, "left_turn_fraction": 0.0, "right_turn_fraction": 0.0, "turn_count": 0,
             "has_left_turn": False, "has_right_turn": False, "intersection_like": False,
             "route_profile": "mostly_straight"}


def route_profile_metrics(ax, ay, turn_rate_thresh: float = 0.12, min_turn_segment_m: float = 4.0) -> dict:
    """compute_route_profile_metrics (control/route_profile.py:55-159): turn
    labels from the heading rate of the smoothed route, turn segments of at least
    `min_turn_segment_m`, and the profile label they make."""
    cx, cy, cyaw, _, _ = smooth_and_compute(ax, ay, window=11, poly=3)
    cx, cy = np.asarray(cx, dtype=float), np.asarray(cy, dtype=float)
    cyaw = np.unwrap(np.asarray(cyaw, dtype=float))
    if cx.size < 2 or cy.size < 2 or cyaw.size < 2:
        return dict(_STRAIGHT)
    ds = np.hypot(np.diff(cx), np.diff(cy)) * MPP
    valid = ds > 1e-6
    if not np.any(valid):
        return dict(_STRAIGHT)
    dth = (np.diff(cyaw) + np.pi) % (2.0 * np.pi) - np.pi
    ds_v, rate = ds[valid], dth[valid] / ds[valid]
    labels = np.where(rate > turn_rate_thresh, 1, np.where(rate < -turn_rate_thresh, -1, 0))
    total = float(ds_v.sum())
    if total <= 1e-9:
        return dict(_STRAIGHT)
    # _normalize_turn_segments (route_profile.py:21-52): runs of one turn sign
    segs, sign_c, length = [], 0, 0.0
    for sign, seg in zip(labels, ds_v):
        sign = int(sign)
        if sign != sign_c or sign == 0:
            if sign_c != 0 and length >= min_turn_segment_m:
                segs.append(sign_c)
            sign_c, length = sign, (float(seg) if sign != 0 else 0.0)
        else:
            length += float(seg)
    if sign_c != 0 and length >= min_turn_segment_m:
        segs.append(sign_c)
    straight = float(ds_v[labels == 0].sum()) / total
    left = float(ds_v[labels == 1].sum()) / total
    right = float(ds_v[labels == -1].sum()) / total
    turns = len(segs)
    has_l, has_r = any(g > 0 for g in segs), any(g < 0 for g in segs)
    if turns == 0 or straight >= 0.9:
        prof = "mostly_straight"
    elif turns == 1 and left >= right:
        prof = "single_left"
    elif turns == 1 and right > left:
        prof = "single_right"
    elif turns >= 2:
        prof = "multi_turn"
    else:
        prof = "mixed"
    return {"straight_fraction": straight, "left_turn_fraction": left, "right_turn_fraction": right,
            "turn_count": turns, "has_left_turn": has_l, "has_right_turn": has_r,
            "intersection_like": turns >= 2 or (has_l and has_r), "route_profile": prof}


def matches_route_profile(m: dict, route_profile=None, min_turns=None, max_turns=None,
                          intersection_required=None) -> bool:
    """control/route_profile.py:162-182."""
    if route_profile is not None and route_profile != "any" and m.get("route_profile") != route_profile:
        return False
    turns = int(m.get("turn_count", 0))
    if min_turns is not None and turns < min_turns:
        return False
    if max_turns is not None and turns > max_turns:
        return False
    inter = bool(m.get("intersection_like", False))
    if intersection_required is True and not inter:
        return False
    if intersection_required is False and inter:
        return False
    return True


# generate_random's ego graph choice (scene_generator.py:254-270): planner, node class
EGO_ROUTE_GRAPHS = {"full_vehicle": ("vehicle-full", "vehicle"), "right_lane": ("vehicle-R", "R"),
                    "left_lane": ("vehicle-L", "L")}


class SceneGenerator:
    """build_scene(options, rng_bundle) -> SceneSpec (scene_generator.py:95-191)."""

    # RedLightRunningScenario.intersections, (y, x) raw (red_light_running.py:23-40)
    INTERSECTIONS_RAW = [(8642, 1564), (8654, 6755), (7250, 1552), (7241, 2446), (7242, 3652), (7242, 4704),
                         (7257, 6773), (6199, 1552), (6197, 2439), (3349, 1545), (3350, 2456), (3350, 3639),
                         (3335, 4714), (3315, 6773), (2456, 1563), (2446, 6757)]

    def __init__(self, cfg=None, map_name: str = "Town01"):
        self.cfg = cfg
        self.map_name = map_name
        self.size = int(getattr(cfg, "size", 128)) if cfg is not None else 128
        self.planners = lane_graph.planners(map_name)
        self._anchors = scenario_anchors(map_name, self.size) if self.size != 128 else None
        self.max_vehicles = getattr(cfg, "max_vehicles", 25) if cfg is not None else 25
        self.traffic_enabled = getattr(cfg, "traffic_enabled", True) if cfg is not None else True
        self._red_light_routes: dict = {}

    # ------------------------------------------------------------ random traffic
    def route_in_range(self, rng: random.Random, planner_key: str, node_cls: str, min_m: float, max_m: float,
                       route_profile=None, min_turns=None, max_turns=None, intersection_required=None,
                       max_attempts: int = 100):
        """find_route_in_range with an explicit planner (scenes/utils.py:125-211):
        random start/end nodes of `node_cls`, the planner's merged shortest path,
        waypoints path[1:] in surface px; accepted when its length is within
        [min_m, max_m] m and its profile matches. -> (rx, ry, length_m, metrics) | None"""
        g = self.planners[planner_key]
        for _ in range(max_attempts):
            start = g.random_node(node_cls, rng)
            end = g.random_node(node_cls, rng)
            if start == end:
                continue
            path = g.find_path_idx(start, end)
            if len(path) < 2:
                continue
            xy = g.surf_xy[path[1:]]  # node_pos_surface of path[1:]
            rx, ry = xy[:, 0].tolist(), xy[:, 1].tolist()
            length = route_length_meters(rx, ry)
            if min_m <= length <= max_m:
                metrics = route_profile_metrics(rx, ry)
                if not matches_route_profile(metrics, route_profile, min_turns, max_turns, intersection_required):
                    continue
                return rx, ry, length, metrics
        return None

    def actor_route(self, lane: str, rng: random.Random):
        """get_actor("vehicle", lane) + find_route (scene_generator.py:330-344,
        scenes/utils.py:74-101): two random nodes of the lane's own graph, the
        interior nodes of the merged path between them; None unless > 5 points."""
        g = self.planners[f"vehicle-{lane}"]
        start = g.random_node(lane, rng)
        end = g.random_node(lane, rng)
        path = g.find_path_idx(start, end)
        xy = g.surf_xy[path[1:-1]]
        rx, ry = xy[:, 0].tolist(), xy[:, 1].tolist()
        return (rx, ry) if len(rx) > 5 else None

    def generate_random(self, num_cars, dist_range, bundle: RNGBundle, traffic_enabled=True, ego_target_speed=12.0,
                        max_retries=20, route_profile=None, route_profile_mix=None, min_turns=None, max_turns=None,
                        intersection_required=None, ego_route_graph="full_vehicle") -> SceneSpec:
        """SceneGenerator.generate_random (scene_generator.py:196-327)."""
        num_cars = num_cars if traffic_enabled else 0
        ego_target_speed = float(ego_target_speed)
        ctx = {"scene": "rdm", "scenario_param_num_vehicles": int(num_cars),
               "scenario_param_route_dist_range": list(dist_range),
               "scenario_param_ego_route_graph": str(ego_route_graph)}
        profile = route_profile
        if route_profile_mix:
            labels = list(route_profile_mix.keys())
            weights = [float(route_profile_mix[k]) for k in labels]
            if any(w < 0.0 for w in weights):
                raise ValueError(f"route_profile_mix must use non-negative weights: {route_profile_mix}")
            if sum(weights) <= 0.0:
                raise ValueError(f"route_profile_mix must contain at least one positive weight: {route_profile_mix}")
            profile = bundle.route_rng.choices(labels, weights=weights, k=1)[0]
            ctx["scenario_param_route_profile_mix"] = dict(route_profile_mix)
        if profile is not None:
            ctx["scenario_param_requested_route_profile"] = profile
        if min_turns is not None:
            ctx["scenario_param_min_turns"] = int(min_turns)
        if max_turns is not None:
            ctx["scenario_param_max_turns"] = int(max_turns)
        if intersection_required is not None:
            ctx["scenario_param_intersection_required"] = bool(intersection_required)
        if max_retries is not None:
            ctx["scenario_param_max_route_attempts"] = int(max_retries)
        if ego_route_graph not in EGO_ROUTE_GRAPHS:
            raise ValueError(f"Unsupported ego_route_graph={ego_route_graph!r}. "
                             "Expected one of: full_vehicle, right_lane, left_lane.")
        key, node_cls = EGO_ROUTE_GRAPHS[ego_route_graph]
        found = None
        for _ in range(max_retries):
            found = self.route_in_range(bundle.route_rng, key, node_cls, dist_range[0], dist_range[1], profile,
                                        min_turns, max_turns, intersection_required)
            if found is not None and len(found[0]) > 1:
                break
            found = None
        if found is None:
            raise RuntimeError(f"Failed to generate a valid ego route in range {dist_range} after {max_retries} "
                               "attempts.")
        rx, ry, length, m = found
        ctx.update({"route_profile": m["route_profile"], "route_turn_count": int(m["turn_count"]),
                    "route_intersection_like": bool(m["intersection_like"]), "route_length_m": float(length),
                    "route_left_turn_fraction": float(m["left_turn_fraction"]),
                    "route_right_turn_fraction": float(m["right_turn_fraction"]),
                    "route_straight_fraction": float(m["straight_fraction"])})
        vehicles = []
        for _ in range(num_cars):
            lane = bundle.traffic_rng.choice(["L", "R"])
            route = self.actor_route(lane, bundle.traffic_rng)
            if route is not None:
                vehicles.append(ActorSpec("vehicle", route[0], route[1], 12.0))
        spec = SceneSpec(rx, ry, 0.0, ego_target_speed, vehicles=vehicles, hero_jitter_seed=None,
                         actor_jitter_seed=None)
        spec.hero_rng_state = _rng_state(bundle.route_np_rng)
        spec.actor_rng_state = _rng_state(bundle.traffic_np_rng)
        spec.context = ctx
        spec.len_route_m = float(length)
        return spec

    # ------------------------------------------------------------ lead_brake
    def lead_brake(self, level: int, g: np.random.Generator, kw: dict) -> SceneSpec:
        ego_start_y = kw.get("anchor_y", int(g.integers(900, 1000)))
        lead_gap_m = kw.get("lead_gap", float(g.uniform(4.5, 12.5)))
        ego_speed = kw.get("ego_speed", float(g.uniform(8.0, 16.0)))
        lead_speed = kw.get("lead_speed", ego_speed + float(g.uniform(-2.0, 2.0)))
        brake_delay = kw.get("brake_delay", float(g.uniform(1.5, 4.0)))
        brake_strength = kw.get("brake_strength", float(g.uniform(2.0, 6.0)))
        x_center = kw.get("anchor_x", 850)
        lane_width = _m2s(2.2)
        ego_step, lead_step, rear_step = _m2s(6.25), _m2s(1.56), _m2s(3.12)
        ego_rx = [x_center] * 6
        ego_ry = [ego_start_y - i * ego_step for i in range(6)]
        lead_y0 = ego_ry[0] - _m2s(lead_gap_m)
        vehicles = [ActorSpec("vehicle", [x_center - 1] * 6, [lead_y0 - i * lead_step for i in range(6)], lead_speed,
                              {"type": "timed_brake",
                               "params": {"start_brake_t": brake_delay, "decel_mps2": brake_strength}})]
        if level >= 2:
            lx = x_center - lane_width
            left_rx = [lx] * 7
            left_ry = [ego_start_y - i * 20 for i in range(7)]
            left_rx.reverse()
            left_ry.reverse()
            left_speed = kw.get("left_speed", float(g.uniform(10.0, 18.0)))
            vehicles.append(ActorSpec("vehicle", left_rx, left_ry, left_speed, None))
        if level >= 3:
            rear_gap_m = kw.get("rear_gap", float(g.uniform(3.0, 6.0)))
            ry0 = ego_ry[0] + _m2s(rear_gap_m)
            rear_speed = kw.get("rear_speed", max(ego_speed - float(g.uniform(1.0, 3.0)), 4.0))
            rbd = kw.get("rear_brake_delay", float(g.uniform(2.0, 5.0)))
            vehicles.append(ActorSpec("vehicle", [x_center] * 6, [ry0 - i * rear_step for i in range(6)], rear_speed,
                                      {"type": "timed_brake",
                                       "params": {"start_brake_t": rbd, "decel_mps2": brake_strength}}))
        spec = SceneSpec(ego_rx, ego_ry, ego_speed, ego_speed, vehicles=vehicles)
        spec.len_route_m = route_length_meters(ego_rx, ego_ry)  # compute_total_dist_m (lead_brake.py:50)
        return spec

    # ------------------------------------------------------------ jaywalk
    def jaywalk(self, level: int, g: np.random.Generator, kw: dict) -> SceneSpec:
        ego_start_y = kw.get("anchor_y", int(g.integers(900, 1000)))
        ego_speed = kw.get("ego_speed", float(g.uniform(8.0, 14.0)))
        ped_x_base = kw.get("anchor_x", 850)
        lane_width = _m2s(1.6)
        cross_offset_m = kw.get("cross_offset", float(g.uniform(-3.0, 3.0)))
        cross_delay = kw.get("cross_delay", float(g.uniform(1.0, 2.5)))
        ped_speed = kw.get("pedestrian_speed", float(g.uniform(1.2, 2.2)))
        ego_step, rear_step = _m2s(6.25), _m2s(3.12)
        yield_duration = kw.get("yield_duration", float(g.uniform(0.8, 1.6)))
        ego_rx = [ped_x_base] * 6
        ego_ry = [ego_start_y - i * ego_step for i in range(6)]
        off = _m2s(cross_offset_m)
        ped_y = ego_ry[2] + _m2s(float(g.uniform(-1.0, 1.6)))
        ped_rx = np.linspace(ped_x_base + lane_width + off, ped_x_base - lane_width + off, 8)
        ped_ry = np.ones_like(ped_rx) * ped_y
        if level == 1:
            beh = {"type": "cross", "params": {"start_delay": cross_delay}}
        elif level == 2:
            beh = {"type": "stop_mid", "params": {"start_delay": cross_delay}}
        else:
            beh = {"type": "yield_return", "params": {"start_delay": cross_delay, "yield_duration": yield_duration}}
        peds = [ActorSpec("pedestrian", list(ped_rx), list(ped_ry), ped_speed, beh)]
        vehicles = []
        if level >= 4:
            rear_gap_m = kw.get("rear_gap", float(g.uniform(3.0, 6.0)))
            ry0 = ego_ry[0] + _m2s(rear_gap_m)
            rear_speed = kw.get("rear_speed", max(ego_speed - float(g.uniform(1.0, 3.0)), 4.0))
            vehicles.append(ActorSpec("vehicle", [ped_x_base] * 6, [ry0 - i * rear_step for i in range(6)],
                                      rear_speed, None))
        spec = SceneSpec(ego_rx, ego_ry, ego_speed, ego_speed, vehicles=vehicles, pedestrians=peds)
        spec.len_route_m = route_length_meters(ego_rx, ego_ry)  # compute_total_dist_m (jaywalk.py:55)
        return spec

    # ------------------------------------------------------------ red light runner
    @staticmethod
    def _direction_key(dx: float, dy: float) -> str:
        if abs(dx) > abs(dy):
            return "east" if dx > 0 else "west"
        return "south" if dy > 0 else "north"

    def _intersection_graph(self):
        return self.planners["vehicle"]  # the 2-lane graph (red_light_running.py:42-45)

    def _select_intersection(self, index=None, anchor_x=None, anchor_y=None) -> np.ndarray:
        """_select_intersection (red_light_running.py:74-107): the first candidate
        (nearest the requested intersection / anchor, else list order) whose
        1200-unit neighbourhood has lane nodes in all four directions."""
        raw = [np.array([float(x), float(y)]) for y, x in self.INTERSECTIONS_RAW]
        if index is not None:
            if not 0 <= int(index) < len(raw):
                raise IndexError(f"intersection_index {int(index)} out of range for red_light_runner.")
            ref = raw[int(index)]
            order = [i for _, i in sorted((np.linalg.norm(c - ref), i) for i, c in enumerate(raw))]
        elif anchor_x is not None and anchor_y is not None:
            ref = np.array([anchor_x * 8.0, anchor_y * 8.0], dtype=float)
            order = [i for _, i in sorted((np.linalg.norm(c - ref), i) for i, c in enumerate(raw))]
        else:
            order = list(range(len(raw)))
        g = self._intersection_graph()
        pos = np.array([np.asarray(p, dtype=float) for p in g.pos])
        for i in order:
            counts = {"north": 0, "south": 0, "east": 0, "west": 0}
            for p in pos:
                d = p - raw[i]
                if np.linalg.norm(d) >= 1200.0:
                    continue
                counts[self._direction_key(d[0], d[1])] += 1
            if all(counts[k] > 0 for k in ("north", "south", "east", "west")):
                return raw[i]
        raise RuntimeError("No valid 4-way intersection candidate found for red_light_runner.")

    def _straight_route(self, center: np.ndarray, start_dir: str, end_dir: str):
        """_sample_straight_route (red_light_running.py:109-161): the best-scored
        start/end lane nodes (distance near 950 units, small lateral offset) whose
        shortest path passes within 180 units of the centre and has >= 6 nodes;
        the route is the path's raw positions / 8."""
        g = self._intersection_graph()

        def candidates(direction):
            out = []
            for n, p in zip(g.ids, g.pos):
                p = np.asarray(p, dtype=float)
                d = p - center
                dist = np.linalg.norm(d)
                if not 150.0 <= dist <= 1500.0 or self._direction_key(d[0], d[1]) != direction:
                    continue
                lateral = abs(d[0]) if direction in ("north", "south") else abs(d[1])
                out.append((abs(dist - 950.0) + 0.2 * lateral, n))
            out.sort(key=lambda item: item[0])
            return [n for _, n in out[:25]]

        ends = candidates(end_dir)
        for s in candidates(start_dir):
            for t in ends:
                try:
                    path = g.shortest_path(s, t)
                except lane_graph.NoPath:
                    continue
                coords = [np.asarray(g.pos[g.index[n]], dtype=float) for n in path]
                if min(np.linalg.norm(c - center) for c in coords) > 180.0 or len(coords) < 6:
                    continue
                return [float(c[0]) / 8.0 for c in coords], [float(c[1]) / 8.0 for c in coords]
        raise RuntimeError(f"Unable to build a valid {start_dir}->{end_dir} route through the selected 4-way "
                           "intersection.")

    def red_light_runner(self, level: int, g: np.random.Generator, kw: dict) -> SceneSpec:
        """RedLightRunningScenario.sample (red_light_running.py:195-245): the ego
        drives south->north through a 4-way intersection on green while an
        adversary crosses west->east on red. Nothing in it is random: the routes
        depend on the selected intersection only, and are cached per centre."""
        if "center" in kw:  # S != 128 anchor (module docstring): synthetic straight routes
            return self._red_light_synthetic(kw)
        center = self._select_intersection(kw.get("intersection_index"), kw.get("anchor_x"), kw.get("anchor_y"))
        key = (float(center[0]), float(center[1]))
        if key not in self._red_light_routes:
            self._red_light_routes[key] = (self._straight_route(center, "south", "north"),
                                           self._straight_route(center, "west", "east"))
        (ego_rx, ego_ry), (adv_rx, adv_ry) = self._red_light_routes[key]
        ego_speed = kw.get("ego_speed", 10.0)
        adv_speed = kw.get("adv_speed", 16.0)
        cx, cy = float(center[0]) / 8.0, float(center[1]) / 8.0
        off, length, width = _m2s(4.0), _m2s(8.0), _m2s(0.45) + 1.0
        tls = [TrafficLightSpec(cx, cy + off, "horizontal", "green", width, length),
               TrafficLightSpec(cx - off, cy, "vertical", "red", width, length)]
        spec = SceneSpec(list(ego_rx), list(ego_ry), ego_speed, ego_speed,
                         vehicles=[ActorSpec("vehicle", list(adv_rx), list(adv_ry), adv_speed, None)],
                         traffic_lights=tls)
        spec.len_route_m = route_length_meters(ego_rx, ego_ry)
        return spec

    def _red_light_synthetic(self, kw: dict) -> SceneSpec:
        """The S != 128 stand-in: straight 20-point routes through the anchor."""
        cx, cy = (float(v) for v in kw["center"])
        span = 950.0 / 8.0
        n = 20
        ego_ry = list(np.linspace(cy + span, cy - span, n))
        ego_rx = [cx + _m2s(1.75)] * n
        adv_rx = list(np.linspace(cx - span, cx + span, n))
        adv_ry = [cy + _m2s(1.75)] * n
        ego_speed = kw.get("ego_speed", 10.0)
        adv_speed = kw.get("adv_speed", 16.0)
        off, length, width = _m2s(4.0), _m2s(8.0), _m2s(0.45) + 1.0
        tls = [TrafficLightSpec(cx, cy + off, "horizontal", "green", width, length),
               TrafficLightSpec(cx - off, cy, "vertical", "red", width, length)]
        return SceneSpec(ego_rx, ego_ry, ego_speed, ego_speed,
                         vehicles=[ActorSpec("vehicle", adv_rx, adv_ry, adv_speed, None)], traffic_lights=tls)

    # ------------------------------------------------------------ dispatch
    def build_scene(self, options: dict, bundle: RNGBundle) -> SceneSpec:
        scene = options.get("scene", "rdm")
        config_file = options.get("config_file")
        if isinstance(scene, str) and scene.endswith(".json") and os.path.exists(scene):
            config_file = scene
        if config_file:  # authored scene / scenario config (scene_generator.py:98-138)
            data = read_scene_file(config_file)
            if "actors" in data:
                spec, len_route, ctx = load_authored_scene(data, options)
                # authored actors are built without np_rng in the reference (fresh-entropy
                # spawn jitter); here they draw it from the scenario generator
                spec.hero_rng_state = _rng_state(bundle.route_np_rng)
                spec.actor_rng_state = _rng_state(bundle.scenario_np_rng)
                spec.context = dict(ctx, scene=data.get("scenario_id") or data.get("scenario"),
                                    config_file=config_file, len_route_px=len_route)
                return spec
            sub = scenario_options_from_config(normalize_scenario_config(data), options)
            return self.build_scene(sub, bundle)
        if scene == "rdm":
            attempts = options.get("max_route_attempts")
            target = options.get("ego_target_speed")
            return self.generate_random(
                options.get("num_vehicles", self.max_vehicles),
                options.get("route_dist_range", [30, 100]),
                bundle,
                traffic_enabled=options.get("traffic_enabled", self.traffic_enabled),
                ego_target_speed=12.0 if target is None else target,
                max_retries=20 if attempts is None else int(attempts),
                route_profile=options.get("route_profile"),
                route_profile_mix=options.get("route_profile_mix"),
                min_turns=options.get("min_turns"),
                max_turns=options.get("max_turns"),
                intersection_required=options.get("intersection_required"),
                ego_route_graph=options.get("ego_route_graph", "full_vehicle"),
            )
        if scene in ("lead_brake", "jaywalk", "red_light_runner"):
            # scenario_options.setdefault("level", scenario_rng.choice([1, 2, 3, 4]))
            # (scene_generator.py:180-183): the draw is made even when a level is given
            drawn = bundle.scenario_rng.choice([1, 2, 3, 4])
            level = options.get("level")
            if level is None:
                level = drawn
            g = bundle.scenario_np_rng
            kw = {k: v for k, v in options.items() if k not in ("scene", "level", "reset_mask")}
            if self._anchors is not None:
                north, cross = self._anchors
                if scene == "red_light_runner" and "center" not in kw and cross:
                    kw["center"] = cross[bundle.scene_seed % len(cross)]
                elif scene != "red_light_runner" and "anchor_x" not in kw and north:
                    kw["anchor_x"], kw["anchor_y"] = north[bundle.scene_seed % len(north)]
            spec = getattr(self, scene)(int(level), g, kw)
            spec.hero_rng_state = _rng_state(bundle.route_np_rng)
            spec.actor_rng_state = _rng_state(g)  # actors share the sampler's generator (deep-copied)
            spec.context = {"scene": scene, "level": int(level)}
            return spec
        raise KeyError(f"unsupported scene {scene!r}")
