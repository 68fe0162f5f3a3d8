"""Host-side seeded scene generation (stays on the host).

What is restated from the reference, same RNG streams and draw order:
  derive_seed / build_rng_bundle       src/randomness.py:13-65
  lead_brake scenario sampler          src/scenes/scenarios/lead_brake.py:18-129
  jaywalk scenario sampler             src/scenes/scenarios/jaywalk.py:28-117
  scenario level draw                  src/managers/scene_generator.py:170-182

What is synthetic (and why): the reference's random-traffic routes and the
red-light-runner routes are shortest paths on lane graphs that ship only as
Python pickles (`assets/Town01/*.pkl`, loaded with `pickle.load` at
`src/planning/map_graph.py:13-19`). Unpickling reference files is not allowed
here, so `RoadGrid` plans routes on the drivable pixels of the Town01 class
map instead: a grid of road-centre cells (cells whose distance to the road edge
exceeds a margin), breadth-first shortest paths from a seeded set of source
cells, waypoints every `cell` px. Routes are in 128-surface coordinates for
every map size, as in the reference (`scene_generator.py:71-75,334`). Ego route
length ranges, vehicle counts and the rule that a background vehicle needs >5
route points follow `scene_generator.py:196-344`.

The generator produces `SceneSpec`s; `scene_pack.pack_scene` turns them into
device records. Step parity is defined on realised scenes (the record), which
is also what the GPU and the oracle are compared on.
"""
from __future__ import annotations

import os

import hashlib
import random
from dataclasses import dataclass

import numpy as np

from scipy import ndimage
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import shortest_path

from .authored import load_authored_scene, normalize_scenario_config, read_scene_file, scenario_options_from_config
from .params import load_class_map
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


class RoadGrid:
    """Road-centre cell graph over the 128-scale Town01 class map."""

    def __init__(self, map_name: str = "Town01", size: int = 128, cell: int = 4, margin: float = 6.0,
                 stride: int = 3, n_sources: int = 128, seed: int = 12345):
        # routes live in 128-surface coordinates for every map size (scene_generator.py:71-75), so
        # plan on the part of the size-S map those coordinates cover (the whole map at S=128)
        classes = window_128(load_class_map(map_name, size))
        self.h, self.w = classes.shape
        drivable = classes == 1
        dist = ndimage.distance_transform_edt(drivable)
        self.cell = cell
        self.stride = stride  # waypoint every stride*cell px (12.5 px lane-graph spacing in the reference)
        gh, gw = self.h // cell, self.w // cell
        cy = (np.arange(gh) * cell + cell // 2)
        cx = (np.arange(gw) * cell + cell // 2)
        ok = dist[np.ix_(cy, cx)] >= margin
        ids = -np.ones((gh, gw), dtype=np.int64)
        nodes = np.argwhere(ok)
        ids[ok] = np.arange(len(nodes))
        self.node_xy = np.stack([cx[nodes[:, 1]], cy[nodes[:, 0]]], axis=1).astype(float)
        rows, cols = [], []
        for dy, dx in ((0, 1), (1, 0)):
            a = ids[: gh - dy, : gw - dx]
            b = ids[dy:, dx:]
            m = (a >= 0) & (b >= 0)
            rows += [a[m], b[m]]
            cols += [b[m], a[m]]
        r = np.concatenate(rows)
        c = np.concatenate(cols)
        n = len(nodes)
        self.graph = csr_matrix((np.ones(len(r)), (r, c)), shape=(n, n))
        # keep the largest connected component only
        from scipy.sparse.csgraph import connected_components
        _, lab = connected_components(self.graph, directed=False)
        big = np.bincount(lab).argmax()
        self.valid = np.flatnonzero(lab == big)
        rng = np.random.default_rng(seed)
        self.sources = rng.choice(self.valid, size=min(n_sources, len(self.valid)), replace=False)
        d, pred = shortest_path(self.graph, directed=False, unweighted=True, indices=self.sources,
                                return_predecessors=True)
        self.dist = d
        self.pred = pred

    def path(self, si: int, target: int) -> np.ndarray:
        """Waypoints (surface px) of the BFS path from source index si to node target."""
        out = []
        node = int(target)
        src = int(self.sources[si])
        while node != src and node >= 0:
            out.append(node)
            node = int(self.pred[si, node])
        out.append(src)
        nodes = out[::-1]
        keep = nodes[::self.stride]
        if keep[-1] != nodes[-1]:
            keep.append(nodes[-1])
        return self.node_xy[np.array(keep)]

    def route_in_range(self, rng: random.Random, min_m: float, max_m: float, max_attempts: int = 100):
        """Random ego route whose length is within [min_m, max_m] meters
        (find_route_in_range, scenes/utils.py:125-211)."""
        for _ in range(max_attempts):
            si = rng.randrange(len(self.sources))
            d = self.dist[si]
            lo = min_m / MPP / self.cell
            hi = max_m / MPP / self.cell
            cand = np.flatnonzero((d >= lo) & (d <= hi))
            if len(cand) == 0:
                continue
            target = int(cand[rng.randrange(len(cand))])
            pts = self.path(si, target)
            length = float(np.sum(np.hypot(np.diff(pts[:, 0]), np.diff(pts[:, 1])))) * MPP
            if min_m <= length <= max_m and len(pts) >= 2:
                return pts
        return None

    def random_route(self, rng: random.Random, min_points: int = 6, max_points: int = 48):
        si = rng.randrange(len(self.sources))
        d = self.dist[si]
        hops = self.stride
        cand = np.flatnonzero(np.isfinite(d) & (d >= (min_points - 1) * hops) & (d <= (max_points - 2) * hops))
        if len(cand) == 0:
            return None
        target = int(cand[rng.randrange(len(cand))])
        return self.path(si, target)


_GRIDS: dict = {}


def window_128(classes: np.ndarray) -> np.ndarray:
    """The region of a size-S class map addressed by 128-surface coordinates."""
    return classes[:1280, :1024]


def road_grid(map_name: str = "Town01", size: int = 128) -> RoadGrid:
    key = (map_name, size)
    if key not in _GRIDS:
        _GRIDS[key] = RoadGrid(map_name, size)
    return _GRIDS[key]


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


class SceneGenerator:
    """build_scene(options, rng_bundle) -> SceneSpec (scene_generator.py:95-191)."""

    def __init__(self, cfg=None, map_name: str = "Town01"):
        self.cfg = cfg
        self.map_name = map_name
        self.size = int(getattr(cfg, "size", 128)) if cfg is not None else 128
        self.grid = road_grid(map_name, self.size)
        self._anchors = scenario_anchors(map_name, self.size) if self.size != 128 else None
        self.max_vehicles = getattr(cfg, "max_vehicles", 25) if cfg is not None else 25
        self.traffic_enabled = getattr(cfg, "traffic_enabled", True) if cfg is not None else True

    # ------------------------------------------------------------ random traffic
    def generate_random(self, num_cars, dist_range, bundle: RNGBundle, traffic_enabled=True, ego_target_speed=12.0,
                        max_retries=20) -> SceneSpec:
        num_cars = num_cars if traffic_enabled else 0
        pts = None
        for _ in range(max_retries):
            pts = self.grid.route_in_range(bundle.route_rng, float(dist_range[0]), float(dist_range[1]))
            if pts is not None and len(pts) > 1:
                break
        if pts is None:
            raise RuntimeError(f"Failed to generate a valid ego route in range {dist_range} after {max_retries} "
                               "attempts.")
        vehicles = []
        for _ in range(num_cars):
            _lane = bundle.traffic_rng.choice(["L", "R"])
            vp = self.grid.random_route(bundle.traffic_rng)
            if vp is None or len(vp) <= 5:
                continue
            vehicles.append(ActorSpec("vehicle", list(vp[:, 0]), list(vp[:, 1]), 12.0))
        spec = SceneSpec(list(pts[:, 0]), list(pts[:, 1]), 0.0, float(ego_target_speed), vehicles=vehicles,
                         hero_jitter_seed=None, actor_jitter_seed=None)
        spec.hero_rng_state = _rng_state(bundle.route_np_rng)
        spec.actor_rng_state = _rng_state(bundle.traffic_np_rng)
        spec.context = {"scene": "rdm", "scenario_param_num_vehicles": int(num_cars),
                        "scenario_param_route_dist_range": list(dist_range)}
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
        return SceneSpec(ego_rx, ego_ry, ego_speed, ego_speed, vehicles=vehicles)

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
        return SceneSpec(ego_rx, ego_ry, ego_speed, ego_speed, vehicles=vehicles, pedestrians=peds)

    # ------------------------------------------------------------ red light runner (synthetic geometry)
    INTERSECTIONS_RAW = [(8642, 1564), (8654, 6755), (7250, 1552), (7241, 2446), (7242, 3652), (7242, 4704),
                         (7257, 6773), (6199, 1552), (6197, 2439), (3349, 1545), (3350, 2456), (3350, 3639),
                         (3335, 4714), (3315, 6773), (2456, 1563), (2446, 6757)]

    def red_light_runner(self, level: int, g: np.random.Generator, kw: dict) -> SceneSpec:
        """Ego drives south->north through a 4-way intersection on green while an
        adversary crosses west->east on red (red_light_running.py:201-245). The
        intersection list is the reference's; routes are straight lines through
        its centre sampled every 12.5 px instead of lane-graph paths."""
        idx = kw.get("intersection_index")
        if idx is None:
            idx = int(g.integers(0, len(self.INTERSECTIONS_RAW)))
        if "center" in kw:
            cx, cy = (float(v) for v in kw["center"])
        else:
            ry_raw, rx_raw = self.INTERSECTIONS_RAW[int(idx)]
            cx, cy = rx_raw / 8.0, ry_raw / 8.0
        span = 950.0 / 8.0
        n = 20
        ego_ry = list(np.linspace(cy + span, cy - span, n))
        ego_rx = [cx + _m2s(1.75)] * n
        adv_rx = list(np.linspace(cx - span, cx + span, n))
        adv_ry = [cy + _m2s(1.75)] * n
        ego_speed = kw.get("ego_speed", 10.0)
        adv_speed = kw.get("adv_speed", 16.0)
        off = _m2s(4.0)
        length = _m2s(8.0)
        width = _m2s(0.45) + 1.0
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
            spec = self.generate_random(
                options.get("num_vehicles", self.max_vehicles),
                options.get("route_dist_range", [30, 100]),
                bundle,
                traffic_enabled=options.get("traffic_enabled", self.traffic_enabled),
                ego_target_speed=options.get("ego_target_speed", 12.0) or 12.0,
                max_retries=int(options.get("max_route_attempts") or 20),
            )
            return spec
        if scene in ("lead_brake", "jaywalk", "red_light_runner"):
            level = options.get("level")
            if level is None:
                level = bundle.scenario_rng.choice([1, 2, 3, 4])
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
