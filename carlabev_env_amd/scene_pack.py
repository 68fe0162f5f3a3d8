"""Scene -> device record packing (host side of `CarlaBEV.reset`).

A `SceneSpec` is the realised content of the reference's actors dict after
`SceneGenerator.build_scene` (`src/managers/scene_generator.py:95-191`):
ego route + speeds, vehicles, pedestrians, traffic lights. `pack_scene`
reproduces what `CarlaBEV.reset` (`envs/carlabev.py:96-148`) then does to it:

  BaseMap.reset -> Scene.load_scene      scene.py:61-88
    ActorManager.spawn_hero              actor_manager.py:36-64 (m/s -> px/s)
    BaseAgent.__init__ (set_route, jitter, initial stanley)  hero.py:52-86
    set_targets(hero.cx, hero.cy)        scenes/utils.py:114-122
    ActorManager.reset_all -> Actor.reset (controller, jitter, behaviour reset)
                                         actor_manager.py:100-109, actor.py:86-108
  Scene.reset_scene metrics               scene.py:49-54
  CaRLRewardFn.reset(rx, ry)              carl_reward_fn.py:121-134
  Stats.reset / RewardFn.reset            stats.py, reward.py:75-78

and writes the result into one fixed-size record (include/cbev_layout.h).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import layout as LY
from .routes import ControllerInit, cumulative_lengths_int

MPP = 40.0 / 128.0  # SURFACE_METERS_PER_PIXEL (envs/geometry.py:6-10)

# palette ids of traffic-light colours (traffic_light.py:46-54)
TL_COLOR = {"red": 6, "yellow": 7, "green": 5, "unknown": 9}


def mps_to_surface(v: float) -> float:
    return float(v) / MPP


@dataclass
class ActorSpec:
    kind: str                     # "vehicle" | "pedestrian"
    rx: list                      # surface route (floats), Actor.rx
    ry: list
    speed_mps: float              # cruise speed (Vehicle default 12.0, Pedestrian 1.5)
    behavior: dict | None = None  # {"type": ..., "params": {...}} (behavior/registry.py)
    jitter: bool = True           # Controller.set_route(jitter_start=True)


@dataclass
class TrafficLightSpec:
    x: float
    y: float
    orientation: str = "horizontal"
    state: str = "red"
    width: float | None = None
    length: float | None = None

    def rect(self):
        """TrafficLight.draw rect (traffic_light.py:58-90): float Rect, truncated, no pad offset."""
        width = float(self.width) if self.width is not None else max(1.0, 0.45 / MPP) + 1.0
        length = float(self.length) if self.length is not None else max(4.0, 8.5 / MPP)
        w, h = (length, width) if self.orientation == "horizontal" else (width, length)
        return int(self.x - w / 2), int(self.y - h / 2), int(w), int(h)


@dataclass
class SceneSpec:
    agent_rx: list                      # ego route (surface floats); packed as int32 like Scene.agent_route
    agent_ry: list
    initial_speed_mps: float = 0.0
    target_speed_mps: float = 12.0
    vehicles: list = field(default_factory=list)
    pedestrians: list = field(default_factory=list)
    traffic_lights: list = field(default_factory=list)
    hero_jitter_seed: int | None = None     # route_np_rng seed (randomness.py:35-65)
    actor_jitter_seed: int | None = None    # traffic_np_rng / scenario_np_rng seed
    hero_rng_state: dict | None = None      # or the exact generator state to draw the jitter from
    actor_rng_state: dict | None = None
    context: dict = field(default_factory=dict)
    len_route_m: float | None = None        # the len_route build_scene returns, when the sampler reports one

    def caps_needed(self):
        n_route = len(self.agent_rx)
        acts = list(self.vehicles) + list(self.pedestrians)
        ra = max([len(a.rx) + 2 for a in acts], default=0)
        return n_route, len(acts), ra, len(self.traffic_lights)


def _generator(state, seed):
    g = np.random.default_rng(seed)
    if state is not None:
        g.bit_generator.state = state
    return g


def behavior_fields(beh: dict | None):
    """(BEH id, P0, P1) for behaviour specs as normalised by behavior/registry.py:94-143."""
    if beh is None:
        return LY.BEH["none"], 0.0, 0.0
    t = beh.get("type", "none")
    p = beh.get("params", {}) or {}
    if t in ("none", "constant_speed"):
        return LY.BEH["none"], 0.0, 0.0
    if t == "timed_brake":
        return LY.BEH[t], float(p.get("start_brake_t", 3.5)), float(p.get("decel_mps2", 1.0))
    if t in ("cross", "stop_mid"):
        return LY.BEH[t], float(p.get("start_delay", 0.0)), 0.0
    if t == "yield_return":
        return LY.BEH[t], float(p.get("start_delay", 0.0)), float(p.get("yield_duration", 1.0))
    raise ValueError(f"unknown behaviour {t!r}")


def init_actor_slot(view: LY.RecordView, a: int, spec: ActorSpec, np_rng, map_size: int = 128):
    """Actor.__init__ + Actor.reset (actor.py:43-108) into slot a."""
    scale = int(1024 / map_size)
    size = int(32 / scale) if spec.kind == "vehicle" else int(16 / scale)
    cruise_mps = max(0.0, float(spec.speed_mps))
    cruise = mps_to_surface(cruise_mps)
    rx = [float(v) for v in spec.rx]
    ry = [float(v) for v in spec.ry]
    ci = ControllerInit(rx, ry, cruise, jitter_start=spec.jitter, np_rng=np_rng)
    n = len(ci.cx)
    ra = view.acx.shape[1]
    if n > ra or len(rx) > ra:
        raise ValueError(f"actor route of {max(n, len(rx))} points exceeds actor_route_cap={ra}")
    beh, p0, p1 = behavior_fields(spec.behavior)
    if beh == LY.BEH["yield_return"] and len(rx) + 1 > min(ra, 64):
        # a StopReturn retreat rebuilds the route as [pos] + initial_route[:idx + 1][::-1]
        # (jaywalk.py:43-54): up to len(rx) + 1 points, which must fit the slot and the
        # device's wave-wide rebuild (one point per lane: at most 64)
        raise ValueError(f"yield_return actor route of {len(rx)} points: its retreat route ({len(rx) + 1} points) "
                         f"must fit actor_route_cap={ra} and 64 points")
    ad, ai = view.ad, view.ai
    ad[LY.AD["X"], a], ad[LY.AD["Y"], a], ad[LY.AD["YAW"], a], ad[LY.AD["V"], a] = ci.x, ci.y, ci.yaw, ci.v
    ad[LY.AD["CT_SPEED"], a] = cruise            # Controller(self.target_speed)
    ad[LY.AD["CRUISE"], a] = cruise
    ad[LY.AD["CRUISE_MPS"], a] = cruise_mps
    ad[LY.AD["T_SPEED"], a] = cruise
    ad[LY.AD["T_SPEED_MPS"], a] = cruise_mps
    ad[LY.AD["TIME"], a] = 0.0
    ad[LY.AD["ELAPSED"], a] = 0.0
    ad[LY.AD["STATE_ELAPSED"], a] = 0.0
    ad[LY.AD["P0"], a], ad[LY.AD["P1"], a] = p0, p1
    ad[LY.AD["GOAL_X"], a] = ad[LY.AD["GOAL_Y"], a] = 0.0
    ai[LY.AI["KIND"], a] = 1 if spec.kind == "vehicle" else 2
    ai[LY.AI["SIZE"], a] = size
    ai[LY.AI["TIDX"], a] = ci.target_idx
    ai[LY.AI["NROUTE"], a] = n
    ai[LY.AI["NRX"], a] = len(rx)
    ai[LY.AI["NINIT"], a] = len(rx)
    ai[LY.AI["BEH"], a] = beh
    ai[LY.AI["BSTATE"], a] = LY.BSTATE["idle"]
    ai[LY.AI["BRAKING"], a] = 0
    ai[LY.AI["HAS_GOAL"], a] = 0
    if beh in (LY.BEH["cross"], LY.BEH["stop_mid"], LY.BEH["yield_return"]):
        # BaseJaywalkBehavior.reset (jaywalk.py:36-41)
        ai[LY.AI["BSTATE"], a] = LY.BSTATE["waiting"]
        ad[LY.AD["T_SPEED_MPS"], a] = 0.0
        ad[LY.AD["T_SPEED"], a] = 0.0
    view.acx[a, :n], view.acy[a, :n], view.acyaw[a, :n] = ci.cx, ci.cy, ci.cyaw
    view.acf[a, :n, 0], view.acf[a, :n, 1] = view.acx[a, :n], view.acy[a, :n]  # float32 rounding
    view.acb[a, :(n + LY.ACB_PTS - 1) // LY.ACB_PTS] = LY.acb_circles(view.acf[a, :n])  # the search's pruning circles
    view.aix[a, :len(rx)], view.aiy[a, :len(rx)] = rx, ry
    view.arx[a, :len(rx)], view.ary[a, :len(rx)] = rx, ry


def pack_scene(view: LY.RecordView, spec: SceneSpec, size: int, scene_id: int = 0) -> dict:
    """Write the realised reset state of `spec` into a zeroed record view.
    Returns the reset-time info (spawn validation etc. is decided by the caller)."""
    hd, hi = view.hd, view.hi
    hd[:] = 0.0
    hi[:] = 0
    view.vis[:] = 0
    # Scene.agent_route: int32 route (scene.py:179-196); spawn_hero m/s -> px/s
    rx = np.asarray(spec.agent_rx, dtype=np.int32)
    ry = np.asarray(spec.agent_ry, dtype=np.int32)
    R = view.cx.shape[0]
    hero_rng = _generator(spec.hero_rng_state, spec.hero_jitter_seed)
    ci = ControllerInit(rx, ry, mps_to_surface(spec.initial_speed_mps), jitter_start=True, np_rng=hero_rng, hero=True)
    n = len(ci.cx)
    if n > R or len(rx) > R:
        raise ValueError(f"ego route of {max(n, len(rx))} points exceeds route_cap={R}")
    hd[LY.HD["X"]], hd[LY.HD["Y"]], hd[LY.HD["YAW"]], hd[LY.HD["V"]] = ci.x, ci.y, ci.yaw, ci.v
    hd[LY.HD["TSPEED"]] = mps_to_surface(spec.target_speed_mps)
    hi[LY.HI["TIDX"]] = ci.target_idx
    hi[LY.HI["NROUTE"]] = n
    hi[LY.HI["NRAW"]] = len(rx)
    view.cx[:n], view.cy[:n], view.cyaw[:n] = ci.cx, ci.cy, ci.cyaw
    view.raw_x[:len(rx)], view.raw_y[:len(rx)] = rx, ry
    cum = cumulative_lengths_int(rx, ry)
    view.raw_cum[:len(rx)] = cum
    hd[LY.HD["ROUTE_TOTAL"]] = cum[-1]
    # targets at the smoothed ego route, all visible (target.py:29-33)
    for i in range(n):
        view.vis[i >> 5] |= np.uint32(1 << (i & 31))
    hd[LY.HD["GOAL_X"]], hd[LY.HD["GOAL_Y"]] = ci.cx[-1], ci.cy[-1]
    d2g = float(np.linalg.norm(np.array([ci.x, ci.y]) - np.array([ci.cx[-1], ci.cy[-1]])))
    hd[LY.HD["D2G"]] = hd[LY.HD["D2G_T1"]] = d2g
    # actors: vehicles first, then pedestrians (ActorManager dict order)
    actors = [a for a in list(spec.vehicles) + list(spec.pedestrians) if len(a.rx) >= 2 and len(a.ry) >= 2]
    A = view.ad.shape[1]
    if len(actors) > A:
        raise ValueError(f"{len(actors)} actors exceed actor_cap={A}")
    actor_rng = _generator(spec.actor_rng_state, spec.actor_jitter_seed)
    for a, act in enumerate(actors):
        # actors are always built with map_size=128 (scene_generator.py:71-75,334), so
        # they stay 4x4 / 2x2 at size 256
        init_actor_slot(view, a, act, actor_rng)
    hi[LY.HI["NACT"]] = len(actors)
    hi[LY.HI["NVEH"]] = sum(1 for a in actors if a.kind == "vehicle")
    T = view.ti.shape[1]
    if len(spec.traffic_lights) > T:
        raise ValueError(f"{len(spec.traffic_lights)} traffic lights exceed tl_cap={T}")
    for k, tl in enumerate(spec.traffic_lights):
        x, y, w, h = tl.rect()
        view.ti[LY.TI["RX"], k], view.ti[LY.TI["RY"], k] = x, y
        view.ti[LY.TI["RW"], k], view.ti[LY.TI["RH"], k] = w, h
        view.ti[LY.TI["COLOR"], k] = TL_COLOR.get(tl.state, 9)
    hi[LY.HI["NTL"]] = len(spec.traffic_lights)
    hi[LY.HI["ACTOR_ID"]] = -1
    hi[LY.HI["SCENE_ID"]] = scene_id
    return {"n_route": n, "n_actors": len(actors)}
