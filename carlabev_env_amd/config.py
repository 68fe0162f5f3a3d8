"""Configuration surface of the batched env (mirror of `CarlaBEV/config/`).

Same field names, defaults and validation rules as the reference's
`EnvConfig` / `RunConfig` (`CarlaBEV/config/env.py:43-207`), the preset
registries for actions (`config/action_profiles.py:35-76`), rewards
(`config/reward_profiles.py:19-45`) and difficulties (`config/difficulty.py:22-47`),
and the reset-option builders (`config/reset.py:15-116`). Validation stays on
the host; the HIP path only receives the resolved numeric constants
(`params.build_params`).
"""
from __future__ import annotations

import os
from typing import Any, Literal

import numpy as np
from pydantic import BaseModel, ConfigDict, Field, model_validator

ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")

ObsMode = Literal["bev_rgb", "bev_semantic", "vector"]
SemanticMaskCh = Literal["binary", "2-class", "4-class", "5-class", "6-class", "7-class"]
TemporalFusionMode = Literal["stack", "vehicle_temporal", "vehicle_weighted"]
ActionMode = Literal["discrete", "continuous"]
RewardMode = Literal["shaping", "carl"]
RenderMode = Literal["human", "rgb_array"]

# --------------------------------------------------------------- presets
ACTION_PROFILES: dict[str, dict[str, Any]] = {
    "discrete9_v1": {"action_mode": "discrete", "discrete_actions": [
        (0.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.0, 0.0, 1.0), (1.0, 1.0, 0.0), (1.0, -1.0, 0.0),
        (0.0, 1.0, 0.0), (0.0, -1.0, 0.0), (0.0, 1.0, 1.0), (0.0, -1.0, 1.0)]},
    "discrete13_v1": {"action_mode": "discrete", "discrete_actions": [
        (0.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.0, 0.0, 1.0), (1.0, 1.0, 0.0), (1.0, 0.5, 0.0),
        (1.0, -0.5, 0.0), (1.0, -1.0, 0.0), (0.0, 1.0, 0.0), (0.0, 0.5, 0.0), (0.0, -0.5, 0.0),
        (0.0, -1.0, 0.0), (0.0, 1.0, 1.0), (0.0, -1.0, 1.0)]},
    "continuous_gsb_v1": {"action_mode": "continuous", "low": (0.0, -1.0, 0.0), "high": (1.0, 1.0, 1.0)},
}

REWARD_PROFILES: dict[str, dict[str, Any]] = {
    "carl_base_v1": {"family": "carl", "parameters": {}},
    "carl_safety_v1": {"family": "carl", "parameters": {
        "lane_center_exponent": 1.5, "lane_center_floor": 0.15, "off_lane_penalty": 0.05,
        "speed_penalty_scale": 4.0, "speed_penalty_floor": 0.05, "ttc_threshold": 5.0,
        "ttc_penalty_floor": 0.05, "reward_scale": 0.85, "comfort_penalty_floor": 0.25}},
    "shaping_base_v1": {"family": "shaping", "parameters": {}},
}

DIFFICULTIES: dict[str, dict[str, Any]] = {
    "rt_no_traffic_v1": {"traffic_enabled": False, "num_vehicles": 0, "route_dist_range": (30, 80)},
    "rt_easy_v1": {"traffic_enabled": True, "num_vehicles": 8, "route_dist_range": (30, 80)},
    "rt_medium_v1": {"traffic_enabled": True, "num_vehicles": 16, "route_dist_range": (40, 100)},
    "rt_hard_v1": {"traffic_enabled": True, "num_vehicles": 25, "route_dist_range": (50, 130)},
}

LEGACY_ACTION_PROFILE_IDS = {"discrete": "discrete9_v1", "continuous": "continuous_gsb_v1"}
LEGACY_REWARD_PROFILE_IDS = {"carl": "carl_base_v1", "shaping": "shaping_base_v1"}


def get_action_profile_spec(profile_id: str) -> dict[str, Any]:
    if profile_id not in ACTION_PROFILES:
        raise KeyError(f"Unknown action_profile_id={profile_id!r}. Available action profiles: "
                       f"{', '.join(sorted(ACTION_PROFILES))}")
    return ACTION_PROFILES[profile_id]


def get_reward_profile_spec(profile_id: str) -> dict[str, Any]:
    if profile_id not in REWARD_PROFILES:
        raise KeyError(f"Unknown reward_profile_id={profile_id!r}. Available reward profiles: "
                       f"{', '.join(sorted(REWARD_PROFILES))}")
    return REWARD_PROFILES[profile_id]


def get_difficulty_spec(difficulty_id: str) -> dict[str, Any]:
    if difficulty_id not in DIFFICULTIES:
        raise KeyError(f"Unknown difficulty_id={difficulty_id!r}. Available difficulty presets: "
                       f"{', '.join(sorted(DIFFICULTIES))}")
    return dict(DIFFICULTIES[difficulty_id], difficulty_id=difficulty_id)


# --------------------------------------------------------------- EnvConfig
class EnvConfig(BaseModel):
    """Field-for-field mirror of `CarlaBEV.config.EnvConfig` (config/env.py:43-181)."""

    model_config = ConfigDict(extra="forbid", validate_assignment=True, populate_by_name=True)

    seed: int = 0
    fps: int = 15
    size: int = 128
    env_id: str = "CarlaBEV-v0"
    map_name: str = "Town01"
    obs_size: tuple[int, int] = (96, 96)
    obs_mode: ObsMode = "bev_semantic"
    semantic_mask_ch: SemanticMaskCh = "6-class"
    temporal_fusion_mode: TemporalFusionMode = "stack"
    fov_masked: bool = False
    ego_anchor_x_frac: float = 0.5
    ego_anchor_y_frac: float = 0.5
    frame_stack: int = 4
    action_mode: ActionMode = "discrete"
    action_profile_id: str | None = None
    render_mode: RenderMode = "human"
    max_actions: int = 5000
    scenes_path: str = "assets/scenes"
    reward_mode: RewardMode = "carl"
    reward_profile_id: str | None = None
    traffic_enabled: bool = True
    max_vehicles: int = 50
    route_direction_metrics_enabled: bool = False

    @model_validator(mode="before")
    @classmethod
    def _normalize_legacy_fields(cls, data: Any):
        if not isinstance(data, dict):
            return data
        d = dict(data)
        if "obs_mode" not in d:
            if d.get("obs_space") == "vector":
                d["obs_mode"] = "vector"
            elif d.get("masked") is False:
                d["obs_mode"] = "bev_rgb"
            else:
                d["obs_mode"] = "bev_semantic"
        d.pop("obs_space", None)
        d.pop("masked", None)
        if "action_mode" not in d and "action_space" in d:
            d["action_mode"] = d["action_space"]
        d.pop("action_space", None)
        if "reward_mode" not in d and "reward_type" in d:
            d["reward_mode"] = "carl" if d["reward_type"] == "carl" else "shaping"
        d.pop("reward_type", None)
        if d.get("action_profile_id") is None:
            d["action_profile_id"] = LEGACY_ACTION_PROFILE_IDS.get(d.get("action_mode", "discrete"), "discrete9_v1")
        if d.get("reward_profile_id") is None:
            d["reward_profile_id"] = LEGACY_REWARD_PROFILE_IDS.get(d.get("reward_mode", "carl"), "carl_base_v1")
        return d

    @model_validator(mode="after")
    def _validate_values(self):
        if self.frame_stack < 1:
            raise ValueError("frame_stack must be >= 1")
        if self.temporal_fusion_mode != "stack":
            if self.obs_mode != "bev_semantic":
                raise ValueError("temporal_fusion_mode requires obs_mode='bev_semantic'")
            if self.frame_stack < 3:
                raise ValueError("temporal_fusion_mode requires frame_stack >= 3")
            if self.semantic_mask_ch not in {"4-class", "5-class", "6-class", "7-class"}:
                raise ValueError("temporal_fusion_mode requires a semantic_mask_ch with a vehicle channel")
        if self.obs_size[0] < 1 or self.obs_size[1] < 1:
            raise ValueError("obs_size dimensions must be >= 1")
        if not 0.0 <= self.ego_anchor_x_frac <= 1.0:
            raise ValueError("ego_anchor_x_frac must be within [0.0, 1.0]")
        if not 0.0 <= self.ego_anchor_y_frac <= 1.0:
            raise ValueError("ego_anchor_y_frac must be within [0.0, 1.0]")
        a = get_action_profile_spec(self.action_profile_id)
        r = get_reward_profile_spec(self.reward_profile_id)
        if a["action_mode"] != self.action_mode:
            raise ValueError(f"action_profile_id={self.action_profile_id!r} resolves to action_mode="
                             f"{a['action_mode']!r}, but EnvConfig.action_mode={self.action_mode!r}")
        if r["family"] != self.reward_mode:
            raise ValueError(f"reward_profile_id={self.reward_profile_id!r} resolves to reward_mode="
                             f"{r['family']!r}, but EnvConfig.reward_mode={self.reward_mode!r}")
        path = os.path.join(ASSET_DIR, f"{self.map_name}-{self.size}-class.npz")
        if not os.path.exists(path):
            raise ValueError(f"map_name='{self.map_name}' is missing required assets: [{path!r}]")
        return self

    @property
    def masked(self) -> bool:
        return self.obs_mode == "bev_semantic"

    @property
    def obs_space(self) -> str:
        return "vector" if self.obs_mode == "vector" else "bev"

    @property
    def action_space(self) -> str:
        return self.action_mode

    @property
    def reward_type(self) -> str:
        return "carl" if self.reward_mode == "carl" else "shaping"


class RunConfig(BaseModel):
    """Mirror of `CarlaBEV.config.RunConfig` (config/env.py:184-207)."""

    model_config = ConfigDict(extra="forbid", validate_assignment=True, populate_by_name=True)

    env: EnvConfig = Field(default_factory=EnvConfig)
    exp_name: str = "carlabev-run"
    num_envs: int = 1
    seed: int = 1
    capture_video: bool = False
    capture_every: int = 50
    video_output_dir: str | None = None
    video_episode_indices: list[int] | None = None
    video_name_prefix: str = "rl-video"
    cuda: bool = True
    torch_deterministic: bool = True

    @model_validator(mode="after")
    def _validate_values(self):
        if self.num_envs < 1:
            raise ValueError("num_envs must be >= 1")
        return self


def validate_env_config(cfg) -> EnvConfig:
    return cfg if isinstance(cfg, EnvConfig) else EnvConfig.model_validate(dict(cfg))


def validate_run_config(cfg) -> RunConfig:
    run = cfg if isinstance(cfg, RunConfig) else RunConfig.model_validate(dict(cfg))
    if run.env.obs_mode == "vector":
        raise ValueError("obs_mode='vector' is not supported through make_env()/wrap_env() yet. "
                         "Use CarlaBEV() directly if you need vector observations.")
    return run


# --------------------------------------------------------------- reset options
class RandomNavigationReset(BaseModel):
    """Mirror of config/reset.py:15-31."""

    model_config = ConfigDict(extra="forbid", validate_assignment=True)

    difficulty_id: str | None = None
    num_vehicles: int = 25
    route_dist_range: tuple[int, int] = (30, 130)
    ego_route_graph: str = "full_vehicle"
    route_profile: str | None = None
    route_profile_mix: dict[str, float] | None = None
    min_turns: int | None = None
    max_turns: int | None = None
    intersection_required: bool | None = None
    max_route_attempts: int | None = None
    scene_seed: int | None = None
    route_seed: int | None = None
    traffic_seed: int | None = None
    scenario_seed: int | None = None


def build_random_navigation_options(request: RandomNavigationReset, *, reset_mask=None) -> dict[str, Any]:
    """config/reset.py:73-116."""
    options: dict[str, Any] = {
        "scene": "rdm",
        "num_vehicles": int(request.num_vehicles),
        "route_dist_range": list(request.route_dist_range),
        "ego_route_graph": request.ego_route_graph,
    }
    for key in ("route_profile", "min_turns", "max_turns", "intersection_required", "max_route_attempts",
                "scene_seed", "route_seed", "traffic_seed", "scenario_seed"):
        val = getattr(request, key)
        if val is not None:
            options[key] = val
    if request.route_profile_mix is not None:
        options["route_profile_mix"] = dict(request.route_profile_mix)
    if request.difficulty_id is not None:
        spec = get_difficulty_spec(request.difficulty_id)
        options.update({"difficulty_id": spec["difficulty_id"], "traffic_enabled": spec["traffic_enabled"],
                        "num_vehicles": int(spec["num_vehicles"]),
                        "route_dist_range": list(spec["route_dist_range"])})
    if reset_mask is not None:
        options["reset_mask"] = np.asarray(reset_mask, dtype=bool)
    return options


def list_action_profile_ids():
    return sorted(ACTION_PROFILES)


def list_reward_profile_ids():
    return sorted(REWARD_PROFILES)


def list_difficulty_ids():
    return sorted(DIFFICULTIES)
