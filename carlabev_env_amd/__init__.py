"""MI355X-native batched step() for CarlaBEV (HIP/gfx950).

Drop-in for the reference's vector env (`CarlaBEV.envs.make_env`): the
per-env step (ego bicycle, scripted actors, route checkpoints, BEV raster,
collision/reward/termination) runs as HIP kernels through libcbev.so; scene
generation stays on the host.
"""
from .config import (EnvConfig, RunConfig, RandomNavigationReset, build_random_navigation_options,
                     validate_env_config, validate_run_config, get_action_profile_spec, get_reward_profile_spec,
                     get_difficulty_spec, list_action_profile_ids, list_reward_profile_ids, list_difficulty_ids)

__version__ = "0.1.0"

__all__ = ["EnvConfig", "RunConfig", "RandomNavigationReset", "build_random_navigation_options",
           "validate_env_config", "validate_run_config", "get_action_profile_spec", "get_reward_profile_spec",
           "get_difficulty_spec", "list_action_profile_ids", "list_reward_profile_ids", "list_difficulty_ids",
           "make_env", "CarlaBEVVectorEnv"]


def __getattr__(name):
    # torch-dependent pieces load lazily so config/scene tooling imports fast
    if name in ("make_env", "CarlaBEVVectorEnv"):
        from . import vector_env
        return getattr(vector_env, name)
    raise AttributeError(name)
