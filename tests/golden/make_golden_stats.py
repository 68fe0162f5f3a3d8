"""Golden vectors for the episode statistics, from the reference's own `Stats`
(`CarlaBEV/src/deeprl/stats.py:19-148`, comfort bounds `comfort.py:3-10,64-70`).

Runs ONLY in the build container (imports the reference through refimport);
writes tests/golden/stats.npz, which tests/test_stats_golden.py checks
tests/stats_ref.py (the restatement the GPU episode test compares the device
with) against. Each stream is one env's Stats object fed a seeded sequence of
per-step `info` dicts shaped as CarlaBEV.step builds them (carlabev.py:159-185:
info["reward"] = {reward, cause}, info["hero"] = {state, comfort metrics}) and
terminated at the end of every episode (`Stats.terminated()`), covering every
cause, windows past the 200-episode history, comfort violations of every bound
and harsh brakes.

  steps[k]     = (stream, reward, cause code, v, accel_long, accel_lat, jerk_long,
                  jerk_lat, yaw_rate, yaw_acc, ends_episode)
  summaries[j] = (stream, the 19 values of get_episode_info in SUMMARY_KEYS order,
                  the termination cause code)
cause codes are carlabev_env_amd.layout.CAUSE (None = 0).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import refimport  # noqa: E402

refimport.setup()

from CarlaBEV.src.deeprl.stats import Stats  # noqa: E402

from carlabev_env_amd.layout import CAUSE  # noqa: E402

SUMMARY_KEYS = ("episode", "return", "length", "mean_reward", "success_rate", "collision_rate", "unfinished_rate",
                "mean_speed", "mean_ttc", "mean_progress", "mean_abs_accel_long", "mean_abs_accel_lat",
                "mean_abs_jerk_long", "mean_abs_jerk_lat", "mean_abs_yaw_rate", "mean_abs_yaw_acc",
                "comfort_violation_rate", "harsh_brake_rate")
TERMINAL = ("collision", "success", "off_road", "out_of_bounds", "max_actions")
COMFORT = ("accel_long", "accel_lat", "jerk_long", "jerk_lat", "yaw_rate", "yaw_acc")
SCALE = {"accel_long": 2.5, "accel_lat": 2.5, "jerk_long": 4.0, "jerk_lat": 4.0, "yaw_rate": 25.0, "yaw_acc": 150.0}


def stream(rng, k, n_episodes, max_len, steps, summaries):
    st = Stats()
    for ep in range(n_episodes):
        length = int(rng.integers(1, max_len + 1))
        end_cause = TERMINAL[int(rng.integers(0, len(TERMINAL)))]
        for t in range(length):
            last = t == length - 1
            cause = end_cause if last else ("ckpt" if rng.random() < 0.1 else None)
            if cause is None:
                r = float(rng.uniform(0.0, 1.0)) if rng.random() < 0.8 else 0.0
            elif cause == "ckpt":
                r = 0.1
            else:
                r = {"success": 1.0, "max_actions": 0.0}.get(cause, -1.0) * (1.0 if rng.random() < 0.7 else 18.0)
            if rng.random() < 0.05:  # large magnitudes stress the window sums
                r *= float(rng.choice([1e3, -1e4, 3.3e5]))
            v = float(rng.uniform(-3.0, 45.0))
            comfort = {c: float(rng.normal(0.0, SCALE[c])) for c in COMFORT}
            if rng.random() < 0.15:  # harsh brake
                comfort["accel_long"] = -float(rng.uniform(2.0001, 9.0))
            if rng.random() < 0.05:  # exactly at a bound: not a violation
                c = COMFORT[int(rng.integers(0, 6))]
                comfort[c] = {"accel_long": 2.0, "accel_lat": -2.0, "jerk_long": 3.0, "jerk_lat": 3.0,
                              "yaw_rate": 20.0, "yaw_acc": -120.0}[c]
            info = {"reward": {"reward": r, "cause": cause},
                    "hero": dict({"state": [0.0, 0.0, 0.0, v]}, **comfort)}
            st.step(info)
            steps.append((k, r, CAUSE[cause], v, *[comfort[c] for c in COMFORT], float(last)))
        s = st.terminated()
        summaries.append((k, *[float(s[key]) for key in SUMMARY_KEYS], CAUSE[s["termination"]]))


def main():
    rng = np.random.default_rng(20261017)
    steps, summaries = [], []
    stream(rng, 0, 230, 6, steps, summaries)    # window wraps past 200 episodes
    stream(rng, 1, 215, 12, steps, summaries)
    stream(rng, 2, 40, 60, steps, summaries)
    stream(rng, 3, 3, 1, steps, summaries)      # 1-step episodes
    path = os.path.join(HERE, "stats.npz")
    np.savez_compressed(path, steps=np.array(steps, dtype=np.float64), summaries=np.array(summaries, dtype=np.float64),
                        keys=np.array(SUMMARY_KEYS))
    print(f"stats.npz: {len(steps)} steps, {len(summaries)} episodes, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
