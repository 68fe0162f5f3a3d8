"""Test-only restatement of the reference's episode statistics
(`CarlaBEV/src/deeprl/stats.py:19-148`, comfort bounds `comfort.py:3-10,64-70`)
fed with per-step values read back from the device, to check the device's
episode summaries (include/cbev_layout.h CBEV_EP_FIELDS).

Each per-step `info` holds what `EpisodeStats.step` reads: the reward, the
step's reward cause (None when none), the hero speed state[3] and the six
comfort metrics of `hero.last_comfort`.
"""
from __future__ import annotations

from collections import deque

import numpy as np

COMFORT_KEYS = ("accel_long", "accel_lat", "jerk_long", "jerk_lat", "yaw_rate", "yaw_acc")
BOUNDS = {"accel_long": 2.0, "accel_lat": 2.0, "yaw_rate": 20.0, "jerk_long": 3.0, "jerk_lat": 3.0, "yaw_acc": 120.0}


class EpisodeStats:  # stats.py:19-84
    def __init__(self):
        self.rewards, self.speeds, self.progress, self.ttc = [], [], [], []
        self.cause = None
        self.comfort_values = {k: [] for k in COMFORT_KEYS}
        self.comfort_step_violations, self.harsh_brake_flags = [], []

    def step(self, info):
        self.rewards.append(info["reward"])
        if info["cause"] is not None:
            self.cause = info["cause"]
        self.speeds.append(info["v"])
        metrics = {k: float(info[k]) for k in COMFORT_KEYS}
        for k, v in metrics.items():
            self.comfort_values[k].append(abs(v))
        violations = sum(int(abs(metrics[k]) > lim) for k, lim in BOUNDS.items())
        self.comfort_step_violations.append(1.0 if violations > 0 else 0.0)
        self.harsh_brake_flags.append(1.0 if metrics["accel_long"] < -BOUNDS["accel_long"] else 0.0)

    @property
    def episode_return(self):
        return float(np.sum(self.rewards))

    def mean(self, vals):
        return float(np.mean(vals)) if vals else 0.0


class Stats:  # stats.py:87-148
    def __init__(self, maxlen=200):
        self.current = EpisodeStats()
        self.history = deque(maxlen=maxlen)
        self.episode = 0

    def reset(self):
        self.current = EpisodeStats()

    def _count(self, name):
        vals = [ep.cause for ep in self.history]
        return vals.count(name) / len(vals) if vals else 0.0

    def terminated(self):
        c = self.current
        vals = [ep.episode_return for ep in self.history]
        summary = {
            "episode": self.episode, "termination": c.cause, "return": c.episode_return, "length": len(c.rewards),
            "mean_reward": np.mean(vals) if vals else 0.0,
            "success_rate": self._count("success"), "collision_rate": self._count("collision"),
            "unfinished_rate": self._count("off_road"),
            "mean_speed": c.mean(c.speeds), "mean_ttc": c.mean(c.ttc), "mean_progress": c.mean(c.progress),
            "mean_abs_accel_long": c.mean(c.comfort_values["accel_long"]),
            "mean_abs_accel_lat": c.mean(c.comfort_values["accel_lat"]),
            "mean_abs_jerk_long": c.mean(c.comfort_values["jerk_long"]),
            "mean_abs_jerk_lat": c.mean(c.comfort_values["jerk_lat"]),
            "mean_abs_yaw_rate": c.mean(c.comfort_values["yaw_rate"]),
            "mean_abs_yaw_acc": c.mean(c.comfort_values["yaw_acc"]),
            "comfort_violation_rate": c.mean(c.comfort_step_violations),
            "harsh_brake_rate": c.mean(c.harsh_brake_flags),
        }
        self.history.append(self.current)
        self.episode += 1
        self.reset()
        return summary
