"""tests/stats_ref.py (the episode-statistics restatement test_gpu_episode.py
checks the device's summaries with) against the reference's own `Stats`
(CarlaBEV/src/deeprl/stats.py:19-148) on the seeded sequences of
tests/golden/stats.npz (made by tests/golden/make_golden_stats.py): every cause,
ckpt steps, history windows past 200 episodes, comfort violations at and past
every bound, harsh brakes, 1-step episodes."""
from __future__ import annotations

import os

import numpy as np

from carlabev_env_amd.layout import CAUSE_NAME
from stats_ref import COMFORT_KEYS, Stats

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "stats.npz")


def test_stats_ref_matches_reference_stats():
    d = np.load(GOLD)
    steps, summ, keys = d["steps"], d["summaries"], [str(k) for k in d["keys"]]
    streams = {}
    got = []
    for row in steps:
        k = int(row[0])
        st = streams.setdefault(k, Stats())
        info = {"reward": float(row[1]), "cause": CAUSE_NAME[int(row[2])], "v": float(row[3])}
        info.update({c: float(row[4 + i]) for i, c in enumerate(COMFORT_KEYS)})
        st.current.step(info)
        if row[10]:
            s = st.terminated()
            got.append((k, [s[key] for key in keys], s["termination"]))
    assert len(got) == len(summ)
    assert max(len(st.history) for st in streams.values()) == 200  # the window wrapped
    for (k, vals, cause), want in zip(got, summ):
        assert k == int(want[0])
        assert CAUSE_NAME[int(want[-1])] == cause
        np.testing.assert_array_equal(np.array(vals, dtype=np.float64), want[1:-1])
