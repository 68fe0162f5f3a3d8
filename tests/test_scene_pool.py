"""Host scene feed (carlabev_env_amd/scene_pool.py): worker processes build the
same packed records as a HostResetBuilder in this process, for the same global
scene ids (scene_seed = seed0 + gid, carlabev.py:96-148)."""
from __future__ import annotations

import numpy as np

from carlabev_env_amd.config import EnvConfig
from carlabev_env_amd.scene_pool import ScenePool, make_builder, scene_options

CAPS = dict(route_cap=64, actor_cap=20, actor_route_cap=288, tl_cap=4)


def test_pool_records_match_in_process_builder():
    cfg = EnvConfig(size=128, obs_size=(128, 128), render_mode="rgb_array").model_dump()
    builder, layout = make_builder(cfg, CAPS)
    pool = ScenePool(cfg, CAPS, "rt_medium_v1", 40_000, layout.record_bytes, workers=2, first_gid=100, stride=3,
                     batch=2)
    try:
        pool.request(5)
        got_ids, got = [], []
        for _ in range(60):
            g, r = pool.poll(timeout=2.0)
            got_ids += g
            got.append(r)
            if len(got_ids) >= 5:
                break
        recs = np.concatenate(got)
        assert sorted(got_ids) == [100, 103, 106, 109, 112]
        for gid, rec in zip(got_ids, recs):
            want = np.zeros(layout.record_bytes, np.uint8)
            builder.build(want, None, dict(scene_options("rt_medium_v1", gid), scene_seed=40_000 + gid))
            assert np.array_equal(rec, want), gid
        assert pool.delivered == 5 and pool.requested == 5
    finally:
        pool.close()


def test_pool_reports_worker_errors():
    cfg = EnvConfig(size=128, obs_size=(128, 128), render_mode="rgb_array").model_dump()
    small = dict(CAPS, actor_cap=2)  # rt_medium's 16 vehicles do not fit
    _, layout = make_builder(cfg, small)
    pool = ScenePool(cfg, small, "rt_medium_v1", 0, layout.record_bytes, workers=1, batch=1)
    try:
        pool.request(1)
        import pytest
        with pytest.raises(RuntimeError, match="actor_cap"):
            for _ in range(60):
                pool.poll(timeout=2.0)
    finally:
        pool.close()


def test_scene_options_mix():
    assert [scene_options("mix3", g)["scene"] for g in range(4)] == ["lead_brake", "jaywalk", "red_light_runner",
                                                                       "lead_brake"]


def test_build_scenes_rejects_repeated_ids():
    """One output row per scene id: a repeated id would leave a row of zeros that
    looks like a record, so build_scenes refuses it before any work."""
    import pytest
    from carlabev_env_amd.scene_pool import build_scenes
    cfg = EnvConfig(size=128, obs_size=(128, 128), render_mode="rgb_array").model_dump()
    _, layout = make_builder(cfg, CAPS)
    with pytest.raises(ValueError, match="repeated scene ids"):
        build_scenes(cfg, CAPS, "rt_easy_v1", 0, layout.record_bytes, [3, 5, 3], workers=1)
