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


def test_build_pool_matches_serial_reset_build():
    """BuildPool (the parallel half of CarlaBEVVectorEnv.reset(options)) writes the
    bytes, spawn validation and scenario context a serial in-process build writes
    for the same (seed, options), in the order asked, over scene kinds with and
    without traffic and scenario samplers."""
    from carlabev_env_amd.scene_pool import BuildPool
    cfg = EnvConfig(size=128, obs_size=(128, 128), render_mode="rgb_array").model_dump()
    builder, layout = make_builder(cfg, CAPS)
    items = [(7_000 + k, dict(scene_options(d, k))) for k, d in
             enumerate(["rt_no_traffic_v1", "rt_medium_v1", "mix3", "rt_easy_v1", "mix3", "mix3", "rt_medium_v1"])]
    items.append((None, dict(scene_options("rt_no_traffic_v1", 0))))  # seed None: the config's seed (carlabev.py:84)
    pool = BuildPool(cfg, CAPS, workers=3, chunk=2)
    try:
        recs, meta = pool.build(items)
    finally:
        pool.close()
    for k, (seed, opts) in enumerate(items):
        want = np.zeros(layout.record_bytes, np.uint8)
        info, _spec, ctx = builder.build(want, seed, opts)
        assert np.array_equal(recs[k], want), k
        assert meta[k] == (info, ctx), k


def test_reset_build_memo_is_exact():
    """HostResetBuilder memoises by (scene seed, options): a repeated reset copies
    the bytes of the first build (which a fresh builder reproduces), and the
    returned dicts are independent copies."""
    cfg = EnvConfig(size=128, obs_size=(128, 128), render_mode="rgb_array").model_dump()
    b1, layout = make_builder(cfg, CAPS)
    b2, _ = make_builder(cfg, CAPS)
    opts = dict(scene_options("rt_medium_v1", 3))
    r1, r2, r3 = (np.zeros(layout.record_bytes, np.uint8) for _ in range(3))
    i1, _, c1 = b1.build(r1, 5, dict(opts, reset_mask=np.ones(4, bool)))
    i2, _, c2 = b1.build(r2, 5, opts)  # the reset mask is not part of the scene
    b2.build(r3, 5, opts)
    assert b1.builds == 1 and b1.memo_hits == 1
    assert np.array_equal(r1, r2) and np.array_equal(r1, r3)
    assert i1 == i2 and c1 == c2 and c1 is not c2
    c2["scene"] = "edited"
    _, _, c4 = b1.build(r2, 5, opts)
    assert c4["scene"] != "edited"
    b1.build(r2, 6, opts)  # another seed: built
    assert b1.builds == 2 and not np.array_equal(r1, r2)


def test_memo_copies_are_deep_and_independent():
    """The memo's plain-data copy (host_reset._copy_plain, in place of
    copy.deepcopy) keeps values and types and shares nothing mutable; objects it
    does not know go through copy.deepcopy."""
    from carlabev_env_amd.host_reset import _copy_plain

    class Box:
        def __init__(self, v):
            self.v = v

    src = {"a": [1, 2.5, None, True, "s", np.int64(3)], "b": {"c": (np.arange(3), [4])}, "d": Box([7])}
    out = _copy_plain(src)
    assert out["a"] == src["a"] and type(out["a"][5]) is np.int64 and isinstance(out["b"]["c"], tuple)
    assert np.array_equal(out["b"]["c"][0], src["b"]["c"][0])
    out["a"].append(9)
    out["b"]["c"][0][0] = 99
    out["b"]["c"][1].append(5)
    out["d"].v.append(8)
    assert src["a"] == [1, 2.5, None, True, "s", 3] and src["b"]["c"][0][0] == 0
    assert src["b"]["c"][1] == [4] and src["d"].v == [7]
