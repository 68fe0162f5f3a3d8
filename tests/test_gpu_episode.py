"""GPU: episode statistics on the device and the vector
env's surface details (observation copies, input validation, action index
errors), through CarlaBEVVectorEnv.

The episode summary is checked against tests/stats_ref.py, a restatement of
`Stats` / `EpisodeStats` (stats.py:19-148) fed with each step's values read
back from the device (the per-step values themselves are parity-tested against
the oracle in test_gpu_parity.py). Bar: integers, causes and contexts exact;
float64 means within 1e-9 (the device sums in step order, NumPy pairwise).
"""
from __future__ import annotations

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from carlabev_env_amd import layout as LY
from carlabev_env_amd._lib import lib
from stats_ref import Stats

pytestmark = pytest.mark.gpu


def _env(n, info_mode="full", **kw):
    from carlabev_env_amd import EnvConfig, make_env
    cfg = EnvConfig(size=128, obs_size=(128, 128), render_mode="rgb_array", obs_mode="bev_semantic")
    return make_env({"env": cfg, "num_envs": n}, info_mode=info_mode, **kw)


def _opts(difficulty="rt_medium_v1"):
    from carlabev_env_amd import RandomNavigationReset, build_random_navigation_options
    return build_random_navigation_options(RandomNavigationReset(difficulty_id=difficulty))


def _step_values(env):
    """What EpisodeStats.step reads, per env, after a step (device values)."""
    recs = env.records_host()
    rew = env.reward.cpu().numpy()
    cause = env.cause.cpu().numpy()
    out = []
    for i in range(env.num_envs):
        v = LY.RecordView(recs[i], env.layout)
        out.append({"reward": float(rew[i]), "cause": LY.CAUSE_NAME.get(int(cause[i])), "v": v.h("V"),
                    "accel_long": v.h("C_AL"), "accel_lat": v.h("C_ALAT"), "jerk_long": v.h("C_JL"),
                    "jerk_lat": v.h("C_JLAT"), "yaw_rate": v.h("C_YR"), "yaw_acc": v.h("C_YACC"),
                    "num_vehicles": v.h("NUM_VEH"), "len_ego_route": v.h("LEN_ROUTE_M")})
    return out


def _check_summary(got: dict, i: int, want: dict, tag):
    ep = got["episode_info"]
    assert got["_episode_info"][i] and ep["_episode"][i], tag
    for k, w in want.items():
        g = ep[k][i]
        if isinstance(w, (list, tuple, np.ndarray)):
            assert np.allclose(np.asarray(g, np.float64), np.asarray(w, np.float64), rtol=1e-12), (tag, k, g, w)
        elif isinstance(w, str) or w is None or isinstance(w, (int, np.integer)):
            assert g == w, (tag, k, g, w)
        else:
            assert np.isclose(g, w, rtol=1e-9, atol=1e-9), (tag, k, g, w)
    assert ep["episode"].dtype == np.int64 and ep["length"].dtype == np.int64 and ep["num_vehicles"].dtype == np.int64
    assert got["episode"]["r"][i] == ep["return"][i] and got["episode"]["l"][i] == ep["length"][i]
    assert 0.0 <= got["episode"]["t"][i] < 600.0


def test_episode_info_matches_stats_restatement():
    """>= 3 episodes in every env (host resets on termination, as the canonical
    loop does): each termination's episode_info equals Stats.terminated() over the
    same steps, the window statistics included; the reset's scenario context is
    merged (carlabev.py:181-182)."""
    n = 10
    env = _env(n)
    obs, infos = env.reset(seed=11, options=_opts())
    ctx = {i: infos["scenario"][i] for i in range(n)}
    stats = [Stats() for _ in range(n)]
    scene = {}
    for i, s in enumerate(_step_values(env)):
        scene[i] = (int(s["num_vehicles"]), s["len_ego_route"])
    episodes = np.zeros(n, np.int64)
    rng = np.random.default_rng(5)
    for t in range(3000):
        a = rng.integers(0, 9, n)
        obs, r, term, trunc, infos = env.step(a)
        vals = _step_values(env)
        done = term.cpu().numpy()
        for i in range(n):
            stats[i].current.step(vals[i])
        if done.any():
            assert "episode_info" in infos
            for i in np.flatnonzero(done):
                want = stats[i].terminated()
                want["num_vehicles"], want["len_ego_route"] = scene[i]
                want.update(ctx[i])
                _check_summary(infos, i, want, (t, i))
                episodes[i] += 1
            assert not infos["_episode_info"][~done].any()
            _, rinfo = env.reset(seed=1000 + t, options=dict(_opts(), reset_mask=done))
            vals = _step_values(env)
            for i in np.flatnonzero(done):
                stats[i].reset()
                ctx[i] = rinfo["scenario"][i]
                scene[i] = (int(vals[i]["num_vehicles"]), vals[i]["len_ego_route"])
        else:
            assert len(infos) == 0 and "episode_info" not in infos
        if episodes.min() >= 3:
            break
    assert episodes.min() >= 3, episodes
    env.close()


def test_episode_info_after_bank_resets_and_held_infos():
    """Bank resets (device-only) carry the bank scene's num_vehicles, route length
    and scenario context into the next episode's summary; infos held across more
    steps than the device ring keeps are read before their rows are recycled."""
    n = 8
    env = _env(n)
    env.reset(seed=3, options=_opts("rt_hard_v1"))
    bank = env.build_bank([500 + k for k in range(5)], _opts("rt_easy_v1"))
    env.attach_bank(bank)
    bank_vals = [LY.RecordView(b, env.layout) for b in bank.cpu().numpy()]
    held = []
    rng = np.random.default_rng(0)
    after_bank = np.zeros(n, bool)
    bank_of = np.full(n, -1)
    checked = 0
    for t in range(2000):
        obs, r, term, trunc, infos = env.step(rng.integers(0, 9, n))
        held.append((t, infos, term.cpu().numpy(), after_bank.copy(), bank_of.copy()))
        done = term.cpu().numpy()
        if done.any():
            bidx = torch.from_numpy(((np.arange(n) + t) % 5).astype(np.int64))  # int64 CPU indices are accepted
            env.reset_from_bank(mask=term, bank_idx=bidx)
            after_bank |= done
            bank_of[done] = bidx.numpy()[done]
        if checked >= 6 and t > 40:
            break
        # read infos 12 steps late (more than the device ring's slots)
        if len(held) > 12:
            t0, inf, dn, ab, bo = held.pop(0)
            if dn.any():
                ep = inf["episode_info"]
                for i in np.flatnonzero(dn):
                    if ab[i]:
                        v = bank_vals[bo[i]]
                        assert ep["num_vehicles"][i] == int(v.h("NUM_VEH"))
                        assert ep["len_ego_route"][i] == v.h("LEN_ROUTE_M")
                        assert ep["difficulty_id"][i] == "rt_easy_v1"
                        checked += 1
    assert checked >= 6
    env.close()


def test_refresh_bank_releases_only_dead_contexts():
    """A fast bank refresh (every step, far more retired scenario contexts than
    the keep window) never releases the context of a scene an env still runs,
    and terminations report the context of the bank scene they were reset from
    (carlabev.py:182); the context table stays bounded."""
    n, B = 6, 4
    env = _env(n)
    env.reset(seed=7, options=_opts("rt_easy_v1"))
    env.attach_bank(env.build_bank([900 + k for k in range(B)], _opts("rt_easy_v1")))
    env.RETIRED_CTX_KEEP = 2  # release as soon as 2 N ids are retired
    host = env._new_record_buffer(B)
    rng = np.random.default_rng(1)
    slot, tag = 0, 0
    env_tag = {}  # env -> tag of the bank scene it was last reset from (None: untagged)
    bank_tag = [None] * B  # build_bank's scenes carry the builder's contexts, no tag
    seen = 0
    for t in range(400):
        obs, r, term, trunc, infos = env.step(rng.integers(0, 9, n))
        done = term.cpu().numpy().astype(bool)
        for i in np.flatnonzero(done):
            if env_tag.get(i) is not None:
                assert infos["episode_info"]["tag"][i] == env_tag[i], (t, i)
                seen += 1
        if done.any():  # env i's j-th masked reset takes bank row (i + j * stride) % B (cbev.h, ABI 7)
            counts = env.reset_counts()
            stride = lib().cbev_bank_stride(B)
            env.reset_terminated()
            for i in np.flatnonzero(done):
                env_tag[i] = bank_tag[(int(i) + int(counts[i]) * stride) % B]
        # refresh the whole bank with fresh tagged scenes every step
        ctxs = []
        for k in range(B):
            env.build_reset_record(host[k], 2000 + tag, _opts("rt_easy_v1"))
            ctxs.append({"tag": tag})
            tag += 1
        slot = env.refresh_bank(slot, host, ctxs)
        bank_tag = [c["tag"] for c in ctxs]
        live = set(env.record_ctx_ids().tolist())
        assert live <= set(env._ctx_table), (t, live - set(env._ctx_table))
        assert len(env._ctx_table) <= 4 * n + 2 * B + 16, len(env._ctx_table)
        if seen >= 4 and t > 50:
            break
    assert tag > 2 * n + env.RETIRED_CTX_KEEP and seen >= 1
    env.close()


def test_obs_copies_and_input_validation():
    env = _env(6, info_mode="none")
    env2 = _env(6, info_mode="none")
    obs0, _ = env.reset(seed=1, options=_opts())
    env2.reset(seed=1, options=_opts())
    o0 = obs0.clone()
    obs1, *_ = env.step(np.zeros(6, np.int64))
    env2.step(np.zeros(6, np.int64))
    assert torch.equal(obs0, o0), "a returned observation must survive the next step (copy_obs)"
    assert obs1.data_ptr() != obs0.data_ptr()
    # Python's negative index: -1 is the last discrete action, identical to 8
    _, r_a, *_ = env.step(np.full(6, -1))
    _, r_b, *_ = env2.step(np.full(6, 8))
    assert torch.equal(r_a, r_b) and torch.equal(env.records, env2.records)
    with pytest.raises(IndexError):
        env.step(np.full(6, 9))
    with pytest.raises(IndexError):
        env.step(np.full(6, -10))
    # device tensors are not synchronised per step: the index error is a flag
    assert env.errors() == 0
    env.step(torch.full((6,), 12, dtype=torch.int32, device=env.device))
    from carlabev_env_amd._lib import ERR_ACTION_INDEX
    assert env.errors() == ERR_ACTION_INDEX and env.errors() == 0
    # reset_from_bank validates its inputs
    env.attach_bank(env.build_bank([7, 8, 9], _opts()))
    with pytest.raises(ValueError):
        env.reset_from_bank(mask=torch.ones(5, dtype=torch.bool, device=env.device))
    with pytest.raises(ValueError):
        env.reset_from_bank(mask=None, bank_idx=torch.zeros(4, dtype=torch.int64))
    env.reset_from_bank(mask=None, bank_idx=torch.tensor([2, 1, 0, 2, 1, 0], dtype=torch.int64))  # CPU int64
    got = env.records_host()
    want = env.bank.cpu().numpy()
    for i, b in enumerate([2, 1, 0, 2, 1, 0]):
        assert np.array_equal(got[i], want[b])
    env.close()
    env2.close()
