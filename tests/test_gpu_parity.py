"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on the
same seeded scenes and action streams.

Bar: palette frames, termination/truncation flags, causes, collision results,
tile ids, target indices, visibility bits and behaviour states bit-exact;
float64 kinematic state and rewards within 1e-9 relative (device libm vs
glibc may differ by one ulp in sin/cos/atan2/hypot; expression order and
no-FMA compilation are identical on both sides).
"""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import oracle as O
from carlabev_env_amd import layout as LY
from carlabev_env_amd._lib import check, lib
from carlabev_env_amd.semantics import gray_lut, rgb_lut, semantic_lut, rgb_to_semantic_mask_ids, PALETTE
from carlabev_env_amd.config import RandomNavigationReset, build_random_navigation_options
from helpers import CAPS_FULL, action_stream, bench_caps, build_records, world

pytestmark = pytest.mark.gpu

P_ = ctypes.c_void_p


def ptr(t):
    return P_(t.data_ptr()) if t is not None else None


class DevWorld:
    def __init__(self, P, padded, caps):
        L = lib()
        LY.check_library_layout(L, caps)  # records are packed with the header's layout
        self.ctx = P_()
        check(L.cbev_create(ctypes.byref(P), ctypes.byref(caps.c()), 0, ctypes.byref(self.ctx)), "create")
        check(L.cbev_set_map(self.ctx, padded.ctypes.data_as(P_), padded.nbytes), "set_map")

    def __del__(self):
        lib().cbev_destroy(self.ctx)


def angles_close(a, b, tol=1e-9):
    """Headings equal modulo 2 pi. A retreat's rebuilt route is np.unwrap'ed: where a
    segment heading sits on the +-pi cut, ulp-level differences in the smoothed
    route (device Savitzky-Golay tables vs the oracle's long-double fit, device vs
    glibc sin/cos in the actor's position) can flip atan2's sign there and offset
    every later heading by exactly 2 pi, which angle_mod and cos/sin absorb."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    d = np.remainder(a - b + np.pi, 2 * np.pi) - np.pi
    return bool(np.all(np.abs(d) <= tol * (1 + np.abs(b))))


def compare_records(a: np.ndarray, b: np.ndarray, layout, tag=""):
    va, vb = LY.RecordView(a, layout), LY.RecordView(b, layout)
    ints = ("TIDX", "NROUTE", "NACT", "TILE", "COLLIDED", "ACTOR_ID", "CAUSE", "TERM", "TRUNC", "EP_LEN",
            "HAS_PREV_COMFORT", "S_PREV_VALID", "KSTEPS", "OFFROAD", "NACTSTATE")
    for k in ints:
        assert va.i(k) == vb.i(k), (tag, k, va.i(k), vb.i(k))
    assert np.array_equal(va.vis, vb.vis), (tag, "vis")
    assert np.array_equal(va.vis_draw, vb.vis_draw), (tag, "vis_draw")
    assert np.allclose(va.hd, vb.hd, rtol=1e-9, atol=1e-9, equal_nan=True), (
        tag, [(n, va.hd[i], vb.hd[i]) for n, i in LY.HD.items()
              if not np.isclose(va.hd[i], vb.hd[i], rtol=1e-9, atol=1e-9, equal_nan=True)])
    n = va.i("NACT")
    assert np.array_equal(va.ai[:, :n], vb.ai[:, :n]), (tag, "actor ints")
    yaw = LY.AD["YAW"]
    rows = [i for i in range(va.ad.shape[0]) if i != yaw]
    assert np.allclose(va.ad[rows, :n], vb.ad[rows, :n], rtol=1e-9, atol=1e-9), (tag, "actor doubles")
    assert angles_close(va.ad[yaw, :n], vb.ad[yaw, :n]), (tag, "actor yaw")
    for a in range(n):  # actor routes (rebuilt on a jaywalk retreat): smoothed up to NROUTE, raw up to NRX
        m, k = va.ai[LY.AI["NROUTE"], a], va.ai[LY.AI["NRX"], a]
        for arr in ("acx", "acy", "arx", "ary"):
            mk = k if arr in ("arx", "ary") else m
            assert np.allclose(getattr(va, arr)[a, :mk], getattr(vb, arr)[a, :mk], rtol=1e-9, atol=1e-9), (tag, arr, a)
        assert angles_close(va.acyaw[a, :m], vb.acyaw[a, :m]), (tag, "acyaw", a)
        # a: the device record; its float32 route copy (the target search's first
        # pass) follows every rebuild of the smoothed route
        assert np.array_equal(va.acf[a, :m, 0], va.acx[a, :m].astype(np.float32)), (tag, "acf x", a)
        assert np.array_equal(va.acf[a, :m, 1], va.acy[a, :m].astype(np.float32)), (tag, "acf y", a)
        # and its pruning circles (acb) hold every block's float32 points
        assert acb_holds(va.acb[a], va.acf[a, :m]), (tag, "acb", a)


def acb_holds(acb, pts) -> bool:
    """Every float32 route point lies inside its block's circle (cbev_layout.h acb)."""
    P = LY.ACB_PTS
    for b in range((len(pts) + P - 1) // P):
        w0, w1 = int(acb[b, 0]), int(acb[b, 1])
        c = np.array([(w0 & 0xFFFF) - 32768, (w0 >> 16) - 32768], np.float64) / 8.0
        q = pts[P * b: P * (b + 1)].astype(np.float64)
        if np.hypot(q[:, 0] - c[0], q[:, 1] - c[1]).max() > w1 / 8.0:
            return False
    return True


def info_of(v, cause):
    """The per-step export cbev_step writes to `info` (include/cbev.h), from an oracle record."""
    o = np.zeros(16, np.float32)
    o[0:7] = v.hd[LY.HD["C_SPEED"]:LY.HD["C_SPEED"] + 7]
    o[7:11] = v.hd[LY.HD["U_GAS"]:LY.HD["U_GAS"] + 4]
    o[11] = v.h("REWARD")
    o[12] = v.h("DIST2WP")
    o[13] = v.i("TILE")
    o[14] = v.i("COLLIDED")
    o[15] = v.i("NACTSTATE")
    return o


class EpisodeStatsOn:
    """The device episode statistics (cbev_set_episode_stats) on a context, as
    the bench's info_mode "full" runs the step: k_ego then updates the per-env
    Stats accumulators and writes a summary row per termination (the kernel
    variant the headline measures). `check(step, term, sample, views, causes)`
    compares this step's rows with the oracle's records of the sampled envs."""
    RING = 4

    def __init__(self, ctx, n):
        self.n = n
        self.stats = torch.zeros((n, LY.STATS_BYTES), dtype=torch.uint8, device="cuda")
        self.rows = torch.zeros((self.RING, n, len(LY.EP)), dtype=torch.float64, device="cuda")
        self.counts = torch.zeros(self.RING, dtype=torch.int32, device="cuda")
        check(lib().cbev_set_episode_stats(ctx, ptr(self.stats), n, ptr(self.rows), ptr(self.counts), self.RING),
              "episode_stats")
        self.episodes = np.zeros(n, np.int64)
        self.rows_seen = 0

    def check(self, step, term_all, sample, views, causes):
        slot = step % self.RING
        cnt = int(self.counts[slot].item())
        assert cnt == int(term_all.sum()), (step, cnt, int(term_all.sum()))
        rows = self.rows[slot, :cnt].cpu().numpy()
        by_env = {int(r[LY.EP["ENV"]]): r for r in rows}
        assert len(by_env) == cnt, (step, "one row per terminated env")
        for j, e in enumerate(sample):
            v = views[j]
            if not v.i("TERM"):
                assert e not in by_env, (step, e)
                continue
            r = by_env[int(e)]
            assert r[LY.EP["CAUSE"]] == causes[j] == v.i("CAUSE"), (step, e)
            assert r[LY.EP["EPISODE"]] == self.episodes[e], (step, e)
            assert r[LY.EP["LENGTH"]] == v.i("EP_LEN"), (step, e)
            assert np.isclose(r[LY.EP["RETURN"]], v.h("EP_RETURN"), rtol=1e-9, atol=1e-12), (step, e)
            ln = max(v.i("EP_LEN"), 1)
            assert np.isclose(r[LY.EP["MEAN_SPEED"]], v.h("EP_SPEED") / ln, rtol=1e-9, atol=1e-12), (step, e)
            self.rows_seen += 1
        for e in np.flatnonzero(term_all):
            self.episodes[e] += 1


def error_flags(ctx):
    f = ctypes.c_int32()
    check(lib().cbev_error_flags(ctx, ctypes.byref(f), 1), "error_flags")
    return f.value


def run_parity(kinds, n_envs, steps, size=128, profile="discrete9_v1", reward="carl_base_v1", seed0=0, anchor_y=0.5,
               act_seed=1234, edit=None, fov=False, caps=CAPS_FULL, options=None, acts=None, on_step=None,
               stats=False):
    """Every env of a small batch stepped on the device and by the oracle, compared
    whole after each step. acts: an explicit (steps, n[, 3]) action array instead of
    the seeded stream; on_step(t, views, causes): sees the oracle's records after
    each step (branch-coverage probes); stats: with the device episode statistics
    on (EpisodeStatsOn), the headline's k_ego variant."""
    cfg, P, padded, layout, builder = world(size, profile, reward, anchor_y, caps=caps)
    if options is None:
        recs, _ = build_records(builder, n_envs, kinds, seed0=seed0)
    else:  # explicit scene options (e.g. more vehicles than the difficulty presets)
        recs, _ = builder.build_many([seed0 + i for i in range(n_envs)],
                                     lambda k, s: dict(options[k % len(options)], scene_seed=s))
    if edit is not None:  # hand-made states on top of the seeded scenes
        edit(recs, layout, P)
    dw = DevWorld(P, padded, caps)
    L = lib()
    S = P.size
    omask = None
    if fov:  # device: the product's mask; oracle: its own restatement, blacked out after the render
        import wrappers as W
        from carlabev_env_amd.fov_mask import fov_corner_mask
        dmask = fov_corner_mask(S)
        check(L.cbev_set_fov_mask(dw.ctx, dmask.ctypes.data_as(P_)), "fov")
        omask = W.fov_mask(S)
    d_recs = torch.from_numpy(recs.copy()).cuda()
    d_frames = torch.zeros((n_envs, S, S), dtype=torch.uint8, device="cuda")
    check(L.cbev_reset(dw.ctx, ptr(d_recs), n_envs, None, 0, None, None, 0, ptr(d_frames), 1, None), "reset")
    orc = O.Oracle(P, padded, caps.c(), layout.record_bytes)
    h_frames = np.zeros((n_envs, S, S), np.uint8)
    for e in range(n_envs):
        orc.reset_obs(recs[e], h_frames[e])
        if omask is not None:
            h_frames[e][omask] = 8  # CBEV_PX_BLACK
    torch.cuda.synchronize()
    assert np.array_equal(d_frames.cpu().numpy(), h_frames), "reset frames differ"
    if acts is None:
        acts = action_stream(P, n_envs, steps, seed=act_seed)
    st = EpisodeStatsOn(dw.ctx, n_envs) if stats else None
    rew = torch.zeros(n_envs, dtype=torch.float64, device="cuda")
    term = torch.zeros(n_envs, dtype=torch.uint8, device="cuda")
    trunc = torch.zeros_like(term)
    cause = torch.zeros(n_envs, dtype=torch.int32, device="cuda")
    info = torch.zeros((n_envs, 16), dtype=torch.float32, device="cuda")
    n_term = 0
    for t in range(steps):
        a = torch.from_numpy(np.ascontiguousarray(acts[t])).cuda()
        check(L.cbev_step(dw.ctx, ptr(d_recs), n_envs, ptr(a), ptr(d_frames), ptr(rew), ptr(term), ptr(trunc),
                          ptr(cause), ptr(info), None), "step")
        h_cause = np.zeros(n_envs, np.int32)
        for e in range(n_envs):
            h_cause[e] = orc.step_one(recs[e], np.ascontiguousarray(acts[t, e]), h_frames[e])
            if omask is not None:
                h_frames[e][omask] = 8  # CBEV_PX_BLACK
        torch.cuda.synchronize()
        df = d_frames.cpu().numpy()
        bad = np.argwhere(df != h_frames)
        assert bad.size == 0, (t, bad[:8], df[tuple(bad[0])], h_frames[tuple(bad[0])])
        dr = d_recs.cpu().numpy()
        for e in range(n_envs):
            compare_records(dr[e], recs[e], layout, tag=(t, e))
        views = [LY.RecordView(recs[e], layout) for e in range(n_envs)]
        assert np.array_equal(term.cpu().numpy(), np.array([v.i("TERM") for v in views], np.uint8))
        assert np.array_equal(trunc.cpu().numpy(), np.array([v.i("TRUNC") for v in views], np.uint8))
        assert np.allclose(rew.cpu().numpy(), [v.h("REWARD") for v in views], rtol=1e-9, atol=1e-12)
        # this step's cause (not the record's sticky last non-None cause) and the per-step export
        assert np.array_equal(cause.cpu().numpy(), h_cause), (t, cause.cpu().numpy(), h_cause)
        want = np.stack([info_of(v, h_cause[e]) for e, v in enumerate(views)])
        got = info.cpu().numpy()
        assert np.array_equal(got[:, 13:], want[:, 13:]), (t, "info ints")
        assert np.allclose(got, want, rtol=1e-6, atol=1e-6), (t, "info")
        if st is not None:
            st.check(t, term.cpu().numpy(), np.arange(n_envs), views, h_cause)
        if on_step is not None:
            on_step(t, views, h_cause)
        n_term += int(term.sum())
    # no raster tile exceeded its LDS window bound (CBEV_ERR_RASTER_WINDOW), no bad action index
    assert error_flags(dw.ctx) == 0
    return n_term


def test_parity_ego_only_config2():
    assert run_parity(["rt_no_traffic_v1"], 48, 150, seed0=10_000) >= 0


def test_parity_random_traffic_config3():
    run_parity(["rt_hard_v1"], 32, 120, seed0=20_000, act_seed=7)


def test_parity_continuous_medium_config4():
    run_parity(["rt_medium_v1"], 24, 100, profile="continuous_gsb_v1", seed0=40_000, act_seed=99)


def test_parity_scenarios_size256_config5():
    run_parity(["mix3"], 24, 100, size=256, seed0=30_000)


def test_parity_jaywalk_retreats():
    """Jaywalk scenes whose yield_return pedestrians retreat within the run (the
    oracle shows the first retreat at step 22 for these seeds): the wave-wide
    route rebuild in k_actors against the oracle's serial one."""
    run_parity(["jaywalk"], 48, 80, seed0=30_000)


def test_parity_fov_masked():
    """EnvConfig.fov_masked: corner triangles blacked out (fov.py:46-68,96-99), step and reset frames."""
    run_parity(["rt_medium_v1"], 16, 40, seed0=77, fov=True)
    run_parity(["mix3"], 8, 20, size=256, seed0=30_100, fov=True)


def test_parity_shaping_reward_and_offcentre_anchor():
    run_parity(["rt_easy_v1", "jaywalk"], 16, 80, reward="shaping_base_v1", anchor_y=0.2, seed0=5)


def _edge_states(recs, layout, P):
    """One env per branch the seeded rollouts rarely reach."""
    V = [LY.RecordView(recs[e], layout) for e in range(recs.shape[0])]
    X, Y, YAW, VEL = (LY.HD[k] for k in ("X", "Y", "YAW", "V"))
    V[1].hd[X] += 40.0  # off the road: NON_DRIVABLE tile (collision) or sidewalk
    V[2].hd[X], V[2].hd[Y] = V[2].hd[LY.HD["GOAL_X"]], V[2].hd[LY.HD["GOAL_Y"]]  # on the goal: success
    V[3].hd[X] += 120.0  # far from the route: out of bounds or off-road
    V[4].hd[VEL] = 60.0  # over the CaRL speed limit, brake/clip paths
    if V[5].i("NACT") > 0:  # on an actor: vehicle / pedestrian collision
        V[5].hd[X], V[5].hd[Y] = V[5].ad[LY.AD["X"], 0], V[5].ad[LY.AD["Y"], 0]
    V[6].hd[YAW], V[6].hd[VEL] = -np.pi / 2, 0.0  # exact multiple of 90 degrees: rotate90 in the step raster
    V[7].hd[YAW] = np.pi  # yaw at the angle_mod wrap
    V[8].hd[VEL] = -3.0  # reversing
    V[9].hd[X] = 3.0  # at the map's left edge: crop clamped against the padding


def test_parity_edge_states_carl():
    run_parity(["rt_medium_v1"], 10, 6, seed0=777, edit=_edge_states)


def test_parity_edge_states_shaping_and_truncation():
    def edit(recs, layout, P):
        _edge_states(recs, layout, P)
        LY.RecordView(recs[0], layout).hi[LY.HI["KSTEPS"]] = P.max_actions - 2  # truncation on step 2
    run_parity(["rt_easy_v1"], 10, 4, reward="shaping_base_v1", seed0=4242, edit=edit)


@pytest.mark.parametrize("ne", ["2", "8", "64"])
def test_parity_ego_workgroup_shapes(ne, monkeypatch):
    """k_ego with 4 (CBEV_EGO_NE=2 is raised to the floor of 4 envs, whose 64
    threads per env stay inside one wave for the shuffle reductions), 8 and the
    most envs per workgroup the LDS admits (read at cbev_create); odd env counts
    leave a partial last workgroup."""
    monkeypatch.setenv("CBEV_EGO_NE", ne)
    run_parity(["rt_no_traffic_v1"], 47, 30, seed0=10_000)
    run_parity(["rt_hard_v1"], 31, 30, seed0=20_000, act_seed=7)
    run_parity(["mix3"], 13, 30, size=256, seed0=30_000)
    run_parity(["rt_easy_v1", "jaywalk"], 9, 30, reward="shaping_base_v1", anchor_y=0.2, seed0=5)


def test_bank_reset_and_wrapper_expansion():
    cfg, P, padded, layout, builder = world()
    n, B, F = 40, 7, 4
    recs, _ = build_records(builder, n, ["rt_medium_v1"], seed0=300)
    bank, _ = build_records(builder, B, ["rt_hard_v1", "jaywalk"], seed0=900)
    dw = DevWorld(P, padded, CAPS_FULL)
    L = lib()
    S = P.size
    d_recs = torch.from_numpy(recs.copy()).cuda()
    d_bank = torch.from_numpy(bank.copy()).cuda()
    ring = torch.zeros((F, n, S, S), dtype=torch.uint8, device="cuda")
    mask = (torch.arange(n) % 3 == 0).to(torch.uint8).cuda()
    bidx = (torch.arange(n) % B).to(torch.int32).cuda()
    check(L.cbev_reset(dw.ctx, ptr(d_recs), n, ptr(d_bank), B, ptr(mask), ptr(bidx), 0, ptr(ring), F, None), "reset")
    torch.cuda.synchronize()
    dr = d_recs.cpu().numpy()
    orc = O.Oracle(P, padded, CAPS_FULL.c(), layout.record_bytes)
    m = mask.cpu().numpy().astype(bool)
    for e in range(n):
        if m[e]:
            assert np.array_equal(dr[e], bank[e % B])
            f = np.zeros((S, S), np.uint8)
            orc.reset_obs(bank[e % B].copy(), f)
            for s in range(F):
                assert np.array_equal(ring[s, e].cpu().numpy(), f)
        else:
            assert np.array_equal(dr[e], recs[e])
    # rotating-offset bank assignment (bank_idx NULL): b = (e + offset) % B
    d2 = torch.from_numpy(recs.copy()).cuda()
    ring2 = torch.zeros((1, n, S, S), dtype=torch.uint8, device="cuda")
    check(L.cbev_reset(dw.ctx, ptr(d2), n, ptr(d_bank), B, None, None, 5, ptr(ring2), 1, None), "reset2")
    torch.cuda.synchronize()
    d2h = d2.cpu().numpy()
    for e in range(n):
        assert np.array_equal(d2h[e], bank[(e + 5) % B])
    # expansion kinds against host restatements
    ring_h = torch.randint(0, 10, (F, n, S, S), dtype=torch.uint8)
    ring_d = ring_h.cuda()
    head = 1
    order = [(head + 1 + f) % F for f in range(F)]
    for mode in ("6-class", "7-class", "binary", "5-class"):
        lut = semantic_lut(mode)
        C = int(max(1, max(int(x).bit_length() for x in lut)))
        C = {"6-class": 6, "7-class": 7, "binary": 1, "5-class": 5}[mode]
        out = torch.zeros((n, F * C, S, S), dtype=torch.float32, device="cuda")
        check(L.cbev_expand_obs(dw.ctx, ptr(ring_d), n, F, head, 0, C, lut.ctypes.data_as(P_), ptr(out), None), "exp")
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        for e in (0, 5, n - 1):
            ref = np.concatenate([rgb_to_semantic_mask_ids(ring_h[s, e].numpy(), mode) for s in order])
            assert np.array_equal(o[e], ref), mode
    g = torch.zeros((n, F, S, S), dtype=torch.uint8, device="cuda")
    check(L.cbev_expand_obs(dw.ctx, ptr(ring_d), n, F, head, 1, 1, gray_lut().ctypes.data_as(P_), ptr(g), None), "g")
    rgb = torch.zeros((n, S, S, 3), dtype=torch.uint8, device="cuda")
    check(L.cbev_expand_obs(dw.ctx, ptr(ring_d), n, F, head, 2, 3, rgb_lut().ctypes.data_as(P_), ptr(rgb), None), "r")
    torch.cuda.synchronize()
    gl = gray_lut()
    assert np.array_equal(g.cpu().numpy(), gl[ring_h.numpy()[order].transpose(1, 0, 2, 3)].astype(np.uint8))
    assert np.array_equal(rgb.cpu().numpy(), PALETTE[ring_h[head].numpy()])


def test_reset_from_cached_bank_frames_matches_render():
    cfg, P, padded, layout, builder = world()
    n, B, F = 48, 9, 4
    recs, _ = build_records(builder, n, ["rt_medium_v1"], seed0=1300)
    bank, _ = build_records(builder, B, ["rt_hard_v1", "jaywalk", "lead_brake"], seed0=1900)
    dw = DevWorld(P, padded, CAPS_FULL)
    L = lib()
    S = P.size
    d_bank = torch.from_numpy(bank.copy()).cuda()
    mask = (torch.arange(n) % 4 != 1).to(torch.uint8).cuda()
    bidx = ((torch.arange(n) * 7) % B).to(torch.int32).cuda()
    outs = []
    for cached in (False, True):
        d_recs = torch.from_numpy(recs.copy()).cuda()
        ring = torch.full((F, n, S, S), 13, dtype=torch.uint8, device="cuda")
        for idx, off in ((bidx, 0), (None, 5)):
            if cached:
                bf = torch.zeros((B, S, S), dtype=torch.uint8, device="cuda")
                check(L.cbev_bank_frames(dw.ctx, ptr(d_bank), B, ptr(bf), None), "bank_frames")
                check(L.cbev_reset_frames(dw.ctx, ptr(d_recs), n, ptr(d_bank), B, ptr(mask), ptr(idx), off, ptr(bf),
                                          ptr(ring), F, None), "reset_frames")
            else:
                check(L.cbev_reset(dw.ctx, ptr(d_recs), n, ptr(d_bank), B, ptr(mask), ptr(idx), off, ptr(ring), F,
                                   None), "reset")
        torch.cuda.synchronize()
        outs.append((d_recs.cpu().numpy(), ring.cpu().numpy()))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1], outs[1][1])


def test_vector_env_surface_and_partial_reset():
    from carlabev_env_amd import EnvConfig, make_env, build_random_navigation_options, RandomNavigationReset
    cfg = EnvConfig(size=128, obs_size=(128, 128), render_mode="rgb_array", obs_mode="bev_semantic")
    env = make_env({"env": cfg, "num_envs": 8})
    assert env.single_observation_space.shape == (24, 128, 128)
    assert env.single_action_space.n == 9
    obs, infos = env.reset(seed=3, options=build_random_navigation_options(
        RandomNavigationReset(difficulty_id="rt_medium_v1")))
    assert tuple(obs.shape) == (8, 24, 128, 128) and obs.dtype == torch.float32
    assert all(i["valid"] for i in infos["spawn_validation"])
    # the reset stack repeats the reset frame (FrameStackObservation padding "reset")
    o = obs.cpu().numpy()
    assert np.array_equal(o[:, 0:6], o[:, 18:24])
    saw_term = False
    for t in range(200):
        a = np.random.default_rng(t).integers(0, 9, 8)
        obs, r, term, trunc, infos = env.step(a)
        assert r.dtype == torch.float64 and term.dtype == torch.bool
        if term.any():
            saw_term = True
            assert "episode_info" in infos and infos["_episode_info"].any()
            obs, _ = env.reset(options={"reset_mask": term.cpu().numpy(), "scene_seed": 1000 + t})
    rgb = env.render()
    assert len(rgb) == 8 and rgb[0].shape == (128, 128, 3)
    assert saw_term
    env.close()


def test_profile_raster_rerenders_the_step():
    """cbev_profile_raster (bench.py's burst-timed roofline) re-renders the frames
    the preceding split step wrote, for traffic scenes at both sizes."""
    for size, kinds in ((128, ["rt_hard_v1"]), (256, ["mix3"])):
        cfg, P, padded, layout, builder = world(size, "discrete9_v1", "carl_base_v1", 0.5)
        n = 48
        recs, _ = build_records(builder, n, kinds, seed0=7)
        dw = DevWorld(P, padded, CAPS_FULL)
        L = lib()
        S = P.size
        d_recs = torch.from_numpy(recs.copy()).cuda()
        d_frames = torch.zeros((n, S, S), dtype=torch.uint8, device="cuda")
        check(L.cbev_reset(dw.ctx, ptr(d_recs), n, None, 0, None, None, 0, ptr(d_frames), 1, None), "reset")
        acts = action_stream(P, n, 3, seed=5)
        rew = torch.zeros(n, dtype=torch.float64, device="cuda")
        term = torch.zeros(n, dtype=torch.uint8, device="cuda")
        trunc = torch.zeros_like(term)
        cause = torch.zeros(n, dtype=torch.int32, device="cuda")
        for t in range(3):
            a = torch.from_numpy(np.ascontiguousarray(acts[t])).cuda()
            check(L.cbev_step(dw.ctx, ptr(d_recs), n, ptr(a), ptr(d_frames), ptr(rew), ptr(term), ptr(trunc),
                              ptr(cause), None, None), "step")
        torch.cuda.synchronize()
        want = d_frames.cpu().numpy()
        again = torch.full_like(d_frames, 0xAA)
        ms = ctypes.c_double()
        check(L.cbev_profile_raster(dw.ctx, ptr(d_recs), n, ptr(again), 3, None, ctypes.byref(ms)), "profile_raster")
        assert ms.value > 0
        got = again.cpu().numpy()
        # the step saved the target bits its render drew (vis_draw) before its
        # collision pass consumed targets: the re-render is the same frame
        assert np.array_equal(got, want), size


CAPS_WIDE = LY.Caps(128, 96, 288, 4)


def test_parity_wide_actor_kernel():
    """k_actors<true>: more than 64 actor slots select the wide kernel. More than 64
    vehicles take the per-lane d_actor_step path (stanley_controller.py:100-123); jaywalk
    scenes in the wide kernel rebuild a retreating pedestrian's route with the whole wave,
    as the narrow kernel does (behavior/jaywalk.py:43-54), with a 288-point route capacity."""
    many = dict(build_random_navigation_options(RandomNavigationReset(difficulty_id="rt_hard_v1")), num_vehicles=72)
    run_parity(None, 6, 40, seed0=50_000, caps=CAPS_WIDE, options=[many])
    run_parity(["jaywalk"], 24, 80, seed0=30_000, caps=CAPS_WIDE)


def _long_route_edit(recs, layout, P):
    """Actor slots 0-3 of every record on 600-point out-and-back routes (300
    points east along the start's row, then back beside it, half a point
    shifted): 38 blocks of 16 points, more than the circles a group holds (18
    blocks at 2 lanes per actor, 20 at 4: cbev.hip actor_cq) and than the 32
    candidate bits. Slots 0-1 return 0.25 px
    beside the outbound leg, so the first minimum is soon on the return leg's
    last blocks (the reference's whole-route scan); slots 2-3 return 3 px away
    and drive the outbound leg."""
    from carlabev_env_amd.scene_pack import ActorSpec, init_actor_slot
    for e in range(len(recs)):
        v = LY.RecordView(recs[e], layout)
        rng = np.random.default_rng(7000 + e)
        for a in range(min(int(v.hi[LY.HI["NACT"]]), 4)):
            x0, y0 = float(v.ad[LY.AD["X"], a]), float(v.ad[LY.AD["Y"], a])
            n = 300
            rx = [x0 + i for i in range(n)] + [x0 + n - 0.5 - i for i in range(n)]
            ry = [y0] * n + [y0 + (0.25 if a < 2 else 3.0)] * n
            init_actor_slot(v, a, ActorSpec("vehicle", rx, ry, 8.0), rng)


def test_parity_long_actor_routes():
    """k_actors' windowed search on routes with more blocks than its circles
    (actor route capacity 640, 25 vehicles: k_actors_g4, 4 lanes per actor in two
    passes of the group loop): every block outside the window is scanned in the
    second round, blocks past the 32nd included (stanley_controller.py:100-123
    scans the whole route)."""
    caps = LY.Caps(128, 25, 640, 4)
    run_parity(["rt_hard_v1"], 8, 40, seed0=61_000, caps=caps, edit=_long_route_edit)


def test_parity_actor_kernel_up_to_64_slots():
    """k_actors<false, 1> (33-64 actor slots; up to 32 launch k_actors_g4): 2
    lanes per actor for 17-32 vehicles, one lane per actor (the whole-route
    search, actor_search<1>) beyond, and the long routes at 2 lanes per actor."""
    caps = LY.Caps(128, 48, 288, 4)
    many = dict(build_random_navigation_options(RandomNavigationReset(difficulty_id="rt_hard_v1")), num_vehicles=40)
    run_parity(None, 6, 40, seed0=52_000, caps=caps, options=[many])
    run_parity(["rt_hard_v1"], 12, 40, seed0=53_000, caps=caps)
    run_parity(["rt_hard_v1"], 8, 30, seed0=61_000, caps=LY.Caps(128, 48, 640, 4), edit=_long_route_edit)


def _sample_envs(n, k=160):
    """>= k env ids spread over the batch: a stride over all of it plus the
    workgroup / env-block / XCD-round boundaries (16-env staged workgroups, 64-env
    blocks, 512-env XCD rounds) and the last env."""
    ids = set(np.linspace(0, n - 1, k).astype(int).tolist())
    for b in (16, 64, 512):
        for j in range(0, n, max(b, n // 16)):
            ids.update(x for x in (j - 1, j, j + 1) if 0 <= x < n)
    ids.add(n - 1)
    return np.array(sorted(ids))


def run_full_size(kinds, n_envs, size=128, profile="discrete9_v1", seed0=0, steps=16, distinct=160, act_seed=1,
                  caps=CAPS_FULL, stats=False, push=0):
    """The HIP path at a benchmarked batch size (grid shapes, XCD placement and
    staging batches of the bench) against the oracle on a sampled subset of envs.
    `distinct` seeded scenes are tiled over the batch (env e gets scene e % distinct);
    every env gets its own action stream, so tiled copies diverge. `caps` are the
    record capacities: bench.CONFIGS' for the bench configurations, so the kernel
    shapes the bench line measures (k_actors skipped at actor_cap 0, the k_ego
    workgroup size, the record layout) are the ones checked here. stats: the device
    episode statistics on (the bench's info_mode "full", EpisodeStatsOn); push:
    envs per step moved off the road before the step (terminations in every step)."""
    cfg, P, padded, layout, builder = world(size, profile, "carl_base_v1", 0.5, caps=caps)
    base, _ = build_records(builder, distinct, kinds, seed0=seed0)
    recs = base[np.arange(n_envs) % distinct].copy()
    dw = DevWorld(P, padded, caps)
    L = lib()
    S = P.size
    rng = np.random.default_rng(act_seed)
    if P.action_kind == 0:
        p = np.ones(P.n_discrete)
        p[1] += 4.0
        acts = rng.choice(P.n_discrete, size=(steps, n_envs), p=p / p.sum()).astype(np.int32)
    else:
        acts = rng.uniform([0, -1, 0], [1, 1, 1], size=(steps, n_envs, 3)).astype(np.float32)
    sample = _sample_envs(n_envs)
    d_recs = torch.from_numpy(recs).cuda()
    d_frames = torch.zeros((n_envs, S, S), dtype=torch.uint8, device="cuda")
    check(L.cbev_reset(dw.ctx, ptr(d_recs), n_envs, None, 0, None, None, 0, ptr(d_frames), 1, None), "reset")
    orc = O.Oracle(P, padded, caps.c(), layout.record_bytes)
    h_recs = recs[sample].copy()
    h_frames = np.zeros((len(sample), S, S), np.uint8)
    rew = torch.zeros(n_envs, dtype=torch.float64, device="cuda")
    term = torch.zeros(n_envs, dtype=torch.uint8, device="cuda")
    trunc = torch.zeros_like(term)
    cause = torch.zeros(n_envs, dtype=torch.int32, device="cuda")
    info = torch.zeros((n_envs, 16), dtype=torch.float32, device="cuda")
    st = EpisodeStatsOn(dw.ctx, n_envs) if stats else None
    prng = np.random.default_rng(act_seed + 1)
    pos = {int(e): j for j, e in enumerate(sample)}
    for t in range(steps):
        if push:  # the same edit on the device records and the oracle's copies
            ids = np.unique(np.concatenate([prng.choice(n_envs, size=push, replace=False), sample[t::7][:4]]))
            sel_p = torch.from_numpy(ids).cuda()
            h = d_recs[sel_p].cpu().numpy()
            for k, e in enumerate(ids):
                LY.RecordView(h[k], layout).hd[LY.HD["X"]] += 60.0
                if int(e) in pos:
                    LY.RecordView(h_recs[pos[int(e)]], layout).hd[LY.HD["X"]] += 60.0
            d_recs[sel_p] = torch.from_numpy(h).cuda()
        a = torch.from_numpy(np.ascontiguousarray(acts[t])).cuda()
        check(L.cbev_step(dw.ctx, ptr(d_recs), n_envs, ptr(a), ptr(d_frames), ptr(rew), ptr(term), ptr(trunc),
                          ptr(cause), ptr(info), None), "step")
        h_cause = np.array([orc.step_one(h_recs[j], np.ascontiguousarray(acts[t, e]), h_frames[j])
                            for j, e in enumerate(sample)], np.int32)
        torch.cuda.synchronize()
        sel = torch.from_numpy(sample).cuda()
        df = d_frames[sel].cpu().numpy()
        bad = np.argwhere(df != h_frames)
        assert bad.size == 0, (t, sample[bad[0][0]], bad[:4])
        dr = d_recs[sel].cpu().numpy()
        for j, e in enumerate(sample):
            compare_records(dr[j], h_recs[j], layout, tag=(t, int(e)))
        views = [LY.RecordView(h_recs[j], layout) for j in range(len(sample))]
        assert np.array_equal(term[sel].cpu().numpy(), [v.i("TERM") for v in views])
        assert np.array_equal(trunc[sel].cpu().numpy(), [v.i("TRUNC") for v in views])
        assert np.array_equal(cause[sel].cpu().numpy(), h_cause)
        assert np.allclose(rew[sel].cpu().numpy(), [v.h("REWARD") for v in views], rtol=1e-9, atol=1e-12)
        got, want = info[sel].cpu().numpy(), np.stack([info_of(v, 0) for v in views])
        assert np.array_equal(got[:, 13:], want[:, 13:]) and np.allclose(got, want, rtol=1e-6, atol=1e-6), t
        if st is not None:
            st.check(t, term.cpu().numpy(), sample, views, h_cause)
    assert error_flags(dw.ctx) == 0
    if st is not None:
        assert st.rows_seen > 0
    return len(sample)


def test_full_size_config2():
    """Config 2 at its bench capacities (actor_cap 0: k_actors is not launched,
    k_ego runs with empty actor groups and its 16-env workgroups)."""
    assert run_full_size(["rt_no_traffic_v1"], 4096, seed0=10_000, caps=bench_caps(2)) >= 128


def test_full_size_config2_stats_on():
    """The headline's kernel variant: config 2 at its bench batch and capacities with
    the device episode statistics on (info_mode "full": k_ego's d_episode_summary
    path), oracle-checked per step; envs pushed off the road terminate every step,
    and each sampled termination's summary row matches the oracle's record."""
    assert run_full_size(["rt_no_traffic_v1"], 4096, seed0=10_000, steps=12, caps=bench_caps(2), stats=True,
                         push=300) >= 128


def run_full_size_folded(n_envs, steps, caps, seed0, bank_seed0, act_seed=1, distinct=96, bank_distinct=48,
                         n_bank=1021, F=2, kinds=("rt_no_traffic_v1",)):
    """The headline's exact kernel variant against the oracle: bench config 2's
    step with the device episode statistics on AND the canonical reset folded into
    the next step (cbev_set_deferred_reset: bench.py's loop of step() +
    reset_terminated(), carlabev.py:96-148,177-185 and deeprl/stats.py:30-148).
    Every step the terminated envs are reset from a bank (cbev_reset_terminated,
    then folded into the next k_ego); every third bank row starts off the road, so
    an env reset from it terminates in the very step that takes the reset (reset
    and terminated in consecutive steps). Every third step the caller edits the
    records (pushes envs off the road), which flushes the pending reset first
    (k_reset_mask): both reset paths, interleaved. The oracle copies each reset
    env's bank row (reset_rows: the same per-env rule) and its reset frame into
    every ring slot; frames (all ring slots), records, reward / term / trunc /
    cause / info and each terminated env's summary row are compared per step on
    a sampled subset, and the per-env reset counts at the end."""
    cfg, P, padded, layout, builder = world(128, "discrete9_v1", "carl_base_v1", 0.5, caps=caps)
    base, _ = build_records(builder, distinct, list(kinds), seed0=seed0)
    recs = base[np.arange(n_envs) % distinct].copy()
    bdist, _ = build_records(builder, bank_distinct, list(kinds), seed0=bank_seed0)
    bank = bdist[np.arange(n_bank) % bank_distinct].copy()
    for b in range(0, n_bank, 3):
        LY.RecordView(bank[b], layout).hd[LY.HD["X"]] += 60.0
    dw = DevWorld(P, padded, caps)
    L = lib()
    S = P.size
    check(L.cbev_set_deferred_reset(dw.ctx, 1), "deferred")
    d_bank = torch.from_numpy(bank).cuda()
    bf = torch.zeros((n_bank, S, S), dtype=torch.uint8, device="cuda")
    check(L.cbev_bank_frames(dw.ctx, ptr(d_bank), n_bank, ptr(bf), None), "bank_frames")
    d_recs = torch.from_numpy(recs).cuda()
    ring = torch.zeros((F, n_envs, S, S), dtype=torch.uint8, device="cuda")
    check(L.cbev_reset(dw.ctx, ptr(d_recs), n_envs, None, 0, None, None, 0, ptr(ring), F, None), "reset")
    orc = O.Oracle(P, padded, caps.c(), layout.record_bytes)
    sample = _sample_envs(n_envs)
    pos = {int(e): j for j, e in enumerate(sample)}
    h_recs = recs[sample].copy()
    h_ring = np.zeros((F, len(sample), S, S), np.uint8)
    for j in range(len(sample)):
        orc.reset_obs(h_recs[j], h_ring[0, j])
        h_ring[1:, j] = h_ring[0, j]
    bank_frame = {}

    def frame_of(b):
        if b not in bank_frame:
            f = np.zeros((S, S), np.uint8)
            orc.reset_obs(bank[b].copy(), f)
            bank_frame[b] = f
        return bank_frame[b]

    rng = np.random.default_rng(act_seed)
    p = np.ones(P.n_discrete)
    p[1] += 4.0
    acts = rng.choice(P.n_discrete, size=(steps, n_envs), p=p / p.sum()).astype(np.int32)
    prng = np.random.default_rng(act_seed + 1)
    rew = torch.zeros(n_envs, dtype=torch.float64, device="cuda")
    term = torch.zeros(n_envs, dtype=torch.uint8, device="cuda")
    trunc = torch.zeros_like(term)
    cause = torch.zeros(n_envs, dtype=torch.int32, device="cuda")
    info = torch.zeros((n_envs, 16), dtype=torch.float32, device="cuda")
    st = EpisodeStatsOn(dw.ctx, n_envs)
    seq = np.zeros(n_envs, np.int64)
    pending = None
    folded = flushed = reset_then_term = resets_seen = 0
    was_reset = np.zeros(len(sample), bool)
    for t in range(steps):
        slot = t % F
        edit = t % 3 == 2
        if pending is not None:
            if edit:  # the caller writes the records: it flushes the pending reset first (cbev.h)
                check(L.cbev_flush(dw.ctx), "flush")
                flushed += 1
            else:
                folded += L.cbev_reset_pending(dw.ctx)
            ids, rows = reset_rows(pending, seq, n_bank)  # the oracle side of either path
            was_reset[:] = False
            for e, b in zip(ids.tolist(), rows.tolist()):
                if e in pos:
                    j = pos[e]
                    h_recs[j] = bank[b]
                    h_ring[:, j] = frame_of(b)
                    was_reset[j] = True
                    resets_seen += 1
            pending = None
        if edit:
            ids = np.unique(np.concatenate([prng.choice(n_envs, size=min(300, n_envs // 6), replace=False),
                                            sample[t::7][:4]]))
            sel_p = torch.from_numpy(ids).cuda()
            h = d_recs[sel_p].cpu().numpy()
            for k, e in enumerate(ids):
                LY.RecordView(h[k], layout).hd[LY.HD["X"]] += 60.0
                if int(e) in pos:
                    LY.RecordView(h_recs[pos[int(e)]], layout).hd[LY.HD["X"]] += 60.0
            d_recs[sel_p] = torch.from_numpy(h).cuda()
        a = torch.from_numpy(np.ascontiguousarray(acts[t])).cuda()
        check(L.cbev_step(dw.ctx, ptr(d_recs), n_envs, ptr(a), ptr(ring[slot]), ptr(rew), ptr(term), ptr(trunc),
                          ptr(cause), ptr(info), None), "step")
        h_cause = np.array([orc.step_one(h_recs[j], np.ascontiguousarray(acts[t, e]), h_ring[slot, j])
                            for j, e in enumerate(sample)], np.int32)
        torch.cuda.synchronize()
        assert L.cbev_reset_pending(dw.ctx) == 0
        sel = torch.from_numpy(sample).cuda()
        dg = ring[:, sel].cpu().numpy()
        bad = np.argwhere(dg != h_ring)
        assert bad.size == 0, (t, "ring", bad[:4])
        dr = d_recs[sel].cpu().numpy()
        for j, e in enumerate(sample):
            compare_records(dr[j], h_recs[j], layout, tag=(t, int(e)))
        views = [LY.RecordView(h_recs[j], layout) for j in range(len(sample))]
        tn = term.cpu().numpy()
        seq += tn.astype(bool)  # the step counts its terminations (the next resets' bank rows)
        assert np.array_equal(tn[sample], [v.i("TERM") for v in views]), t
        assert np.array_equal(trunc[sel].cpu().numpy(), [v.i("TRUNC") for v in views]), t
        assert np.array_equal(cause[sel].cpu().numpy(), h_cause), t
        assert np.allclose(rew[sel].cpu().numpy(), [v.h("REWARD") for v in views], rtol=1e-9, atol=1e-12), t
        got, want = info[sel].cpu().numpy(), np.stack([info_of(v, 0) for v in views])
        assert np.array_equal(got[:, 13:], want[:, 13:]) and np.allclose(got, want, rtol=1e-6, atol=1e-6), t
        st.check(t, tn, sample, views, h_cause)
        reset_then_term += int(np.sum(was_reset & (tn[sample] != 0)))
        pending = tn.astype(bool)
        check(L.cbev_reset_terminated(dw.ctx, ptr(d_recs), n_envs, ptr(d_bank), n_bank, ptr(bf), ptr(ring), F, None),
              "reset_terminated")
    check(L.cbev_flush(dw.ctx), "flush")
    assert np.array_equal(_counts(L, dw, n_envs), seq)
    assert error_flags(dw.ctx) == 0
    if caps.actor_cap == 0:  # the fold (k_ego) needs a context without actor slots
        assert folded >= steps // 2 and flushed >= 2, (folded, flushed)
    assert st.rows_seen > 0 and resets_seen > 0 and reset_then_term > 0, (st.rows_seen, resets_seen, reset_then_term)


def test_full_size_config2_stats_folded_reset():
    """The bench's headline variant (statistics on + the folded reset) at config
    2's batch and capacities, against the oracle (run_full_size_folded)."""
    run_full_size_folded(4096, 15, bench_caps(2), 10_000, 14_000)


def test_full_size_config3_masked_reset():
    """Config 3 (rt_hard traffic, 25 actor slots of 288-point routes) at its bench
    batch with the statistics on and the canonical reset every step (k_reset_mask:
    actor contexts take no fold), against the oracle."""
    run_full_size_folded(4096, 12, bench_caps(3), 20_000, 24_000, act_seed=7, distinct=64, bank_distinct=32,
                         n_bank=509, kinds=("rt_hard_v1", "rt_medium_v1"))


def test_stats_folded_reset_small():
    """The same at an odd batch (partial k_ego workgroups) and a 3-slot ring."""
    run_full_size_folded(45, 24, bench_caps(2), 10_200, 14_200, distinct=45, bank_distinct=17, n_bank=53, F=3)


def test_parity_stats_on_small():
    """Every env, every step, with the episode statistics on (odd batch: partial
    k_ego workgroups), at config 2's and config 5's capacities."""
    run_parity(["rt_no_traffic_v1"], 37, 120, seed0=10_000, caps=bench_caps(2), stats=True)
    run_parity(["mix3"], 19, 60, size=256, seed0=30_000, caps=bench_caps(5), stats=True)


def test_parity_carl_safety_v1_branches():
    """carl_safety_v1 (config/reward_profiles.py:25-37) on rt_hard traffic: the
    lane-centre term with exponent 1.5 (the general pow, carl_reward_fn.py:248),
    the 0.05 off-lane factor on sidewalk / far-off-lane steps (P > 0 there,
    carl_reward_fn.py:254) and the TTC threshold of 5 s (carl_reward_fn.py:273);
    each branch is hit in some step (counted on the oracle's records, which the
    device records equal)."""
    hits = {"pow": 0, "off_lane": 0, "off_lane_pos": 0, "ttc": 0}

    def probe(t, views, causes):
        for v in views:
            if 0.15 < v.h("P_LANE") < 1.0:
                hits["pow"] += 1
            if v.h("P_OFF") == 0.05:
                hits["off_lane"] += 1
                hits["off_lane_pos"] += v.h("REWARD") > 0
            if v.h("P_TTC") == 0.5:
                hits["ttc"] += 1

    run_parity(["rt_hard_v1"], 29, 100, reward="carl_safety_v1", seed0=20_000, act_seed=7, caps=bench_caps(3),
               on_step=probe)
    assert all(v > 0 for v in hits.values()), hits


def test_parity_discrete13_every_index():
    """discrete13_v1 (config/action_profiles.py:51): the 13-entry table, every index
    0..12 and every negative index -13..-1 (Python's discrete_actions[int(a)]
    counts from the end, envs/spaces.py:43-47), on rt_medium traffic."""
    n, steps = 26, 120
    rng = np.random.default_rng(13)
    acts = rng.integers(-13, 13, size=(steps, n)).astype(np.int32)
    acts[0] = np.arange(-13, 13)
    acts[1] = np.arange(-13, 13)[::-1]
    assert set(np.unique(acts).tolist()) == set(range(-13, 13))
    run_parity(["rt_medium_v1"], n, steps, profile="discrete13_v1", seed0=600, caps=bench_caps(4), acts=acts)


def test_full_size_config3():
    run_full_size(["rt_hard_v1"], 4096, seed0=20_000, act_seed=7, caps=bench_caps(3))


def test_full_size_config4_shard():
    run_full_size(["rt_medium_v1"], 8192, profile="continuous_gsb_v1", seed0=40_000, act_seed=99, caps=bench_caps(4))


def test_full_size_config5():
    run_full_size(["mix3"], 2048, size=256, seed0=30_000, steps=12, caps=bench_caps(5))


def test_full_size_caps_full():
    """The test capacities (CAPS_FULL: 32 actor slots, 8-env k_ego workgroups) at a
    bench batch size, so both workgroup shapes run full-size."""
    run_full_size(["rt_medium_v1"], 4096, seed0=40_000, act_seed=3, steps=10)


@pytest.mark.parametrize("config", [2, 3, 4, 5])
def test_parity_bench_caps_small(config):
    """Every step of a small odd-sized batch at each bench configuration's record
    capacities (bench.CONFIGS), compared whole against the oracle; the odd env
    counts leave partial k_ego workgroups and k_actors / k_raster tails."""
    caps = bench_caps(config)
    if config == 2:
        run_parity(["rt_no_traffic_v1"], 37, 150, seed0=10_000, caps=caps)
        run_parity(["rt_no_traffic_v1"], 5, 60, seed0=10_500, act_seed=77, caps=caps)
    elif config == 3:
        run_parity(["rt_hard_v1"], 29, 100, seed0=20_000, act_seed=7, caps=caps)
    elif config == 4:
        run_parity(["rt_medium_v1"], 23, 100, profile="continuous_gsb_v1", seed0=40_000, act_seed=99, caps=caps)
    else:
        run_parity(["mix3"], 19, 80, size=256, seed0=30_000, caps=caps)


def _bank_world(n, B, F, caps, kinds, seed0, bank_seed0):
    cfg, P, padded, layout, builder = world(caps=caps)
    recs, _ = build_records(builder, n, kinds, seed0=seed0)
    bank, _ = build_records(builder, B, kinds, seed0=bank_seed0)
    dw = DevWorld(P, padded, caps)
    L = lib()
    S = P.size
    d_bank = torch.from_numpy(bank.copy()).cuda()
    bf = torch.zeros((B, S, S), dtype=torch.uint8, device="cuda")
    check(L.cbev_bank_frames(dw.ctx, ptr(d_bank), B, ptr(bf), None), "bank_frames")
    d_recs = torch.from_numpy(recs.copy()).cuda()
    ring = torch.zeros((F, n, S, S), dtype=torch.uint8, device="cuda")
    check(L.cbev_reset(dw.ctx, ptr(d_recs), n, None, 0, None, None, 0, ptr(ring), F, None), "reset")
    return P, layout, dw, d_bank, bf, d_recs, ring


def reset_rows(mask_np, tcount, B):
    """The bank rows a masked reset hands out (include/cbev.h, ABI 7): env e takes
    (e + j * cbev_bank_stride(B)) % B, j = tcount[e], its terminations so far
    (counted by the steps)."""
    ids = np.flatnonzero(mask_np)
    stride = lib().cbev_bank_stride(B)
    rows = (ids.astype(np.int64) + tcount[ids].astype(np.int64) * stride) % B
    return ids, rows


def _want_reset(L, dw, d_recs, ring, d_bank, bf, mask_np, tcount, F):
    """cbev_reset_frames with the bank rows the masked reset hands out (reset_rows)."""
    n, B = d_recs.shape[0], d_bank.shape[0]
    ids, rows = reset_rows(mask_np, tcount, B)
    bidx = np.zeros(n, np.int32)
    bidx[ids] = rows
    want_r, want_f = d_recs.clone(), ring.clone()
    m = torch.from_numpy(mask_np.astype(np.uint8)).cuda()
    check(L.cbev_reset_frames(dw.ctx, ptr(want_r), n, ptr(d_bank), B, ptr(m), ptr(torch.from_numpy(bidx).cuda()),
                              0, ptr(bf), ptr(want_f), F, None), "reset_frames")
    return want_r, want_f, len(ids)


def _cursor(L, dw):
    c = ctypes.c_int64()
    check(L.cbev_bank_cursor(dw.ctx, ctypes.byref(c)), "cursor")
    return c.value


def _counts(L, dw, n):
    out = np.zeros(n, np.uint32)
    check(L.cbev_reset_counts(dw.ctx, out.ctypes.data_as(P_), n), "reset_counts")
    return out


def test_reset_terminated_matches_masked_reset():
    """cbev_reset_terminated (the canonical loop's reset from the last step's term
    buffer) = cbev_reset_frames with mask = that step's terminations and the bank
    rows of the per-env rule (reset_rows: env e takes (e + j * stride) % B after
    its j-th termination); each step counts its terminations."""
    n, B, F = 45, 11, 4
    P, layout, dw, d_bank, bf, d_recs, ring = _bank_world(n, B, F, bench_caps(3), ["rt_hard_v1", "rt_medium_v1"],
                                                           2100, 2900)
    L = lib()
    rew = torch.zeros(n, dtype=torch.float64, device="cuda")
    term = torch.zeros(n, dtype=torch.uint8, device="cuda")
    trunc = torch.zeros_like(term)
    cause = torch.zeros(n, dtype=torch.int32, device="cuda")
    acts = action_stream(P, n, 12, seed=7)
    seq = np.zeros(n, np.int64)
    rng = np.random.default_rng(5)
    total = 0
    for t in range(12):
        # push a random subset off the road so every round terminates some envs
        h = d_recs.cpu().numpy()
        for e in rng.choice(n, size=int(rng.integers(0, 9)), replace=False):
            LY.RecordView(h[e], layout).hd[LY.HD["X"]] += 60.0
        d_recs.copy_(torch.from_numpy(h))
        a = torch.from_numpy(np.ascontiguousarray(acts[t])).cuda()
        check(L.cbev_step(dw.ctx, ptr(d_recs), n, ptr(a), ptr(ring[t % F]), ptr(rew), ptr(term), ptr(trunc),
                          ptr(cause), None, None), "step")
        torch.cuda.synchronize()
        tn = term.cpu().numpy().astype(bool)
        seq += tn
        assert np.array_equal(_counts(L, dw, n), seq), t
        want_r, want_f, k = _want_reset(L, dw, d_recs, ring, d_bank, bf, tn, seq, F)
        total += k
        check(L.cbev_reset_terminated(dw.ctx, ptr(d_recs), n, ptr(d_bank), B, ptr(bf), ptr(ring), F, None), "reset_term")
        torch.cuda.synchronize()
        assert torch.equal(d_recs, want_r), t
        assert torch.equal(ring, want_f), t
        assert _cursor(L, dw) == total, t
    assert total > 20 and seq.max() >= 2  # some env walked past its first bank row
    # n must match the last step's
    assert L.cbev_reset_terminated(dw.ctx, ptr(d_recs), n - 1, ptr(d_bank), B, ptr(bf), ptr(ring), F, None) != 0


def test_reset_masked_mass_termination_and_edits():
    """The cursor reset when most of a large batch terminates at once (every env
    pushed off the road: the ranking must not depend on the count), with the mask
    edited in place between the step and the reset (term |= extra, term[i] = 0:
    the reset reads the buffer when it runs), an unaligned mask view, and a step
    with no reset (the cursor moves only when a reset runs)."""
    n, B, F = 4099, 5003, 1
    P, layout, dw, d_bank, bf, d_recs, ring = _bank_world(n, B, F, bench_caps(2), ["rt_no_traffic_v1"], 6000, 16000)
    L = lib()
    rew = torch.zeros(n, dtype=torch.float64, device="cuda")
    term = torch.zeros(n, dtype=torch.uint8, device="cuda")
    trunc = torch.zeros_like(term)
    cause = torch.zeros(n, dtype=torch.int32, device="cuda")
    acts = action_stream(P, n, 6, seed=3)
    rng = np.random.default_rng(11)
    seq = np.zeros(n, np.int64)

    def step(t, push):
        h = d_recs.cpu().numpy()
        for e in push:
            LY.RecordView(h[e], layout).hd[LY.HD["X"]] += 60.0
        d_recs.copy_(torch.from_numpy(h))
        a = torch.from_numpy(np.ascontiguousarray(acts[t])).cuda()
        check(L.cbev_step(dw.ctx, ptr(d_recs), n, ptr(a), ptr(ring[0]), ptr(rew), ptr(term), ptr(trunc), ptr(cause),
                          None, None), "step")
        torch.cuda.synchronize()
        seq[:] += term.cpu().numpy().astype(bool)  # the step counts its terminations

    # 1: (almost) every env terminates
    step(0, range(n))
    m = term.cpu().numpy().astype(bool)
    assert m.sum() > n // 2
    want_r, want_f, k = _want_reset(L, dw, d_recs, ring, d_bank, bf, m, seq, F)
    check(L.cbev_reset_terminated(dw.ctx, ptr(d_recs), n, ptr(d_bank), B, ptr(bf), ptr(ring), F, None), "reset_term")
    torch.cuda.synchronize()
    assert torch.equal(d_recs, want_r) and torch.equal(ring, want_f)
    assert _cursor(L, dw) == seq.sum()
    # 2: a step whose terminations are not reset: they are counted all the same
    step(1, rng.choice(n, size=300, replace=False))
    assert term.cpu().numpy().sum() > 0 and np.array_equal(_counts(L, dw, n), seq)
    # 3: in-place edits of the term buffer before the reset
    step(2, rng.choice(n, size=700, replace=False))
    extra = torch.from_numpy((rng.random(n) < 0.05).astype(np.uint8)).cuda()
    term |= extra
    term[:17] = 0
    m = term.cpu().numpy().astype(bool)
    want_r, want_f, k = _want_reset(L, dw, d_recs, ring, d_bank, bf, m, seq, F)
    check(L.cbev_reset_terminated(dw.ctx, ptr(d_recs), n, ptr(d_bank), B, ptr(bf), ptr(ring), F, None), "reset_term")
    torch.cuda.synchronize()
    assert torch.equal(d_recs, want_r) and torch.equal(ring, want_f)
    assert np.array_equal(_counts(L, dw, n), seq)
    # 4: cbev_reset_masked with an arbitrary mask at an odd byte offset (byte-wise mask loads)
    buf = torch.zeros(n + 3, dtype=torch.uint8, device="cuda")
    mview = buf[3:]
    mh = rng.random(n) < 0.4
    mview.copy_(torch.from_numpy(mh.astype(np.uint8) * 7))  # any nonzero byte selects
    want_r, want_f, k = _want_reset(L, dw, d_recs, ring, d_bank, bf, mh, seq, F)
    check(L.cbev_reset_masked(dw.ctx, ptr(d_recs), n, ptr(mview), ptr(d_bank), B, ptr(bf), ptr(ring), F, None),
          "reset_masked")
    torch.cuda.synchronize()
    assert torch.equal(d_recs, want_r) and torch.equal(ring, want_f)
    # 5: the same mask again straight away (no step, so no new termination between):
    # every selected env takes the same row again, and nothing moves the counts
    h5 = d_recs.cpu().numpy()
    for e in np.flatnonzero(mh)[:50]:
        LY.RecordView(h5[e], layout).hd[LY.HD["X"]] += 1.0  # an edit the second reset must undo
    d_recs.copy_(torch.from_numpy(h5))
    check(L.cbev_reset_masked(dw.ctx, ptr(d_recs), n, ptr(mview), ptr(d_bank), B, ptr(bf), ptr(ring), F, None),
          "reset_masked again")
    torch.cuda.synchronize()
    assert torch.equal(d_recs, want_r) and torch.equal(ring, want_f)
    assert np.array_equal(_counts(L, dw, n), seq) and _cursor(L, dw) == seq.sum()


def test_reset_cursor_advances_under_graph_replay():
    """The per-env termination counts live on the device: a step +
    cbev_reset_terminated captured once in a HIP graph and replayed hands out each
    env's next row after each new termination (each replay = the eager calls,
    reset_rows), the steps inside the graph counting the terminations."""
    n, B, F = 45, 17, 2
    P, layout, dw, d_bank, bf, d_recs, ring = _bank_world(n, B, F, bench_caps(2), ["rt_no_traffic_v1"], 3100, 3900)
    L = lib()
    rew = torch.zeros(n, dtype=torch.float64, device="cuda")
    term = torch.zeros(n, dtype=torch.uint8, device="cuda")
    trunc = torch.zeros_like(term)
    cause = torch.zeros(n, dtype=torch.int32, device="cuda")
    a = torch.zeros(n, dtype=torch.int32, device="cuda")
    check(L.cbev_step(dw.ctx, ptr(d_recs), n, ptr(a), ptr(ring[0]), ptr(rew), ptr(term), ptr(trunc), ptr(cause),
                      None, None), "step")
    torch.cuda.synchronize()
    sel = (np.arange(n) % 4 == 1)
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):  # reads the term buffer of the step before it
            check(L.cbev_reset_terminated(dw.ctx, ptr(d_recs), n, ptr(d_bank), B, ptr(bf), ptr(ring), F,
                                          P_(torch.cuda.current_stream().cuda_stream)), "reset_term (capture)")
    torch.cuda.synchronize()
    seq = _counts(L, dw, n).astype(np.int64)  # capture runs nothing
    total = 0
    for rep in range(4):
        h = d_recs.cpu().numpy()  # push the selected envs off the road: the next step terminates them
        for e in np.flatnonzero(sel):
            LY.RecordView(h[e], layout).hd[LY.HD["X"]] += 60.0
        d_recs.copy_(torch.from_numpy(h))
        check(L.cbev_step(dw.ctx, ptr(d_recs), n, ptr(a), ptr(ring[0]), ptr(rew), ptr(term), ptr(trunc),
                          ptr(cause), None, None), "step")
        torch.cuda.synchronize()
        tn = term.cpu().numpy().astype(bool)
        seq += tn
        assert np.array_equal(_counts(L, dw, n), seq), rep
        want_r, want_f, k = _want_reset(L, dw, d_recs, ring, d_bank, bf, tn, seq, F)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(d_recs, want_r) and torch.equal(ring, want_f), rep
        total += k
    assert total >= 8 and seq.max() >= 3


def _same_records(a, b, layout):
    """Records equal but for RS_FAST's bits above bit 0 (device scratch: a folded
    reset's bank row for k_raster, k_ego -> k_raster of one step)."""
    o = layout.off["hi"] + 4 * LY.HI["RS_FAST"]
    a, b = a.clone(), b.clone()
    for r in (a, b):
        v = r.view(r.shape[0], -1)[:, o:o + 4].contiguous().view(torch.int32) & 1
        r.view(r.shape[0], -1)[:, o:o + 4] = v.view(torch.uint8).view(r.shape[0], 4)
    return torch.equal(a, b)


def _deferred_pair(n, B, F, caps, seed0, bank_seed0, stats=True):
    """Two contexts on the same scenes and bank: reset_terminated launched at once
    (A) and deferred into the next step (B, cbev_set_deferred_reset); with the
    device episode statistics on in both (stats: the headline's k_ego variant)."""
    cfg, P, padded, layout, builder = world(caps=caps)
    recs, _ = build_records(builder, n, ["rt_no_traffic_v1"], seed0=seed0)
    bank, _ = build_records(builder, B, ["rt_no_traffic_v1"], seed0=bank_seed0)
    L = lib()
    S = P.size
    out = []
    for deferred in (0, 1):
        dw = DevWorld(P, padded, caps)
        check(L.cbev_set_deferred_reset(dw.ctx, deferred), "deferred")
        d_bank = torch.from_numpy(bank.copy()).cuda()
        bf = torch.zeros((B, S, S), dtype=torch.uint8, device="cuda")
        check(L.cbev_bank_frames(dw.ctx, ptr(d_bank), B, ptr(bf), None), "bank_frames")
        d_recs = torch.from_numpy(recs.copy()).cuda()
        ring = torch.zeros((F, n, S, S), dtype=torch.uint8, device="cuda")
        check(L.cbev_reset(dw.ctx, ptr(d_recs), n, None, 0, None, None, 0, ptr(ring), F, None), "reset")
        bufs = dict(rew=torch.zeros(n, dtype=torch.float64, device="cuda"),
                    term=torch.zeros(n, dtype=torch.uint8, device="cuda"),
                    trunc=torch.zeros(n, dtype=torch.uint8, device="cuda"),
                    cause=torch.zeros(n, dtype=torch.int32, device="cuda"),
                    info=torch.zeros((n, 16), dtype=torch.float32, device="cuda"))
        if stats:
            bufs["stats"] = EpisodeStatsOn(dw.ctx, n)
        out.append((dw, d_bank, bf, d_recs, ring, bufs))
    return P, layout, out


_T0 = slice(8 * 200 + 16, 8 * 200 + 24)  # cbev_episode_stats.t0 (the device clock at the episode's reset)


def _same_stats(a, b, step, n):
    """The two contexts' episode statistics after `step`: per-env accumulators
    (all but the reset clock stamp t0), this step's summary rows (by env; all
    columns but the elapsed SECONDS) and their count."""
    sa, sb = a.stats.cpu().numpy(), b.stats.cpu().numpy()
    keep = np.ones(sa.shape[1], bool)
    keep[_T0] = False
    if not np.array_equal(sa[:, keep], sb[:, keep]):
        return False
    slot = step % a.RING
    ca, cb = min(int(a.counts[slot].item()), n), min(int(b.counts[slot].item()), n)
    if ca != cb:
        return False
    ra, rb_ = a.rows[slot, :ca].cpu().numpy(), b.rows[slot, :cb].cpu().numpy()
    ra, rb_ = ra[np.argsort(ra[:, LY.EP["ENV"]])], rb_[np.argsort(rb_[:, LY.EP["ENV"]])]
    cols = [c for c in range(ra.shape[1]) if c != LY.EP["SECONDS"]]
    return bool(np.array_equal(ra[:, cols], rb_[:, cols]))


def test_deferred_reset_matches_immediate():
    """The canonical reset folded into the next step's k_ego (cbev_set_deferred_reset)
    leaves exactly the state the immediate k_reset_mask + step leave: records, every
    frame-stack slot, reward / term / trunc / cause / info, the episode statistics
    (accumulators, summary rows) and the per-env reset counts, step
    after step. Covered: envs pushed off the road (resets in most steps), in-place
    edits of the term buffer between the step and the reset (the folded reset reads
    the buffer when the next step runs), a reset read straight away (cbev_flush, and
    cbev_expand_obs flushing by itself), a step with no reset before it, the frame
    ring's slots in turn, an odd batch (partial k_ego workgroup)."""
    for n, B, F in ((45, 13, 4), (4099, 6007, 4)):
        P, layout, ctxs = _deferred_pair(n, B, F, bench_caps(2), 7000, 17000)
        L = lib()
        S = P.size
        acts = action_stream(P, n, 16, seed=21)
        rng = np.random.default_rng(3)
        folded = rows_seen = 0
        for t in range(16):
            push = rng.choice(n, size=min(n, int(rng.integers(1, 9)) * max(1, n // 40)), replace=False)
            extra = torch.from_numpy((rng.random(n) < 0.03).astype(np.uint8)).cuda()
            folded += L.cbev_reset_pending(ctxs[1][0].ctx)
            for dw, d_bank, bf, d_recs, ring, b in ctxs:
                if t % 2 == 0:  # the caller writes the records: it flushes first (cbev.h)
                    check(L.cbev_flush(dw.ctx), "flush")
                    h = d_recs.cpu().numpy()
                    for e in push:
                        LY.RecordView(h[e], layout).hd[LY.HD["X"]] += 60.0
                    d_recs.copy_(torch.from_numpy(h))
                a = torch.from_numpy(np.ascontiguousarray(acts[t])).cuda()
                check(L.cbev_step(dw.ctx, ptr(d_recs), n, ptr(a), ptr(ring[t % F]), ptr(b["rew"]), ptr(b["term"]),
                                  ptr(b["trunc"]), ptr(b["cause"]), ptr(b["info"]), None), "step")
            torch.cuda.synchronize()
            (dA, _, _, rA, gA, bA), (dB, _, _, rB, gB, bB) = ctxs
            assert L.cbev_reset_pending(dB.ctx) == 0
            for k in ("rew", "term", "trunc", "cause", "info"):
                assert torch.equal(bA[k], bB[k]), (n, t, k)
            assert _same_stats(bA["stats"], bB["stats"], t, n), (n, t, "episode stats")
            rows_seen += int(bA["stats"].counts[t % bA["stats"].RING].item())
            assert _same_records(rA, rB, layout), (n, t, "records")
            assert torch.equal(gA, gB), (n, t, "ring")
            if t % 5 == 4:  # no reset before the next step
                continue
            for dw, d_bank, bf, d_recs, ring, b in ctxs:
                if t % 3 == 1:  # in-place edit of the mask before the reset
                    b["term"] |= extra
                check(L.cbev_reset_terminated(dw.ctx, ptr(d_recs), n, ptr(d_bank), B, ptr(bf), ptr(ring), F, None),
                      "reset_terminated")
            torch.cuda.synchronize()
            assert L.cbev_reset_pending(dA.ctx) == 0 and L.cbev_reset_pending(dB.ctx) == 1, t
            if t % 4 == 2:  # the reset observed right away: flush
                check(L.cbev_flush(dB.ctx), "flush")
                torch.cuda.synchronize()
                assert _same_records(rA, rB, layout) and torch.equal(gA, gB), (n, t, "flushed reset")
            elif t % 4 == 3:  # ... or through an observation call, which flushes by itself
                out = torch.zeros((n, S, S, 3), dtype=torch.uint8, device="cuda")
                check(L.cbev_expand_obs(dB.ctx, ptr(gB[0][None]), n, 1, 0, 2, 3, rgb_lut().ctypes.data_as(P_),
                                        ptr(out), None), "expand")
                torch.cuda.synchronize()
                assert L.cbev_reset_pending(dB.ctx) == 0
                assert _same_records(rA, rB, layout) and torch.equal(gA, gB), (n, t, "observed reset")
        for dw, *_ in ctxs:
            check(L.cbev_flush(dw.ctx), "flush")
        torch.cuda.synchronize()
        (dA, _, _, rA, gA, bA), (dB, _, _, rB, gB, bB) = ctxs
        assert _same_records(rA, rB, layout) and torch.equal(gA, gB)
        assert _cursor(L, dA) == _cursor(L, dB) and _cursor(L, dA) > 0
        assert np.array_equal(_counts(L, dA, n), _counts(L, dB, n))
        assert folded >= 3, folded  # steps that took a pending reset
        assert rows_seen > 0


def _graph_pair(n, B, F, seed0, bank_seed0, capture_reset):
    """Deferred context B, one step + reset captured into a graph (capture_reset:
    the reset_terminated inside the capture too), against an eager context A with
    the deferral off; both on the same scenes, bank and statistics."""
    caps = bench_caps(2)
    P, layout, ctxs = _deferred_pair(n, B, F, caps, seed0, bank_seed0)
    L = lib()
    (dA, bankA, bfA, rA, gA, bA), (dB, bankB, bfB, rB, gB, bB) = ctxs
    check(L.cbev_set_deferred_reset(dA.ctx, 0), "deferred off")
    a0 = torch.zeros(n, dtype=torch.int32, device="cuda")

    def push(d_recs, every):
        h = d_recs.cpu().numpy()
        for e in range(0, n, every):
            LY.RecordView(h[e], layout).hd[LY.HD["X"]] += 60.0
        d_recs.copy_(torch.from_numpy(h))

    def step(dw, d_recs, ring, b, a):
        check(L.cbev_step(dw.ctx, ptr(d_recs), n, ptr(a), ptr(ring[0]), ptr(b["rew"]), ptr(b["term"]), ptr(b["trunc"]),
                          ptr(b["cause"]), ptr(b["info"]), P_(torch.cuda.current_stream().cuda_stream)), "step")

    def reset(dw, d_recs, ring, d_bank, bf):
        check(L.cbev_reset_terminated(dw.ctx, ptr(d_recs), n, ptr(d_bank), B, ptr(bf), ptr(ring), F,
                                      P_(torch.cuda.current_stream().cuda_stream)), "reset_terminated")

    for ctx_ in ((dA, rA, gA, bA), (dB, rB, gB, bB)):
        push(ctx_[1], 3)
        step(ctx_[0], ctx_[1], ctx_[2], ctx_[3], a0)
    torch.cuda.synchronize()
    assert int(bA["term"].sum()) > 0
    if not capture_reset:
        reset(dB, rB, gB, bankB, bfB)  # recorded (and the fold's scratch allocated) before the capture
        assert L.cbev_reset_pending(dB.ctx) == 1
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    side.wait_stream(torch.cuda.current_stream())
    acts = torch.ones(n, dtype=torch.int32, device="cuda")
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            if capture_reset:
                reset(dB, rB, gB, bankB, bfB)
            step(dB, rB, gB, bB, acts)
    torch.cuda.synchronize()
    for rep in range(4):
        if rep == 2:  # more terminations between replays (nothing is pending outside the graph)
            assert L.cbev_reset_pending(dB.ctx) == 0
            check(L.cbev_flush(dB.ctx), "flush")
            torch.cuda.synchronize()
            for d_recs in (rA, rB):
                push(d_recs, 5)
        reset(dA, rA, gA, bankA, bfA)
        step(dA, rA, gA, bA, acts)
        g.replay()
        torch.cuda.synchronize()
        for k in ("rew", "term", "trunc", "cause", "info"):
            assert torch.equal(bA[k], bB[k]), (rep, k)
        assert _same_records(rA, rB, layout), (rep, "records")
        assert torch.equal(gA, gB), (rep, "ring")
    check(L.cbev_flush(dB.ctx), "flush")
    torch.cuda.synchronize()
    assert np.array_equal(_counts(L, dA, n), _counts(L, dB, n)) and _cursor(L, dA) > 0


def test_folded_step_under_graph_capture():
    """a cbev_step captured while a reset is pending carries the
    folded reset (each replay resets the envs the term buffer selects, then
    steps), also when the capture records the reset itself on a fresh context
    (nothing is allocated under the capture). Each replay equals the eager
    reset_terminated + step."""
    _graph_pair(45, 13, 2, 7100, 17100, capture_reset=False)
    _graph_pair(45, 13, 2, 7200, 17200, capture_reset=True)


def test_vector_env_reads_after_deferred_reset():
    """CarlaBEVVectorEnv defers reset_terminated into the next step; reading the
    observation, the records or the term flags straight after it sees the reset
    (the accessors flush), exactly as an env with the deferral off."""
    from carlabev_env_amd import EnvConfig, make_env
    cfg = EnvConfig(size=128, obs_size=(128, 128), render_mode="rgb_array", obs_mode="bev_semantic")
    import bench
    envs = [make_env({"env": cfg, "num_envs": 24}, info_mode="none", caps=dict(bench.CONFIGS[2]["caps"]),
                     defer_reset=d) for d in (False, True)]
    opts = build_random_navigation_options(RandomNavigationReset(difficulty_id="rt_no_traffic_v1"))
    for env in envs:
        env.reset(seed=5, options=opts)
        env.attach_bank(env.build_bank([900 + k for k in range(11)], opts))
        env.auto_obs = False
    rng = np.random.default_rng(2)
    seen = folded = 0
    for t in range(60):
        a = rng.integers(0, 9, 24)
        outs = []
        for env in envs:
            env.step(a)
            if t % 7 == 0:  # push some envs off the road so resets happen
                h = env.records_host()
                for e in range(0, 24, 5):
                    LY.RecordView(h[e], env.layout).hd[LY.HD["X"]] += 60.0
                env.records.copy_(torch.from_numpy(h))
            env.reset_terminated()
            if env is envs[1]:
                folded += lib().cbev_reset_pending(env._ctx)  # recorded, not launched
            outs.append((env._obs().clone(), env.records.clone(), env.term.clone()))
        assert torch.equal(outs[0][0], outs[1][0]), t
        assert _same_records(outs[0][1], outs[1][1], envs[0].layout), t
        assert torch.equal(outs[0][2], outs[1][2]), t
        seen += int(outs[0][2].sum())
    assert seen > 0 and folded == 60
    # and a step takes a recorded reset (nothing read in between): the same state
    for env in envs:
        env.step(np.zeros(24, np.int64))
        h = env.records_host()
        for e in range(0, 24, 3):
            LY.RecordView(h[e], env.layout).hd[LY.HD["X"]] += 60.0
        env.records.copy_(torch.from_numpy(h))
        env.step(np.ones(24, np.int64))
        env.reset_terminated()
        env.step(np.ones(24, np.int64))  # takes the reset
        env.step(np.zeros(24, np.int64))
    assert _same_records(envs[0].records, envs[1].records, envs[0].layout)
    assert torch.equal(envs[0].ring, envs[1].ring)
    assert torch.equal(envs[0].reward, envs[1].reward)
    for env in envs:
        env.close()
