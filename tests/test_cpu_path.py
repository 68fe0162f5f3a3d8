"""CPU-side tests: the C-ABI library surface, host scene packing, and the
oracle's end-to-end step against the reference's own behavioural contracts.
No GPU calls are made here."""
from __future__ import annotations

import ctypes
import math

import numpy as np
import pytest

import oracle as O
import raster_ref
from carlabev_env_amd import layout as LY
from carlabev_env_amd import _lib
from carlabev_env_amd.params import CbevParams, fov_geometry
from helpers import CAPS_FULL, action_stream, build_records, world


# ------------------------------------------------------------ C-ABI surface
def test_library_loads_and_exports_every_symbol():
    L = _lib.lib()
    for name in _lib.EXPORTED_SYMBOLS:
        assert hasattr(L, name), name
    assert L.cbev_abi_version() == 7
    assert L.cbev_bank_stride(8192) % 2 == 1 and L.cbev_bank_stride(1) == 0 and L.cbev_bank_stride(0) == -1
    assert L.cbev_params_size() == ctypes.sizeof(CbevParams)


def test_header_declares_exactly_the_exported_symbols():
    import re
    text = open(LY.HEADER.replace("cbev_layout.h", "cbev.h")).read()
    declared = set(re.findall(r"^\s*(?:int|void|const char\*)\s+(cbev_\w+)\(", text, re.M))
    assert declared == set(_lib.EXPORTED_SYMBOLS)


@pytest.mark.parametrize("caps", [(128, 32, 64, 4), (128, 0, 2, 0), (256, 50, 200, 8), (64, 1, 8, 1)])
def test_layout_matches_library(caps):
    L = _lib.lib()
    c = LY.Caps(*caps)
    out = LY.CbevLayout()
    assert L.cbev_layout_of(ctypes.byref(c.c()), ctypes.byref(out)) == 0
    py = LY.Layout.make(c)
    for name, off in py.off.items():
        assert getattr(out, name) == off, name
    assert out.record_bytes == py.record_bytes
    assert out.vis_words == py.vis_words


def test_field_names_match_header():
    L = _lib.lib()
    for g, key in enumerate(("HD", "HI", "AD", "AI", "TI")):
        names = L.cbev_field_names(g).decode().strip(",").split(",")
        assert names == LY.NAMES[key]


def test_fov_geometry_matches_reference_formula():
    # fov.py:30-44: anchor round((S-1)*frac), crop max(S, ceil(2*hypot))
    assert fov_geometry(128) == (64, 64, 182)
    assert fov_geometry(256) == (128, 128, 363)
    ax, ay, c = fov_geometry(128, 0.5, 0.75)
    assert (ax, ay) == (64, 95) and c == max(128, math.ceil(2 * math.hypot(64, 95)))


# ------------------------------------------------------------ host packing
def test_scene_generation_is_deterministic_and_valid():
    cfg, P, padded, layout, builder = world()
    a, meta_a = build_records(builder, 6, ["rt_hard_v1"], seed0=100)
    b, meta_b = build_records(builder, 6, ["rt_hard_v1"], seed0=100)
    assert np.array_equal(a, b)
    for info, spec, ctx in meta_a:
        assert info["valid"]
        assert len(spec.vehicles) <= 25


# ------------------------------------------------------------ oracle end-to-end
def _rollout(kinds, n_envs=6, steps=120, size=128, profile="discrete9_v1", reward="carl_base_v1", anchor_y=0.5):
    cfg, P, padded, layout, builder = world(size, profile, reward, anchor_y)
    recs, meta = build_records(builder, n_envs, kinds)
    orc = O.Oracle(P, padded, CAPS_FULL.c(), layout.record_bytes)
    S = P.size
    frames = np.zeros((n_envs, S, S), np.uint8)
    acts = action_stream(P, n_envs, steps)
    causes = []
    for e in range(n_envs):
        orc.reset_obs(recs[e], frames[e])
        v = LY.RecordView(recs[e], layout)
        ref = raster_ref.render(P, padded, v, reset=True)
        assert np.array_equal(frames[e], ref), "reset frame mismatch vs numpy restatement"
    for t in range(steps):
        for e in range(n_envs):
            c = orc.step_one(recs[e], np.ascontiguousarray(acts[t, e]), frames[e])
            causes.append(c)
            v = LY.RecordView(recs[e], layout)
            # ego overlay sits at the anchor (validate_simulator_semantics.py:366-414)
            assert frames[e, P.anchor_y, P.anchor_x] == 8
            # ego at crop centre +-1.5 px (test_seeded_scene_consistency.py:128-138)
            xm, ym = orc.crop_origin(v.h("X"), v.h("Y"))
            hx, hy = P.pad + v.h("X") - xm, P.pad + v.h("Y") - ym
            if 0 < xm < P.render_w - P.crop and 0 < ym < P.render_h - P.crop:
                assert abs(hx - P.crop / 2) <= 1.5 and abs(hy - P.crop / 2) <= 1.5
    return recs, frames, causes, layout


def test_oracle_rollout_random_traffic():
    recs, frames, causes, layout = _rollout(["rt_hard_v1", "rt_medium_v1"], n_envs=4, steps=100)
    assert set(causes) <= set(range(8))


def test_oracle_rollout_scenarios_and_continuous():
    _rollout(["mix3"], n_envs=6, steps=80, profile="continuous_gsb_v1")


def test_oracle_rollout_size256_and_offcentre_anchor():
    _rollout(["rt_easy_v1"], n_envs=2, steps=40, size=256)
    _rollout(["rt_no_traffic_v1"], n_envs=2, steps=40, anchor_y=0.2)


def test_oracle_raster_matches_numpy_restatement_mid_episode():
    """Render the same record with the C oracle (via a no-op step replay) and with
    the vectorised NumPy restatement: paint order, crop, rotate, compose."""
    cfg, P, padded, layout, builder = world()
    recs, meta = build_records(builder, 4, ["rt_hard_v1"], seed0=7)
    orc = O.Oracle(P, padded, CAPS_FULL.c(), layout.record_bytes)
    acts = action_stream(P, 4, 60)
    frame = np.zeros((P.size, P.size), np.uint8)
    for t in range(60):
        for e in range(4):
            before = recs[e].copy()
            orc.step_one(recs[e], np.ascontiguousarray(acts[t, e]), frame)
            # the frame is drawn after dynamics and before collision consumption:
            # rebuild that state = post-step record with the pre-step visibility
            # bits, which the step also kept as vis_draw
            mid = recs[e].copy()
            vmid, vbef = LY.RecordView(mid, layout), LY.RecordView(before, layout)
            assert np.array_equal(vmid.vis_draw, vbef.vis)
            vmid.vis[:] = vbef.vis
            ref = raster_ref.render(P, padded, vmid)
            assert np.array_equal(frame, ref), (t, e, np.argwhere(frame != ref)[:5])


def test_shaping_reward_rollout_terminates_with_reference_causes():
    recs, frames, causes, layout = _rollout(["rt_easy_v1"], n_envs=3, steps=60, reward="shaping_base_v1")
    assert set(causes) <= {0, 1, 2, 3, 4, 5, 6, 7}


def test_create_refuses_records_k_ego_cannot_stage():
    """k_ego stages at least 4 records per workgroup (its shuffle reductions stay
    inside a wave): capacities whose staged ranges exceed the LDS budget at 4 envs
    are refused at cbev_create (no GPU work: the check precedes any launch)."""
    import ctypes
    from carlabev_env_amd import layout as LY
    _, P, _, _, _ = world()
    L = _lib.lib()
    ctx = ctypes.c_void_p()
    rc = L.cbev_create(ctypes.byref(P), ctypes.byref(LY.Caps(4096, 0, 2, 0).c()), 0, ctypes.byref(ctx))
    assert rc == -1 and b"k_ego" in L.cbev_last_error()


def test_pack_refuses_retreat_routes_beyond_the_wave_rebuild():
    """A StopReturn (yield_return) actor's retreat route ([pos] + initial_route[:idx+1][::-1],
    jaywalk.py:43-54) is rebuilt by one wave, one point per lane: scene_pack refuses
    initial routes whose retreat could exceed 64 points, whatever actor_route_cap is."""
    from carlabev_env_amd.scene_pack import ActorSpec, SceneSpec, pack_scene
    layout = LY.Layout.make(CAPS_FULL)
    assert CAPS_FULL.actor_route_cap > 64
    beh = {"type": "yield_return", "params": {"start_delay": 0.5, "yield_duration": 1.0}}
    for n, ok in ((63, True), (64, False)):
        ped = ActorSpec("pedestrian", [300.0 + 0.5 * i for i in range(n)], [400.0] * n, 1.6, beh)
        spec = SceneSpec([500.0, 500.0, 500.0], [700.0, 690.0, 680.0], 0.0, 12.0, pedestrians=[ped])
        buf = np.zeros(layout.record_bytes, np.uint8)
        if ok:
            pack_scene(LY.RecordView(buf, layout), spec, 128)
        else:
            with pytest.raises(ValueError, match="64 points"):
                pack_scene(LY.RecordView(buf, layout), spec, 128)


def test_library_layout_check_refuses_a_mismatch():
    """check_library_layout: the header's layout when the library agrees; a refusal
    naming the groups when a library computes another (a stale build)."""
    L = _lib.lib()
    lay = LY.check_library_layout(L, CAPS_FULL)
    assert lay.record_bytes == LY.Layout.make(CAPS_FULL).record_bytes

    class Shifted:  # a library whose actor groups sit 64 bytes later
        @staticmethod
        def cbev_layout_of(c, out):
            rc = L.cbev_layout_of(c, out)
            out._obj.ai += 64
            return rc
    with pytest.raises(RuntimeError, match="ai"):
        LY.check_library_layout(Shifted, CAPS_FULL)


def test_acb_circles_hold_their_blocks():
    """layout.acb_circles: per block of ACB_PTS route points, a fixed-point circle
    holding every point (the actor target search skips a block by it), as
    scene_pack writes it."""
    rng = np.random.default_rng(5)
    for n in (1, 15, 16, 17, 64, 276):
        pts = (rng.uniform(0, 1200, 2) + np.cumsum(rng.normal(0, 9, (n, 2)), 0)).astype(np.float32)
        acb = LY.acb_circles(pts)
        assert acb.shape == ((n + LY.ACB_PTS - 1) // LY.ACB_PTS, 2)
        for b in range(len(acb)):
            w0, w1 = int(acb[b, 0]), int(acb[b, 1])
            c = np.array([(w0 & 0xFFFF) - 32768, (w0 >> 16) - 32768]) / 8.0
            q = pts[LY.ACB_PTS * b: LY.ACB_PTS * (b + 1)].astype(np.float64)
            d = np.hypot(q[:, 0] - c[0], q[:, 1] - c[1])
            assert d.max() <= w1 / 8.0 and w1 / 8.0 <= d.max() + 0.25 + 1e-9


def test_retreat_route_check_flags_long_stop_return_routes():
    """records whose yield_return actor has a route the narrow k_actors
    cannot retreat along (more than 63 points) are found before they reach the
    device (CarlaBEVVectorEnv.attach_bank / refresh_bank / load_scenes refuse
    them); scene_pack's own records never are."""
    caps = LY.Caps(64, 4, 288, 4)
    cfg, P, padded, layout, builder = world(caps=caps)
    recs, _ = build_records(builder, 6, ["mix3"], seed0=30_000)
    o = layout.off
    hi = recs[:, o["hi"]:o["hi"] + 4 * len(LY.HI)].copy().view(np.int32)
    ai = recs[:, o["ai"]:o["ai"] + 4 * len(LY.AI) * 4].copy().view(np.int32).reshape(6, len(LY.AI), 4)
    assert not LY.retreat_route_violations(hi, ai, caps).any()
    ai[2, LY.AI["BEH"], 0] = LY.BEH["yield_return"]
    ai[2, LY.AI["NRX"], 0] = 64
    hi[2, LY.HI["NACT"]] = max(hi[2, LY.HI["NACT"]], 1)
    got = LY.retreat_route_violations(hi, ai, caps)
    assert got.tolist() == [False, False, True, False, False, False]
    # the wide kernel (more than 64 actor slots) rebuilds any retreat serially: nothing to refuse
    assert not LY.retreat_route_violations(hi, ai, LY.Caps(64, 72, 128, 0)).any()
