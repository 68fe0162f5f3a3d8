"""Drop-in batched replacement of the reference's vector env.

`make_env(cfg)` mirrors `CarlaBEV.envs.make_env` (`envs/__init__.py:108-120`):
the reference returns a single-process `gymnasium.vector.SyncVectorEnv` over
`num_envs` copies of `CarlaBEV` wrapped by `wrap_env` (Resize -> SemanticMask
/ Grayscale -> FrameStack -> Flatten -> RecordEpisodeStatistics), with
autoreset DISABLED. `CarlaBEVVectorEnv` exposes the same surface —
`reset(seed, options)` with `options["reset_mask"]` partial resets,
`step(actions) -> (obs, rewards, terminations, truncations, infos)`,
`render()`, `close()`, `num_envs`, single/batched observation and action
spaces — but every env's state lives in HBM and one step is three HIP
launches through libcbev.so (include/cbev.h).

Host/device split: scene generation and reset-time packing run on the host
(`scene_gen`, `scene_pack`, as the reference's `src/managers/` does); the step,
the observation raster, rewards, termination and the wrapper stack run on the
GPU. Observations, rewards and flags are returned as torch tensors on the
env's device (no host round trip); `infos` follow gymnasium's vector-info
convention (`infos[key]` arrays + `infos["_key"]` masks).
"""
from __future__ import annotations

import ctypes
import os
import weakref
from collections import deque
from collections.abc import Mapping

import numpy as np
import torch

from . import layout as LY
from ._lib import check, lib
from .config import EnvConfig, RunConfig, validate_run_config, get_action_profile_spec
from .params import CbevParams, build_params, load_class_map, padded_map
from .host_reset import HostResetBuilder
from .scene_gen import SceneGenerator
from .semantics import gray_lut, rgb_lut, semantic_lut, semantic_mask_channels, PALETTE
from . import obs_pipeline as OP
from .fov_mask import fov_corner_mask
from .spaces import batch_space, make_box, make_discrete

DEFAULT_CAPS = dict(route_cap=128, actor_cap=32, actor_route_cap=288, tl_cap=4)


def _ptr(t: torch.Tensor | None):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


# episode_info keys (Stats.get_episode_info, stats.py:127-148, + carlabev.py:180-181)
# -> summary row column (include/cbev_layout.h CBEV_EP_FIELDS) and the Python
# type of the reference's value, which sets the batched array's dtype the way
# SyncVectorEnv._add_info does (int -> int64, float -> float64, str -> object)
_EP_KEYS = (("episode", "EPISODE", int), ("termination", "CAUSE", str), ("return", "RETURN", float),
            ("length", "LENGTH", int), ("mean_reward", "MEAN_REWARD", float),
            ("success_rate", "SUCCESS_RATE", float), ("collision_rate", "COLLISION_RATE", float),
            ("unfinished_rate", "UNFINISHED_RATE", float), ("mean_speed", "MEAN_SPEED", float),
            ("mean_ttc", "MEAN_TTC", float), ("mean_progress", "MEAN_PROGRESS", float),
            ("mean_abs_accel_long", "MEAN_ABS_AL", float), ("mean_abs_accel_lat", "MEAN_ABS_ALAT", float),
            ("mean_abs_jerk_long", "MEAN_ABS_JL", float), ("mean_abs_jerk_lat", "MEAN_ABS_JLAT", float),
            ("mean_abs_yaw_rate", "MEAN_ABS_YR", float), ("mean_abs_yaw_acc", "MEAN_ABS_YACC", float),
            ("comfort_violation_rate", "VIOL_RATE", float), ("harsh_brake_rate", "HARSH_RATE", float),
            ("num_vehicles", "NUM_VEH", int), ("len_ego_route", "LEN_ROUTE_M", float))
EP_RING = 8  # device slots of per-step episode rows (cbev_set_episode_stats)


def _batched(values: dict, n: int) -> dict:
    """{key: {env: value}} -> SyncVectorEnv._add_info's arrays + "_key" masks."""
    out = {}
    for key, per_env in values.items():
        first = next(iter(per_env.values()))
        if isinstance(first, (bool, int, float, np.number)) and not isinstance(first, bool):
            arr = np.zeros(n, dtype=np.int64 if isinstance(first, (int, np.integer)) else np.float64)
        elif isinstance(first, bool):
            arr = np.zeros(n, dtype=np.bool_)
        else:
            arr = np.full(n, None, dtype=object)
        mask = np.zeros(n, dtype=np.bool_)
        for i, v in per_env.items():
            arr[i] = v
            mask[i] = True
        out[key], out[f"_{key}"] = arr, mask
    return out


class StepInfos(Mapping):
    """`infos` of one step() in info_mode="full": the vector-env dict the
    reference returns ({} or {"episode_info": ..., "_episode_info": mask,
    "episode": ..., "_episode": mask}), built from the device's episode rows the
    first time it is read. Not reading it costs no host work and no sync."""

    __slots__ = ("_env", "_step", "_stream", "_d", "__weakref__")

    def __init__(self, env, step: int, stream):
        # stream: the torch Stream the step was queued on, held (not its raw
        # handle) so reading the infos never synchronises a destroyed stream
        self._env, self._step, self._stream, self._d = env, step, stream, None

    def _get(self) -> dict:
        if self._d is None:
            self._d = self._env._materialize_infos(self._step, self._stream)
            self._env = None
        return self._d

    def __getitem__(self, key):
        return self._get()[key]

    def __iter__(self):
        return iter(self._get())

    def __len__(self):
        return len(self._get())

    def __repr__(self):
        return repr(self._get())


class CarlaBEVVectorEnv:
    metadata = {"autoreset_mode": "disabled", "render_modes": ["rgb_array"], "render_fps": 60}

    def __init__(self, cfg, *, num_envs: int | None = None, device=None, caps: dict | None = None,
                 info_mode: str = "full", scene_generator=None, wrappers: bool = True, copy_obs: bool = True,
                 defer_reset: bool = True, reset_pool=None):
        """wrappers=False gives the base `CarlaBEV` observation of every env, as a
        `SyncVectorEnv` of unwrapped `CarlaBEV(cfg)` would: (S, S, 3) uint8 RGB for the
        BEV modes, float32[7] for obs_mode="vector" (carlabev.py:233-244, spaces.py:54-61).
        The reference only allows "vector" on the bare env (config/env.py:310-314).

        copy_obs=True (default) returns a fresh observation tensor from every step() /
        reset(), as SyncVectorEnv(copy=True) returns fresh arrays; copy_obs=False returns
        the env's own buffer, which the next step() / reset() overwrites in place
        (throughput loops that consume obs before stepping again).

        defer_reset=True (default) lets reset_terminated() fold into the next step's
        first kernel (cbev_set_deferred_reset): every accessor of the env's state
        (records, ring, term, frames(), observations, render, the bank calls) applies a
        recorded reset first, so what the caller observes is unchanged. It takes
        effect only when the records have no actor slots (caps actor_cap == 0:
        k_ego is the step's first kernel) and no resize is configured; otherwise
        reset_terminated() launches at once. A tensor taken from records / ring /
        term before reset_terminated() shows the pre-reset state until the next
        step or accessor applies it.

        caps: the record capacities (layout.Caps fields). The default, DEFAULT_CAPS with
        actor_cap >= max_vehicles + 4, holds any scene the generator makes: actor
        routes up to 288 points (the longest lane-graph route has 276), which costs
        about 64 * actor_cap * actor_route_cap bytes per record (about 470 KB at 29
        actor slots) in the records, the bank and every reset copy. Ego-only scenes
        fit caps=dict(actor_cap=0, actor_route_cap=2) (3.3 KB per env, and the reset
        folds into the step); SceneSpec.caps_needed() gives a scene's own needs.

        reset_pool: a scene_pool.BuildPool (created before this process touched the
        GPU) that builds the distinct scenes a reset(options) needs in worker
        processes; records are byte-identical to the in-process build. Built scenes
        are memoised either way (HostResetBuilder), so a repeated (seed, options)
        reset, such as the reference's canonical loop without seeds, is a copy."""
        if isinstance(cfg, RunConfig):
            raw = cfg
        elif isinstance(cfg, dict) and "env" in cfg:
            raw = cfg
        else:
            raw = {"env": cfg}
        run = validate_run_config(raw) if wrappers else (
            raw if isinstance(raw, RunConfig) else RunConfig.model_validate(dict(raw)))
        self.wrappers = bool(wrappers)
        self.copy_obs = bool(copy_obs)
        self.run_cfg = run
        self.cfg: EnvConfig = run.env
        self.num_envs = int(num_envs if num_envs is not None else run.num_envs)
        self.info_mode = info_mode
        if device is None:
            if not torch.cuda.is_available():
                raise RuntimeError("CarlaBEVVectorEnv needs a ROCm GPU (torch.cuda); there is no CPU fallback")
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self.S = int(self.cfg.size)
        self.F = int(self.cfg.frame_stack) if self.wrappers else 1
        self.classes = load_class_map(self.cfg.map_name, self.S)
        self.params: CbevParams = build_params(self.cfg, self.classes)
        self.map_host, pitch = padded_map(self.classes, self.params.pad)
        assert pitch == self.params.map_pitch
        c = dict(DEFAULT_CAPS)
        # rdm scenes default to EnvConfig.max_vehicles vehicles (scene_generator.py:100); scenarios add <= 3
        c["actor_cap"] = max(c["actor_cap"], int(self.cfg.max_vehicles) + 4)
        c.update(caps or {})
        self.caps = LY.Caps(**c)
        L = lib()
        self.layout = LY.check_library_layout(L, self.caps)
        self.rb = self.layout.record_bytes
        ctx = ctypes.c_void_p()
        check(L.cbev_create(ctypes.byref(self.params), ctypes.byref(self.caps.c()), self.device.index or 0,
                            ctypes.byref(ctx)), "cbev_create")
        self._ctx = ctx
        check(L.cbev_set_map(ctx, self.map_host.ctypes.data_as(ctypes.c_void_p), self.map_host.nbytes), "cbev_set_map")
        if self.cfg.fov_masked:  # FovRenderSpec(mask_fov=fov_masked), world.py:40-46
            self.fov_mask = fov_corner_mask(self.cfg.size)
            check(L.cbev_set_fov_mask(ctx, self.fov_mask.ctypes.data_as(ctypes.c_void_p)), "cbev_set_fov_mask")
        N, S, F = self.num_envs, self.S, self.F
        dev = self.device
        # ResizeObservation(obs_size) (envs/__init__.py:62): frames are rendered at S x S and
        # resized on the device into the (h, w) frame ring
        self.obs_hw = (int(self.cfg.obs_size[0]), int(self.cfg.obs_size[1])) if self.wrappers else (S, S)
        self.resize = self.obs_hw != (S, S)
        if self.resize:
            check(L.cbev_set_obs_size(ctx, self.obs_hw[0], self.obs_hw[1]), "cbev_set_obs_size")
        h, w = self.obs_hw
        # records, frame ring and term flags: reached through the properties below,
        # which apply a deferred reset first
        self._reset_pending = False
        self._records = torch.zeros((N, self.rb), dtype=torch.uint8, device=dev)
        self._ring = torch.zeros((F, N, h, w), dtype=torch.uint8, device=dev)
        # render-size frame of the current step (render(), carlabev.py:233-249); the
        # newest ring slot itself when there is no resize
        self.full = torch.zeros((N, S, S), dtype=torch.uint8, device=dev) if self.resize else None
        self.head = 0
        self.reward = torch.zeros(N, dtype=torch.float64, device=dev)
        self._term = torch.zeros(N, dtype=torch.uint8, device=dev)
        self.trunc = torch.zeros(N, dtype=torch.uint8, device=dev)
        self.cause = torch.zeros(N, dtype=torch.int32, device=dev)
        self.info = torch.zeros((N, 16), dtype=torch.float32, device=dev)
        # device addresses of the per-step buffers (allocated once here): the step's
        # host path passes them as plain ints instead of re-reading tensor metadata
        self._p_step = tuple(t.data_ptr() for t in (self._records, self.reward, self._term, self.trunc, self.cause,
                                                      self.info))
        self._p_ring, self._slot_bytes = self._ring.data_ptr(), N * h * w
        # the canonical reset folded into the next step (frames are rendered straight
        # into the ring only without a resize)
        check(L.cbev_set_deferred_reset(ctx, 1 if (defer_reset and not self.resize) else 0), "cbev_set_deferred_reset")
        self._p_full = self.full.data_ptr() if self.full is not None else None
        self._dev_index = dev.index if dev.index is not None else torch.cuda.current_device()
        # spaces (envs/spaces.py:27-61 + wrapper spaces)
        aspec = get_action_profile_spec(self.cfg.action_profile_id)
        self.discrete = aspec["action_mode"] == "discrete"
        if self.discrete:
            self.single_action_space = make_discrete(len(aspec["discrete_actions"]))
        else:
            self.single_action_space = make_box(np.asarray(aspec["low"], np.float32),
                                                np.asarray(aspec["high"], np.float32), (3,), np.float32)
        if not self.wrappers:
            if self.cfg.obs_mode == "vector":
                self.single_observation_space = make_box(-np.inf, np.inf, (7,), np.float32)
                self.obs_buf = torch.zeros((N, 7), dtype=torch.float32, device=dev)
            else:
                self.single_observation_space = make_box(0, 255, (S, S, 3), np.uint8)
                self.obs_buf = torch.zeros((N, S, S, 3), dtype=torch.uint8, device=dev)
        elif self.cfg.masked:
            self.channels = semantic_mask_channels(self.cfg.semantic_mask_ch)
            C = len(self.channels)
            fusion = self.cfg.temporal_fusion_mode
            Cw = OP.fused_channels(self.cfg.semantic_mask_ch, fusion, F)
            self.single_observation_space = make_box(0.0, 1.0, (Cw, h, w), np.float32)
            self._obs_kind, self._obs_lut, self._obs_ch = OP.FUSION_KIND[fusion], semantic_lut(self.cfg.semantic_mask_ch), C
            self.obs_buf = torch.zeros((N, Cw, h, w), dtype=torch.float32, device=dev)
        else:
            self.single_observation_space = make_box(0, 255, (F, h, w), np.uint8)
            self._obs_kind = OP.KIND_GRAY_RAW if self.resize else OP.KIND_GRAY
            self._obs_lut, self._obs_ch = gray_lut(), 1
            self.obs_buf = torch.zeros((N, F, h, w), dtype=torch.uint8, device=dev)
        self.observation_space = batch_space(self.single_observation_space, N)
        self.action_space = batch_space(self.single_action_space, N)
        seed = getattr(run, "seed", self.cfg.seed)
        self.single_action_space.seed(seed)
        self.generator = scene_generator or SceneGenerator(self.cfg, self.cfg.map_name)
        self.builder = HostResetBuilder(self.cfg, self.classes, self.params, self.layout, self.generator)
        self._ctx_id_off = self.layout.off["hi"] + 4 * LY.HI["CTX_ID"]  # byte offset of a record's CTX_ID
        self.reset_pool = reset_pool
        self.pool_builds = 0  # scenes reset() had the pool build
        self.scene_context = [dict() for _ in range(N)]
        # scenario contexts by id (records carry CTX_ID): bank rows' ids stay, an env's
        # host-reset id is released at its next host reset
        self._ctx_table: dict[int, dict] = {0: {}}
        self._ctx_next = 1
        self._env_ctx = np.zeros(N, dtype=np.int64)
        self._pending: deque = deque()  # (step, weakref(StepInfos)) not yet read
        self._ep_step = 0
        if info_mode == "full":  # Stats on the device (cbev_set_episode_stats)
            self._ep_stats = torch.zeros((N, LY.STATS_BYTES), dtype=torch.uint8, device=dev)
            self._ep_rows = torch.zeros((EP_RING, N, len(LY.EP)), dtype=torch.float64, device=dev)
            self._ep_counts = torch.zeros(EP_RING, dtype=torch.int32, device=dev)
            check(L.cbev_set_episode_stats(ctx, _ptr(self._ep_stats), N, _ptr(self._ep_rows), _ptr(self._ep_counts),
                                           EP_RING), "cbev_set_episode_stats")
        self.bank = None
        self._all_mask = None  # uint8 ones: reset_from_bank(mask=None) without bank_idx
        self._bank_ctx_ids = None  # scenario-context id per bank row set by refresh_bank
        self._retired_ctx: deque = deque()  # ids of overwritten bank rows, released oldest first
        # (id, step) of scenario contexts reset() replaced: released once no unread
        # StepInfos can refer to them (those of steps up to EP_RING back are read by then)
        self._host_retired: deque = deque()
        self._stepped = False
        self._step_stream = 0
        self.auto_obs = True  # reset_from_bank also expands the wire observation
        self._closed = False

    # ------------------------------------------------------------------ state (deferred reset applied first)
    def flush(self):
        """Apply a reset_terminated() the next step has not taken yet (cbev_flush;
        stream-ordered, no sync). Every accessor below calls it."""
        if self._reset_pending:
            self._reset_pending = False
            check(lib().cbev_flush(self._ctx), "cbev_flush")

    @property
    def records(self) -> torch.Tensor:
        self.flush()
        return self._records

    @property
    def ring(self) -> torch.Tensor:
        self.flush()
        return self._ring

    @property
    def term(self) -> torch.Tensor:
        self.flush()
        return self._term

    # ------------------------------------------------------------------ helpers
    def _stream(self):
        # the caller's current stream on the env's device (raw handle: no Stream object per call)
        return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(self._dev_index))

    def _new_record_buffer(self, n: int) -> np.ndarray:
        return np.zeros((n, self.rb), dtype=np.uint8)

    def build_reset_record(self, buf: np.ndarray, seed, options: dict, env_index: int = 0):
        return self.builder.build(buf, seed, options)

    def _check_records(self, recs, what: str):
        """Refuse device or host records a StopReturn actor of which the narrow
        k_actors could not retreat (layout.retreat_route_violations)."""
        if self.caps.actor_cap == 0 or self.caps.actor_cap > 64:
            return
        o = self.layout.off
        nhi, nai = 4 * len(LY.HI), 4 * len(LY.AI) * self.caps.actor_cap
        if isinstance(recs, torch.Tensor):
            hi = recs[:, o["hi"]:o["hi"] + nhi].cpu().numpy()
            ai = recs[:, o["ai"]:o["ai"] + nai].cpu().numpy()
        else:
            hi, ai = recs[:, o["hi"]:o["hi"] + nhi], recs[:, o["ai"]:o["ai"] + nai]
        hi = np.ascontiguousarray(hi).view(np.int32).reshape(len(hi), len(LY.HI))
        ai = np.ascontiguousarray(ai).view(np.int32).reshape(len(ai), len(LY.AI), self.caps.actor_cap)
        bad = np.flatnonzero(LY.retreat_route_violations(hi, ai, self.caps))
        if bad.size:
            raise ValueError(f"{what}: record {int(bad[0])} (of {bad.size}) has a yield_return actor whose retreat "
                             f"route would exceed min(actor_route_cap, 64) points (scene_pack refuses such actors)")

    def _mask_array(self, mask) -> np.ndarray:
        if mask is None:
            return np.ones(self.num_envs, dtype=bool)
        if isinstance(mask, torch.Tensor):
            mask = mask.detach().to("cpu").numpy()
        m = np.asarray(mask, dtype=bool).reshape(-1)
        if m.size != self.num_envs:
            raise ValueError(f"reset_mask has {m.size} entries, expected {self.num_envs}")
        return m

    # ------------------------------------------------------------------ scene bank (device-side reset)
    def attach_bank(self, bank_records: torch.Tensor, contexts=None):
        """Use a pre-built scene bank (B packed records on this device) for partial resets
        without per-reset host work."""
        if bank_records.device != self.device or bank_records.dtype != torch.uint8 or bank_records.shape[1] != self.rb:
            raise ValueError("bank must be a (B, record_bytes) uint8 tensor on the env device")
        self._check_records(bank_records, "attach_bank")
        self.flush()  # a deferred reset reads the old bank
        self.bank = bank_records.contiguous()
        self.bank_contexts = contexts
        # reset observations of the bank, rendered once; reset_from_bank then only copies
        B, S = self.bank.shape[0], self.S
        self.bank_frames = torch.empty((B, S, S), dtype=torch.uint8, device=self.device)
        self._p_bank, self._p_bank_frames = self.bank.data_ptr(), self.bank_frames.data_ptr()
        check(lib().cbev_bank_frames(self._ctx, _ptr(self.bank), B, _ptr(self.bank_frames), self._stream()),
              "cbev_bank_frames")

    RETIRED_CTX_KEEP = 1 << 16  # contexts of overwritten bank rows checked for release past this many

    def refresh_bank(self, slot0: int, records: np.ndarray, contexts=None) -> int:
        """Write k fresh scene records (uint8[k][record_bytes], e.g. from a ScenePool)
        into bank rows slot0, slot0 + 1, ... (wrapping) and render their cached reset
        frames; stream-ordered, no sync. Returns the next slot.

        contexts: the k scenes' scenario-context dicts (ScenePool.poll(contexts=True));
        each gets an id written into its record's CTX_ID, so episodes reset from the
        row report it in episode_info as the reference merges _scenario_context
        (carlabev.py:182). The id of an overwritten row is retired: envs may still run
        that scene, so once more than RETIRED_CTX_KEEP (or 2 N) ids are retired, the
        pending infos are read and the retired ids no env's record carries any more are
        released (one device read of the records' CTX_ID words)."""
        if self.bank is None:
            raise RuntimeError("no scene bank attached")
        self.flush()  # a deferred reset reads the rows about to be overwritten
        B, k = self.bank.shape[0], int(records.shape[0])
        if k == 0:
            return slot0
        if records.shape[1] != self.rb or k > B:
            raise ValueError(f"expected at most {B} records of {self.rb} bytes")
        self._check_records(records, "refresh_bank")
        if contexts is not None:
            if len(contexts) != k:
                raise ValueError(f"{len(contexts)} contexts for {k} records")
            records = np.array(records, copy=True)
            if self._bank_ctx_ids is None or self._bank_ctx_ids.shape[0] != B:
                self._bank_ctx_ids = np.zeros(B, dtype=np.int64)
            ci = LY.HI["CTX_ID"]
            for j in range(k):
                row = (slot0 + j) % B
                old = int(self._bank_ctx_ids[row])
                if old:
                    self._retired_ctx.append(old)
                cid = self._new_ctx_id(contexts[j])
                self._bank_ctx_ids[row] = cid
                LY.RecordView(records[j], self.layout).hi[ci] = cid
            if len(self._retired_ctx) > max(self.RETIRED_CTX_KEEP, 2 * self.num_envs):
                self._release_retired_contexts()
        src = torch.from_numpy(np.ascontiguousarray(records)).pin_memory()
        done = 0
        s = slot0 % B
        while done < k:
            m = min(k - done, B - s)
            self.bank[s:s + m].copy_(src[done:done + m], non_blocking=True)
            check(lib().cbev_bank_frames(self._ctx, _ptr(self.bank[s:s + m]), m, _ptr(self.bank_frames[s:s + m]),
                                         self._stream()), "cbev_bank_frames")
            done += m
            s = (s + m) % B
        self._refresh_keep = src  # the pinned staging must outlive the async copy
        return s

    def record_ctx_ids(self) -> np.ndarray:
        """CTX_ID of every env's record as it is now (synchronises)."""
        o = self.layout.off["hi"] + 4 * LY.HI["CTX_ID"]
        return self.records[:, o:o + 4].contiguous().view(torch.int32).reshape(-1).cpu().numpy()

    def _release_retired_contexts(self):
        """Forget the retired scenario contexts that no env runs and no unread
        StepInfos refers to (the pending ones are read first)."""
        self._flush_pending(all_=True)
        live = set(self.record_ctx_ids().tolist())
        keep = deque()
        while self._retired_ctx:
            cid = self._retired_ctx.popleft()
            if cid in live:
                keep.append(cid)
            else:
                self._ctx_table.pop(cid, None)
        self._retired_ctx = keep

    def termination_count(self) -> int:
        """Episodes terminated so far on this env's device context (synchronises)."""
        n = ctypes.c_int64()
        check(lib().cbev_termination_count(self._ctx, ctypes.byref(n)), "cbev_termination_count")
        return int(n.value)

    def _new_ctx_id(self, ctx: dict) -> int:
        cid = self._ctx_next
        self._ctx_next += 1
        self._ctx_table[cid] = ctx
        return cid

    def build_bank(self, seeds, options: dict | None = None) -> torch.Tensor:
        """B seeded scenes as device records; each carries its scene scalars and the
        id of its scenario context, so a bank reset reports them in episode_info."""
        options = dict(options or {})
        host = self._new_record_buffer(len(seeds))
        for k, s in enumerate(seeds):
            _, _, ctx = self.build_reset_record(host[k], s, dict(options, scene_seed=int(s)))
            LY.RecordView(host[k], self.layout).hi[LY.HI["CTX_ID"]] = self._new_ctx_id(ctx)
        return torch.from_numpy(host).to(self.device)

    def reset_terminated(self):
        """The canonical loop's reset(reset_mask=terminated) on the device: every env
        whose `term` flag is set when the launch runs (the last step's, including any
        in-place edit of env.term since) <- its next bank row (env e takes
        bank[(e + j * stride) % B], j = its terminations so far, stride =
        cbev_bank_stride(B) coprime with B, so each env walks the whole bank before a
        scene repeats for it), reset frame into every frame-stack slot. One launch
        (or none: folded into the next step), no host sync."""
        if self.bank is None:
            raise RuntimeError("no scene bank attached")
        if not self._stepped:
            raise RuntimeError("reset_terminated before any step()")
        if self.resize:
            return self._reset_masked(self._term)
        # cbev_reset_terminated: recorded for the next step to fold in (cbev_set_deferred_reset)
        # or launched at once; its mask is the term buffer of the last step (this env's)
        check(lib().cbev_reset_terminated(self._ctx, self._p_step[0], self.num_envs, self._p_bank, self.bank.shape[0],
                                          self._p_bank_frames, self._p_ring, self.F, self._stream()),
              "cbev_reset_terminated")
        self._reset_pending = bool(lib().cbev_reset_pending(self._ctx))
        if not self.auto_obs:
            return None
        return self._obs()

    def _reset_masked(self, mask: torch.Tensor):
        N, B = self.num_envs, self.bank.shape[0]
        rec = self._p_step[0]
        if self.resize:
            check(lib().cbev_reset_masked(self._ctx, rec, N, mask.data_ptr(), self._p_bank, B, self._p_bank_frames,
                                          self._p_full, 1, self._stream()), "cbev_reset_masked")
            self._resize_into_ring(mask, all_slots=True)
        else:
            check(lib().cbev_reset_masked(self._ctx, rec, N, mask.data_ptr(), self._p_bank, B, self._p_bank_frames,
                                          self._p_ring, self.F, self._stream()), "cbev_reset_masked")
        if not self.auto_obs:
            return None
        return self._obs()

    def bank_rows_used(self) -> int:
        """Bank rows the masked resets (reset_terminated, reset_from_bank without
        bank_idx) have handed out since the env was created (synchronises)."""
        n = ctypes.c_int64()
        check(lib().cbev_bank_cursor(self._ctx, ctypes.byref(n)), "cbev_bank_cursor")
        return int(n.value)

    def reset_counts(self) -> np.ndarray:
        """Per-env termination counts j (uint32[N], synchronises): a masked reset of
        env e takes bank row (e + j * cbev_bank_stride(B)) % B."""
        out = np.zeros(self.num_envs, np.uint32)
        check(lib().cbev_reset_counts(self._ctx, out.ctypes.data_as(ctypes.c_void_p), self.num_envs),
              "cbev_reset_counts")
        return out

    @staticmethod
    def bank_rows_between(c0: np.ndarray, c1: np.ndarray, n_bank: int) -> np.ndarray:
        """The bank rows the canonical loop's resets took between two reset_counts()
        readings (each termination reset: counts c0 + 1 .. c1)."""
        c0, c1 = c0.astype(np.int64), c1.astype(np.int64)
        d = c1 - c0
        e = np.repeat(np.arange(len(c0), dtype=np.int64), d)
        j = np.repeat(c0 + 1, d) + (np.arange(int(d.sum()), dtype=np.int64) - np.repeat(np.cumsum(d) - d, d))
        return (e + j * int(lib().cbev_bank_stride(n_bank))) % n_bank

    def reset_from_bank(self, mask: torch.Tensor | None = None, bank_idx: torch.Tensor | None = None):
        """Device-only partial reset from the scene bank, reset frame into every
        frame-stack slot. One launch, no host sync.
        Without bank_idx: the envs selected by mask (all when None; its contents as
        the launch reads them) take the bank rows of their termination counts
        (reset_terminated's per-env rule; reset_terminated is this with mask = env.term).
        With bank_idx: env i (mask[i]) <- bank[bank_idx[i]]; the cursor is untouched."""
        if self.bank is None:
            raise RuntimeError("no scene bank attached")
        N, B = self.num_envs, self.bank.shape[0]
        if mask is not None:
            mask = torch.as_tensor(mask)
            if mask.numel() != N:
                raise ValueError(f"reset mask has {mask.numel()} entries, expected {N}")
            mask = mask.reshape(N).to(device=self.device, dtype=torch.uint8).contiguous()
        if bank_idx is None:
            if mask is None:
                if self._all_mask is None:
                    self._all_mask = torch.ones(N, dtype=torch.uint8, device=self.device)
                mask = self._all_mask
            return self._reset_masked(mask)
        bank_idx = torch.as_tensor(bank_idx)  # the kernels read N int32 bank rows on this device
        if bank_idx.numel() != N:
            raise ValueError(f"bank_idx has {bank_idx.numel()} entries, expected {N}")
        bank_idx = bank_idx.reshape(N).to(device=self.device, dtype=torch.int32).contiguous()
        if self.resize:
            check(lib().cbev_reset_frames(self._ctx, _ptr(self.records), N, _ptr(self.bank), B, _ptr(mask),
                                          _ptr(bank_idx), 0, _ptr(self.bank_frames), _ptr(self.full), 1,
                                          self._stream()), "cbev_reset_frames")
            self._resize_into_ring(mask, all_slots=True)
        else:
            check(lib().cbev_reset_frames(self._ctx, _ptr(self.records), N, _ptr(self.bank), B, _ptr(mask),
                                          _ptr(bank_idx), 0, _ptr(self.bank_frames), _ptr(self.ring), self.F,
                                          self._stream()), "cbev_reset_frames")
        if not self.auto_obs:
            return None
        return self._obs()

    def load_scenes(self, records: torch.Tensor):
        """Every env <- records[i] (N packed records on this device, e.g. the seeded
        start scenes), reset observation rendered into every frame-stack slot; the
        bank and its cursor are untouched. One launch."""
        N = self.num_envs
        if records.device != self.device or records.dtype != torch.uint8 or tuple(records.shape) != (N, self.rb):
            raise ValueError(f"expected a ({N}, {self.rb}) uint8 tensor on {self.device}")
        records = records.contiguous()
        self._check_records(records, "load_scenes")
        dst = self.full if self.resize else self.ring
        check(lib().cbev_reset(self._ctx, _ptr(self.records), N, _ptr(records), N, None, None, 0, _ptr(dst),
                               1 if self.resize else self.F, self._stream()), "cbev_reset")
        if self.resize:
            self._resize_into_ring(None, all_slots=True)

    def _resize_into_ring(self, mask: torch.Tensor | None, all_slots: bool):
        """ResizeObservation + the mask/grayscale colour test of self.full into the ring:
        the newest slot after a step, every slot of the masked envs after a reset."""
        h, w = self.obs_hw
        N = self.num_envs
        dst = self.ring[0] if all_slots else self.ring[self.head]
        check(lib().cbev_resize_obs(self._ctx, _ptr(self.full), N, _ptr(mask), 0 if self.cfg.masked else 1, _ptr(dst),
                                    self.F if all_slots else 1, N * h * w, self._stream()), "cbev_resize_obs")

    # ------------------------------------------------------------------ gymnasium surface
    def reset(self, seed=None, options=None):
        options = dict(options or {})
        mask = self._mask_array(options.pop("reset_mask", None))
        N = self.num_envs
        if seed is None:
            seeds = [None] * N
        elif isinstance(seed, (int, np.integer)):
            seeds = [int(seed) + i for i in range(N)]
        else:
            seeds = list(seed)
        idx = np.flatnonzero(mask)
        host = self._new_record_buffer(max(len(idx), 1))
        spawn_infos = []
        # contexts replaced by earlier resets that no StepInfos can still refer to:
        # released (StepInfos of steps <= _ep_step - EP_RING have been read or dropped,
        # _flush_pending); this reset's replaced ones wait their turn
        while self._host_retired and self._host_retired[0][1] <= self._ep_step - EP_RING:
            self._ctx_table.pop(self._host_retired.popleft()[0], None)
        key_of_seed = {}  # memo keys, once per distinct seed of this call

        def key_of(i):
            sd = seeds[i]
            try:
                k = key_of_seed.get(sd, key_of_seed)
            except TypeError:  # an unhashable seed: its own key
                return self.builder.memo_key(sd, options)
            if k is key_of_seed:
                k = key_of_seed[sd] = self.builder.memo_key(sd, options)
            return k

        if self.reset_pool is not None and len(idx) > 1:
            # the distinct scenes not memoised yet, built by the pool's workers and
            # memoised here; the loop below then copies them
            todo = {}
            for i in idx.tolist():
                key = key_of(i)
                if key is not None and key not in todo and self.builder.memo_get(key) is None:
                    todo[key] = i
            if len(todo) > 1:
                recs, meta = self.reset_pool.build([(seeds[i], options) for i in todo.values()])
                for key, rec, (info, ctx) in zip(todo, recs, meta):
                    self.builder.memo_put(key, rec, info, None, ctx)
                self.pool_builds += len(todo)
        ctx_ids = host[:, self._ctx_id_off:self._ctx_id_off + 4].view(np.int32)[:, 0] if len(idx) else None
        for k, i in enumerate(idx.tolist()):
            info, spec, ctx = self.builder.build(host[k], seeds[i], options, key_of(i))
            spawn_infos.append(info)
            self.scene_context[i] = ctx
            old = int(self._env_ctx[i])
            if old:
                self._host_retired.append((old, self._ep_step))
            cid = self._new_ctx_id(ctx)
            self._env_ctx[i] = cid
            ctx_ids[k] = cid  # the record's CTX_ID
        if len(idx):
            staging = torch.from_numpy(host[:len(idx)]).to(self.device)
            bank_idx = np.zeros(N, dtype=np.int32)
            bank_idx[idx] = np.arange(len(idx), dtype=np.int32)
            bidx = torch.from_numpy(bank_idx).to(self.device)
            m = torch.from_numpy(mask.astype(np.uint8)).to(self.device)
            if self.resize:
                check(lib().cbev_reset(self._ctx, _ptr(self.records), N, _ptr(staging), len(idx), _ptr(m), _ptr(bidx),
                                       0, _ptr(self.full), 1, self._stream()), "cbev_reset")
                self._resize_into_ring(m, all_slots=True)
            else:
                check(lib().cbev_reset(self._ctx, _ptr(self.records), N, _ptr(staging), len(idx), _ptr(m), _ptr(bidx),
                                       0, _ptr(self.ring), self.F, self._stream()), "cbev_reset")
        obs = self._obs()
        infos = {}
        if len(idx):
            infos["spawn_validation"] = np.array([None] * N, dtype=object)
            infos["_spawn_validation"] = mask.copy()
            infos["scenario"] = np.array([None] * N, dtype=object)
            infos["_scenario"] = mask.copy()
            for k, i in enumerate(idx):
                infos["spawn_validation"][i] = spawn_infos[k]
                infos["scenario"][i] = self.scene_context[i]
        return obs, infos

    def _actions_tensor(self, actions) -> torch.Tensor:
        if isinstance(actions, torch.Tensor) and actions.device == self.device and actions.is_contiguous() and (
                actions.dtype == (torch.int32 if self.discrete else torch.float32)):
            return actions  # device indices out of range set CBEV_ERR_ACTION_INDEX (errors())
        if self.discrete and not (isinstance(actions, torch.Tensor) and actions.device.type != "cpu"):
            # host actions: the reference's discrete_actions[int(action)] IndexError (spaces.py:46)
            n = self.single_action_space.n
            a_np = np.asarray(actions.cpu() if isinstance(actions, torch.Tensor) else actions).reshape(-1)
            bad = (a_np < -n) | (a_np >= n)
            if bad.any():
                raise IndexError(f"discrete action {a_np[bad][0]} out of range for Discrete({n})")
        a = torch.as_tensor(actions, device=self.device)
        if self.discrete:
            a = a.reshape(self.num_envs).to(torch.int32).contiguous()
        else:
            a = a.reshape(self.num_envs, 3).to(torch.float32).contiguous()
        return a

    def step_async_only(self, actions):
        """Enqueue one step; returns nothing and never synchronises (bench path)."""
        a = self._actions_tensor(actions)
        if self.info_mode == "full":
            self._flush_pending()
            self._ep_step += 1
        self.head = (self.head + 1) % self.F
        frames = self._p_full if self.resize else self._p_ring + self.head * self._slot_bytes
        rec, rew, term, trunc, cause, info = self._p_step
        stream = self._stream()
        check(lib().cbev_step(self._ctx, rec, self.num_envs, a.data_ptr(), frames, rew, term, trunc, cause, info,
                              stream), "cbev_step")
        self._reset_pending = False  # taken by this step (or launched before it)
        self._step_stream = stream.value or 0  # the step's rows are waited for on this stream (StepInfos)
        self._stepped = True
        if self.resize:
            self._resize_into_ring(None, all_slots=False)
        return a

    def errors(self, clear: bool = True) -> int:
        """CBEV_ERR_* bits the kernels raised since the last call (synchronises the
        device): ERR_ACTION_INDEX (1) = a device action tensor held a discrete index outside
        [-n, n), the reference's IndexError; that env stepped action 0.
        ERR_RASTER_WINDOW (2) = a raster tile's crop window exceeded its LDS bound
        (an internal invariant the GPU parity tests assert; that frame is not valid).
        ERR_RETREAT_ROUTE (4) = a StopReturn actor's retreat route would exceed 64
        points (records not written by scene_pack, which refuses such actors)."""
        flags = ctypes.c_int32()
        check(lib().cbev_error_flags(self._ctx, ctypes.byref(flags), 1 if clear else 0), "cbev_error_flags")
        return int(flags.value)

    def step(self, actions):
        self.step_async_only(actions)
        obs = self._obs()
        rew = self.reward.clone()
        term = self.term.bool()
        trunc = self.trunc.bool()
        infos = self.step_infos()
        if self.info_mode == "device":
            infos = {"cause": self.cause.clone(), "comfort": self.info[:, :11].clone()}
        return obs, rew, term, trunc, infos

    def _obs(self):
        """The wire observation of every env. copy_obs: expanded straight into a
        new tensor (from torch's caching allocator, on the current stream), so the
        caller's earlier observations stay as they were without a clone pass (at
        config 2 a wire observation is 6.4 GB: expanding it once costs ≈ 1.3 ms, a
        clone 2.5 ms more); otherwise into the env's one buffer."""
        out = torch.empty_like(self.obs_buf) if self.copy_obs else self.obs_buf
        if not self.wrappers:
            if self.cfg.obs_mode == "vector":
                check(lib().cbev_vector_obs(self._ctx, _ptr(self.records), self.num_envs, _ptr(out),
                                            self._stream()), "cbev_vector_obs")
            else:
                check(lib().cbev_expand_obs(self._ctx, _ptr(self.frames()[None]), self.num_envs, 1, 0, 2, 3,
                                            rgb_lut().ctypes.data_as(ctypes.c_void_p), _ptr(out),
                                            self._stream()), "cbev_expand_obs")
            return out
        check(lib().cbev_expand_obs(self._ctx, _ptr(self.ring), self.num_envs, self.F, self.head, self._obs_kind,
                                    self._obs_ch, self._obs_lut.ctypes.data_as(ctypes.c_void_p), _ptr(out),
                                    self._stream()), "cbev_expand_obs")
        return out

    def step_infos(self):
        """`infos` of the step just queued: a StepInfos (info_mode="full"), read
        from the device only when accessed; {} otherwise."""
        if self.info_mode != "full":
            return {}
        infos = StepInfos(self, self._ep_step - 1, self._step_stream_obj())
        self._pending.append((self._ep_step - 1, weakref.ref(infos)))
        return infos

    def _step_stream_obj(self):
        """The torch Stream of the last step (its raw handle kept by step_async_only)."""
        if not self._step_stream:
            return None
        cur = torch.cuda.current_stream(self.device)
        if cur.cuda_stream == self._step_stream:
            return cur
        return torch.cuda.ExternalStream(self._step_stream, device=self.device)

    def _flush_pending(self, all_: bool = False):
        """Read the StepInfos whose device rows the next step would recycle (or all,
        all_=True) if the caller still holds them; forget the rest."""
        limit = self._ep_step + 1 - EP_RING  # step self._ep_step zeroes the slot of this step
        while self._pending and (all_ or self._pending[0][0] <= limit):
            _, ref = self._pending.popleft()
            obj = ref()
            if obj is not None:
                obj._get()

    def _materialize_infos(self, step: int, stream=None) -> dict:
        """Vector-env infos of `step` from its device rows (SyncVectorEnv._add_info
        layout: {"episode_info": {key: array, "_key": mask}, "_episode_info": mask,
        "episode": {"r", "l", "t"} + masks, "_episode": mask}; {} when no env
        terminated). The scenario context is merged as carlabev.py:181-182 does.
        Waits for the stream the step was launched on (`stream`, a torch Stream
        the StepInfos holds; None: the legacy default stream), not the whole device: RCCL gathers and the
        caller's other streams keep running. A step's rows stay valid until
        EP_RING - 1 newer steps are queued, and _flush_pending reads them before
        that, so a step enqueues no event or other marker for its infos."""
        if stream is not None:
            stream.synchronize()
        else:
            torch.cuda.default_stream(self.device).synchronize()
        slot = step % EP_RING
        cnt = min(int(self._ep_counts[slot].item()), self.num_envs)  # a slot holds at most N rows
        if cnt == 0:
            return {}
        rows = self._ep_rows[slot, :cnt].cpu().numpy()
        rows = rows[np.argsort(rows[:, LY.EP["ENV"]], kind="stable")]
        N = self.num_envs
        env_ids = rows[:, LY.EP["ENV"]].astype(np.int64)
        summary: dict = {}
        for key, col, typ in _EP_KEYS:
            c = rows[:, LY.EP[col]]
            if key == "termination":
                vals = [LY.CAUSE_NAME.get(int(v)) for v in c]
            elif typ is int:
                vals = [int(v) for v in c]
            else:
                vals = [float(v) for v in c]
            summary[key] = dict(zip(env_ids.tolist(), vals))
        for j, i in enumerate(env_ids.tolist()):
            ctx = self._ctx_table.get(int(rows[j, LY.EP["CTX_ID"]]), {})
            for k, v in ctx.items():
                summary.setdefault(k, {})[i] = v
        done = np.zeros(N, dtype=np.bool_)
        done[env_ids] = True
        episode = {"r": dict(zip(env_ids.tolist(), rows[:, LY.EP["RETURN"]].tolist())),
                   "l": dict(zip(env_ids.tolist(), rows[:, LY.EP["LENGTH"]].astype(np.int64).tolist())),
                   "t": dict(zip(env_ids.tolist(), np.round(rows[:, LY.EP["SECONDS"]], 6).tolist()))}
        return {"episode_info": _batched(summary, N), "_episode_info": done,
                "episode": _batched(episode, N), "_episode": done.copy()}

    def render(self):
        """Tuple of per-env (S, S, 3) uint8 RGB frames, like SyncVectorEnv.render()."""
        ids = self.frames().to("cpu").numpy()
        rgb = PALETTE[ids]
        return tuple(rgb[i] for i in range(self.num_envs))

    def render_device(self) -> torch.Tensor:
        out = torch.empty((self.num_envs, self.S, self.S, 3), dtype=torch.uint8, device=self.device)
        check(lib().cbev_expand_obs(self._ctx, _ptr(self.frames()[None]), self.num_envs, 1, 0, 2, 3,
                                    rgb_lut().ctypes.data_as(ctypes.c_void_p), _ptr(out), self._stream()),
              "cbev_expand_obs")
        return out

    def frames(self) -> torch.Tensor:
        """Newest render-size palette-id frames (N, S, S) uint8 (compact observation)."""
        return self.full if self.resize else self.ring[self.head]  # self.ring applies a deferred reset

    def records_host(self) -> np.ndarray:
        return self.records.to("cpu").numpy()

    def close(self):
        if not self._closed and getattr(self, "_ctx", None):
            torch.cuda.synchronize(self.device)
            lib().cbev_destroy(self._ctx)
            self._ctx = None
            self._closed = True

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def make_env(cfg, eval: bool = False, **kwargs) -> CarlaBEVVectorEnv:  # noqa: A002 - reference signature
    """Mirror of `CarlaBEV.envs.make_env(cfg, eval=False)` (envs/__init__.py:108-120)."""
    env = CarlaBEVVectorEnv(cfg, **kwargs)
    if eval:
        env.single_action_space.seed(999)
    return env
