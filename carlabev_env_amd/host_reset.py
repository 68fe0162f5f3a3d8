"""Host half of `CarlaBEV.reset` (carlabev.py:96-148): seeds -> scene -> record.

Kept free of torch/HIP so the same builder feeds the device (vector_env) and
the CPU tests/oracle with byte-identical records.

A reset's scene is a pure function of its seeds and options (every random draw
comes from the RNG bundle built from them, carlabev.py:83-94), so built
records are memoised by (scene seed, options): the reference's canonical loop
resets with `options={"reset_mask": done, ...}` and no seed, which makes every
env rebuild the scene of `cfg.seed` on every reset (carlabev.py:84); here the
repeated build is a copy of the same bytes.
"""
from __future__ import annotations

import copy
import os
from collections import OrderedDict

import numpy as np

from . import layout as LY
from .params import CbevParams
from .scene_gen import SceneGenerator, build_rng_bundle
from .scene_pack import pack_scene
from .semantics import PALETTE


def _freeze(v):
    """A hashable, order-preserving form of an options value (TypeError if none)."""
    if isinstance(v, dict):
        return ("d",) + tuple((k, _freeze(x)) for k, x in v.items())
    if isinstance(v, (list, tuple)):
        return ("l",) + tuple(_freeze(x) for x in v)
    if isinstance(v, np.ndarray):
        return ("a", v.dtype.str, v.shape, v.tobytes())
    if isinstance(v, np.generic):
        return v.item()
    hash(v)
    return v


def _copy_plain(v):
    """copy.deepcopy for the plain data of spawn infos and scenario contexts
    (dicts, lists, tuples, arrays, scalars, strings), several times faster; any
    other object goes through copy.deepcopy."""
    if isinstance(v, dict):
        return {k: _copy_plain(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_copy_plain(x) for x in v]
    if isinstance(v, tuple):
        return tuple(_copy_plain(x) for x in v)
    if v is None or isinstance(v, (str, int, float, bool, np.generic)):
        return v
    if isinstance(v, np.ndarray):
        return v.copy()
    return copy.deepcopy(v)


_NO_KEY = object()


class HostResetBuilder:
    MEMO_BYTES = 256 << 20  # memoised records kept (least recently used dropped first)

    def __init__(self, cfg, classes: np.ndarray, params: CbevParams, layout: LY.Layout,
                 generator: SceneGenerator | None = None):
        self.cfg = cfg
        self.classes = classes
        self.P = params
        self.layout = layout
        self.generator = generator or SceneGenerator(cfg, cfg.map_name)
        self._memo: OrderedDict = OrderedDict()
        self._memo_bytes = 0
        self.memo_hits = 0
        self.builds = 0

    def memo_key(self, seed, options: dict):
        """(scene seed, options) of a reset, or None when an option is not hashable.
        An authored scene file is keyed by its path, size and mtime too."""
        opts = {k: v for k, v in options.items() if k != "reset_mask"}
        scene_seed = int(opts.get("scene_seed", self.cfg.seed if seed is None else seed))
        try:
            key = (scene_seed, _freeze(opts))
        except TypeError:
            return None
        for f in (opts.get("config_file"), opts.get("scene")):
            if isinstance(f, str) and f.endswith(".json") and os.path.exists(f):
                st = os.stat(f)
                key += ((f, st.st_size, st.st_mtime_ns),)
        return key

    def spawn_validation(self, view: LY.RecordView) -> dict:
        """Scene.spawn_validation_info (scene.py:142-170) on a packed record."""
        x, y = view.h("X"), view.h("Y")
        h, w = self.classes.shape
        tx = int(np.clip(round(float(x)), 0, w - 1))
        ty = int(np.clip(round(float(y)), 0, h - 1))
        tile = int(self.classes[ty, tx])
        if tile == 0:  # BLOCKING_CLASSES = {NON_DRIVABLE}
            return {"valid": False, "reason": "hero_on_obstacle", "tile": PALETTE[tile].tolist()}
        pad, hw = self.P.pad, self.P.hero_w
        hx, hy = round(pad + x) - hw // 2, round(pad + y) - hw // 2
        for a in range(view.i("NACT")):
            sz = int(view.ai[LY.AI["SIZE"], a])
            ax = round(pad + view.ad[LY.AD["X"], a]) - sz // 2
            ay = round(pad + view.ad[LY.AD["Y"], a]) - sz // 2
            if hw and sz and hx < ax + sz and hy < ay + sz and hx + hw > ax and hy + hw > ay:
                kind = "vehicle" if view.ai[LY.AI["KIND"], a] == 1 else "pedestrian"
                return {"valid": False, "reason": "hero_overlaps_actor", "actor_type": kind,
                        "actor_id": 0 if kind == "vehicle" else 1}
        return {"valid": True, "reason": "ok", "tile": PALETTE[tile].tolist()}

    def memo_get(self, key):
        """(record, spawn_validation, spec, scenario_context) memoised for `key`, or None."""
        hit = self._memo.get(key) if key is not None else None
        if hit is not None:
            self._memo.move_to_end(key)
        return hit

    def memo_put(self, key, rec: np.ndarray, info, spec, ctx):
        if key is None or rec.nbytes > self.MEMO_BYTES:
            return
        if key in self._memo:
            self._memo_bytes -= self._memo.pop(key)[0].nbytes
        self._memo[key] = (np.array(rec, copy=True), _copy_plain(info), spec, _copy_plain(ctx))
        self._memo_bytes += rec.nbytes
        while self._memo_bytes > self.MEMO_BYTES:
            _, (old, *_rest) = self._memo.popitem(last=False)
            self._memo_bytes -= old.nbytes

    def build(self, buf: np.ndarray, seed, options: dict, key=_NO_KEY):
        """Fill `buf` (one record) for CarlaBEV.reset(seed, options).
        Returns (spawn_validation, spec, scenario_context); a repeated (seed,
        options) copies the memoised bytes (the spec object is shared, the dicts
        are copies). `key`: memo_key(seed, options) when the caller has it."""
        if key is _NO_KEY:
            key = self.memo_key(seed, options)
        hit = self.memo_get(key)
        if hit is not None:
            rec, info, spec, ctx = hit
            buf[:] = rec
            self.memo_hits += 1
            return _copy_plain(info), spec, _copy_plain(ctx)
        info, spec, ctx = self._build(buf, seed, options)
        self.builds += 1
        self.memo_put(key, buf, info, spec, ctx)
        return info, spec, ctx

    def _build(self, buf: np.ndarray, seed, options: dict):
        scene_seed = int(options.get("scene_seed", self.cfg.seed if seed is None else seed))
        bundle = build_rng_bundle(scene_seed=scene_seed, route_seed=options.get("route_seed"),
                                  traffic_seed=options.get("traffic_seed"),
                                  scenario_seed=options.get("scenario_seed"))
        max_attempts = int(options.get("max_reset_attempts", 10))
        view = LY.RecordView(buf, self.layout)
        info, spec = None, None
        for _ in range(max_attempts):
            spec = self.generator.build_scene(options, bundle)
            buf[:] = 0
            pack_scene(view, spec, self.cfg.size, scene_id=scene_seed)
            info = self.spawn_validation(view)
            if info["valid"]:
                break
        else:
            raise RuntimeError(f"Failed to reset into a valid initial state after {max_attempts} attempts: {info}")
        # the scene scalars episode_info reports (carlabev.py:180-181), carried by the record
        view.hd[LY.HD["NUM_VEH"]] = float(len(spec.vehicles))
        view.hd[LY.HD["LEN_ROUTE_M"]] = spec.len_route_m if spec.len_route_m is not None else route_length_m(spec)
        ctx = dict(spec.context)
        for k in ("scene", "level", "difficulty_id"):
            if options.get(k) is not None:
                ctx[k] = options[k]
        ctx["scenario_param_scene_seed"] = scene_seed
        ctx["scenario_param_route_seed"] = bundle.route_seed
        ctx["scenario_param_traffic_seed"] = bundle.traffic_seed
        return info, spec, ctx

    def build_many(self, seeds, options_fn) -> tuple[np.ndarray, list]:
        out = np.zeros((len(seeds), self.layout.record_bytes), dtype=np.uint8)
        meta = []
        for k, s in enumerate(seeds):
            meta.append(self.build(out[k], s, options_fn(k, s)))
        return out, meta


def route_length_m(spec) -> float:
    rx = np.asarray(spec.agent_rx, dtype=float)
    ry = np.asarray(spec.agent_ry, dtype=float)
    return float(np.sum(np.hypot(np.diff(rx), np.diff(ry)))) * (40.0 / 128.0)
