"""Host half of `CarlaBEV.reset` (carlabev.py:96-148): seeds -> scene -> record.

Kept free of torch/HIP so the same builder feeds the device (vector_env) and
the CPU tests/oracle with byte-identical records.
"""
from __future__ import annotations

import numpy as np

from . import layout as LY
from .params import CbevParams
from .scene_gen import SceneGenerator, build_rng_bundle
from .scene_pack import pack_scene
from .semantics import PALETTE


class HostResetBuilder:
    def __init__(self, cfg, classes: np.ndarray, params: CbevParams, layout: LY.Layout,
                 generator: SceneGenerator | None = None):
        self.cfg = cfg
        self.classes = classes
        self.P = params
        self.layout = layout
        self.generator = generator or SceneGenerator(cfg, cfg.map_name)

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

    def build(self, buf: np.ndarray, seed, options: dict):
        """Fill `buf` (one zeroed record) for CarlaBEV.reset(seed, options).
        Returns (spawn_validation, spec, scenario_context)."""
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
