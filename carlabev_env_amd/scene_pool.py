"""Host scene feed for fresh seeded resets (host half).

The reference builds a new scene on every reset (`CarlaBEV.reset`,
carlabev.py:96-148 -> `SceneGenerator.build_scene`, scene_generator.py:95-191),
on the CPU, one env at a time. Here the device resets from a scene bank
(`CarlaBEVVectorEnv.reset_from_bank`), so the host's job is to keep that bank
supplied with fresh scenes at the rate the device terminates episodes.

`ScenePool` runs that host work in worker processes (spawned, so they never
inherit a process that has touched the GPU): each builds packed records for
the global scene ids it is handed, seeded as the reference seeds a reset
(scene_seed = seed0 + global id, randomness.py:13-65), and returns the bytes.
The caller drains finished scenes without blocking (`poll`) and writes them
into bank slots (`CarlaBEVVectorEnv.refresh_bank`).
"""
from __future__ import annotations

import multiprocessing as mp
import queue
import time

import numpy as np


def scene_options(difficulty: str, gid: int) -> dict:
    """Reset options of global scene id `gid`: random navigation at a difficulty
    preset, or "mix3" = lead_brake / jaywalk / red_light_runner by gid % 3."""
    from .config import RandomNavigationReset, build_random_navigation_options
    if difficulty == "mix3":
        return {"scene": ("lead_brake", "jaywalk", "red_light_runner")[gid % 3]}
    return build_random_navigation_options(RandomNavigationReset(difficulty_id=difficulty))


def make_builder(cfg_dict: dict, caps: dict):
    """The HostResetBuilder a CarlaBEVVectorEnv with this config and these
    capacities uses (vector_env.py), without torch or the GPU."""
    from . import layout as LY
    from .config import EnvConfig
    from .host_reset import HostResetBuilder
    from .params import build_params, load_class_map
    from .scene_gen import SceneGenerator
    cfg = EnvConfig.model_validate(cfg_dict)
    classes = load_class_map(cfg.map_name, int(cfg.size))
    params = build_params(cfg, classes)
    layout = LY.Layout.make(LY.Caps(**caps))
    return HostResetBuilder(cfg, classes, params, layout, SceneGenerator(cfg, cfg.map_name)), layout


def _worker(cfg_dict, caps, difficulty, seed0, tasks, results):
    builder, layout = make_builder(cfg_dict, caps)
    rb = layout.record_bytes
    while True:
        task = tasks.get()
        if task is None:
            return
        gids = task
        out = np.zeros((len(gids), rb), np.uint8)
        ctxs = []
        try:
            for k, gid in enumerate(gids):
                _, _, ctx = builder.build(out[k], None, dict(scene_options(difficulty, gid), scene_seed=seed0 + gid))
                ctxs.append(ctx)
        except Exception as exc:  # noqa: BLE001 - reported to the caller by poll()
            results.put((None, f"{type(exc).__name__}: {exc}", None))
            continue
        results.put((gids, out.tobytes(), ctxs))


class ScenePool:
    """`workers` processes building packed scene records for global ids
    first_gid, first_gid + stride, ... in order of request."""

    def __init__(self, cfg_dict: dict, caps: dict, difficulty: str, seed0: int, record_bytes: int, workers: int = 4,
                 first_gid: int = 0, stride: int = 1, batch: int = 16):
        ctx = mp.get_context("spawn")
        self.rb = record_bytes
        self.batch = batch
        self._tasks = ctx.Queue()
        self._results = ctx.Queue()
        self._next = first_gid
        self._stride = stride
        self.requested = 0
        self.delivered = 0
        self.workers = workers
        self._procs = [ctx.Process(target=_worker, args=(cfg_dict, caps, difficulty, seed0, self._tasks, self._results),
                                   daemon=True) for _ in range(workers)]
        for p in self._procs:
            p.start()

    def request_gids(self, gids):
        """Queue scenes for explicit global ids (in batches)."""
        gids = [int(g) for g in gids]
        for i in range(0, len(gids), self.batch):
            self._tasks.put(gids[i:i + self.batch])
            self.requested += len(gids[i:i + self.batch])

    def request(self, n: int):
        """Queue n more scenes (in batches)."""
        while n > 0:
            k = min(n, self.batch)
            self._tasks.put([self._next + self._stride * i for i in range(k)])
            self._next += self._stride * k
            self.requested += k
            n -= k

    def poll(self, max_scenes: int | None = None, timeout: float = 0.0, contexts: bool = False):
        """Finished scenes, without blocking beyond `timeout` seconds for the first
        batch: (global ids, records uint8[k][record_bytes]), plus the scenes'
        scenario-context dicts when contexts=True (for refresh_bank's CTX_IDs)."""
        gids, recs, ctxs = [], [], []
        n = 0
        deadline = time.perf_counter() + timeout
        while max_scenes is None or n < max_scenes:
            try:
                wait = max(0.0, deadline - time.perf_counter()) if not recs else 0.0
                g, b, c = self._results.get(timeout=wait) if wait > 0 else self._results.get_nowait()
            except queue.Empty:
                break
            if g is None:
                raise RuntimeError(f"scene pool worker failed: {b}")
            gids.extend(g)
            recs.append(np.frombuffer(b, np.uint8).reshape(len(g), self.rb))
            ctxs.extend(c)
            n += len(g)
        self.delivered += n
        out = np.concatenate(recs) if recs else np.zeros((0, self.rb), np.uint8)
        return (gids, out, ctxs) if contexts else (gids, out)

    def close(self):
        for _ in self._procs:
            self._tasks.put(None)
        for p in self._procs:
            p.join(timeout=10)
            if p.is_alive():
                p.terminate()


def _build_worker(cfg_dict, caps, tasks, results):
    builder, layout = make_builder(cfg_dict, caps)
    rb = layout.record_bytes
    while True:
        task = tasks.get()
        if task is None:
            return
        tag, items = task
        out = np.zeros((len(items), rb), np.uint8)
        meta = []
        try:
            for k, (seed, options) in enumerate(items):
                info, _spec, ctx = builder.build(out[k], seed, options)
                meta.append((info, ctx))
        except Exception as exc:  # noqa: BLE001 - reported to the caller by build()
            results.put((tag, None, f"{type(exc).__name__}: {exc}"))
            continue
        results.put((tag, out.tobytes(), meta))


class BuildPool:
    """Worker processes building the records of explicit (seed, options) resets,
    for `CarlaBEVVectorEnv.reset` when a reset needs many distinct scenes
    (make_env(cfg, reset_pool=BuildPool(...))). The workers are spawned, so
    create the pool before the calling process touches the GPU (a process that
    has initialised HIP must not start programs: the pool's workers are started
    here, once). Each worker runs the HostResetBuilder the env runs (same config,
    same capacities), so the records are the bytes an in-process build writes
    (tests/test_scene_pool.py)."""

    def __init__(self, cfg_dict: dict, caps: dict, workers: int = 4, chunk: int = 4):
        from . import layout as LY
        ctx = mp.get_context("spawn")
        self.rb = LY.Layout.make(LY.Caps(**caps)).record_bytes
        self.cfg_dict, self.caps, self.chunk, self.workers = dict(cfg_dict), dict(caps), max(1, chunk), workers
        self._tasks, self._results = ctx.Queue(), ctx.Queue()
        self._procs = [ctx.Process(target=_build_worker, args=(self.cfg_dict, self.caps, self._tasks, self._results),
                                   daemon=True) for _ in range(workers)]
        for p in self._procs:
            p.start()
        self._tag = 0

    def build(self, items, timeout: float = 600.0):
        """items: [(seed, options)] -> (uint8[k][record_bytes], [(spawn_validation, scenario_context)]),
        in the order given; blocks until every scene is built."""
        items = list(items)
        out = np.zeros((len(items), self.rb), np.uint8)
        meta = [None] * len(items)
        pending = {}
        for i in range(0, len(items), self.chunk):
            self._tag += 1
            pending[self._tag] = i
            self._tasks.put((self._tag, items[i:i + self.chunk]))
        deadline = time.perf_counter() + timeout
        while pending:
            try:
                tag, data, m = self._results.get(timeout=max(0.1, deadline - time.perf_counter()))
            except queue.Empty:
                raise TimeoutError(f"BuildPool: {len(pending)} chunks not built in {timeout:.0f} s") from None
            if tag not in pending:
                continue  # a chunk of an earlier, failed call
            i = pending.pop(tag)
            if data is None:
                raise RuntimeError(f"scene build worker failed: {m}")
            k = len(m)
            out[i:i + k] = np.frombuffer(data, np.uint8).reshape(k, self.rb)
            meta[i:i + k] = m
        return out, meta

    def close(self):
        for _ in self._procs:
            self._tasks.put(None)
        for p in self._procs:
            p.join(timeout=10)
            if p.is_alive():
                p.terminate()


def build_scenes(cfg_dict: dict, caps: dict, difficulty: str, seed0: int, record_bytes: int, gids,
                 workers: int = 8, timeout: float = 1800.0) -> np.ndarray:
    """Packed records of the scenes of `gids` (uint8[len(gids)][record_bytes], in
    gid order), built by `workers` spawned processes: the same bytes the
    in-process HostResetBuilder writes (tests/test_scene_pool.py)."""
    gids = [int(g) for g in gids]
    if len(set(gids)) != len(gids):  # one output row per gid: a repeated gid would leave a row unfilled
        from collections import Counter
        dup = sorted(g for g, c in Counter(gids).items() if c > 1)[:8]
        raise ValueError(f"build_scenes: repeated scene ids {dup}")
    out = np.zeros((len(gids), record_bytes), np.uint8)
    if not gids:
        return out
    where = {g: i for i, g in enumerate(gids)}
    pool = ScenePool(cfg_dict, caps, difficulty, seed0, record_bytes, workers=max(1, workers),
                     batch=max(1, min(64, len(gids) // (4 * max(1, workers)) or 1)))
    try:
        pool.request_gids(gids)
        done = 0
        deadline = time.perf_counter() + timeout
        while done < len(gids):
            if time.perf_counter() > deadline:
                raise TimeoutError(f"built {done} of {len(gids)} scenes in {timeout:.0f} s")
            got, recs = pool.poll(timeout=5.0)
            if not got and not any(pr.is_alive() for pr in pool._procs):
                raise RuntimeError("every scene worker exited (a spawned worker re-imports the caller's __main__: "
                                   "guard the caller's top-level code with `if __name__ == '__main__'`)")
            for k, g in enumerate(got):
                out[where[g]] = recs[k]
            done += len(got)
    finally:
        pool.close()
    return out
