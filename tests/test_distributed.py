"""Multi-rank env sharding on CPU (gloo, world size 2).

Each rank builds the scenes of its global env ids, steps them (the CPU oracle
stands in for the device step: this test covers the sharding and the gather,
not the kernels) and gathers frames / rewards / termination flags to rank 0,
which compares them with a single-process run over all envs.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

N_PER_RANK, STEPS, SEED0, ACT0 = 3, 6, 10_000, 1234


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(rank_ids, seed0, act0):
    import oracle as O
    from carlabev_env_amd import layout as LY
    from helpers import world, scene_options
    cfg, P, padded, layout, builder = world()
    n = len(rank_ids)
    recs = np.zeros((n, layout.record_bytes), np.uint8)
    for k, g in enumerate(rank_ids):
        builder.build(recs[k], None, dict(scene_options("rt_medium_v1"), scene_seed=seed0 + int(g)))
    orc = O.Oracle(P, padded, LY.Caps(128, 32, 64, 4).c(), layout.record_bytes)
    frames = np.zeros((n, P.size, P.size), np.uint8)
    acts = np.stack([np.random.default_rng(act0 + int(g)).integers(0, P.n_discrete, STEPS) for g in rank_ids],
                    axis=1).astype(np.int32)
    for t in range(STEPS):
        orc.step(recs, n, np.ascontiguousarray(acts[t]), frames)
    views = [LY.RecordView(recs[k], layout) for k in range(n)]
    rew = np.array([v.h("REWARD") for v in views])
    term = np.array([v.i("TERM") for v in views], np.uint8)
    return frames, rew, term


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from carlabev_env_amd.sharding import gather_frames, rank_env_ids
        ids = rank_env_ids(rank, N_PER_RANK)
        frames, rew, term = _run(ids, SEED0, ACT0)
        out = gather_frames(torch.from_numpy(frames), torch.from_numpy(rew), torch.from_numpy(term))
        if rank == 0:
            q.put(tuple(t.numpy() for t in out))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_sharded_gather_matches_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _run(np.arange(world * N_PER_RANK), SEED0, ACT0)
    assert np.array_equal(got[0], ref[0])
    assert np.array_equal(got[1], ref[1])
    assert np.array_equal(got[2], ref[2])


def test_rank_ids_and_seeds():
    from carlabev_env_amd.sharding import action_seeds, rank_env_ids, scene_seeds
    assert list(rank_env_ids(1, 4)) == [4, 5, 6, 7]
    assert scene_seeds(2, 3, 10_000) == [10_006, 10_007, 10_008]
    assert action_seeds(0, 2, 99) == [99, 100]
