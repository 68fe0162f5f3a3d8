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


def test_bench_launcher_dry_run_two_ranks():
    """`bench.py --gpus 2` started by hand spawns two ranks itself (gloo rehearsal:
    rendezvous, the packed one-collective gather, max-over-ranks timing) and
    rank 0 reports n_gpus 2."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3",
                          "--envs", "4", "--config", "4"], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["dry_run"] and rec["gather_ok"]
    from carlabev_env_amd.sharding import payload_bytes
    assert rec["gather_bytes_per_step"] == payload_bytes(4, 128)  # nibble-packed frames
    assert payload_bytes(4, 128) == (4 * 128 * 128 // 2 + 14 * 4 + 15) // 16 * 16
    # config 4 at its bench size (8192 envs per rank): the packed payload is half
    # the unpacked one, and rank 0's ingress at 8 ranks over 7 xGMI links halves
    b = rec["at_config_size"]
    assert b["envs_per_rank"] == 8192 and b["bytes_packed"] == payload_bytes(8192, 128)
    assert abs(b["bytes_unpacked"] - 2 * b["bytes_packed"]) <= 14 * 8192
    assert 0.43 < b["rank0_ingress_ms_packed"] < 0.45 and 0.87 < b["rank0_ingress_ms_unpacked"] < 0.89


def test_pack_frames_roundtrip_cpu():
    from carlabev_env_amd.sharding import pack_frames, unpack_frames
    fr = torch.randint(0, 16, (3, 64, 64), dtype=torch.uint8)
    pk = pack_frames(fr)
    assert pk.shape == (3, 2048)
    f0 = fr.reshape(3, -1)
    assert torch.equal(pk, f0[:, 0::2] | (f0[:, 1::2] << 4))
    assert torch.equal(unpack_frames(pk, 64), fr)


def _packed_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from carlabev_env_amd.sharding import FrameGather
        n, S = 5, 16
        g = FrameGather(n, S, "cpu")  # nibble-packed frames, two buffers used in turn
        send_ptrs = [b.data_ptr() for b in g.send]
        for step in range(5):  # buffers are reused across steps
            gen = torch.Generator().manual_seed(100 * rank + step)
            fr = torch.randint(0, 16, (n, S, S), dtype=torch.uint8, generator=gen)
            rew = torch.randn(n, dtype=torch.float64, generator=gen)
            term = (torch.rand(n, generator=gen) < 0.5).to(torch.uint8)
            trunc = (torch.rand(n, generator=gen) < 0.5).to(torch.uint8)
            cause = torch.randint(-1, 6, (n,), dtype=torch.int32, generator=gen)
            g.gather(fr, rew, term, trunc, cause)
            assert [b.data_ptr() for b in g.send] == send_ptrs
            if rank == 0:
                q.put((step, tuple(t.clone().numpy() for t in g.gathered())))
        g.wait()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_packed_gather_all_fields():
    """The nibble-packed, double-buffered asynchronous gather (sharding.FrameGather)
    round-trips every palette id 0..15 and the reward / cause / flag fields of
    both ranks over five steps, reusing its two send buffers."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_packed_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(5)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n, S = 5, 16
    for step, (fr, rew, cause, term, trunc) in got:
        for r in range(world):
            gen = torch.Generator().manual_seed(100 * r + step)
            e_fr = torch.randint(0, 16, (n, S, S), dtype=torch.uint8, generator=gen).numpy()
            e_rew = torch.randn(n, dtype=torch.float64, generator=gen).numpy()
            e_term = (torch.rand(n, generator=gen) < 0.5).to(torch.uint8).numpy()
            e_trunc = (torch.rand(n, generator=gen) < 0.5).to(torch.uint8).numpy()
            e_cause = torch.randint(-1, 6, (n,), dtype=torch.int32, generator=gen).numpy()
            sl = slice(r * n, (r + 1) * n)
            assert np.array_equal(fr[sl], e_fr) and np.array_equal(rew[sl], e_rew)
            assert np.array_equal(term[sl], e_term) and np.array_equal(trunc[sl], e_trunc)
            assert np.array_equal(cause[sl], e_cause)


def test_rank_ids_and_seeds():
    from carlabev_env_amd.sharding import action_seeds, rank_env_ids, scene_seeds
    assert list(rank_env_ids(1, 4)) == [4, 5, 6, 7]
    assert scene_seeds(2, 3, 10_000) == [10_006, 10_007, 10_008]
    assert action_seeds(0, 2, 99) == [99, 100]
