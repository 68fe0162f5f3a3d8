"""Env sharding across GPUs (one process per GPU).

Envs are independent units (`SyncVectorEnv` steps them separately,
envs/__init__.py:116-119): rank r owns global env ids [r*N, (r+1)*N). Scene
seeds and action streams derive from the global id, so an env's trajectory is
the same whatever the GPU count. The only collective is the optional gather of
the compact uint8 class-id frames (+ reward/flags) to rank 0 (config 4's wire
format), one `torch.distributed.gather` per step (RCCL over xGMI on GPUs, gloo
in the CPU tests).
"""
from __future__ import annotations

import numpy as np


def rank_env_ids(rank: int, envs_per_rank: int) -> np.ndarray:
    """Global env ids owned by `rank`."""
    return np.arange(rank * envs_per_rank, (rank + 1) * envs_per_rank, dtype=np.int64)


def scene_seeds(rank: int, envs_per_rank: int, seed0: int) -> list[int]:
    """scene_seed = seed0 + global_env_id."""
    return [int(seed0 + g) for g in rank_env_ids(rank, envs_per_rank)]


def action_seeds(rank: int, envs_per_rank: int, seed0: int) -> list[int]:
    """Per-env action stream seed default_rng(seed0 + global_env_id)."""
    return [int(seed0 + g) for g in rank_env_ids(rank, envs_per_rank)]


def gather_frames(frames, reward=None, term=None, dst: int = 0, group=None):
    """Gather every rank's frames (and optionally reward/term) to `dst`.

    Returns (frames[world*N, S, S], reward[world*N] | None, term[world*N] | None)
    on `dst`, None elsewhere. Rank order = global env id order.
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    outs = []
    for t in (frames, reward, term):
        if t is None:
            outs.append(None)
            continue
        t = t.contiguous()
        buf = [torch.empty_like(t) for _ in range(world)] if rank == dst else None
        dist.gather(t, buf, dst=dst, group=group)
        outs.append(torch.cat(buf) if rank == dst else None)
    return tuple(outs) if rank == dst else None
