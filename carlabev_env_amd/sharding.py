"""Env sharding across GPUs (one process per GPU).

Envs are independent units (`SyncVectorEnv` steps them separately,
envs/__init__.py:116-119): rank r owns global env ids [r*N, (r+1)*N). Scene
seeds and action streams derive from the global id, so an env's trajectory is
the same whatever the GPU count. The only collective is the optional gather of
the compact uint8 class-id frames + reward/flags/cause to rank 0 (config 4's
wire format): ONE `torch.distributed.gather` per step (RCCL over xGMI on GPUs,
gloo in the CPU tests) of a packed per-rank payload into a receive buffer
allocated once.

Per-rank payload (bytes, N envs of S x S):
    [0, N*S*S)            frames, uint8 palette ids, env-major
    [N*S*S, +8N)          reward float64
    [+8N, +12N)           cause int32 (layout.CAUSE ids)
    [+12N, +13N)          terminated uint8
    [+13N, +14N)          truncated uint8
    (padded to a 16-byte multiple)
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


def payload_bytes(n: int, s: int) -> int:
    raw = n * s * s + 14 * n
    return (raw + 15) // 16 * 16


class FrameGather:
    """One collective per step: every rank's frames + reward/cause/term/trunc to `dst`.

    The send buffer and (on `dst`) the (world, payload) receive buffer are
    allocated once; `gather()` packs this rank's step outputs into the send
    buffer (one device copy of the frames + four small copies) and issues a
    single `dist.gather` whose receive list is views of the receive buffer, so
    no per-step allocation and no concatenation. The gathered arrays are
    exposed as views (`frames`, `reward`, `cause`, `term`, `trunc`) in global
    env id order.
    """

    def __init__(self, n: int, s: int, device, dst: int = 0, group=None):
        import torch
        import torch.distributed as dist
        self.n, self.s, self.dst, self.group = int(n), int(s), int(dst), group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.nbytes = payload_bytes(self.n, self.s)
        self.send = torch.zeros(self.nbytes, dtype=torch.uint8, device=device)
        self._send_views = self._views(self.send)
        self.recv = None
        self._recv_list = None
        if self.rank == self.dst:
            self.recv = torch.zeros((self.world, self.nbytes), dtype=torch.uint8, device=device)
            self._recv_list = list(self.recv.unbind(0))
            per = [self._views(self.recv[r]) for r in range(self.world)]
            # global-id order views over the receive buffer (rank-major = global env id order)
            self.frames_by_rank = [v[0] for v in per]
            self.reward_by_rank = [v[1] for v in per]
            self.cause_by_rank = [v[2] for v in per]
            self.term_by_rank = [v[3] for v in per]
            self.trunc_by_rank = [v[4] for v in per]

    def _views(self, buf):
        import torch
        n, s = self.n, self.s
        o = n * s * s
        frames = buf[:o].view(n, s, s)
        reward = buf[o:o + 8 * n].view(torch.float64)
        cause = buf[o + 8 * n:o + 12 * n].view(torch.int32)
        term = buf[o + 12 * n:o + 13 * n]
        trunc = buf[o + 13 * n:o + 14 * n]
        return frames, reward, cause, term, trunc

    @property
    def bytes_per_step(self) -> int:
        """Bytes that arrive at `dst` per step (the other ranks' payloads)."""
        return (self.world - 1) * self.nbytes

    def pack(self, frames, reward, term, trunc=None, cause=None):
        f, r, c, te, tr = self._send_views
        f.copy_(frames.reshape(self.n, self.s, self.s), non_blocking=True)
        r.copy_(reward, non_blocking=True)
        te.copy_(term, non_blocking=True)
        if trunc is not None:
            tr.copy_(trunc, non_blocking=True)
        if cause is not None:
            c.copy_(cause, non_blocking=True)

    def gather(self, frames, reward, term, trunc=None, cause=None):
        """Pack and gather. Returns the (world, payload) receive buffer on `dst`, None elsewhere."""
        import torch.distributed as dist
        self.pack(frames, reward, term, trunc, cause)
        dist.gather(self.send, self._recv_list, dst=self.dst, group=self.group)
        return self.recv

    # convenience accessors on dst: world*N rows in global env id order
    def gathered(self):
        import torch
        if self.rank != self.dst:
            return None
        return (torch.cat(self.frames_by_rank), torch.cat(self.reward_by_rank), torch.cat(self.cause_by_rank),
                torch.cat(self.term_by_rank), torch.cat(self.trunc_by_rank))


def gather_frames(frames, reward=None, term=None, dst: int = 0, group=None):
    """One-shot gather (tests / occasional use): returns (frames[world*N,S,S],
    reward[world*N], term[world*N]) on `dst`, None elsewhere. Step loops keep a
    `FrameGather` instead, which allocates its buffers once."""
    import torch
    n, s = frames.shape[0], frames.shape[-1]
    g = FrameGather(n, s, frames.device, dst=dst, group=group)
    z64 = torch.zeros(n, dtype=torch.float64, device=frames.device)
    z8 = torch.zeros(n, dtype=torch.uint8, device=frames.device)
    g.gather(frames, reward if reward is not None else z64, term if term is not None else z8)
    out = g.gathered()
    if out is None:
        return None
    f, r, _c, t, _tr = out
    return f, (r if reward is not None else None), (t.to(term.dtype) if term is not None else None)
