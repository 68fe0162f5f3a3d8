"""Env sharding across GPUs (one process per GPU).

Envs are independent units (`SyncVectorEnv` steps them separately,
envs/__init__.py:116-119): rank r owns global env ids [r*N, (r+1)*N). Scene
seeds and action streams derive from the global id, so an env's trajectory is
the same whatever the GPU count. The only collective is the optional gather of
the compact class-id frames + reward/flags/cause to rank 0 (config 4's
wire format): ONE asynchronous `torch.distributed.gather` per step (RCCL over
xGMI on GPUs, gloo in the CPU tests) of a packed per-rank payload into receive
buffers allocated once, double-buffered so it overlaps the next step.

Per-rank payload (bytes, N envs of S x S, F = N*S*S/2):
    [0, F)                frames, nibble-packed palette ids (pack_frames), env-major
    [F, +8N)              reward float64
    [F+8N, +4N)           cause int32 (layout.CAUSE ids)
    [F+12N, +N)           terminated uint8
    [F+13N, +N)           truncated uint8
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


def payload_bytes(n: int, s: int, packed: bool = True) -> int:
    """Per-rank gather payload: frames (nibble-packed: S*S/2 bytes per env) + 14 bytes per env."""
    raw = n * (s * s // 2 if packed else s * s) + 14 * n
    return (raw + 15) // 16 * 16


def _raw_stream(t, stream):
    """`stream` (a raw hipStream_t) or, when None, the caller's current torch stream
    on t's device: the pack / unpack kernels are then ordered with the step kernels
    that wrote the frames and with the collective that reads them."""
    import ctypes
    import torch
    if stream is not None:
        return stream
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(t.device.index))


def pack_frames(frames, out=None, ctx=None, stream=None):
    """Palette-id frames (n, S, S) uint8 -> nibble-packed (n, S*S/2): byte j =
    pixel 2j | pixel 2j+1 << 4. Device tensors go through the HIP kernel
    (cbev_pack_frames, needs the env's C-ABI context; on `stream`, default the
    current torch stream); CPU tensors (gloo) through torch."""
    import torch
    n = frames.shape[0]
    flat = frames.reshape(n, -1)
    if out is None:
        out = torch.empty((n, flat.shape[1] // 2), dtype=torch.uint8, device=frames.device)
    if frames.is_cuda:
        import ctypes
        from ._lib import check, lib
        check(lib().cbev_pack_frames(ctx, ctypes.c_void_p(flat.data_ptr()), n, ctypes.c_void_p(out.data_ptr()),
                                     _raw_stream(flat, stream)), "cbev_pack_frames")
    else:
        torch.bitwise_or(flat[:, 0::2], flat[:, 1::2] << 4, out=out)
    return out


def unpack_frames(packed, s: int, ctx=None, stream=None):
    """Inverse of pack_frames: (n, S*S/2) -> (n, S, S) palette ids."""
    import torch
    n = packed.shape[0]
    out = torch.empty((n, s, s), dtype=torch.uint8, device=packed.device)
    if packed.is_cuda:
        import ctypes
        from ._lib import check, lib
        check(lib().cbev_unpack_frames(ctx, ctypes.c_void_p(packed.data_ptr()), n, ctypes.c_void_p(out.data_ptr()),
                                       _raw_stream(packed, stream)), "cbev_unpack_frames")
    else:
        flat = out.view(n, -1)
        flat[:, 0::2] = packed & 15
        flat[:, 1::2] = packed >> 4
    return out


class FrameGather:
    """One collective per step: every rank's frames + reward/cause/term/trunc to `dst`.

    Wire format: the frames nibble-packed (palette ids are <= 15: half the bytes
    of the uint8 frames), then reward float64, cause int32, term and trunc uint8
    per env (`payload_bytes`). `buffers` send (and, on `dst`, receive) buffers
    are allocated once and used in turn: `gather()` packs this rank's step
    outputs into the next buffer on the caller's stream and issues ONE
    asynchronous `dist.gather` of it (RCCL runs it on its own stream, overlapped
    with the next steps' kernels), then returns. A buffer is reused only after
    its previous gather completed (`Work.wait()`: a stream dependency on the
    GPU, no host sync). `gathered()` waits for the latest gather and returns the
    unpacked arrays in global env id order on `dst`.
    """

    def __init__(self, n: int, s: int, device, dst: int = 0, group=None, packed: bool = True, buffers: int = 2,
                 ctx=None, stream_fn=None):
        import torch
        import torch.distributed as dist
        self.n, self.s, self.dst, self.group = int(n), int(s), int(dst), group
        self.packed, self.ctx, self.stream_fn = bool(packed), ctx, stream_fn
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.fbytes = self.n * self.s * self.s // (2 if self.packed else 1)
        self.nbytes = payload_bytes(self.n, self.s, self.packed)
        self.send = [torch.zeros(self.nbytes, dtype=torch.uint8, device=device) for _ in range(buffers)]
        self._send_views = [self._views(b) for b in self.send]
        self.recv = self._recv_list = None
        if self.rank == self.dst:
            self.recv = [torch.zeros((self.world, self.nbytes), dtype=torch.uint8, device=device)
                         for _ in range(buffers)]
            self._recv_list = [list(r.unbind(0)) for r in self.recv]
        self._work = [None] * buffers
        self._next = 0
        self._last = None

    def _views(self, buf):
        import torch
        n, o = self.n, self.fbytes
        frames = buf[:o].view(n, -1)
        reward = buf[o:o + 8 * n].view(torch.float64)
        cause = buf[o + 8 * n:o + 12 * n].view(torch.int32)
        term = buf[o + 12 * n:o + 13 * n]
        trunc = buf[o + 13 * n:o + 14 * n]
        return frames, reward, cause, term, trunc

    @property
    def bytes_per_step(self) -> int:
        """Bytes that arrive at `dst` per step (the other ranks' payloads)."""
        return (self.world - 1) * self.nbytes

    def pack(self, k, frames, reward, term, trunc=None, cause=None):
        f, r, c, te, tr = self._send_views[k]
        if self.packed:
            pack_frames(frames.reshape(self.n, self.s, self.s), out=f, ctx=self.ctx,
                        stream=self.stream_fn() if self.stream_fn else None)
        else:
            f.copy_(frames.reshape(self.n, -1), non_blocking=True)
        r.copy_(reward, non_blocking=True)
        te.copy_(term, non_blocking=True)
        if trunc is not None:
            tr.copy_(trunc, non_blocking=True)
        if cause is not None:
            c.copy_(cause, non_blocking=True)

    def gather(self, frames, reward, term, trunc=None, cause=None):
        """Pack into the next buffer and issue its gather asynchronously; returns the Work."""
        import torch.distributed as dist
        k = self._next
        if self._work[k] is not None:  # the buffer's previous gather must be done with it
            self._work[k].wait()
            self._work[k] = None
        self.pack(k, frames, reward, term, trunc, cause)
        self._work[k] = dist.gather(self.send[k], self._recv_list[k] if self._recv_list else None, dst=self.dst,
                                    group=self.group, async_op=True)
        self._last = k
        self._next = (k + 1) % len(self.send)
        return self._work[k]

    def wait(self):
        """Make the caller wait for every outstanding gather (a stream dependency on the GPU)."""
        for k, w in enumerate(self._work):
            if w is not None:
                w.wait()
                self._work[k] = None

    def gathered(self):
        """On dst: (frames[world*N,S,S], reward, cause, term, trunc) of the latest gather, in
        global env id order (frames unpacked); None elsewhere."""
        import torch
        if self.rank != self.dst or self._last is None:
            return None
        k = self._last
        if self._work[k] is not None:
            self._work[k].wait()
            self._work[k] = None
        per = [self._views(self.recv[k][r]) for r in range(self.world)]
        if self.packed:
            fr = torch.cat([unpack_frames(v[0], self.s, ctx=self.ctx,
                                          stream=self.stream_fn() if self.stream_fn else None) for v in per])
        else:
            fr = torch.cat([v[0].view(self.n, self.s, self.s) for v in per])
        return (fr, torch.cat([v[1] for v in per]), torch.cat([v[2] for v in per]), torch.cat([v[3] for v in per]),
                torch.cat([v[4] for v in per]))


def gather_frames(frames, reward=None, term=None, dst: int = 0, group=None, ctx=None):
    """One-shot gather (tests / occasional use): returns (frames[world*N,S,S],
    reward[world*N], term[world*N]) on `dst`, None elsewhere. Step loops keep a
    `FrameGather` instead, which allocates its buffers once. Device frames need
    the env's C-ABI context (`ctx`) for the pack / unpack kernels."""
    import torch
    n, s = frames.shape[0], frames.shape[-1]
    g = FrameGather(n, s, frames.device, dst=dst, group=group, ctx=ctx, buffers=1)
    z64 = torch.zeros(n, dtype=torch.float64, device=frames.device)
    z8 = torch.zeros(n, dtype=torch.uint8, device=frames.device)
    g.gather(frames, reward if reward is not None else z64, term if term is not None else z8)
    out = g.gathered()
    g.wait()
    if out is None:
        return None
    f, r, _c, t, _tr = out
    return f, (r if reward is not None else None), (t.to(term.dtype) if term is not None else None)
