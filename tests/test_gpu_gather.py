"""GPU tests of config 4's gather leg on one GPU: the HIP
nibble pack / unpack kernels (cbev_pack_frames / cbev_unpack_frames) against
the torch packing, and sharding.FrameGather's device path (pack on the env's
stream, one RCCL gather, unpack on rank 0) inside a world-size-1 "nccl" group
over real cbev_step outputs. The reference has no multi-process path
(SyncVectorEnv, CarlaBEV/envs/__init__.py:116-119); the wire format is ours, so
the bar is a bit-exact round trip of the step's own outputs.
"""
from __future__ import annotations

import ctypes
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from carlabev_env_amd._lib import lib
from carlabev_env_amd.sharding import FrameGather, pack_frames, payload_bytes, unpack_frames
from helpers import bench_caps, world

pytestmark = pytest.mark.gpu

P_ = ctypes.c_void_p


class Ctx:
    def __init__(self, size):
        cfg, P, padded, layout, builder = world(size=size, caps=bench_caps(2))
        self.ctx = P_()
        assert lib().cbev_create(ctypes.byref(P), ctypes.byref(bench_caps(2).c()), 0, ctypes.byref(self.ctx)) == 0
        assert lib().cbev_set_map(self.ctx, padded.ctypes.data_as(P_), padded.nbytes) == 0

    def __del__(self):
        lib().cbev_destroy(self.ctx)


def torch_pack(fr):
    flat = fr.reshape(fr.shape[0], -1)
    return flat[:, 0::2] | (flat[:, 1::2] << 4)


@pytest.mark.parametrize("S", [64, 128, 256])
def test_pack_unpack_frames_device(S):
    """Every palette id 0..15 in both nibbles, an odd env count, on a side stream
    (the default stream argument is the current torch stream), and unpacking
    from a receive-buffer view at a nonzero rank offset."""
    c = Ctx(S)
    n = 7
    g = torch.Generator().manual_seed(S)
    fr = torch.randint(0, 16, (n, S, S), dtype=torch.uint8, generator=g)
    fr[0].view(-1)[:512] = torch.arange(512, dtype=torch.int64).remainder(16).to(torch.uint8)  # all (lo, hi) pairs
    fr[0].view(-1)[512:1024] = (torch.arange(512) // 16).remainder(16).to(torch.uint8)
    want = torch_pack(fr)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        d = fr.cuda()
        pk = pack_frames(d, ctx=c.ctx)
        # a gather receive buffer: world x payload rows; rank 2's packed frames at its offset
        nb = payload_bytes(n, S)
        recv = torch.zeros((3, nb), dtype=torch.uint8, device="cuda")
        recv[2, :n * S * S // 2].copy_(pk.reshape(-1))
        out = unpack_frames(recv[2, :n * S * S // 2].view(n, -1), S, ctx=c.ctx)
    side.synchronize()
    assert torch.equal(pk.cpu(), want)
    assert torch.equal(out.cpu(), fr)
    # misaligned buffers are refused, not mis-read
    assert lib().cbev_pack_frames(c.ctx, P_(d.data_ptr() + 4), 1, P_(pk.data_ptr()), None) != 0
    assert lib().cbev_unpack_frames(c.ctx, P_(pk.data_ptr() + 1), 1, P_(d.data_ptr()), None) != 0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_frame_gather_device_world1():
    """FrameGather(ctx, stream_fn) in a world-size-1 RCCL group over three real
    cbev_step outputs of config 4's shape (continuous rt_medium, 128x128
    semantic): gathered() equals the env's frames / reward / cause / term / trunc
    bit for bit, with the two send buffers reused; then the same without
    stream_fn (current-stream default) on a side stream."""
    import torch.distributed as dist
    from carlabev_env_amd import EnvConfig, build_random_navigation_options, RandomNavigationReset
    from carlabev_env_amd.vector_env import CarlaBEVVectorEnv
    dev = torch.device("cuda", 0)
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                device_id=dev)
    try:
        cfg = EnvConfig(size=128, obs_size=(128, 128), obs_mode="bev_semantic", render_mode="rgb_array",
                        action_mode="continuous", action_profile_id="continuous_gsb_v1")
        n = 37
        import bench
        env = CarlaBEVVectorEnv({"env": cfg, "num_envs": n}, device=dev, caps=bench.CONFIGS[4]["caps"])
        env.reset(seed=40_000, options=build_random_navigation_options(
            RandomNavigationReset(difficulty_id="rt_medium_v1")))
        rng = np.random.default_rng(99)
        for stream_fn in (env._stream, None):
            g = FrameGather(n, 128, dev, ctx=env._ctx, stream_fn=stream_fn)
            assert g.bytes_per_step == 0 and len(g.send) == 2
            side = torch.cuda.Stream(dev)
            with torch.cuda.stream(side):
                for t in range(3):
                    a = torch.from_numpy(rng.uniform([0, -1, 0], [1, 1, 1], size=(n, 3)).astype(np.float32)).to(dev)
                    env.step(a)
                    g.gather(env.frames(), env.reward, env.term, env.trunc, env.cause)
                    fr, rew, cause, term, trunc = g.gathered()
                    want = (env.frames().clone(), env.reward.clone(), env.cause.clone(), env.term.clone(),
                            env.trunc.clone())
                    side.synchronize()
                    assert torch.equal(fr, want[0]), t
                    assert torch.equal(rew, want[1]) and torch.equal(cause, want[2]), t
                    assert torch.equal(term, want[3]) and torch.equal(trunc, want[4]), t
                g.wait()
            side.synchronize()
        env.close()
    finally:
        if own:
            dist.destroy_process_group()
