"""Observation/action spaces identical to the reference's.

Gymnasium is not installed in this image; when it is importable its
`spaces.Discrete` / `spaces.Box` are used directly, otherwise these minimal
duck-typed equivalents (same attributes: n, shape, dtype, low, high, seed,
sample, contains) stand in. Definitions follow `envs/spaces.py:27-61` and the
wrapper spaces of `wrappers/rgb_to_semantic.py:236-241,266-268`.
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - exercised only where gymnasium exists
    from gymnasium import spaces as _gs
except Exception:  # noqa: BLE001
    _gs = None


class Discrete:
    def __init__(self, n: int, seed=None):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.dtype(np.int64)
        self._rng = np.random.default_rng(seed)

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        return [seed]

    def sample(self):
        return np.int64(self._rng.integers(self.n))

    def contains(self, x) -> bool:
        try:
            return 0 <= int(x) < self.n
        except (TypeError, ValueError):
            return False

    def __repr__(self):
        return f"Discrete({self.n})"

    def __eq__(self, other):
        return isinstance(other, Discrete) and other.n == self.n


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        self.dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low)
        self.shape = tuple(int(s) for s in shape)
        self.low = np.broadcast_to(np.asarray(low, dtype=self.dtype), self.shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=self.dtype), self.shape).copy()
        self._rng = np.random.default_rng(seed)

    def seed(self, seed=None):
        self._rng = np.random.default_rng(seed)
        return [seed]

    def sample(self):
        if self.dtype.kind == "f":
            return self._rng.uniform(self.low, self.high).astype(self.dtype)
        return self._rng.integers(self.low, self.high.astype(np.int64) + 1).astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    def __eq__(self, other):
        return (isinstance(other, Box) and other.shape == self.shape and other.dtype == self.dtype
                and np.array_equal(other.low, self.low) and np.array_equal(other.high, self.high))


def make_discrete(n):
    return _gs.Discrete(n) if _gs is not None else Discrete(n)


def make_box(low, high, shape=None, dtype=np.float32):
    if _gs is not None:
        return _gs.Box(low=low, high=high, shape=shape, dtype=dtype)
    return Box(low, high, shape, dtype)


def batch_space(space, n: int):
    """gymnasium.vector.utils.batch_space for Discrete/Box."""
    if isinstance(space, Discrete) or (_gs is not None and isinstance(space, _gs.Discrete)):
        return make_box(0, space.n - 1, (n,), np.int64) if _gs is None else _gs.MultiDiscrete(np.full(n, space.n))
    return make_box(np.broadcast_to(space.low, (n, *space.shape)), np.broadcast_to(space.high, (n, *space.shape)),
                    (n, *space.shape), space.dtype)
