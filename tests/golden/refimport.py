"""Import selected pure-Python modules of the reference (read-only, /root/reference).

Test infrastructure only: used by `make_golden.py` in the build container to
capture golden input/output vectors from the reference's own arithmetic. It is
never imported by the product, by `-m gpu` tests or on the GPU box (the
reference tree does not exist there).

Mechanics:
- parent packages whose `__init__` pulls gymnasium/pygame
  (`CarlaBEV/__init__.py:1`, `CarlaBEV/envs/__init__.py:1`,
  `CarlaBEV/config/__init__.py` -> `config/env.py:18` -> `envs/utils.py:2`,
  `CarlaBEV/src/gui/__init__.py:1`) are registered as bare namespace modules
  so their `__init__` is skipped;
- a minimal `pygame` stand-in provides only the names the hero/actor modules
  touch at import/construction time (Sprite base class, Rect, Vector2/3,
  draw.rect). None of the captured numbers flows through it: the captured
  vectors are the bicycle/Stanley/behaviour/reward arithmetic, which is
  NumPy/math in the reference;
- bytecode is neither written into nor read from the reference tree
  (`sys.pycache_prefix` points at a private temp dir, so any `__pycache__`
  shipped next to the reference sources is ignored).
"""
from __future__ import annotations

import sys
import tempfile
import types

REF = "/root/reference"

sys.dont_write_bytecode = True
sys.pycache_prefix = tempfile.mkdtemp(prefix="refpyc_")


def _bare_pkg(name: str, path: str) -> None:
    mod = types.ModuleType(name)
    mod.__path__ = [path]
    sys.modules[name] = mod


class _Rect:
    """Stand-in with the attributes hero/actor construction touches."""

    def __init__(self, x=0, y=0, w=0, h=0):
        self.x, self.y, self.w, self.h = int(x), int(y), int(w), int(h)

    @property
    def center(self):
        return (self.x + self.w // 2, self.y + self.h // 2)

    @center.setter
    def center(self, c):
        self.x = int(c[0]) - self.w // 2
        self.y = int(c[1]) - self.h // 2


class _Vec2:
    def __init__(self, x=0.0, y=0.0):
        self.x, self.y = float(x), float(y)

    def __iter__(self):
        return iter((self.x, self.y))

    def __len__(self):
        return 2

    def __getitem__(self, i):
        return (self.x, self.y)[i]


class _Vec3(_Vec2):
    def __init__(self, x=0.0, y=0.0, z=0.0):
        super().__init__(x, y)
        self.z = float(z)


def _install_pygame_stub() -> None:
    if "pygame" in sys.modules:
        return
    pg = types.ModuleType("pygame")
    sprite = types.ModuleType("pygame.sprite")

    class Sprite:  # noqa: D401 - stand-in base class
        def __init__(self, *a, **k):
            pass

    sprite.Sprite = Sprite
    pmath = types.ModuleType("pygame.math")
    pmath.Vector2 = _Vec2
    pmath.Vector3 = _Vec3
    draw = types.ModuleType("pygame.draw")
    draw.rect = lambda surf, color, rect, *a, **k: rect
    pg.sprite, pg.math, pg.draw, pg.Rect = sprite, pmath, draw, _Rect
    sys.modules.update({"pygame": pg, "pygame.sprite": sprite, "pygame.math": pmath, "pygame.draw": draw})


def setup() -> None:
    _install_pygame_stub()
    _bare_pkg("CarlaBEV", f"{REF}/CarlaBEV")
    _bare_pkg("CarlaBEV.envs", f"{REF}/CarlaBEV/envs")
    _bare_pkg("CarlaBEV.config", f"{REF}/CarlaBEV/config")
    _bare_pkg("CarlaBEV.src", f"{REF}/CarlaBEV/src")
    _bare_pkg("CarlaBEV.src.gui", f"{REF}/CarlaBEV/src/gui")
