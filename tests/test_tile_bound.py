"""k_raster's LDS window bound (csrc/cbev.hip Tiles::lds_bytes) against the
worst case over every heading (tools/tile_window_bound.py): a window larger
than the constant would be clamped and flagged (CBEV_ERR_RASTER_WINDOW), so the
constants must cover every heading, and the launch's residency (4 workgroups
of 128 x 128 tiles per CU) follows from them."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import tile_window_bound as twb  # noqa: E402


def _constants():
    src = open(os.path.join(ROOT, "carlabev_env_amd", "csrc", "cbev.hip")).read()
    m = re.search(r"lds_bytes = TC == 64 \? (\d+) : TR == 64 \? (\d+) : (\d+);", src)
    assert m, "Tiles::lds_bytes not found"
    return {(64, 64): int(m.group(1)), (128, 64): int(m.group(2)), (128, 128): int(m.group(3))}


def test_lds_bytes_cover_every_heading():
    """The constant holds the sampled worst case plus one spare row of its pitch."""
    for (tc, tr), have in _constants().items():
        need, (_, _, _, nc) = twb.bound(tc, tr)
        spare = 16 * nc + 4
        assert need + spare <= have, f"{tc} x {tr}: window needs {need} + {spare} B, Tiles::lds_bytes is {have}"
        assert have - need < 640, f"{tc} x {tr}: {have} B reserved for a {need} B worst case"


def test_128_tiles_keep_four_workgroups_per_cu():
    assert 163840 // _constants()[(128, 128)] == 4
