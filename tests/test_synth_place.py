"""The synthetic arenas' frame placement (tools/synth/synthgen.py `place`): frames
longer than 64 bytes start on a 128-byte line, frames of <= 64 bytes take 64-byte slots after
them, no two frames overlap, and the numpy and torch forms agree (CPU only)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "synth"))
import synthgen  # noqa: E402


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_place_alignment_and_no_overlap(seed):
    import torch
    rng = np.random.default_rng(seed)
    ln = rng.choice([60, 64, 65, 80, 128, 129, 192, 594, 1350, 1518], 5000)
    alen = (ln + 63) & ~63
    off, total = synthgen.place(alen, np)
    ot, tt = synthgen.place(torch.tensor(alen), torch)
    assert np.array_equal(ot.numpy(), off) and tt == total
    big = alen > 64
    assert (off[big] % 128 == 0).all() and (off % 64 == 0).all()
    o = np.argsort(off)
    assert (off[o][:-1] + alen[o][:-1] <= off[o][1:]).all()
    assert off.max() + alen[np.argmax(off)] <= total
    # padding only rounds the long frames up to whole lines
    assert total == int(((alen[big] + 127) // 128 * 128).sum()) + 64 * int((~big).sum())


def test_place_empty_and_all_short():
    off, total = synthgen.place(np.zeros(0, dtype=np.int64), np)
    assert total == 0 and len(off) == 0
    off, total = synthgen.place(np.full(7, 64, dtype=np.int64), np)
    assert list(off) == [64 * k for k in range(7)] and total == 448
