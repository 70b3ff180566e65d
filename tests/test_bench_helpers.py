"""CPU tests of bench.py's host-side helpers (no GPU): the slab parity leg's sweep window that shifts
along z both ways, and the staged-model byte counts the roofline objects use."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_z_shift_window_covers_both_z_directions(oracle):
    for seed, first, sweeps in ((1234, 5, 3), (1234, 0, 2), (99, 17, 3), (1234, 100, 4)):
        s0 = bench.z_shift_window(seed, first, sweeps)
        assert s0 >= first
        plans = [oracle.sweep_plan(seed, s, 2.5) for s in range(s0, s0 + sweeps)]
        zdirs = {d > 0 for _, f, d in plans if f == 2}
        assert zdirs == {True, False}, (seed, first, s0, plans)
        # the first such window: no earlier start in [first, s0) has both directions
        for s in range(first, s0):
            early = [oracle.sweep_plan(seed, t, 2.5) for t in range(s, s + sweeps)]
            assert {d > 0 for _, f, d in early if f == 2} != {True, False}
        assert bench.z_shifts(seed, s0, sweeps) == ["xyz"[f] + ("+" if d > 0 else "-") for _, f, d in plans]


def test_z_shift_window_single_sweep_is_first():
    assert bench.z_shift_window(1234, 7, 1) == 7


def test_staged_bytes_model():
    # per non-empty visited cell 12 B x stencil particles + 54 B of counts + 12 B x own
    n = np.array([0, 3, 5], np.int64)
    s = np.array([40, 50, 60], np.int64)
    assert bench.staged_bytes(n, s) == (12 * 50 + 54 + 12 * 3) + (12 * 60 + 54 + 12 * 5)
    # stencil counts of a uniform periodic box: 27 x the per-cell count
    g = np.full(4 * 4 * 4, 2, np.int64)
    assert np.all(bench.stencil_counts(g, (4, 4, 4)) == 54)
