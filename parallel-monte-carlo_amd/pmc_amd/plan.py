"""Per-sweep plan (colour order, shift axis f, shift distance d) from the C ABI.

Reference: FY_Shuffle / itoa (start.cu:34-44,153-157) and f, d (kernel.cu:683-684); here a
host Philox stream keyed by the seed, so every rank derives the same plan without a broadcast.
"""
from __future__ import annotations

import ctypes as C

from ._lib import check, lib


def sweep_plan(seed: int, sweep: int, w: float = 2.5, flags: int = 0):
    """flags: pmc_params.flags (0: colours grouped by z parity; PMC_FLAG_FULL_SHUFFLE: all 8 shuffled)."""
    order = (C.c_int * 8)()
    f = C.c_int()
    d = C.c_float()
    check("pmc_sweep_plan_ex", lib().pmc_sweep_plan_ex(seed, sweep, w, flags, C.byref(order), C.byref(f),
                                                       C.byref(d)))
    return list(order), f.value, d.value
