"""pmc_amd -- MI355X-native checkerboard Metropolis Monte Carlo (subsweep + shiftCells hot path).

Host mirror of qingye3/parallel-monte-carlo's call surface over the C ABI in include/pmc.h;
the compute runs in hand-written HIP kernels for gfx950 (csrc/).  See DESIGN.md.
"""
from ._lib import PmcError, build, lib  # noqa: F401
from .engine import PmcContext, colour_offset, device_count, hbm_probe, selftest_detmath  # noqa: F401

__all__ = ["PmcContext", "PmcError", "build", "lib", "colour_offset", "device_count", "hbm_probe", "selftest_detmath"]
