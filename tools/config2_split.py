"""Config 2 (one colour phase of 64^3 / 1e6): the phase as ONE launch against the same phase as two
ordered plane-range launches (planes [0, 32) and [32, 64): each about one round of the chip's wave
slots), for rocprofv3 counter passes (tools/config2_split.sh) -- prices the memory-side re-reads of the
phase's second round of waves.  Each rep runs the full phase, then the two halves
of the SAME colour and sweep index on the state the full phase left (the bytes a phase reads depend
only on the counts, which a phase does not change)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "parallel-monte-carlo_amd"))

import pmc_amd  # noqa: E402


def main() -> int:
    ctx = pmc_amd.PmcContext(64)
    ctx.init_lattice(1_000_000)
    ctx.start(0, 4)                       # away from the lattice start
    ctx.synchronize()
    for rep in range(4):
        colour, sweep = rep % 8, 10 + rep
        ctx.phase(colour, sweep)          # one launch (grid: all 16384 two-cell waves)
        ctx.synchronize()
        ctx.phase_range(colour, sweep, 0, 32)
        ctx.synchronize()
        ctx.phase_range(colour, sweep, 32, 64)
        ctx.synchronize()
    print("config2_split: 4 reps of full phase + two halves")
    return 0


if __name__ == "__main__":
    sys.exit(main())
