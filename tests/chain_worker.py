"""pmc_sweep under a given PMC_SWEEP_CHAINS (read once per process, so each count runs in its own
process; tests/test_gpu_chains.py).  Writes out.npz (state, counters, energy, the chain layout).

  PMC_SWEEP_CHAINS=k python tests/chain_worker.py OUT CPS_X CPS_Y CPS_Z ATOMS FIRST COUNT
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "parallel-monte-carlo_amd"))


def main() -> int:
    out = sys.argv[1]
    cx, cy, cz, atoms, first, count = (int(v) for v in sys.argv[2:8])
    import numpy as np
    import pmc_amd

    ctx = pmc_amd.PmcContext(cx, cps_y=cy, cps_z=cz)
    ctx.init_lattice(atoms)
    for s in range(first, first + count):
        ctx.sweep(s)
    disk, n = ctx.copy_out()
    np.savez(out + ".npz", disk=disk, n=n)
    with open(out + ".json", "w") as f:
        json.dump({"stats": ctx.stats(), "energy": ctx.energy(), "flags": ctx.error_flags(),
                   "layout": ctx.sweep_layout()}, f)
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
