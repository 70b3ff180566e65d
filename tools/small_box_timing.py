"""Small boxes: per-sweep time of eager launches (8 subsweep + 8 fallback + 1
shift launches per sweep) against pmc_run_small (one launch per 32 sweeps on XCD 0), alternating,
both from the same start state; the two paths' final states must be bitwise equal."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parallel-monte-carlo_amd")]
import pmc_amd  # noqa: E402

cps = int(sys.argv[1]) if len(sys.argv) > 1 else 16
atoms = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000
sweeps = int(sys.argv[3]) if len(sys.argv) > 3 else 320
ctx = pmc_amd.PmcContext(cps)
ctx.init_lattice(atoms)
for s in range(5):
    ctx.sweep(s)
ctx.synchronize()
d0, n0 = ctx.copy_out()
res = {"cps": cps, "atoms": atoms, "sweeps": sweeps, "eager_ms": [], "small_ms": []}
for rep in range(3):
    for mode in ("eager", "small"):
        ctx.copy_in(d0, n0)
        ctx.synchronize()
        # warm the clock with the same path
        if mode == "eager":
            for s in range(64):
                ctx.sweep(100 + s)
        else:
            ctx.run_small(100, 64)
        ctx.copy_in(d0, n0)
        ctx.synchronize()
        t0 = time.perf_counter()
        if mode == "eager":
            for s in range(sweeps):
                ctx.sweep(1000 + s)
        else:
            ctx.run_small(1000, sweeps)
        ctx.synchronize()
        res[f"{mode}_ms"].append((time.perf_counter() - t0) / sweeps * 1e3)
        d, n = ctx.copy_out()
        res[f"{mode}_state"] = (d, n)
de, ne = res.pop("eager_state")
ds, ns = res.pop("small_state")
mask = np.arange(16)[None, :] < ne.astype(np.int64)[:, None]
same = bool(np.array_equal(ne, ns)) and bool(np.array_equal(de.reshape(-1, 3, 16).view(np.uint32)[np.broadcast_to(mask[:, None, :], (len(ne), 3, 16))],
                                                            ds.reshape(-1, 3, 16).view(np.uint32)[np.broadcast_to(mask[:, None, :], (len(ne), 3, 16))]))
res["state_bitwise_equal"] = same
res["error_flags"] = ctx.error_flags()
print(json.dumps(res))
