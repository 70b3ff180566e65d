"""Per-sweep time of eager sweeps (pmc_sweep) at one box size, for A/B of the small-launch path
(PMC_SMALL_LAUNCH: colour phases of at most that many cells run as one full-capacity launch of one
cell per wave; 0 disables it).  Prints the final state's checksum so runs can be compared bitwise.
python tools/small_launch_timing.py <cps> <atoms> [sweeps]"""
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parallel-monte-carlo_amd")]
import pmc_amd  # noqa: E402

cps, atoms = int(sys.argv[1]), int(sys.argv[2])
sweeps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
ctx = pmc_amd.PmcContext(cps)
ctx.init_lattice(atoms)
for s in range(5):
    ctx.sweep(s)
ctx.synchronize()
d0, n0 = ctx.copy_out()
for s in range(100):          # clock warm-up with the same path
    ctx.sweep(100 + s)
ctx.copy_in(d0, n0)
ctx.synchronize()
t0 = time.perf_counter()
for s in range(sweeps):
    ctx.sweep(1000 + s)
ctx.synchronize()
dt = (time.perf_counter() - t0) / sweeps * 1e3
d, n = ctx.copy_out()
h = hashlib.sha256(n.tobytes())
for c in range(len(n)):
    pass
mask_ok = True
import numpy as np
m = np.arange(16)[None, :] < n.astype(np.int64)[:, None]
h.update(d.reshape(-1, 3, 16).view(np.uint32)[np.broadcast_to(m[:, None, :], (len(n), 3, 16))].tobytes())
print(json.dumps({"cps": cps, "atoms": atoms, "sweeps": sweeps, "small_launch": os.environ.get("PMC_SMALL_LAUNCH", "default"),
                  "ms_per_sweep": dt, "state_sha": h.hexdigest()[:16], "error_flags": ctx.error_flags()}))
