"""Time one colour phase of the subsweep at 128^3/1e7 for several n_moves (ablation)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "parallel-monte-carlo_amd"))
import torch  # noqa: E402,F401
import pmc_amd  # noqa: E402

cps = int(os.environ.get("CPS", "128"))
atoms = int(os.environ.get("ATOMS", "10000000"))
for nm in [int(v) for v in os.environ.get("MOVES", "0,1,5,10,20").split(",")]:
    ctx = pmc_amd.PmcContext(cps, n_moves=nm)
    ctx.init_lattice(atoms)
    # equilibrate a little with the standard chain so the state is not the lattice
    ctx.synchronize()
    for s in range(2):   # one launch per phase (pmc_sweep would split phases over plane chains)
        for c in range(8):
            ctx.phase(c, s)
        ctx.shift(s)
    ctx.synchronize()
    reps = int(os.environ.get("REPS", "5"))
    times = []
    for s in range(reps):
        t0 = time.perf_counter()
        for c in range(8):
            ctx.phase(c, 100 + s)
        ctx.synchronize()
        times.append((time.perf_counter() - t0) / 8)
    times.sort()
    dt = times[len(times) // 2]
    st = ctx.stats()
    print(f"n_moves={nm:3d}  phase_ms={dt*1e3:.4f}  evaluated/trials={st['evaluated']/max(1,st['trials']):.3f}", flush=True)
    ctx.close()
