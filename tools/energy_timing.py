"""Time pmc_energy (k_energy, the cell-list calc_energy of kernel.cu:452-470) at 128^3 / 1e7 and
check it against the oracle's orc_energy on the same state (bitwise, fixed-point sums)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parallel-monte-carlo_amd"), os.path.join(REPO, "oracle")]
import pmc_amd  # noqa: E402
import pmc_oracle  # noqa: E402  (checker only)

cps = int(sys.argv[1]) if len(sys.argv) > 1 else 128
atoms = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
ctx = pmc_amd.PmcContext(cps)
ctx.init_lattice(atoms)
ctx.start(0, 2)
ctx.synchronize()
e = ctx.energy()
t0 = time.perf_counter()
reps = 10
for _ in range(reps):
    e = ctx.energy()
dt = (time.perf_counter() - t0) / reps
disk, n = ctx.copy_out()
st = pmc_oracle.OracleState(pmc_oracle.make_params(cps=cps))
st.disk[:] = disk
st.n[:] = n
pmc_oracle.set_threads(16)
eo = st.energy()
print(json.dumps({"cps": cps, "atoms": atoms, "energy_gpu": e, "energy_oracle": eo, "equal": e == eo,
                  "ms_per_call_incl_sync": dt * 1e3}))
