"""Debug: GPU shiftCells vs the oracle on one state; prints the first mismatching slots."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parallel-monte-carlo_amd"), os.path.join(REPO, "oracle")]
import torch  # noqa: E402
import pmc_amd  # noqa: E402
import pmc_oracle  # noqa: E402

f, d = int(sys.argv[1]), float(sys.argv[2])
ctx = pmc_amd.PmcContext(16)
ctx.init_lattice(10_000)
ctx.start(0, 2)
disk, n = ctx.copy_out()
st = pmc_oracle.OracleState(pmc_oracle.make_params(cps=16))
st.disk[:] = disk
st.n[:] = n
dev = torch.device("cuda")
din = torch.from_numpy(disk).to(dev)
nin = torch.from_numpy(n).to(dev)
dout = torch.zeros_like(din)
nout = torch.zeros_like(nin)
torch.cuda.synchronize()
ctx.shiftCells(din, nin, dout, nout, f, d)
ctx.synchronize()
torch.cuda.synchronize()
assert st.shift_cells(f, d) == 0
gd, gn = dout.cpu().numpy().reshape(-1, 3, 16), nout.cpu().numpy()
od = st.disk.reshape(-1, 3, 16)
print("counts equal:", np.array_equal(gn, st.n))
bad = 0
for c in range(len(gn)):
    k = gn[c]
    if not np.array_equal(gd[c, :, :k], od[c, :, :k]):
        if bad < 6:
            print("cell", c, "xyz", c % 16, (c // 16) % 16, c // 256, "n", k)
            print("  gpu", gd[c, f, :k])
            print("  orc", od[c, f, :k])
            print("  in ", disk.reshape(-1, 3, 16)[c, f, :n[c]])
        bad += 1
print("bad cells", bad)
