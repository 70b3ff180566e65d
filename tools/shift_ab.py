"""Time shiftCells at 128^3/1e7 per axis (A/B of shift kernels via PMC_SHIFT_NORUN)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "parallel-monte-carlo_amd"))
import torch  # noqa: E402
import pmc_amd  # noqa: E402

ctx = pmc_amd.PmcContext(128)
ctx.init_lattice(10_000_000)
ctx.start(0, 1)
disk, n = ctx.copy_out()
dev = torch.device("cuda")
din = torch.from_numpy(disk).to(dev)
nin = torch.from_numpy(n).to(dev)
dout = torch.zeros_like(din)
nout = torch.zeros_like(nin)
for f in range(3):
    for d in (0.7, -0.9):
        ctx.shiftCells(din, nin, dout, nout, f, d)
        ctx.synchronize()
        t = []
        for _ in range(20):
            t0 = time.perf_counter()
            ctx.shiftCells(din, nin, dout, nout, f, d)
            ctx.synchronize()
            t.append(time.perf_counter() - t0)
        t.sort()
        print(f"f={f} d={d:+.1f}  {t[len(t)//2]*1e3:.4f} ms", flush=True)
