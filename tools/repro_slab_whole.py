"""Repro probe for an intermittent mismatch seen twice in test_gpu_c_slab_driver_equals_whole_box
[16-10000-True]: the whole-box context's counts read back as all zeros.  Repeats the test body and,
on a mismatch, reads the whole box again (a late host copy shows as a second read that is right)."""
import gc
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parallel-monte-carlo_amd")]
import torch  # noqa: E402
import pmc_amd as pmc  # noqa: E402
from pmc_amd.slab import SlabDriver  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
bad = 0
for it in range(reps):
    for rccl in (False, True):
        drv = SlabDriver(cps=16, nz_local=16, rank=0, world=1, atoms_per_rank=10_000, use_rccl=rccl)
        whole = pmc.PmcContext(16, cps_z=16)
        whole.init_lattice(10_000)
        drv.run(10, 8)
        for s in range(10, 18):
            whole.sweep(s)
        torch.cuda.synchronize()
        d_slab, n_slab = drv.owned()
        disk, n = whole.copy_out()
        ok = np.array_equal(n_slab, n)
        if not ok:
            bad += 1
            disk2, n2 = whole.copy_out()
            print(f"it {it} rccl {rccl}: mismatch; whole n sum {int(n.sum())}, reread sum {int(n2.sum())}, "
                  f"reread equal {np.array_equal(n_slab, n2)}, slab sum {int(n_slab.sum())}", flush=True)
        drv.ctx.close()
        whole.close()
        del drv, whole
        gc.collect()
print(f"done: {bad} mismatches in {2 * reps} runs", flush=True)
