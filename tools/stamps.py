"""Section timing of the subsweep from per-wave s_memtime stamps (analysis build, -DPMC_STAMPS).

  PMC_LIB_PATH=.../lib_stamps.so python tools/stamps.py

Stamps per cell visit (main launch): 0 entry, 1 stencil table + count load issued, 2 row loads
issued, 3 RNG done, 4 own count known, 5 shuffle done, 6 own cell + neighbours staged (v11), 7 far pad,
8 moves done, 9 written back.
"""
import ctypes as C
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "parallel-monte-carlo_amd"))
import torch  # noqa: E402,F401
import pmc_amd  # noqa: E402

cps = int(os.environ.get("CPS", "128"))
atoms = int(os.environ.get("ATOMS", "10000000"))
ctx = pmc_amd.PmcContext(cps)
ctx.init_lattice(atoms)
for s in range(3):
    ctx.sweep(s)
ctx.synchronize()
L = pmc_amd._lib.lib()
L.pmc_debug_stamps.restype = C.c_int
L.pmc_debug_stamps.argtypes = [C.c_size_t, C.c_void_p]
ncell = (cps // 2) ** 3
names = ["stencil+cnt", "row loads", "rng", "count wait", "shuffle", "own+nb staging", "far pad", "moves", "writeback"]   # spec v11: own cell staged first
for rep in range(2):
    assert L.pmc_debug_stamps(ncell, None) == 0
    t0 = time.perf_counter()
    ctx.phase(rep, 100 + rep)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    raw = np.zeros((ncell, 16), np.uint64)
    assert L.pmc_debug_stamps(ncell, raw.ctypes.data) == 0
    st = raw[:, :10].copy()
    full = np.all(st > 0, axis=1)
    s = st[full].astype(np.int64)
    base = int(st[st[:, 0] > 0, 0].min())
    span = int(st[full, 9].max()) - base
    d = np.diff(s, axis=1)
    life = s[:, 9] - s[:, 0]
    print(f"phase {rep}: wall {dt*1e3:.3f} ms, stamp span {span} ticks -> {span/dt/1e6:.0f} MHz-equiv; "
          f"visits {full.sum()} of {ncell}")
    for k, nm in enumerate(names):
        print(f"  {nm:14s} mean {d[:, k].mean():8.0f}  median {np.median(d[:, k]):8.0f}  "
              f"share {d[:, k].mean() / life.mean() * 100:5.1f}%")
    print(f"  lifetime mean {life.mean():.0f} median {np.median(life):.0f} p99 {np.percentile(life, 99):.0f}")
    # two cells per wave: cell A = even colour-cell index, B = odd (B's loads go out after A's visit)
    idx = np.nonzero(full)[0]
    for nm_ab, sel in (("A (even)", idx % 2 == 0), ("B (odd)", idx % 2 == 1)):
        dd = d[sel]
        print(f"  cell {nm_ab}: " + ", ".join(f"{nm} {dd[:, k].mean():.0f}" for k, nm in enumerate(names)))
    starts = np.sort(st[full, 0].astype(np.int64) - base)
    print(f"  start quantiles (ticks): " + " ".join(f"{q}%:{np.percentile(starts, q):.0f}" for q in (1, 10, 50, 90, 99)))
    ends = np.sort(st[full, 9].astype(np.int64) - base)
    print(f"  end quantiles (ticks):   " + " ".join(f"{q}%:{np.percentile(ends, q):.0f}" for q in (1, 10, 50, 90, 99, 100)))
