# Occupancy of 3x3x4-cell windows (the cells whose particles can reach one cell's stencil after one
# shiftCells): max / mean / std over a 32^3 box at 4.768 particles per cell, C oracle, sweeps from the
# lattice start.  Bounds the "skip the overflow-fallback launch when no cell can overflow" idea
# (DESIGN section 10, item 5).  Run: python tools/window_stats.py
import sys, time
import numpy as np
sys.path.insert(0, "oracle")
import pmc_oracle as o
o.build()
o.set_threads(8)
cps = 32
atoms = int(round(4.768 * cps**3))
st = o.OracleState(o.make_params(cps=cps))
st.init_lattice(atoms)
def wstats(n):
    n3 = n.reshape(cps, cps, cps).astype(np.int64)  # z, y, x
    out = {}
    for f, ax in ((0, 2), (1, 1), (2, 0)):
        s = np.zeros_like(n3)
        shape = [3, 3, 3]; shape[ax] = 4
        for dz in range(shape[0]):
            for dy in range(shape[1]):
                for dx in range(shape[2]):
                    s += np.roll(n3, (-dz, -dy, -dx), axis=(0, 1, 2))
        out[f] = (s.max(), s.mean(), s.std())
    return out
t0 = time.time()
done = 0
for target in (0, 10, 40, 100, 200, 400):
    if target > done:
        st.run(done, target - done); done = target
    w = wstats(st.n)
    print(done, "max n", st.n.max(), " ".join(f"f{f}: max {m} mean {a:.1f} std {s:.2f}" for f, (m, a, s) in w.items()), f"{time.time()-t0:.0f}s", flush=True)
