"""pmc_sweep's plane chains (PMC_SWEEP_CHAINS = 1, 2, 4): each colour phase split into one launch per
chain of planes, on streams of their own, ordered only at runs of equal z parity by the neighbours'
previous runs (the slab driver's rule).  Every chain count gives the oracle's whole-box run bit for
bit -- occupied slots, counts, the four counters, the energy -- over sweeps that shift along x, y and
z in both directions (start.cu:237-260).  The variable is read once per process: one process per
count.  Tolerance: none.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(REPO, "tests", "chain_worker.py")


def _window(oracle, count):
    for s in range(0, 400):
        plans = [oracle.sweep_plan(1234, s + k, 2.5) for k in range(count)]
        if {f for _, f, _ in plans} == {0, 1, 2} and {d > 0 for _, f, d in plans if f == 2} == {True, False}:
            return s
    raise AssertionError("no window")


@pytest.mark.parametrize("chains,cps,atoms,want", [
    (4, (32, 32, 32), 120_000, [(0, 8), (8, 16), (16, 24), (24, 32)]),
    (4, (16, 12, 20), 11_000, [(0, 4), (4, 10), (10, 14), (14, 20)]),   # ragged even borders
    (4, (16, 16, 12), 9_000, [(0, 6), (6, 12)]),                         # too thin for 4: two chains
    (2, (16, 16, 16), 10_000, [(0, 8), (8, 16)]),
    (2, (12, 8, 10), 2_500, [(0, 4), (4, 10)]),          # ragged halves
    (2, (8, 8, 8), 1_500, [(0, 4), (4, 8)]),              # the thinnest box that still splits
    (2, (16, 16, 6), 4_000, [(0, 6)]),                    # too thin: one launch per phase
    (1, (16, 16, 16), 10_000, [(0, 16)]),
])
def test_sweep_chains_equal_oracle(oracle, tmp_path, chains, cps, atoms, want):
    count = 6
    first = _window(oracle, count)
    out = str(tmp_path / "out")
    env = dict(os.environ, PMC_SWEEP_CHAINS=str(chains))
    p = subprocess.run([sys.executable, WORKER, out] + [str(v) for v in cps] + [str(atoms), str(first), str(count)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    z = np.load(out + ".npz")
    with open(out + ".json") as f:
        j = json.load(f)
    assert [tuple(b) for b in j["layout"]] == want
    cx, cy, cz = cps
    st = oracle.OracleState(oracle.make_params(cps=cx, cps_y=cy, cps_z=cz))
    assert st.init_lattice(atoms) == 0
    assert st.run(first, count) == 0
    assert np.array_equal(z["n"], st.n), "cell counts differ"
    assert oracle.valid_slots_equal(z["disk"], z["n"], st.disk, st.n, 16), "particle coordinates differ"
    assert j["stats"] == st.stats.as_dict()
    assert j["energy"] == st.energy()
    assert j["flags"] == 0
