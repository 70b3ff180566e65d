"""The oracle's reference-quirk flags (include/pmc.h PMC_FLAG_QUIRK_*) on CPU:
the flags are accepted and change exactly what they name.  The GPU kernels are held to the oracle
with the same flags in tests/test_gpu_quirks.py."""
import numpy as np
import pytest

R1, R2, S1, FULL = 2, 4, 8, 1


def _state(oracle, flags, atoms=1000, cps=8):
    st = oracle.OracleState(oracle.make_params(cps=cps, flags=flags))
    assert st.init_lattice(atoms) == 0
    return st


def test_quirk_flags_accepted_unknown_refused(oracle):
    for f in (R1, R2, S1, R1 | R2 | S1, FULL | R1 | R2 | S1):
        oracle.OracleState(oracle.make_params(cps=8, flags=f))
    with pytest.raises(ValueError):
        oracle.OracleState(oracle.make_params(cps=8, flags=16))


def test_r1_rotation_is_the_reference_shuffle_with_random_int_zero():
    """random_shuffle (subsweep.h:50-58) with random_int always 0 (subsweep.h:38-40: (int) of a
    uniform in (0, 1] is 0): slot i swaps with slot 0 for i = n-1 .. 0, leaving slot l holding
    particle (l + 1) mod n -- the permutation PMC_FLAG_QUIRK_R1 uses."""
    for n in range(1, 20):
        slots = list(range(n))
        for i in range(n - 1, -1, -1):
            j = 0
            slots[i], slots[j] = slots[j], slots[i]
        assert slots == [(l + 1) % n for l in range(n)], n


def test_r2_same_numbers_every_visit(oracle):
    """R2: a colour phase from the same state gives the same result at any sweep index; without it
    the sweep index changes the draws."""
    out = {}
    for flags in (0, R2):
        res = []
        for s in (3, 11):
            st = _state(oracle, flags)
            st.subsweep(oracle.colour_offset(5), s)
            res.append((st.disk.copy(), st.n.copy(), st.stats.as_dict()))
        out[flags] = res
    (d0, n0, s0), (d1, n1, s1) = out[R2]
    assert np.array_equal(n0, n1) and np.array_equal(d0.view(np.uint32), d1.view(np.uint32)) and s0 == s1
    (d0, n0, _), (d1, n1, _) = out[0]
    assert not np.array_equal(d0.view(np.uint32), d1.view(np.uint32))


def test_r1_changes_only_the_visit_order(oracle):
    """R1 changes the result of a phase (the rotation replaces the random permutation) but not the
    particle count or the number of trials."""
    a, b = _state(oracle, 0), _state(oracle, R1)
    a.subsweep(oracle.colour_offset(2), 7)
    b.subsweep(oracle.colour_offset(2), 7)
    assert np.array_equal(a.n, b.n)
    assert a.stats.as_dict()["trials"] == b.stats.as_dict()["trials"]
    assert not np.array_equal(a.disk.view(np.uint32), b.disk.view(np.uint32))


@pytest.mark.parametrize("f", [0, 1, 2])
@pytest.mark.parametrize("d", [1.0, -1.0])
def test_s1_integer_offset(oracle, f, d):
    """S1: the offset added to particles taken from the neighbour cell is (int)(w*dir) = +-2 at
    w = 2.5 instead of +-2.5.  The same particles move; each moved coordinate along the shift axis
    differs from the default's by exactly 0.5, every other coordinate is equal."""
    a, b = _state(oracle, 0), _state(oracle, S1)
    assert a.shift_cells(f, d) == 0 and b.shift_cells(f, d) == 0
    assert np.array_equal(a.n, b.n)
    da, db = a.disk3(), b.disk3()
    mask = np.arange(a.nmax)[None, :] < a.n[:, None]
    for k in range(3):
        diff = (db[:, k, :] - da[:, k, :])[mask]
        if k != f:
            assert not diff.any()
        else:
            moved = diff != 0
            assert moved.any()
            assert np.all(np.abs(diff[moved] - np.float32(-0.5 if d > 0 else 0.5)) < 1e-4), np.unique(diff)


def test_quirk_runs_deterministic(oracle):
    a, b = _state(oracle, R1 | R2 | S1), _state(oracle, R1 | R2 | S1)
    assert a.run(10, 4) == 0 and b.run(10, 4) == 0
    assert np.array_equal(a.disk.view(np.uint32), b.disk.view(np.uint32)) and a.energy() == b.energy()
