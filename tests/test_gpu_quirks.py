"""Reference-quirk flags on the GPU (include/pmc.h PMC_FLAG_QUIRK_*):
R1 (random_int == 0: the own cell visited in the fixed rotation, subsweep.h:38-58), R2
(curand_init(1234, id, 0) every launch: the same numbers at every visit, subsweep.h:256-259) and S1
(int s[3]: the integer shift offset, shiftCells.h:31,105).  With R1/R2 every colour phase runs the
full-capacity kernel instantiated with the quirk bits; S1 has its own shift instantiations; the
default kernels are not touched (their ISA is byte-identical to the build without the flags).  Each
case equals the C oracle (which applies the same flags) bit for bit: counts, every occupied slot,
the four counters, the energy.  Tolerance: none."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

R1, R2, S1, FULL = 2, 4, 8, 1


def _window(oracle, count):
    """First sweep of a window whose plans shift along x, y and z both ways (S1 on every axis)."""
    for s in range(0, 400):
        plans = [oracle.sweep_plan(1234, s + k, 2.5) for k in range(count)]
        if {f for _, f, _ in plans} == {0, 1, 2} and {d > 0 for _, f, d in plans if f == 2} == {True, False}:
            return s
    raise AssertionError("no window")


@pytest.mark.parametrize("flags,nmax", [
    (R1, 16), (R2, 16), (S1, 16), (R1 | R2, 16), (R1 | R2 | S1, 16), (FULL | R1 | R2 | S1, 16),
    (R1 | R2 | S1, 32), (R1 | S1, 24), (R2, 12),
])
def test_quirks_whole_box_equal_oracle(pmc, oracle, flags, nmax):
    count = 8
    first = _window(oracle, count)
    ctx = pmc.PmcContext(16, nmax=nmax, flags=flags)
    ctx.init_lattice(10_000)
    r = ctx.start(first, count)
    st = oracle.OracleState(oracle.make_params(cps=16, nmax=nmax, flags=flags))
    assert st.init_lattice(10_000) == 0
    assert st.run(first, count) == 0
    disk, n = ctx.copy_out()
    assert np.array_equal(n, st.n), "cell counts differ"
    assert oracle.valid_slots_equal(disk, n, st.disk, st.n, nmax), "particle coordinates differ"
    o = st.stats.as_dict()
    for k in ("de_fixed", "accepted", "trials", "evaluated"):
        assert r[k] == o[k], k
    assert r["e_final"] == st.energy()
    assert ctx.error_flags() == 0
    ctx.close()


def test_quirks_change_the_trajectory(pmc, oracle):
    """Each flag changes the run (the flags are not ignored): R1, R2 and S1 states all differ from
    the default and from each other after a few sweeps; the default run is the corrected semantics."""
    first = _window(oracle, 8)
    states = {}
    for flags in (0, R1, R2, S1):
        ctx = pmc.PmcContext(16, flags=flags)
        ctx.init_lattice(10_000)
        ctx.start(first, 8)
        d, n = ctx.copy_out()
        states[flags] = (d.copy(), n.copy())
        ctx.close()
    keys = list(states)
    for i, a in enumerate(keys):
        for b in keys[i + 1:]:
            da, na = states[a]
            db, nb = states[b]
            assert not (np.array_equal(na, nb) and np.array_equal(da.view(np.uint32), db.view(np.uint32))), (a, b)


def test_quirk_r2_same_numbers_every_visit(pmc, oracle):
    """R2: a colour phase from the same state draws the same numbers whatever the sweep index."""
    outs = []
    for s in (3, 11):
        ctx = pmc.PmcContext(16, flags=R2)
        ctx.init_lattice(10_000)
        ctx.phase(5, s)
        outs.append(ctx.copy_out() + (ctx.stats(),))
        ctx.close()
    (d0, n0, s0), (d1, n1, s1) = outs
    assert np.array_equal(n0, n1) and np.array_equal(d0.view(np.uint32), d1.view(np.uint32))
    assert s0 == s1


def test_quirks_slab_ranks_equal_oracle(pmc, oracle):
    """The C slab driver (in-process transport, 4 ranks of the 16^3 box) with all three quirks: the
    interior, boundary and deferred-plane launches and the halo shifts all take the quirk
    instantiations; the ranks' owned planes equal the oracle's whole-box run."""
    import threading
    from pmc_amd.engine import LocalGroup
    from pmc_amd.slab import SlabDriver
    world, cps, atoms, count = 4, 16, 10_000, 8
    flags = R1 | R2 | S1
    first = _window(oracle, count)
    pmc.lib()
    group = LocalGroup(world)
    res, errs = [None] * world, []

    def rank_main(r):
        try:
            d = SlabDriver(cps=cps, nz_local=cps // world, rank=r, world=world, atoms_total=atoms,
                           local_group=group, flags=flags)
            d.run(first, count)
            d.ctx.synchronize()
            res[r] = (d.owned(), d.ctx.stats(), d.ctx.error_flags(), d)
        except Exception as e:  # noqa: BLE001
            errs.append((r, repr(e)))
            group.close()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(240)
    assert not errs, errs
    st = oracle.OracleState(oracle.make_params(cps=cps, flags=flags))
    assert st.init_lattice(atoms) == 0
    assert st.run(first, count) == 0
    nz, plane, row = cps // world, cps * cps, 3 * 16
    tot = dict.fromkeys(("de_fixed", "accepted", "trials", "evaluated"), 0)
    for r, ((d, n), s, fl, _) in enumerate(res):
        ref = slice(r * nz * plane, (r + 1) * nz * plane)
        assert np.array_equal(n, st.n[ref]), f"rank {r}: counts differ"
        assert oracle.valid_slots_equal(d, n, st.disk[ref.start * row:ref.stop * row], st.n[ref], 16), r
        assert fl == 0
        for k in tot:
            tot[k] += s[k]
    assert tot == st.stats.as_dict()
    for *_, drv in res:
        drv.ctx.close()
    group.close()


def test_quirks_refused_where_unsupported(pmc):
    """Two-plane halos and the persistent small-box kernel refuse R1/R2 (loudly, not silently)."""
    with pytest.raises(pmc.PmcError):
        pmc.PmcContext(16, cps_z=16, nz_local=8, z0=0, halo=2, flags=R1)
    ctx = pmc.PmcContext(16, flags=R2)
    ctx.init_lattice(10_000)
    with pytest.raises(pmc.PmcError):
        ctx.run_small(0, 2)
    ctx.close()
    with pytest.raises(pmc.PmcError):
        pmc.PmcContext(16, flags=16)     # no such flag
