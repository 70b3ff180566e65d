"""The product slab driver (pmc_slab_sweep, C) at world sizes > 1 on ONE GPU.

W slab contexts live in one process, one host thread per rank, and exchange their halos through
the in-process transport (pmc_local_group): the same schedule, streams, events, peers and message
lists the driver hands to RCCL on a multi-GPU node, carried as device-to-device copies.  Each W is
compared bit for bit with the C oracle's whole-box run (every occupied slot, counts, the four
counters; the energy to rounding of the per-slab sums), over sweeps that shift along x, y and z
in both directions (start.cu:237-260 is the loop being partitioned), plus a snapshot restart.
Tolerance: none for state and counters.
"""
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run_ranks(world, fn, timeout=240):
    """fn(rank) in one thread per rank; re-raise the first failure."""
    out, err = [None] * world, [None] * world

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException as e:  # noqa: BLE001 -- reported below
            err[r] = e

    th = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
    assert not any(t.is_alive() for t in th), "a rank thread is still running"
    for e in err:
        if e is not None:
            raise e
    return out


def _window(oracle, count):
    """First sweep s of a window [s, s+count) whose plans shift along x, y, and z both ways."""
    for s in range(0, 400):
        plans = [oracle.sweep_plan(1234, s + k, 2.5) for k in range(count)]
        fs = {f for _, f, _ in plans}
        zdirs = {d > 0 for _, f, d in plans if f == 2}
        if fs == {0, 1, 2} and zdirs == {True, False}:
            return s
    raise AssertionError("no window")


FULL = 1   # PMC_FLAG_FULL_SHUFFLE: the reference-like colour order (up to 8 runs, 8 exchanges a sweep)


@pytest.mark.parametrize("world,cps,cps_y,cps_z,atoms,flags", [
    (2, 16, 16, 16, 10_000, 0),
    (3, 16, 16, 12, 7_500, 0),
    (4, 16, 16, 16, 10_000, 0),
    (8, 16, 16, 16, 10_000, 0),      # 2 planes per rank: no interior launch at all
    (4, 32, 32, 32, 120_000, 0),
    (2, 12, 20, 16, 9_000, 0),       # rectangular x/y
    (2, 16, 16, 16, 10_000, FULL),
    (4, 16, 16, 16, 10_000, FULL),
    (4, 32, 32, 32, 120_000, FULL),
])
def test_c_slab_driver_world_equals_oracle(pmc, oracle, world, cps, cps_y, cps_z, atoms, flags):
    from pmc_amd.engine import LocalGroup
    from pmc_amd.slab import SlabDriver
    nz = cps_z // world
    count = 8
    first = _window(oracle, count)
    if flags:   # the window has runs of one colour parity shorter than 4 (more exchanges)
        runs = [sum(1 for k in range(1, 8) if o[k] % 2 != o[k - 1] % 2) + 1
                for o, _, _ in (oracle.sweep_plan(1234, first + j, 2.5, flags) for j in range(count))]
        assert max(runs) > 2, runs
    pmc.lib()
    group = LocalGroup(world)
    drivers = [None] * world

    def rank_main(r):
        d = SlabDriver(cps=cps, cps_y=cps_y, nz_local=nz, rank=r, world=world, atoms_total=atoms,
                       local_group=group, flags=flags)
        drivers[r] = d
        d.run(first, count)
        d.ctx.synchronize()
        obs = d.ctx.slab_observables()          # collective: whole-box sums over the ranks
        return d.owned(), d.ctx.stats(), d.ctx.energy(), d.ctx.error_flags(), obs

    res = _run_ranks(world, rank_main)
    st = oracle.OracleState(oracle.make_params(cps=cps, cps_y=cps_y, cps_z=cps_z, flags=flags))
    assert st.init_lattice(atoms) == 0
    assert st.run(first, count) == 0
    plane, row = cps * cps_y, 3 * 16
    tot = {"de_fixed": 0, "accepted": 0, "trials": 0, "evaluated": 0}
    e_sum = 0.0
    for r, ((d, n), s, e, fl, _) in enumerate(res):
        ref = slice(r * nz * plane, (r + 1) * nz * plane)
        assert np.array_equal(n, st.n[ref]), f"rank {r}: counts differ"
        assert oracle.valid_slots_equal(d, n, st.disk[ref.start * row:ref.stop * row], st.n[ref], 16), \
            f"rank {r}: coordinates differ"
        assert fl == 0
        for k in tot:
            tot[k] += s[k]
        e_sum += e
    assert tot == st.stats.as_dict()
    assert int(sum(int(n.sum()) for (_, n), *_ in res)) == atoms
    assert e_sum == pytest.approx(st.energy(), rel=1e-9, abs=1e-9)
    # pmc_slab_observables: every rank gets the whole box's counters and its energy, summed in
    # fixed point -- equal to the oracle's whole-box values exactly
    for *_, (obs, e_all) in res:
        assert obs == st.stats.as_dict()
        assert e_all == st.energy()
    for d in drivers:
        d.ctx.close()
    group.close()


@pytest.mark.parametrize("halo", [1, 2])
def test_c_slab_driver_world3_restart(pmc, oracle, tmp_path, halo):
    """Per-rank snapshots + halo refill through the in-process transport: a fresh group restored
    from the snapshots repeats the last sweeps bit for bit (one- and two-plane halos)."""
    from pmc_amd.engine import LocalGroup
    from pmc_amd.slab import SlabDriver
    world, cps, cps_z, atoms = 3, 16, 12, 7_500
    nz = cps_z // world
    first = _window(oracle, 6)
    pmc.lib()
    group = LocalGroup(world)
    paths = [str(tmp_path / f"rank{r}.pmcsnap") for r in range(world)]
    keep = []

    def part1(r):
        d = SlabDriver(cps=cps, nz_local=nz, rank=r, world=world, atoms_total=atoms, local_group=group, halo=halo)
        keep.append(d)
        d.run(first, 3)
        d.ctx.save_snapshot(paths[r], first + 3)
        d.run(first + 3, 3)
        return d.owned(), d.ctx.stats()

    a = _run_ranks(world, part1)
    for d in keep:
        d.ctx.close()
    group.close()
    group2 = LocalGroup(world)
    keep2 = []

    def part2(r):
        d = SlabDriver(cps=cps, nz_local=nz, rank=r, world=world, local_group=group2, halo=halo)
        keep2.append(d)
        s = d.ctx.load_snapshot(paths[r])
        d.ctx.slab_exchange()
        d.run(s, 3)
        return d.owned(), d.ctx.stats()

    b = _run_ranks(world, part2)
    for r in range(world):
        (d1, n1), s1 = a[r]
        (d2, n2), s2 = b[r]
        assert np.array_equal(n1, n2)
        assert oracle.valid_slots_equal(d1, n1, d2, n2, 16)
        assert s1 == s2
    for d in keep2:
        d.ctx.close()
    group2.close()


def test_local_group_missing_rank_fails_not_hangs(pmc):
    """A rank that never joins an exchange breaks the group after the barrier timeout: the caller
    gets an error instead of a hang."""
    from pmc_amd.engine import LocalGroup
    from pmc_amd._lib import PmcError
    from pmc_amd.slab import SlabDriver
    pmc.lib()
    os.environ["PMC_LOCAL_GROUP_TIMEOUT_MS"] = "1500"
    try:
        group = LocalGroup(2)
    finally:
        del os.environ["PMC_LOCAL_GROUP_TIMEOUT_MS"]
    d = SlabDriver(cps=16, nz_local=8, rank=0, world=2, local_group=group)
    with pytest.raises(PmcError):
        d.ctx.slab_exchange()
    with pytest.raises(PmcError):   # the group stays broken
        d.ctx.slab_exchange()
    d.ctx.close()
    group.close()


# defaults: split shift and deferred z exchanges on (in the window, sweeps 16 and 17 defer; the last
# deferred one is flushed by finish)
_ROUND3 = {"PMC_SLAB_SPLIT_SHIFT": "0", "PMC_SLAB_DEFER_Z": "0"}   # round 3's schedule
_BFULL = {"PMC_BOUNDARY_FULL": "1"}
_DIRECT = {"PMC_SLAB_DIRECT_HALO": "1"}   # one rank, no transport: boundary launches write the halo


@pytest.mark.parametrize("chains,env,world,cps,nz,atoms", [
    (1, {}, 4, 16, 4, 10_000),
    (3, {}, 2, 32, 16, 120_000),       # interior chains [1,6), [6,10), [10,15)
    (3, {}, 4, 32, 8, 120_000),        # [1,4), [4,6), [6,7)
    (2, _ROUND3, 4, 32, 8, 120_000),   # no split shift, no deferral
    (3, _ROUND3, 2, 32, 16, 120_000),
    (2, _BFULL, 4, 32, 8, 120_000),    # full-capacity boundary launches
    (2, _BFULL, 2, 16, 8, 10_000),
    (2, _DIRECT, 1, 32, 32, 120_000),  # direct halo writes (one rank without a transport), z shifts
    (2, {**_DIRECT, **_ROUND3}, 1, 16, 16, 10_000),
])
def test_c_slab_driver_chain_count(pmc, oracle, chains, env, world, cps, nz, atoms):
    """PMC_SLAB_CHAINS=1 (one interior chain per rank: every phase one launch on the context
    stream) and =3 (three interior chains on three streams beside the exchange stream), with the
    default split shift (x/y shifts: the halo the last exchange fills shifted on the exchange
    stream, every other plane on the context stream without waiting for that exchange) and deferred
    z exchanges (a z shift's halo plane carried by the next sweep's first run exchange when that run
    does not read it), without both (PMC_SLAB_SPLIT_SHIFT=0, PMC_SLAB_DEFER_Z=0), and with
    PMC_BOUNDARY_FULL=1 (boundary phases as one full-capacity launch), and PMC_SLAB_DIRECT_HALO=1 (one
    rank without a transport: the boundary launches write each row into the periodic halo too),
    through the in-process transport, equal the oracle's whole box over 8 sweeps with shifts along
    x, y and z both ways.  Subprocess: the switches are read once per process."""
    import subprocess
    import sys
    code = r'''
import sys, threading, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2], sys.argv[3]]
import pmc_amd, pmc_oracle
from test_gpu_multirank import _run_ranks, _window
from pmc_amd.engine import LocalGroup
from pmc_amd.slab import SlabDriver
world, cps, nz, atoms, chains = (int(v) for v in sys.argv[4:9])
first = _window(pmc_oracle, 8)
pmc_amd.lib()
g = LocalGroup(world)
keep = []
def main(r):
    if world == 1:   # one rank without a transport: periodic halos by local copies (or direct writes)
        d = SlabDriver(cps=cps, nz_local=nz, rank=0, world=1, atoms_total=atoms, transport="local")
    else:
        d = SlabDriver(cps=cps, nz_local=nz, rank=r, world=world, atoms_total=atoms, local_group=g)
    keep.append(d)
    lay = d.ctx.slab_layout()
    d.run(first, 8)
    assert d.ctx.error_flags() == 0, d.ctx.error_flags()
    return d.owned(), d.ctx.stats(), lay
res = _run_ranks(world, main)
st = pmc_oracle.OracleState(pmc_oracle.make_params(cps=cps, cps_z=world * nz))
st.init_lattice(atoms)
st.run(first, 8)
plane, row = cps * cps, 48
tot = {}
for r, ((d, n), s, lay) in enumerate(res):
    assert len(lay) == chains and lay[0][0] == 1 and lay[-1][1] == nz - 1, lay
    ref = slice(r * nz * plane, (r + 1) * nz * plane)
    assert np.array_equal(n, st.n[ref])
    assert pmc_oracle.valid_slots_equal(d, n, st.disk[ref.start * row:ref.stop * row], st.n[ref], 16)
    for k, v in s.items():
        tot[k] = tot.get(k, 0) + v
assert tot == st.stats.as_dict()
print("ok")
'''
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code, os.path.join(repo, "parallel-monte-carlo_amd"),
                          os.path.join(repo, "oracle"), os.path.join(repo, "tests"),
                          str(world), str(cps), str(nz), str(atoms), str(chains)],
                         env=dict(os.environ, PMC_SLAB_CHAINS=str(chains), **env),
                         capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "ok" in out.stdout


def _world_vs_oracle(pmc, oracle, world, cps, nz, atoms, first, count, lattice_cps_z=0, threads=16, halo=1):
    """World ranks of the C slab driver (in-process transport, one GPU) over `count` sweeps of the
    cps x cps x world*nz box against the oracle's whole-box run: every occupied slot, counts, the
    four counters (summed over ranks and through pmc_slab_observables) and the energy."""
    from pmc_amd.engine import LocalGroup
    from pmc_amd.slab import SlabDriver
    pmc.lib()
    group = LocalGroup(world)
    drivers = [None] * world

    def rank_main(r):
        d = SlabDriver(cps=cps, nz_local=nz, rank=r, world=world, atoms_total=atoms, local_group=group,
                       lattice_cps_z=lattice_cps_z, halo=halo)
        drivers[r] = d
        d.run(first, count)
        d.ctx.synchronize()
        obs = d.ctx.slab_observables()
        return d.owned(), d.ctx.stats(), d.ctx.error_flags(), obs

    res = _run_ranks(world, rank_main, timeout=600)
    for d in drivers:      # device memory back before the oracle's host arrays grow
        d.ctx.close()
    group.close()
    oracle.set_threads(threads)
    st = oracle.OracleState(oracle.make_params(cps=cps, cps_z=world * nz))
    assert st.init_lattice(atoms) == 0
    assert int(st.n.sum()) == atoms
    assert st.run(first, count) == 0
    plane, row = cps * cps, 3 * 16
    tot = {"de_fixed": 0, "accepted": 0, "trials": 0, "evaluated": 0}
    for r, ((d, n), s, fl, _) in enumerate(res):
        ref = slice(r * nz * plane, (r + 1) * nz * plane)
        assert np.array_equal(n, st.n[ref]), f"rank {r}: counts differ"
        assert oracle.valid_slots_equal(d, n, st.disk[ref.start * row:ref.stop * row], st.n[ref], 16), \
            f"rank {r}: coordinates differ"
        assert fl == 0
        for k in tot:
            tot[k] += s[k]
    o = st.stats.as_dict()
    assert tot == o
    assert o["trials"] > 0 and o["accepted"] > 0
    assert sum(int(n.sum()) for (_, n), *_ in res) == atoms
    e = st.energy()
    for *_, (obs, e_all) in res:
        assert obs == o
        assert e_all == e
    return o


@pytest.mark.timeout(400)
def test_slab_long_run_world4_64_equals_oracle(pmc, oracle):
    """4 slab ranks of the 64^3 / 1e6 box over 24 sweeps from the lattice start (the counts spread
    from 4-5 per cell through the relaxation; every exchange kind recurs many times): bitwise equal
    to the oracle's whole-box run."""
    _world_vs_oracle(pmc, oracle, 4, 64, 16, 1_000_000, 0, 24)


@pytest.mark.timeout(400)
def test_config4_world8_128_equals_oracle(pmc, oracle):
    """BASELINE config 4 at its workload: the 128^3-cell, 1e7-particle box in 8 z-slabs of 16
    planes (pmc_init_lattice_global: every rank starts from its planes of the one-GPU lattice),
    three sweeps of the product slab driver -- sweeps 13-15 shift along z in both directions --
    against the oracle's whole-box run bit for bit (start.cu:237-260 is the loop partitioned)."""
    plans = [oracle.sweep_plan(1234, s, 2.5) for s in (13, 14, 15)]
    assert {(f, d > 0) for _, f, d in plans} >= {(2, True), (2, False)}
    _world_vs_oracle(pmc, oracle, world=8, cps=128, nz=16, atoms=10_000_000, first=13, count=3)


@pytest.mark.timeout(400)
def test_config4_world8_128_halo2_equals_oracle(pmc, oracle):
    """Config 4 at its workload with two-plane halos (one exchange per sweep, the neighbour's
    boundary plane visited redundantly in the first run): sweeps 13-15, whose z shifts include the
    case that exchanges the stale halo before shiftCells (sweep 13: first run parity 1, +z), bit for
    bit against the oracle's whole box."""
    _world_vs_oracle(pmc, oracle, world=8, cps=128, nz=16, atoms=10_000_000, first=13, count=3, halo=2)


def _window_h2(oracle, count=8):
    """First sweep of a window with shifts along x, y and z whose z shifts cover all four cases of
    the two-plane-halo schedule: first-run parity a = 0 with dir < 0 and a = 1 with dir > 0 (the
    halo shiftCells reads is stale: one plane exchanged first, T shifts the boundary plane) and the
    two fresh ones."""
    for s in range(0, 1000):
        ks = []
        for k in range(count):
            o, f, d = oracle.sweep_plan(1234, s + k, 2.5)
            ks.append((f, o[0] % 2, -1 if d <= 0 else 1))
        z = {(a, dr) for f, a, dr in ks if f == 2}
        if {f for f, _, _ in ks} == {0, 1, 2} and z == {(0, -1), (0, 1), (1, -1), (1, 1)}:
            return s
    raise AssertionError("no window")


@pytest.mark.parametrize("world,cps,nz,atoms", [
    (1, 32, 32, 120_000),      # one rank: the halos are its own planes (periodic)
    (2, 16, 8, 10_000),
    (3, 16, 4, 7_500),
    (4, 32, 8, 120_000),
    (8, 16, 2, 10_000),        # 2 planes per rank: the send planes are the whole slab
])
def test_c_slab_driver_halo2_equals_oracle(pmc, oracle, world, cps, nz, atoms):
    """Two-plane halos (pmc_params.halo = 2, slab_sweep_h2) through the in-process transport over a
    window of 8 sweeps with shifts along x, y and both z cases of each first-run parity, against the
    oracle's whole box: every occupied slot, counts, the four counters (the redundant halo visits
    count nowhere), the energy, no error flag."""
    first = _window_h2(oracle)
    o = _world_vs_oracle(pmc, oracle, world=world, cps=cps, nz=nz, atoms=atoms, first=first, count=8, halo=2)
    assert o["evaluated"] > 0


@pytest.mark.timeout(600)
def test_config5_world8_256_equals_oracle(pmc, oracle):
    """BASELINE config 5 at its workload: 8 slabs of 256x256x32 cells, together the 256^3-cell box
    with the 8e7-particle lattice (each rank keeps its planes of it, pmc_init_lattice_planes), two
    sweeps with z shifts both ways, against the oracle's whole 256^3 box bit for bit."""
    plans = [oracle.sweep_plan(1234, s, 2.5) for s in (13, 14)]
    assert {(f, d > 0) for _, f, d in plans} == {(2, True), (2, False)}
    _world_vs_oracle(pmc, oracle, world=8, cps=256, nz=32, atoms=80_000_000, first=13, count=2,
                     lattice_cps_z=256)


def test_bench_parity_leg_slab_world4(pmc, oracle):
    """bench.py's N > 1 parity leg (parity_leg_slab) at world 4 on one GPU: four slab ranks in
    threads over the in-process transport, a thread-level gather standing in for dist.gather.
    Every rank restores its timed-start storage, reruns the sample's sweep through the slab driver
    and contributes to pmc_slab_observables; rank 0 compares the gathered whole box with the oracle's
    sweep from the same state: every occupied slot, the four counters, the energy (kernel.cu:452-470),
    all exact.  This is the collective rerun and observables path the driver's SCALE line uses."""
    import sys
    import threading
    from pmc_amd.engine import LocalGroup
    from pmc_amd.slab import SlabDriver
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    import bench
    world, cps, nz, atoms, first = 4, 32, 8, 120_000, 5
    plane, row = cps * cps, 3 * 16
    pmc.lib()
    group = LocalGroup(world)
    bar = threading.Barrier(world, timeout=120)
    parts = [None] * world
    whole_box = {}

    def make_thread_gather(rank):
        def gather(disk_s, n_s):
            parts[rank] = (disk_s[plane * row:(nz + 1) * plane * row].copy(), n_s[plane:(nz + 1) * plane].copy())
            bar.wait()
            out = None
            if rank == 0:
                out = (np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]))
            bar.wait()
            return out
        return gather

    drivers = [None] * world

    def rank_main(r):
        d = SlabDriver(cps=cps, nz_local=nz, rank=r, world=world, atoms_total=atoms, local_group=group)
        drivers[r] = d
        d.run(0, first)                                 # warm-up sweeps 0..first-1
        d.ctx.synchronize()
        disk_s, n_s = d.ctx.copy_out()                  # the timed region's start state (storage)
        gather = make_thread_gather(r)
        whole = gather(disk_s, n_s)
        if r == 0:                                      # the oracle's sample sweep on the whole box
            st = oracle.OracleState(oracle.make_params(cps=cps, cps_z=world * nz))
            st.disk[:] = whole[0]
            st.n[:] = whole[1]
            assert st.run(first, 1) == 0
            whole_box["ost"] = st
        bar.wait()
        return bench.parity_leg_slab(d.ctx, d.sweep, d.finish, disk_s, n_s, first, 0.0, gather,
                                     whole_box.get("ost"), r)

    res = _run_ranks(world, rank_main, timeout=300)
    for d in drivers:
        d.ctx.close()
    group.close()
    assert all(v is None for v in res[1:])
    rec = res[0]
    assert rec["state_bitwise_equal"] is True
    assert rec["counters_equal"] is True
    assert rec["energy_rel_err"] == 0.0 and rec["acceptance_rel_err"] == 0.0


def test_energy_refuses_pending_z_exchange(pmc, oracle):
    """A z-shift sweep whose halo the next sweep's first run does not read leaves that exchange deferred
    (PMC_SLAB_DEFER_Z, default on) until the next sweep, pmc_slab_finish or pmc_slab_observables; the energy kernel reads halo neighbours, so
    pmc_energy refuses the state meanwhile (PMC_ERR_ARG, no silent stale halo and no collective flush
    inside a local call).  After pmc_slab_finish it equals the oracle's whole-box energy."""
    from pmc_amd._lib import PmcError
    from pmc_amd.slab import SlabDriver
    def deferred(s):   # a z shift whose halo the next sweep's first run does not read (pmc_slab_sweep)
        _, f, dz = oracle.sweep_plan(1234, s, 2.5)
        return f == 2 and oracle.sweep_plan(1234, s + 1, 2.5)[0][0] % 2 == (0 if dz > 0 else 1)
    s_z = next(s for s in range(1, 200) if deferred(s))
    d = SlabDriver(cps=16, nz_local=16, rank=0, world=1, atoms_total=10_000, transport="local")
    for s in range(s_z + 1):
        d.sweep(s)
    with pytest.raises(PmcError, match="pending"):
        d.ctx.energy()
    d.finish()
    st = oracle.OracleState(oracle.make_params(cps=16))
    assert st.init_lattice(10_000) == 0
    assert st.run(0, s_z + 1) == 0
    assert d.ctx.energy() == pytest.approx(st.energy(), rel=1e-9, abs=1e-9)
    assert d.ctx.error_flags() == 0
    d.ctx.close()
