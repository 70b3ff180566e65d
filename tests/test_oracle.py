"""CPU tests of the oracle: pinned against the reference's own data file (dumpR3.txt frames),
lattice energies derived from the reference's definitions, published Philox KATs and statistical
known answers of an independent textbook Metropolis code (tests/golden/known_answers.json)."""
import json
import math
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "dumpR3_frames.npz")


# ---------------------------------------------------------------------------------------------
# primitives
# ---------------------------------------------------------------------------------------------
def test_philox_kat(oracle):
    # Random123 kat_vectors, philox4x32_10
    assert oracle.philox([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert oracle.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert oracle.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_logf_accuracy(oracle):
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.random(4000), [2.0**-24, 0.5, 0.70710678, 0.9999999, 1.0 - 2.0**-24]])
    for x in xs.astype(np.float32):
        x = float(x)
        if x <= 0:
            continue
        ref = math.log(x)
        assert abs(oracle.logf(x) - ref) <= 3e-7 * max(1.0, abs(ref))


def test_recip_accuracy(oracle):
    rng = np.random.default_rng(2)
    for x in np.concatenate([rng.uniform(1e-4, 200.0, 4000), [1e-4, 1.0, 6.25, 1.5]]).astype(np.float32):
        r = oracle.recip(float(x))
        assert abs(r * float(x) - 1.0) < 2.5e-7


def test_det_sincos_accuracy(oracle):
    for k in range(0, 2**23, 2**23 // 997):
        u = float(np.float32((2 * k + 1) * 2.0**-24))
        s, c = oracle.det_sincos_2pi(u)
        assert abs(s - math.sin(2 * math.pi * u)) < 1.2e-7
        assert abs(c - math.cos(2 * math.pi * u)) < 1.2e-7


def test_normals_moments(oracle):
    import ctypes as C
    g = (C.c_float * 3)()
    vals = []
    for i in range(20000):
        w = oracle.philox([i, 7, 0, 0], [1234, 0])
        oracle.lib().orc_move_normals(C.byref((C.c_uint32 * 4)(*w)), C.byref(g))
        vals.extend(g)
    v = np.array(vals)
    assert abs(v.mean()) < 0.02 and abs(v.std() - 1) < 0.02
    assert abs(np.mean(v**4) - 3) < 0.15


def test_pair_energy_and_cutoff(oracle):
    rc2 = oracle.cutoff_r2(2.5)
    # the r^2 cutoff is the reference's sqrtf(r2) > w predicate (subsweep.h:96-99)
    assert np.sqrt(np.float32(rc2)) <= np.float32(2.5)
    assert np.sqrt(np.nextafter(np.float32(rc2), np.float32(10))) > np.float32(2.5)
    for r in (0.9, 1.0, 1.122462, 1.5, 2.0, 2.49):
        e = oracle.pair_energy(r, 0.0, 0.0, rc2)
        ref = 4 * (r**-12 - r**-6)
        assert e == pytest.approx(ref, rel=2e-6, abs=1e-7)
    assert oracle.pair_energy(2.6, 0.0, 0.0, rc2) == 0.0
    assert np.isfinite(oracle.pair_energy(0.0, 0.0, 0.0, rc2))


def test_sweep_plan(oracle):
    fs = []
    for s in range(300):
        order, f, d = oracle.sweep_plan(1234, s)
        assert sorted(order) == list(range(8))
        assert f in (0, 1, 2)
        assert -1.25 < d < 1.25 and d != 0.0
        fs.append(f)
    assert set(fs) == {0, 1, 2}
    assert oracle.sweep_plan(1234, 3) == oracle.sweep_plan(1234, 3)
    assert oracle.sweep_plan(1234, 3) != oracle.sweep_plan(1235, 3)


def test_sweep_plan_grouped_by_z_parity(oracle):
    """Spec v9 default: the 4 colours of one z parity (colour % 2, itoa start.cu:153-157), then the
    other 4, each group shuffled; either parity first.  PMC_FLAG_FULL_SHUFFLE: one shuffle of all 8
    (the reference's FY_Shuffle) -- same shift (f, d) either way."""
    firsts, orders, ungrouped = set(), set(), 0
    for s in range(400):
        order, f, d = oracle.sweep_plan(1234, s)
        par = [c % 2 for c in order]
        assert par[:4] == [par[0]] * 4 and par[4:] == [1 - par[0]] * 4, order
        firsts.add(par[0])
        orders.add(tuple(order[:4]))
        o2, f2, d2 = oracle.sweep_plan(1234, s, flags=1)
        assert sorted(o2) == list(range(8)) and (f2, d2) == (f, d)
        p2 = [c % 2 for c in o2]
        ungrouped += p2[:4] != [p2[0]] * 4
    assert firsts == {0, 1}
    assert len(orders) == 48                  # 2 parities x 4! orders of the first group
    assert ungrouped > 200                    # the full shuffle is not grouped


def test_fixed_point(oracle):
    f = oracle.lib().orc_to_fixed
    assert f(1.0) == 2**32 and f(-1.0) == -(2**32)
    assert f(0.5 / 2**32) == 1 and f(-0.5 / 2**32) == -1 and f(0.49 / 2**32) == 0
    assert f(1e30) == 2**62


# ---------------------------------------------------------------------------------------------
# pinned against the reference's data (dumpR3.txt) and definitions
# ---------------------------------------------------------------------------------------------
def test_init_r_matches_dumpR3_frame0(oracle):
    """Frame 0 of the reference trajectory is its init_r lattice for N=64 (kernel.cu:78-89)."""
    g = np.load(GOLDEN)
    st = oracle.OracleState(oracle.make_params(cps=4, nmax=10))
    r = st.init_r(64).reshape(3, 64).T
    assert np.array_equal(r.astype(np.float64), g["positions"][0])


@pytest.mark.parametrize("k", range(5))
def test_energy_matches_reference_calc_energy(oracle, k):
    """The cell-list energy equals calc_energy (kernel.cu:452-470) on the reference frames."""
    g = np.load(GOLDEN)
    pos = g["positions"][k].astype(np.float32)
    st = oracle.OracleState(oracle.make_params(cps=4, nmax=10))
    r = np.ascontiguousarray(pos.T).reshape(-1)
    assert st.assign(r) == 0
    assert int(st.n.max()) == int(g["max_occupancy"][k])
    assert st.energy() == pytest.approx(float(g["energy_calc"][k]), rel=2e-6, abs=2e-6)


@pytest.mark.parametrize("atoms,ref", [(64, -3.132843), (800, -2873.914743), (1000, -3982.336447)])
def test_lattice_energy_known_answers(oracle, atoms, ref):
    st = oracle.OracleState(oracle.make_params(cps=4, nmax=32))
    assert st.init_lattice(atoms) == 0
    assert int(st.n.sum()) == atoms
    assert st.energy() == pytest.approx(ref, rel=2e-8, abs=2e-6)


def test_lattice_cube_root_exact(oracle):
    """start.cu:208 truncates int(cbrt(float(1e6))) to 99; the build uses the exact cube root."""
    st = oracle.OracleState(oracle.make_params(cps=8))
    r = st.init_r(1000).reshape(3, -1)
    assert len(np.unique(r[0])) == 10


# ---------------------------------------------------------------------------------------------
# algorithm invariants
# ---------------------------------------------------------------------------------------------
def _in_cells(st):
    p = st.p
    d3 = st.disk3()
    cps = (p.cps_x, p.cps_y, p.cps_z)
    idx = np.arange(st.cells)
    coords = (idx % cps[0], (idx // cps[0]) % cps[1], idx // (cps[0] * cps[1]))
    mask = np.arange(st.nmax)[None, :] < st.n[:, None]
    for k in range(3):
        L = cps[k] * 2.5
        lb = (coords[k] * 2.5 - L / 2).astype(np.float32)[:, None]
        v = d3[:, k, :]
        lbb = np.broadcast_to(lb, v.shape)
        if not np.all((v[mask] >= lbb[mask]) & (v[mask] <= lbb[mask] + np.float32(2.5))):
            return False
    return True


def test_subsweep_invariants(oracle):
    st = oracle.OracleState(oracle.make_params(cps=8))
    st.init_lattice(1000)
    n0 = st.n.copy()
    for colour in range(8):
        st.subsweep(oracle.colour_offset(colour), 0)
    assert np.array_equal(st.n, n0)
    assert _in_cells(st)
    s = st.stats.as_dict()
    # fraction of trial moves that stay in the cell: ~ 0.84042^3 for uniform start (SURVEY s.4)
    assert 0.45 < s["evaluated"] / s["trials"] < 0.75
    # most in-cell moves of a dilute lattice are accepted, but not all
    assert 0.3 < s["accepted"] / s["evaluated"] < 1.0
    # only colour-phase cells move: a second identical run reproduces bit for bit
    st2 = oracle.OracleState(oracle.make_params(cps=8))
    st2.init_lattice(1000)
    for colour in range(8):
        st2.subsweep(oracle.colour_offset(colour), 0)
    assert np.array_equal(st.disk, st2.disk)


def test_subsweep_thread_count_invariant(oracle):
    a = oracle.OracleState(oracle.make_params(cps=16))
    b = oracle.OracleState(oracle.make_params(cps=16))
    a.init_lattice(10000)
    b.init_lattice(10000)
    oracle.set_threads(0)
    a.run(0, 2)
    oracle.set_threads(4)
    b.run(0, 2)
    oracle.set_threads(0)
    assert np.array_equal(a.n, b.n) and oracle.valid_slots_equal(a.disk, a.n, b.disk, b.n, 16)
    assert a.stats.as_dict() == b.stats.as_dict()


@pytest.mark.parametrize("f,d", [(0, 0.9), (1, -0.3), (2, 1.2), (2, -1.2499)])
def test_shift_is_translation(oracle, f, d):
    """shiftCells (fixed copy, float s) = translation x_f -> x_f - d (mod L) + re-bin; the
    root copy's int s[3] breaks this."""
    st = oracle.OracleState(oracle.make_params(cps=8))
    st.init_lattice(2000)
    st.run(0, 3)
    before = st.positions().astype(np.float64)
    e0 = st.energy()
    assert st.shift_cells(f, d) == 0
    after = st.positions().astype(np.float64)
    assert len(after) == len(before)
    assert _in_cells(st)
    L = 20.0
    exp = before.copy()
    exp[:, f] = (exp[:, f] - d + L / 2) % L - L / 2
    key = lambda a: a[np.lexsort((a[:, 2], a[:, 1], a[:, 0]))]  # noqa: E731
    diff = np.abs(key(np.round(after, 3)) - key(np.round(exp, 3)))
    diff = np.minimum(diff, np.abs(diff - L))
    assert diff.max() < 2e-3
    assert st.energy() == pytest.approx(e0, rel=1e-5)


def test_energy_bookkeeping(oracle):
    st = oracle.OracleState(oracle.make_params(cps=8))
    st.init_lattice(2000)
    e0 = st.energy()
    st.run(0, 20)
    e1 = st.energy()
    assert abs(e0 + st.stats.de_fixed / 2**32 - e1) < 1e-3
    assert int(st.n.sum()) == 2000


def _known_answer(name):
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "known_answers.json")
    with open(path) as f:
        return json.load(f)["models"][name]


def _oracle_mean_energy(oracle, n_atoms, flags, equil, sweeps, every=5, chains=8, blocks=20):
    """<E> of `chains` independent oracle chains (Philox seeds 1000..) of the 4^3-cell box (L = 10)
    in threads (the C calls release the GIL): every chain equilibrates `equil` sweeps from the
    lattice, then records the energy after every `every`-th sweep; the standard error is that of the
    pooled batch means (`blocks` per chain)."""
    import threading
    res = [None] * chains

    def chain(k):
        st = oracle.OracleState(oracle.make_params(cps=4, seed=1000 + k, flags=flags))
        assert st.init_lattice(n_atoms) == 0
        assert st.run(0, equil) == 0
        res[k] = st.run_trace(equil, sweeps, every)

    th = [threading.Thread(target=chain, args=(k,)) for k in range(chains)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    bm = np.concatenate([r.reshape(blocks, -1).mean(1) for r in res])
    return float(bm.mean()), float(bm.std(ddof=1) / np.sqrt(len(bm)))


@pytest.mark.slow
@pytest.mark.parametrize("model,n_atoms,flags,sweeps", [
    ("n64", 64, 0, 60_000),
    ("n64", 64, 1, 60_000),      # the reference-like full colour shuffle
    ("n305", 305, 0, 20_000),    # 4.77 particles per cell: the density of BASELINE configs 3-5
])
def test_mean_energy_known_answer(oracle, model, n_atoms, flags, sweeps):
    """The oracle's move/shuffle/accept/shift chain samples the Boltzmann distribution of the
    reference's model: its <E> equals the known answer of an INDEPENDENT textbook Metropolis code
    (tools/textbook_mc.c: no cells, full minimum image, truncated LJ subsweep.h:90-103, accept rule
    subsweep.h:209-216; tests/golden/known_answers.json from tools/make_known_answers.py, 8 seeds
    each: N=64 -21.262 +- 0.007, N=305 -477.64 +- 0.08 in L=10, beta=0.3, sigma=0.5, rc=2.5).
    Tolerance: 3 sigma of the combined standard error (this run's pooled batch means, the known
    answer's), no flat allowance: 0.24-0.26% of <E> at N=64, 0.10% at N=305.  The GPU equals the oracle
    bit for bit, so this pins the GPU chain too.  The reference's own chain cannot be reproduced
    (cuRAND XORWOW re-seeded per launch, subsweep.h:256-259)."""
    ka = _known_answer(model)
    assert ka["N"] == n_atoms and ka["se_rel"] <= 0.003
    mean, se = _oracle_mean_energy(oracle, n_atoms, flags, equil=1000 if n_atoms == 64 else 2000, sweeps=sweeps)
    tol = 3.0 * math.hypot(se, ka["se"])
    assert abs(mean - ka["mean"]) < tol, (mean, se, ka["mean"], ka["se"])
    assert tol < 0.003 * abs(ka["mean"])


def test_known_answer_tool_reproduces(tmp_path):
    """tools/textbook_mc.c is the committed generator of the known answers: it builds and, for the
    first seed of the N=64 model over a short window, lands within 5 of its own standard errors of
    the committed pooled answer; the committed file names the tool's current source hash."""
    import hashlib
    import subprocess
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(repo, "tools", "textbook_mc.c")
    with open(os.path.join(repo, "tests", "golden", "known_answers.json")) as f:
        ka_all = json.load(f)
    assert ka_all["tool_sha256"] == hashlib.sha256(open(src, "rb").read()).hexdigest()
    exe = str(tmp_path / "textbook_mc")
    subprocess.run(["gcc", "-O2", "-std=c11", "-o", exe, src, "-lm"], check=True)
    ka = ka_all["models"]["n64"]
    out = subprocess.run([exe, "64", "10", "0.3", "0.5", "2.5", "1000", "10000", "10", "101"],
                         capture_output=True, text=True, check=True).stdout
    r = json.loads(out)
    assert abs(r["mean"] - ka["mean"]) < 5 * math.hypot(r["se"], ka["se"])
    assert 0.80 < r["acceptance"] < 0.83


def test_subsweep_range_split_equals_full(oracle):
    """A colour phase split into plane ranges (interior first, then boundaries -- the slab
    driver's order) equals the unsplit phase: cells of one colour are independent."""
    import ctypes as C
    a = oracle.OracleState(oracle.make_params(cps=8))
    b = oracle.OracleState(oracle.make_params(cps=8))
    a.init_lattice(2000)
    b.init_lattice(2000)
    for colour in (0, 3, 5, 6):
        o = oracle.colour_offset(colour)
        a.subsweep(o, 7)
        for lo, hi in ((1, 7), (0, 1), (7, 8)):
            oracle.lib().orc_subsweep_range(C.byref(b.p), b.disk, b.n, o[0], o[1], o[2], 7, lo, hi,
                                            C.byref(b.stats))
    assert np.array_equal(a.disk, b.disk)
    assert a.stats.as_dict() == b.stats.as_dict()


def test_to_fixed_f32_equals_to_fixed(oracle):
    """pmc_to_fixed_f32 (integer-only, used per pair by the GPU energy kernel) equals
    pmc_to_fixed((double)f): random floats over the energy range, every binade, exact half-way
    points of the 2^-32 grid, the 2^30 clamp, zeros and subnormals."""
    import numpy as np
    L = oracle.lib()
    rng = np.random.default_rng(11)
    vals = list(rng.standard_normal(20000).astype(np.float32) * np.float32(3.0))
    vals += list((rng.random(20000) * 2 - 1).astype(np.float32) * np.float32(2.0 ** -30))
    for e in range(-40, 34):
        for m in (1.0, 1.5, 1.0000001, 1.9999999, 1.25):
            vals += [np.float32(m * 2.0 ** e), np.float32(-m * 2.0 ** e)]
    for k in range(0, 2000):
        vals += [np.float32((k + 0.5) * 2.0 ** -32), np.float32(-(k + 0.5) * 2.0 ** -32)]
    vals += [np.float32(0.0), np.float32(-0.0), np.float32(2.0 ** 30), np.float32(2.0 ** 30) * np.float32(1.0000001),
             np.float32(-3e38), np.float32(1e-40), np.float32(-1e-40)]
    bad = [v for v in vals if L.orc_to_fixed(float(v)) != L.orc_to_fixed_f32(float(v))]
    assert not bad, bad[:5]


def test_ideal_gas_uniform_density(oracle):
    """beta = 0 (ideal gas): every in-cell trial is accepted (T = -log u > 0 = beta*dE), so the
    move + shift chain must spread the lattice into a uniform density (pyramid step 5).
    Per-axis position histograms over snapshots, 10 bins each, within 8% of uniform; counts
    conserved; no cell over nmax."""
    st = oracle.OracleState(oracle.make_params(cps=4, beta=0.0))
    st.init_lattice(200)
    st.run(0, 200)
    pos = []
    for s in range(200, 1000, 10):
        st.run(s, 10)
        pos.append(st.positions())
    pos = np.concatenate(pos)
    assert len(pos) == 200 * 80
    assert st.stats.accepted == st.stats.evaluated        # beta = 0: every evaluated move accepted
    assert st.stats.evaluated < st.stats.trials           # out-of-cell proposals still rejected
    for k in range(3):
        h, _ = np.histogram(pos[:, k], bins=10, range=(-5.0, 5.0))
        assert h.sum() == len(pos)
        assert np.all(np.abs(h / (len(pos) / 10) - 1.0) < 0.08), h


def test_oracle_sanitizers_clean(oracle):
    """the oracle under ASan + UBSan (oracle/asan_main.c: whole boxes with both colour
    orders, odd boxes, nmax overflow in assign and shift, a slab with halo planes and the shift of
    halo planes, the energy, the primitives).  Any finding aborts with a nonzero status.  (It found
    one: orc_shift_cells_planes read past the storage for a z range whose dir-neighbour halo is
    not stored; that request is now refused, here and in the GPU launcher.)"""
    import subprocess
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    b = subprocess.run(["make", "-C", here, "sanitize"], capture_output=True, text=True)
    assert b.returncode == 0, b.stderr[-2000:]
    r = subprocess.run([os.path.join(here, "build", "orc_sanitize")], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
                                UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1"))
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert r.stdout.strip().endswith("clean")


@pytest.mark.parametrize("beta", [-0.1, float("inf"), float("nan")])
def test_params_reject_bad_beta(oracle, beta):
    """beta must be finite and >= 0 (the library's normalise() refuses the same)."""
    st_params = oracle.make_params(cps=4, beta=beta)
    with pytest.raises(Exception):
        oracle.OracleState(st_params)

