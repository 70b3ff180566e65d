"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle, bit for bit.

Tolerance: none -- disk/n occupied slots, acceptance counters and the fixed-point energy sums
must be identical (bitwise), which is stricter than the north-star's 1e-6 relative bound on
mean energy and acceptance.  Sizes: BASELINE.json configs 1-3 (16^3/1e4, 64^3/1e6, 128^3/1e7).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ctx(pmc, cps, **kw):
    return pmc.PmcContext(cps, **kw)


def _ostate(oracle, cps, **kw):
    return oracle.OracleState(oracle.make_params(cps=cps, **kw))


def _assert_same(oracle, ctx, st, nmax, sl=None):
    disk, n = ctx.copy_out()
    assert np.array_equal(n if sl is None else n[sl], st.n if sl is None else st.n[sl]), "cell counts differ"
    assert oracle.valid_slots_equal(disk, n, st.disk, st.n, nmax, sl), "particle coordinates differ"


def test_detmath_device_equals_host(pmc, oracle):
    rng = np.random.default_rng(7)
    words = rng.integers(0, 2**32, size=(20000, 4), dtype=np.uint64).astype(np.uint32)
    words[:4] = [[0, 0, 0, 0], [0xFFFFFFFF] * 4, [0x200, 0x1FF, 0x80000000, 0x7FFFFFFF], [1, 2, 3, 4]]
    out_f, out_d = pmc.selftest_detmath(words)
    rc2 = oracle.cutoff_r2(2.5)
    import ctypes as C
    for i in range(0, len(words), 97):
        w = [int(v) for v in words[i]]
        g = (C.c_float * 3)()
        oracle.lib().orc_move_normals(C.byref((C.c_uint32 * 4)(*w)), C.byref(g))
        assert np.float32(g[0]).view(np.uint32) == out_f[i, 0].view(np.uint32)
        assert np.float32(g[1]).view(np.uint32) == out_f[i, 1].view(np.uint32)
        assert np.float32(g[2]).view(np.uint32) == out_f[i, 2].view(np.uint32)
        u = lambda x: np.float32(((x >> 9) * 2 + 1) * 2.0**-24)  # noqa: E731
        dx, dy, dz = (np.float32(u(w[k]) * np.float32(5.0) - np.float32(2.5)) for k in (1, 2, 3))
        e = oracle.pair_energy(float(dx), float(dy), float(dz), rc2)
        assert np.float32(e).view(np.uint32) == out_f[i, 3].view(np.uint32)
        T = -oracle.logf(float(u(w[0])))
        assert np.float32(T).view(np.uint32) == np.float32(out_d[i, 0]).view(np.uint32)
        assert oracle.lib().orc_to_fixed(float(out_f[i, 3])) == int(out_d[i, 1])


def test_create_ordered_after_busy_null_stream(pmc):
    """pmc_create's zeroing is ordered before the context's own work.  A spin kernel keeps the null
    stream (torch's default stream) busy; a context created meanwhile must still bin the lattice,
    because its zeroing runs on its own (non-blocking) stream and completes inside pmc_create.  The
    round-2 library zeroed with hipMemset on the null stream, which the context stream does not
    wait for: the zeroing of n then landed after init_lattice's counts (the intermittent all-zero
    count readback of test_gpu_c_slab_driver_equals_whole_box)."""
    import torch
    assert torch.cuda.current_stream().cuda_stream == 0, "torch's current stream is not the null stream"
    torch.cuda._sleep(200_000_000)          # ~0.1-2 s of spinning on the null stream
    ctx = pmc.PmcContext(16)
    ctx.init_lattice(10_000)
    disk, n = ctx.copy_out()                 # on the context stream: the spin may still be running
    busy = not torch.cuda.default_stream().query()
    torch.cuda.synchronize()
    assert int(n.sum()) == 10_000, f"counts read back wrong while the null stream was busy={busy}"
    n2 = ctx.copy_out()[1]
    assert np.array_equal(n, n2), "counts changed after the null stream drained"


@pytest.mark.parametrize("cps,atoms", [(16, 10_000), (64, 1_000_000)])
def test_lattice_assign_parity(pmc, oracle, cps, atoms):
    ctx = _ctx(pmc, cps)
    ctx.init_lattice(atoms)
    st = _ostate(oracle, cps)
    assert st.init_lattice(atoms) == 0
    _assert_same(oracle, ctx, st, 16)
    assert int(st.n.sum()) == atoms


def test_all_colour_phases_parity_16(pmc, oracle):
    ctx = _ctx(pmc, 16)
    ctx.init_lattice(10_000)
    st = _ostate(oracle, 16)
    st.init_lattice(10_000)
    for sweep in (0, 5):
        for colour in range(8):
            ctx.phase(colour, sweep)
            st.subsweep(oracle.colour_offset(colour), sweep)
            _assert_same(oracle, ctx, st, 16)
    s = ctx.stats()
    o = st.stats.as_dict()
    assert s == o, (s, o)
    assert s["trials"] > 0 and 0 < s["accepted"] < s["evaluated"] < s["trials"]


@pytest.mark.parametrize("f,d", [(0, 0.7), (1, -1.1), (2, 1.2499), (2, -1.25), (0, -1e-7)])
def test_shift_parity(pmc, oracle, f, d):
    import torch
    ctx = _ctx(pmc, 16)
    ctx.init_lattice(10_000)
    ctx.start(0, 2)  # decorrelate from the lattice
    disk, n = ctx.copy_out()
    st = _ostate(oracle, 16)
    st.disk[:] = disk
    st.n[:] = n
    dev = torch.device("cuda")
    din = torch.from_numpy(disk).to(dev)
    nin = torch.from_numpy(n).to(dev)
    dout = torch.zeros_like(din)
    nout = torch.zeros_like(nin)
    ctx.shiftCells(din, nin, dout, nout, f, d)
    ctx.synchronize()
    assert st.shift_cells(f, d) == 0
    got_d, got_n = dout.cpu().numpy(), nout.cpu().numpy()
    assert np.array_equal(got_n, st.n)
    assert oracle.valid_slots_equal(got_d, got_n, st.disk, st.n, 16)
    assert int(got_n.sum()) == 10_000


@pytest.mark.parametrize("cps,atoms", [(6, 600), (12, 5000), (20, 30000), ((10, 6, 14), 2500)])
@pytest.mark.parametrize("f,d", [(0, 0.9), (1, -0.6), (2, 1.1), (2, -1.2), (0, -0.8), (1, 0.5)])
def test_shift_sizes_parity(pmc, oracle, cps, atoms, f, d):
    """shiftCells at other box sizes (6, 12, 20 cells per side; 10 x 6 x 14) along every axis, both
    directions: k_shift_run's runs of 4 cells along the shift axis end short (6, 10, 14) or exactly."""
    cx, cy, cz = cps if isinstance(cps, tuple) else (cps, cps, cps)
    ctx = _ctx(pmc, cx, cps_y=cy, cps_z=cz)
    ctx.init_lattice(atoms)
    ctx.start(0, 1)
    disk, n = ctx.copy_out()
    st = _ostate(oracle, cx, cps_y=cy, cps_z=cz)
    st.disk[:] = disk
    st.n[:] = n
    import torch
    dev = torch.device("cuda")
    din = torch.from_numpy(disk).to(dev)
    nin = torch.from_numpy(n).to(dev)
    dout = torch.zeros_like(din)
    nout = torch.zeros_like(nin)
    ctx.shiftCells(din, nin, dout, nout, f, d)
    ctx.synchronize()
    assert st.shift_cells(f, d) == 0
    got_d, got_n = dout.cpu().numpy(), nout.cpu().numpy()
    assert np.array_equal(got_n, st.n)
    assert oracle.valid_slots_equal(got_d, got_n, st.disk, st.n, 16)


@pytest.mark.parametrize("nmax", [8, 12, 20, 24])
@pytest.mark.parametrize("f,d", [(0, 0.9), (1, -0.6), (2, 1.1), (2, -1.2)])
def test_shift_nmax_not_whole_lines_parity(pmc, oracle, nmax, f, d):
    """shiftCells on the packed layout where a cell's record (12*nmax bytes) is not a whole number of
    64-B lines: the whole-line store path must stop at the record's end (at nmax 8 a
    cell of 6+ particles rounds up to 128 B of a 96-B record).  The output buffer carries a guard
    tail that must stay untouched."""
    import torch
    cps, atoms = 10, (1800 if nmax == 8 else 2600)
    ctx = _ctx(pmc, cps, nmax=nmax)
    ctx.init_lattice(atoms)
    ctx.start(0, 1)
    disk, n = ctx.copy_out()
    st = _ostate(oracle, cps, nmax=nmax)
    st.disk[:] = disk
    st.n[:] = n
    dev = torch.device("cuda")
    guard = 64
    din = torch.from_numpy(disk).to(dev)
    nin = torch.from_numpy(n).to(dev)
    dbuf = torch.full((disk.size + guard,), 7.0, dtype=torch.float32, device=dev)
    dout = dbuf[:disk.size]
    nout = torch.zeros_like(nin)
    ctx.shiftCells(din, nin, dout, nout, f, d)
    ctx.synchronize()
    assert st.shift_cells(f, d) == 0
    got_d, got_n = dout.cpu().numpy(), nout.cpu().numpy()
    assert np.array_equal(got_n, st.n)
    assert oracle.valid_slots_equal(got_d, got_n, st.disk, st.n, nmax)
    assert np.all(dbuf[disk.size:].cpu().numpy() == 7.0), "shiftCells wrote past the output buffer"


@pytest.mark.parametrize("nmax", [8, 12])
def test_full_sweeps_nmax_parity(pmc, oracle, nmax):
    """Whole sweeps (8 phases + shiftCells in the context's packed state) at nmax 8 and 12."""
    cps, atoms = 12, (3000 if nmax == 8 else 4300)
    ctx = _ctx(pmc, cps, nmax=nmax)
    ctx.init_lattice(atoms)
    r = ctx.start(0, 3)
    st = _ostate(oracle, cps, nmax=nmax)
    st.init_lattice(atoms)
    st.run(0, 3)
    _assert_same(oracle, ctx, st, nmax)
    o = st.stats.as_dict()
    assert r["accepted"] == o["accepted"] and r["trials"] == o["trials"], (r, o)


def test_full_sweeps_parity_16(pmc, oracle):
    ctx = _ctx(pmc, 16)
    ctx.init_lattice(10_000)
    st = _ostate(oracle, 16)
    st.init_lattice(10_000)
    r = ctx.start(0, 6)
    assert st.run(0, 6) == 0
    _assert_same(oracle, ctx, st, 16)
    o = st.stats.as_dict()
    for k in ("de_fixed", "accepted", "trials", "evaluated"):
        assert r[k] == o[k], k
    assert r["e_final"] == st.energy()
    # energy bookkeeping: E_final ~= E_initial + sum(accepted dE) (float rounding only)
    assert abs(r["e_initial"] + r["de_fixed"] / 2**32 - r["e_final"]) < 1e-3 * abs(r["e_final"])


@pytest.mark.parametrize("beta", [0.0, 1e-30, 0.3, 7.5, 3e37])
def test_acceptance_paths_parity(pmc, oracle, beta):
    """accept_move (subsweep.h:209-216) on the device is one float compare of s = dE/4 against a
    per-move bound F (largest float with 4*beta*F < T, parked by the RNG lanes; +inf for beta = 0);
    it equals the oracle's beta*dE < T in double bit for bit.  beta = 0: every evaluated move is
    accepted (pyramid step 5 on the GPU); 1e-30: the bound estimates overflow to +inf and clamp to
    FLT_MAX; 3e37: 4*beta overflows float (the bound works in double)."""
    ctx = _ctx(pmc, 16, beta=beta)
    ctx.init_lattice(10_000)
    st = _ostate(oracle, 16, beta=beta)
    st.init_lattice(10_000)
    r = ctx.start(0, 3)
    assert st.run(0, 3) == 0
    _assert_same(oracle, ctx, st, 16)
    o = st.stats.as_dict()
    for k in ("de_fixed", "accepted", "trials", "evaluated"):
        assert r[k] == o[k], k
    if beta == 0.0:
        assert r["accepted"] == r["evaluated"] > 0


@pytest.mark.parametrize("n_moves", [0, 1, 7, 11, 23, 42])
def test_move_count_chunking_parity(pmc, oracle, n_moves):
    """Move counts across the RNG chunk boundaries (the two-cell prologue parks 10 moves per cell,
    further chunks hold 16; the single-cell path 16 per chunk) give the oracle's result bit for bit."""
    ctx = _ctx(pmc, 16, n_moves=n_moves)
    ctx.init_lattice(10_000)
    st = _ostate(oracle, 16, n_moves=n_moves)
    st.init_lattice(10_000)
    r = ctx.start(0, 2)
    assert st.run(0, 2) == 0
    _assert_same(oracle, ctx, st, 16)
    o = st.stats.as_dict()
    for k in ("de_fixed", "accepted", "trials", "evaluated"):
        assert r[k] == o[k], k


@pytest.mark.parametrize("cps", [(10, 6, 14), (14, 10, 6)])
def test_odd_colour_count_parity(pmc, oracle, cps):
    """Rectangular boxes whose colour phases hold an odd number of cells (the last wave of the
    two-cell main launch visits one cell) equal the oracle bit for bit."""
    cx, cy, cz = cps
    atoms = 3 * cx * cy * cz
    ctx = _ctx(pmc, cx, cps_y=cy, cps_z=cz)
    ctx.init_lattice(atoms)
    st = _ostate(oracle, cx, cps_y=cy, cps_z=cz)
    st.init_lattice(atoms)
    r = ctx.start(0, 3)
    assert st.run(0, 3) == 0
    _assert_same(oracle, ctx, st, 16)
    o = st.stats.as_dict()
    for k in ("de_fixed", "accepted", "trials", "evaluated"):
        assert r[k] == o[k], k


def test_graph_replay_equals_oracle(pmc, oracle):
    """pmc_run_graph (the sweep loop start.cu:237-260 captured as one hipGraph and replayed, SURVEY
    8f row 4) equals the C oracle bit for bit -- every occupied slot, counts, the four counters --
    over 6 sweeps replayed as 2 + 4 (two graphs), and equals eager launches byte for byte."""
    a = _ctx(pmc, 16)
    b = _ctx(pmc, 16)
    a.init_lattice(10_000)
    b.init_lattice(10_000)
    for s in range(6):
        a.sweep(s)
    b.run_graph(0, 2)
    b.run_graph(2, 4)
    st = _ostate(oracle, 16)
    st.init_lattice(10_000)
    assert st.run(0, 6) == 0
    _assert_same(oracle, b, st, 16)
    assert b.stats() == st.stats.as_dict()
    da, na = a.copy_out()
    db, nb = b.copy_out()
    assert np.array_equal(na, nb) and np.array_equal(da.view(np.uint32), db.view(np.uint32))
    assert a.stats() == b.stats()


@pytest.mark.parametrize("cps,atoms", [((16, 16, 16), 10_000), ((8, 8, 8), 1_500), ((12, 8, 6), 1_800),
                                       ((20, 20, 20), 24_000), ((24, 24, 24), 40_000)])
def test_small_box_persistent_equals_oracle(pmc, oracle, cps, atoms):
    """pmc_run_small (whole sweeps in one launch on XCD 0, in-kernel barriers) equals the oracle bit
    for bit over 40 sweeps (two launches of 32 + 8), 512 participants looping over up to 4 cells per
    colour phase at 24^3.  (pmc_start does not take this path by default -- the eager
    one-launch-per-phase sweep is faster at every size -- only with PMC_SMALL=1.)"""
    cx, cy, cz = cps
    ctx = _ctx(pmc, cx, cps_y=cy, cps_z=cz)
    ctx.init_lattice(atoms)
    ctx.run_small(7, 40)
    st = _ostate(oracle, cx, cps_y=cy, cps_z=cz)
    st.init_lattice(atoms)
    assert st.run(7, 40) == 0
    _assert_same(oracle, ctx, st, 16)
    assert ctx.stats() == st.stats.as_dict()
    assert ctx.error_flags() == 0
    assert ctx.energy() == st.energy()


def test_single_colour_parity_64(pmc, oracle):
    """BASELINE config 2: 64^3 cells, 1e6 particles, one colour phase."""
    ctx = _ctx(pmc, 64)
    ctx.init_lattice(1_000_000)
    st = _ostate(oracle, 64)
    st.init_lattice(1_000_000)
    oracle.set_threads(8)
    ctx.phase(5, 3)
    st.subsweep(oracle.colour_offset(5), 3)
    _assert_same(oracle, ctx, st, 16)
    assert ctx.stats() == st.stats.as_dict()


def test_graph_sweeps_parity_64(pmc, oracle):
    """Sweeps replayed as one hipGraph of single-chain launches on the 64^3 / 1e6 box: each colour
    phase is one solo launch of 32768 cells, which ends in single-cell waves (k_subsweep_mixed).
    Bitwise equal to the oracle over 3 sweeps."""
    oracle.set_threads(16)
    ctx = _ctx(pmc, 64)
    ctx.init_lattice(1_000_000)
    ctx.run_graph(5, 3)
    st = _ostate(oracle, 64)
    st.init_lattice(1_000_000)
    assert st.run(5, 3) == 0
    _assert_same(oracle, ctx, st, 16)
    assert ctx.stats() == st.stats.as_dict()
    assert ctx.error_flags() == 0


def test_long_run_parity_64(pmc, oracle):
    """BASELINE config 2's box (64^3 cells, 1e6 particles) over 30 full sweeps from the lattice start,
    through the relaxation where the cell counts spread (the lattice's 4-5 per cell becomes 0-13): every
    occupied slot, the counts, the four counters and the energy equal the oracle's bit for bit at
    sweeps 10 and 30.  Tolerance: none."""
    oracle.set_threads(16)
    ctx = _ctx(pmc, 64)
    ctx.init_lattice(1_000_000)
    st = _ostate(oracle, 64)
    st.init_lattice(1_000_000)
    for first, count in ((0, 10), (10, 20)):
        r = ctx.start(first, count)
        assert st.run(first, count) == 0
        _assert_same(oracle, ctx, st, 16)
        assert ctx.stats() == st.stats.as_dict()
        assert r["e_final"] == st.energy()
        assert ctx.error_flags() == 0
    _, n = ctx.copy_out()
    assert n.max() > 8      # the counts did spread: the staging's overflow passes (slots >= 8) ran


def test_full_sweeps_parity_128(pmc, oracle):
    """BASELINE config 3 (128^3 cells, 1e7 particles): two full sweeps -- all 8 colour phases and
    shiftCells, one shift along z -- compared with the oracle bit for bit (every occupied slot,
    counts, the four counters, the energy).  Tolerance: none."""
    oracle.set_threads(16)
    s0 = next(s for s in range(100) if oracle.sweep_plan(1234, s, 2.5)[1] == 2)
    ctx = _ctx(pmc, 128)
    ctx.init_lattice(10_000_000)
    st = _ostate(oracle, 128)
    st.init_lattice(10_000_000)
    r = ctx.start(s0, 2)
    assert st.run(s0, 2) == 0
    _assert_same(oracle, ctx, st, 16)
    o = st.stats.as_dict()
    for k in ("de_fixed", "accepted", "trials", "evaluated"):
        assert r[k] == o[k], k
    assert r["e_final"] == st.energy()


def test_single_colour_parity_128(pmc, oracle):
    """BASELINE config 3 size: 128^3 cells, 1e7 particles; one colour phase compared bitwise,
    then size-independent properties over full sweeps."""
    ctx = _ctx(pmc, 128)
    ctx.init_lattice(10_000_000)
    st = _ostate(oracle, 128)
    st.init_lattice(10_000_000)
    _assert_same(oracle, ctx, st, 16)
    oracle.set_threads(16)
    ctx.phase(2, 11)
    st.subsweep(oracle.colour_offset(2), 11)
    _assert_same(oracle, ctx, st, 16)
    assert ctx.stats(reset=True) == st.stats.as_dict()
    # full sweeps: particle conservation, every particle inside its cell's closed box, E bookkeeping
    e0 = ctx.energy()
    r = ctx.start(20, 3)
    disk, n = ctx.copy_out()
    assert int(n.sum()) == 10_000_000
    assert ctx.error_flags() == 0
    d3 = disk.reshape(-1, 3, 16)
    idx = np.arange(128**3)
    cx, cy, cz = idx % 128, (idx // 128) % 128, idx // (128 * 128)
    mask = np.arange(16)[None, :] < n[:, None]
    for k, cc in enumerate((cx, cy, cz)):
        lb = (cc * 2.5 - 160.0).astype(np.float32)[:, None]
        v = d3[:, k, :]
        assert np.all((v[mask] >= np.broadcast_to(lb, v.shape)[mask]) &
                      (v[mask] <= np.broadcast_to(lb + 2.5, v.shape)[mask]))
    assert r["e_initial"] == pytest.approx(e0)
    assert abs(r["e_initial"] + r["de_fixed"] / 2**32 - r["e_final"]) < 1e-4 * abs(r["e_final"])


@pytest.mark.parametrize("env,nmax", [({"PMC_SUBSWEEP_CAP": "64", "PMC_SMALL_LAUNCH": "0"}, 32),
                                      ({"PMC_FORCE_ADDR64": "1"}, 16),
                                      ({"PMC_FORCE_ADDR64": "1", "PMC_SUBSWEEP_CAP": "64", "PMC_SMALL_LAUNCH": "0"}, 16),
                                      ({"PMC_SMALL_LAUNCH": "0"}, 16),
                                      ({"PMC_MIXED_SINGLES": "5", "PMC_SMALL_LAUNCH": "0"}, 16),
                                      ({"PMC_MIXED_SINGLES": "5", "PMC_SMALL_LAUNCH": "0", "PMC_SUBSWEEP_CAP": "64"}, 16)])
def test_fallback_and_addr64_paths(oracle, env, nmax):
    """Test hooks for launch variants the default configs never take, each bit-identical to the
    oracle: PMC_SUBSWEEP_CAP forces a tiny LDS capacity, so (almost) every cell goes to the
    full-capacity fallback launch; PMC_FORCE_ADDR64 forces the 64-bit disk addressing used for
    buffers of 4 GiB and more; PMC_SMALL_LAUNCH=0 takes this 8^3 box through the main two-cell
    launch + fallback instead of the one-launch full-capacity path small boxes default to.  Runs in
    a subprocess (the hooks are read once).  PMC_MIXED_SINGLES=5 ends every launch's XCD runs in
    single-cell waves (k_subsweep_mixed, the default for solo launches of <= 32768 cells), with and
    without forced overflow of those single-cell waves."""
    import os
    import subprocess
    import sys
    code = r'''
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import pmc_amd, pmc_oracle
nmax = int(sys.argv[3])
ctx = pmc_amd.PmcContext(8, nmax=nmax)
ctx.init_lattice(4000)
r = ctx.start(0, 3)
disk, n = ctx.copy_out()
st = pmc_oracle.OracleState(pmc_oracle.make_params(cps=8, nmax=nmax))
st.init_lattice(4000)
st.run(0, 3)
assert np.array_equal(n, st.n)
assert pmc_oracle.valid_slots_equal(disk, n, st.disk, st.n, nmax)
assert r["accepted"] == st.stats.accepted and r["trials"] == st.stats.trials
print("ok", r["accepted"])
'''
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code, os.path.join(repo, "parallel-monte-carlo_amd"),
                          os.path.join(repo, "oracle"), str(nmax)], env=dict(os.environ, **env),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.startswith("ok")


@pytest.mark.parametrize("env", [{"PMC_ENERGY_ROWS_CAP": "0"}, {"PMC_ENERGY_ROWS_CAP": "40"},
                                 {"PMC_ENERGY_LEGACY": "1"}])
def test_energy_paths_equal_oracle(oracle, env):
    """The cell-list energy's launch variants, each bitwise equal to orc_energy: interior cells by
    row segments + edge cells per cell (default); every segment over a tiny staging capacity, so the
    per-cell kernel takes the queued segments (ROWS_CAP 0 / 40); the per-cell kernel alone (LEGACY).
    Whole boxes (16^3, 20x12x14) and a slab with halos.  Subprocess: the hooks are read once."""
    import os
    import subprocess
    import sys
    code = r'''
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import pmc_amd, pmc_oracle
for cps, cy, cz, atoms in ((16, 16, 16, 10000), (20, 12, 14, 9000), (8, 8, 8, 1500)):
    ctx = pmc_amd.PmcContext(cps, cps_y=cy, cps_z=cz)
    ctx.init_lattice(atoms)
    ctx.start(0, 2)
    st = pmc_oracle.OracleState(pmc_oracle.make_params(cps=cps, cps_y=cy, cps_z=cz))
    disk, n = ctx.copy_out()
    st.disk[:] = disk; st.n[:] = n
    assert ctx.energy() == st.energy(), (cps, ctx.energy(), st.energy())
# slab with halo planes: the slab's energy equals the oracle's over the same storage
from pmc_amd.slab import SlabDriver
d = SlabDriver(cps=16, nz_local=8, rank=0, world=1, atoms_per_rank=5000, use_rccl=False)
d.run(3, 2)
e = d.ctx.energy()
disk, n = d.ctx.copy_out()
stp = pmc_oracle.OracleState(pmc_oracle.make_params(cps=16, cps_z=8, nz_local=8, halo=1))
stp.disk[:] = disk; stp.n[:] = n
assert e == stp.energy(), (e, stp.energy())
print("ok")
'''
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code, os.path.join(repo, "parallel-monte-carlo_amd"),
                          os.path.join(repo, "oracle")], env=dict(os.environ, **env),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "ok" in out.stdout


def test_energy_nmax32_and_dense_box_fast(oracle, pmc):
    """the energy's row-segment kernel cannot stage a cell's partner list at nmax > 16,
    and a box denser than the configs' 4.77 per cell overflows its staging capacity.  Both go to
    per-cell kernels that keep the whole chip busy (nmax 32: every cell per cell, MODE 0; over-full
    segments: the MODE-2 queue over up to 8192 waves): bitwise equal to orc_energy and fast -- a
    48^3 box at nmax 32 and a 48^3 box at 7.5 particles per cell (whose near-lattice segments
    overflow the staging) each under 2 ms per call, ~20x the expected time (the fixed 64-wave queue grid of round 3
    took ~100x the per-cell time)."""
    import time
    for nmax, atoms in ((32, 530_000), (16, 830_000)):
        ctx = pmc.PmcContext(48, nmax=nmax)
        ctx.init_lattice(atoms)
        ctx.energy()                      # warm-up (first launch of each kernel)
        t0 = time.perf_counter()
        for _ in range(5):
            e = ctx.energy()
        dt = (time.perf_counter() - t0) / 5
        disk, n = ctx.copy_out()
        st = oracle.OracleState(oracle.make_params(cps=48, nmax=nmax))
        st.disk[:] = disk
        st.n[:] = n
        oracle.set_threads(8)
        assert e == st.energy(), (nmax, e, st.energy())
        oracle.set_threads(0)
        assert dt < 0.002, (nmax, atoms, dt)
        ctx.close()


@pytest.mark.parametrize("rccl", [False, True])
def test_gpu_c_slab_driver_forced_fallback(rccl):
    """PMC_SUBSWEEP_CAP=64 sends (almost) every cell of the C slab driver's interior launches to
    the overflow queue and its fallback launch, beside the boundary launches on the aux stream.
    Bit-identical to the whole box over x/y/z shifts.  Subprocess: the hook is read once."""
    import os
    import subprocess
    import sys
    code = r'''
import sys, numpy as np
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import torch, pmc_amd, pmc_oracle
from pmc_amd.slab import SlabDriver
rccl = sys.argv[3] == "1"
drv = SlabDriver(cps=16, nz_local=8, rank=0, world=1, atoms_per_rank=5000, use_rccl=rccl)
whole = pmc_amd.PmcContext(16, cps_z=8)
whole.init_lattice(5000)
drv.run(11, 6)
for s in range(11, 17):
    whole.sweep(s)
torch.cuda.synchronize()
d_slab, n_slab = drv.owned()
disk, n = whole.copy_out()
assert np.array_equal(n_slab, n)
assert pmc_oracle.valid_slots_equal(d_slab, n_slab, disk, n, 16)
assert drv.ctx.stats() == whole.stats()
assert drv.ctx.error_flags() == 0
print("ok", drv.ctx.stats())
'''
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code, os.path.join(repo, "parallel-monte-carlo_amd"),
                          os.path.join(repo, "oracle"), "1" if rccl else "0"],
                         env=dict(os.environ, PMC_SUBSWEEP_CAP="64", PMC_SMALL_LAUNCH="0"), capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert any(line.startswith("ok") for line in out.stdout.splitlines()), out.stdout[-2000:]   # (RCCL may print too)


@pytest.mark.parametrize("nz,atoms,two_streams", [(16, 10_000, True), (16, 10_000, False), (4, 2_500, True)])
def test_gpu_slab_single_rank_equals_whole_box(pmc, nz, atoms, two_streams):
    """The HIP slab path (halo planes, global z images, plane exchange through torch tensors)
    with one rank reproduces the whole-box run bit for bit -- with the boundary planes on their
    own stream beside the interior (the multi-GPU schedule) and with the one-stream schedule."""
    import torch
    from slab_legacy import SlabSimulation
    sim = SlabSimulation.create(cps=16, nz_local=nz, rank=0, world=1, atoms_per_rank=atoms)
    if not two_streams:
        sim.bstream = None
    whole = pmc.PmcContext(16, cps_z=nz)
    whole.init_lattice(atoms)
    sim.run(0, 4)
    for s in range(4):
        whole.sweep(s)
    torch.cuda.synchronize()
    d_slab, n_slab = sim.owned()
    disk, n = whole.copy_out()
    assert np.array_equal(n_slab.cpu().numpy().reshape(-1), n)
    import pmc_oracle
    assert pmc_oracle.valid_slots_equal(d_slab.cpu().numpy().reshape(-1), n, disk, n, 16)
    assert sim.ctx.stats() == whole.stats()
    if nz != 16:
        return
    # energies: slab pairs across the (self-)boundary count half on each side -> same total
    assert sim.ctx.energy() == pytest.approx(whole.energy(), rel=1e-12, abs=1e-9)


@pytest.mark.gpu
def test_gpu_init_lattice_global_slab_planes(pmc, oracle):
    """Strong-scaling start state (bench --strong): a slab's pmc_init_lattice_global holds exactly
    the owned planes of the whole-box lattice, slot for slot; the slabs together hold every particle."""
    cps, atoms, nz = 16, 10_000, 8
    whole = pmc.PmcContext(cps)
    whole.init_lattice(atoms)
    dw, nw = whole.copy_out()
    plane = cps * cps
    total = 0
    for z0 in (0, nz):
        sl = pmc.PmcContext(cps, cps_z=cps, nz_local=nz, z0=z0, halo=1)
        sl.init_lattice_global(atoms)
        d, n = sl.copy_out()
        own = slice(plane, plane * (nz + 1))
        ref = slice(z0 * plane, (z0 + nz) * plane)
        assert np.array_equal(n[own], nw[ref])
        row = 3 * 16
        assert oracle.valid_slots_equal(d[own.start * row:own.stop * row], n[own],
                                        dw[ref.start * row:ref.stop * row], nw[ref], 16)
        total += int(n[own].sum())
    assert total == atoms


@pytest.mark.gpu
@pytest.mark.parametrize("nz,atoms,rccl,halo", [(16, 10_000, False, 1), (16, 10_000, True, 1), (4, 2_500, True, 1),
                                               (16, 10_000, True, 2), (4, 2_500, False, 2)])
def test_gpu_c_slab_driver_equals_whole_box(pmc, oracle, nz, atoms, rccl, halo):
    """The C slab driver (pmc_slab_*: interior chains, boundary chain with the halo exchange; with
    rccl=True through a one-rank RCCL communicator sending to itself, the multi-GPU transport path;
    halo=2: the one-exchange-per-sweep schedule with two halo planes per side) equals the whole-box
    run and the C oracle's bit for bit: every occupied slot, counts, counters and the energy.
    Sweeps 10-17 shift along x and y (10-12: the halo planes shifted locally) and along z in both
    directions (13-17: one halo plane shifted locally, the other received); after the last one
    every halo plane must equal the periodic image of its owned plane."""
    import torch
    from pmc_amd.slab import SlabDriver
    drv = SlabDriver(cps=16, nz_local=nz, rank=0, world=1, atoms_per_rank=atoms, use_rccl=rccl, halo=halo)
    whole = pmc.PmcContext(16, cps_z=nz)
    whole.init_lattice(atoms)
    assert int(whole.copy_out()[1].sum()) == atoms, "whole box: lattice not binned"
    drv.run(10, 8)
    for s in range(10, 18):
        whole.sweep(s)
    torch.cuda.synchronize()
    d_slab, n_slab = drv.owned()
    disk, n = whole.copy_out()
    assert int(n_slab.sum()) == atoms, "slab: particles lost"
    assert int(n.sum()) == atoms, f"whole box: particles lost (sum {int(n.sum())}, stats {whole.stats()})"
    assert np.array_equal(n_slab, n)
    assert oracle.valid_slots_equal(d_slab, n_slab, disk, n, 16)
    st = oracle.OracleState(oracle.make_params(cps=16, cps_z=nz))     # and the oracle's run itself
    assert st.init_lattice(atoms) == 0
    assert st.run(10, 8) == 0
    assert np.array_equal(n_slab, st.n)
    assert oracle.valid_slots_equal(d_slab, n_slab, st.disk, st.n, 16)
    assert drv.ctx.stats() == st.stats.as_dict()
    d_all, n_all = drv.ctx.copy_out()
    plane, row = 16 * 16, 3 * 16
    d_all = d_all.reshape(nz + 2 * halo, plane * row)
    n_all = n_all.reshape(nz + 2 * halo, plane)
    for k in range(halo):   # storage plane of local z is z + halo
        for hz, image in ((halo - 1 - k, halo + nz - 1 - k), (halo + nz + k, halo + k)):
            assert np.array_equal(n_all[hz], n_all[image])
            assert oracle.valid_slots_equal(d_all[hz], n_all[hz], d_all[image], n_all[image], 16)
    assert drv.ctx.stats() == whole.stats()
    assert drv.ctx.error_flags() == 0
    assert drv.ctx.energy() == pytest.approx(whole.energy(), rel=1e-12, abs=1e-9)
    obs, e_all = drv.ctx.slab_observables()   # one rank: the RCCL all-reduce (or local) of itself
    assert obs == whole.stats() and e_all == whole.energy()
    assert e_all == st.energy()


@pytest.mark.gpu
def test_gpu_c_slab_driver_timing_and_restart(pmc, oracle, tmp_path):
    """Per-launch HIP-event timing of the C driver, and snapshot + halo refill: 2 sweeps, save,
    2 more; a fresh driver restored from the snapshot repeats the last 2 bit for bit."""
    from pmc_amd.slab import SlabDriver
    drv = SlabDriver(cps=16, nz_local=16, rank=0, world=1, atoms_per_rank=10_000)
    drv.ctx.slab_timing(True)
    drv.run(0, 2)
    t = drv.ctx.slab_timing(True)
    # nz = 16: per phase one launch of each interior chain (planes [1, 8) and [8, 15))
    assert t["n_subsweep"] == 2 * 16 and t["n_shift"] == 2 and t["subsweep_ms"] > 0 and t["shift_ms"] > 0
    drv.run(0, 1)
    k = drv.ctx.timing_kinds(True)   # interior (both chains), shift, boundary (exchange stream)
    assert k["n_subsweep"] == 16 and k["n_boundary"] == 8 and k["n_shift"] == 1 and k["boundary_ms"] > 0
    drv.ctx.slab_timing(False)
    drv = SlabDriver(cps=16, nz_local=16, rank=0, world=1, atoms_per_rank=10_000)
    drv.run(0, 2)
    path = str(tmp_path / "slab.pmcsnap")
    drv.ctx.save_snapshot(path, 2)
    drv.run(2, 2)
    d1, n1 = drv.owned()
    s1 = drv.ctx.stats()
    drv2 = SlabDriver(cps=16, nz_local=16, rank=0, world=1)
    first = drv2.ctx.load_snapshot(path)
    drv2.ctx.slab_exchange()
    drv2.run(first, 2)
    d2, n2 = drv2.owned()
    assert np.array_equal(n1, n2)
    assert oracle.valid_slots_equal(d1, n1, d2, n2, 16)
    assert drv2.ctx.stats() == s1


@pytest.mark.gpu
@pytest.mark.parametrize("slab,rccl", [(False, False), (True, False), (True, True)])
def test_bench_rewarm_restores_state(pmc, oracle, slab, rccl):
    """bench.py's clock re-warm (hot-path sweeps on the timed start state, then device-to-device
    restore) leaves the run bit-identical to one without it: every occupied slot, counts, the
    counters of the following sweeps and the energy; for the slab driver the other streams are
    ordered after the save and the restore copies (a torn save broke the ΔE bookkeeping once)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from pmc_amd.slab import SlabDriver

    def make():
        if not slab:
            c = pmc.PmcContext(16)
            c.init_lattice(10_000)
            return c, c.sweep, (lambda: None), (lambda: c.copy_out()), None
        d = SlabDriver(cps=16, nz_local=16, rank=0, world=1, atoms_per_rank=10_000, use_rccl=rccl)
        return d.ctx, d.sweep, d.finish, d.owned, (lambda: d.ctx.slab_exchange())

    res = []
    for use in (False, True):
        ctx, sweep, finish, state, relink = make()
        for s in range(3):
            sweep(s)
        finish()
        ctx.synchronize()
        ctx.stats(reset=True)
        if use:
            bench.rewarm(ctx, sweep, finish, first=3, count=3, relink=relink)
        for s in range(3, 6):
            sweep(s)
        finish()
        ctx.synchronize()
        d, n = state()
        res.append((d, n, ctx.stats(), ctx.energy(), ctx.error_flags()))
    (d0, n0, s0, e0, f0), (d1, n1, s1, e1, f1) = res
    assert np.array_equal(n0, n1)
    assert oracle.valid_slots_equal(d0, n0, d1, n1, 16)
    assert s0 == s1 and e0 == e1 and f0 == f1 == 0


@pytest.mark.gpu
def test_timing_pause_samples_launches(pmc):
    """pmc_timing_pause: launches issued while paused carry no events and are not counted; the
    collected sums cover exactly the unpaused sweeps (bench.py times every 4th sweep this way).  A
    sweep is 8 launches per plane chain (pmc_sweep_layout); the phase spans cover 8 phases per timed
    sweep when there are several chains."""
    ctx = pmc.PmcContext(16)
    ctx.init_lattice(10_000)
    chains = len(ctx.sweep_layout())
    ctx.timing_kinds(True)
    for s in range(4):
        ctx.timing_pause(s % 2 == 1)
        ctx.sweep(s)
    k = ctx.timing_kinds(False)
    assert k["n_subsweep"] == 2 * 8 * chains and k["n_shift"] == 2 and k["subsweep_ms"] > 0
    span, n = ctx.phase_spans()
    assert (n, span > 0) == ((16, True) if chains > 1 else (0, False))
    ctx.timing_kinds(True)      # a new collection starts unpaused
    ctx.sweep(4)
    k = ctx.timing_kinds(False)
    assert k["n_subsweep"] == 8 * chains and k["n_shift"] == 1


@pytest.mark.gpu
def test_slab_halo_parameter_validation(pmc):
    """pmc_params.halo: 0 (whole box), 1 or 2 (slabs); 2 refuses the reference-like colour order (its
    schedule needs two runs per sweep), other values are refused; a two-plane-halo context stores
    nz_local + 4 planes and its plane spans reach the outer halos."""
    with pytest.raises(pmc.PmcError, match="halo must be"):
        pmc.PmcContext(16, cps_z=16, nz_local=8, z0=0, halo=3)
    with pytest.raises(pmc.PmcError, match="two runs per sweep"):
        pmc.PmcContext(16, cps_z=16, nz_local=8, z0=0, halo=2, flags=1)
    ctx = pmc.PmcContext(16, cps_z=16, nz_local=8, z0=8, halo=2)
    d, n = ctx.copy_out()
    assert n.size == 16 * 16 * (8 + 4)
    ctx.close()
