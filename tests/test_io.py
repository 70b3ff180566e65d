"""Trajectory dump / restart: the host formats of the C ABI, on the CPU.

The dump writer is pinned byte for byte against the reference's own trajectory file
(dumpR3.txt frames 0 and 1, written by create_dump, kernel.cu:510-536; bytes kept in
tests/golden/dumpR3_frames.npz by make_golden.py).  disk_to_r (kernel.cu:500-510) is checked
against a numpy restatement, the snapshot by round trips and by restarting the C oracle (TEST
INFRASTRUCTURE) from a snapshot: the continued run equals the uninterrupted one bit for bit.
"""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "dumpR3_frames.npz")


@pytest.fixture(scope="module")
def io(pmc):
    import pmc_amd.io as io
    return io


def test_dump_writer_matches_reference_frame0(io, oracle, tmp_path):
    """Frame 0 of dumpR3.txt is the init_r lattice (N=64, L=10) in create_dump's text format."""
    g = np.load(GOLDEN)
    st = oracle.OracleState(oracle.make_params(cps=4, nmax=10))
    r = st.init_r(64).reshape(3, 64)
    path = tmp_path / "dump.txt"
    io.write_dump(path, 0, r, (-5, -5, -5), (5, 5, 5), append=False)
    assert path.read_bytes() == bytes(g["frame_text_0"])


def test_dump_reader_roundtrip_reference_frame1(io, tmp_path):
    """Frame 1 (disk_to_r order after one sweep): read it, write it back -> identical bytes."""
    g = np.load(GOLDEN)
    src = tmp_path / "ref.txt"
    src.write_bytes(bytes(g["frame_text_0"]) + bytes(g["frame_text_1"]))
    ts, r, lo, hi = io.read_dump(src, 1)
    assert ts == 1 and r.shape == (3, 64)
    assert lo == (-5.0, -5.0, -5.0) and hi == (5.0, 5.0, 5.0)
    assert np.allclose(r.T, g["positions"][1], atol=5e-7)
    out = tmp_path / "out.txt"
    io.write_dump(out, 1, r, lo, hi, append=False)
    assert out.read_bytes() == bytes(g["frame_text_1"])
    ts0, r0, _, _ = io.read_dump(src, 0)
    assert ts0 == 0 and np.array_equal(r0.T.astype(np.float64), g["positions"][0])


def test_dump_reader_errors(io, pmc, tmp_path):
    g = np.load(GOLDEN)
    src = tmp_path / "ref.txt"
    src.write_bytes(bytes(g["frame_text_0"]))
    with pytest.raises(pmc.PmcError) as e:
        io.read_dump(src, 1)
    assert e.value.code == -4                      # PMC_ERR_RANGE: no such frame
    with pytest.raises(pmc.PmcError):
        io.read_dump(tmp_path / "missing.txt", 0)
    bad = tmp_path / "bad.txt"
    bad.write_bytes(bytes(g["frame_text_0"])[:400])   # truncated atom lines
    with pytest.raises(pmc.PmcError):
        io.read_dump(bad, 0)


def _disk_to_r_np(disk, n, nmax):
    d3 = disk.reshape(-1, 3, nmax)
    xs = [[], [], []]
    for c in range(n.size):
        for j in range(int(n[c])):
            for d in range(3):
                xs[d].append(d3[c, d, j])
    return np.array(xs, np.float32)


def test_disk_to_r_order(io, oracle):
    st = oracle.OracleState(oracle.make_params(cps=8))
    st.init_lattice(1000)
    st.run(0, 2)
    r = io.disk_to_r(st.disk, st.n, st.nmax)
    assert r.shape == (3, int(st.n.sum()))
    assert np.array_equal(r, _disk_to_r_np(st.disk, st.n, st.nmax))


def test_snapshot_roundtrip_and_oracle_restart(io, oracle, tmp_path):
    """Snapshot after 3 sweeps, restore into a fresh state, run sweeps 3..5: equals 0..5."""
    p = oracle.make_params(cps=16)
    full = oracle.OracleState(p)
    full.init_lattice(10_000)
    full.run(0, 6)

    a = oracle.OracleState(p)
    a.init_lattice(10_000)
    a.run(0, 3)
    path = tmp_path / "s.pmcsnap"
    io.write_snapshot(path, a.p, 3, a.stats.as_dict(), a.disk, a.n)
    assert not os.path.exists(str(path) + ".tmp")
    q, sweep, stats, disk, n = io.read_snapshot(path, cells=a.cells)
    assert sweep == 3 and stats == a.stats.as_dict()
    assert (q.cps_x, q.nmax, q.n_moves, q.seed, q.beta) == (16, 16, 10, 1234, a.p.beta)
    assert oracle.valid_slots_equal(disk, n, a.disk, a.n, a.nmax)
    # padding slots come back zeroed; a header-only read needs no arrays
    hdr = io.read_snapshot(path, cells=0)
    assert hdr[1] == 3 and hdr[3] is None

    b = oracle.OracleState(p)
    b.disk[:] = disk
    b.n[:] = n
    for k, v in stats.items():
        setattr(b.stats, k, v)
    b.run(sweep, 3)
    assert oracle.valid_slots_equal(b.disk, b.n, full.disk, full.n, full.nmax)
    assert b.stats.as_dict() == full.stats.as_dict()


def test_snapshot_integrity(io, oracle, pmc, tmp_path):
    st = oracle.OracleState(oracle.make_params(cps=4, nmax=10))
    st.init_lattice(64)
    path = tmp_path / "s.pmcsnap"
    io.write_snapshot(path, st.p, 7, {}, st.disk, st.n)
    raw = bytearray(path.read_bytes())
    bad = tmp_path / "flip.pmcsnap"
    raw[-5] ^= 0x40                                  # one coordinate bit
    bad.write_bytes(bytes(raw))
    with pytest.raises(pmc.PmcError, match="checksum"):
        io.read_snapshot(bad, cells=st.cells)
    short = tmp_path / "short.pmcsnap"
    short.write_bytes(path.read_bytes()[:-10])
    with pytest.raises(pmc.PmcError, match="truncated"):
        io.read_snapshot(short, cells=st.cells)
    with pytest.raises(pmc.PmcError, match="cell count"):
        io.read_snapshot(path, cells=st.cells + 1)
    notsnap = tmp_path / "x.pmcsnap"
    notsnap.write_bytes(b"hello world" * 20)
    with pytest.raises(pmc.PmcError, match="PMCSNAP1"):
        io.read_snapshot(notsnap, cells=0)


def test_snapshot_read_refuses_other_nmax(io, oracle, pmc, tmp_path):
    """The reader sizes nothing by the file: buffers for nmax 8 and a snapshot with nmax 10 are
    refused before any write (pmc_io.cpp wrote past a smaller caller buffer)."""
    import ctypes as C
    import numpy as np
    st = oracle.OracleState(oracle.make_params(cps=4, nmax=10))
    st.init_lattice(64)
    path = tmp_path / "s.pmcsnap"
    io.write_snapshot(path, st.p, 7, {}, st.disk, st.n)
    from pmc_amd._lib import Params, lib
    q = Params()
    q.nmax = 8
    disk = np.full(st.cells * 3 * 8, 7.0, np.float32)
    n = np.full(st.cells, 3, np.int16)
    rc = lib().pmc_snapshot_read(str(path).encode(), C.byref(q), None, None, disk.ctypes.data, n.ctypes.data,
                                 st.cells)
    assert rc == -1                                       # PMC_ERR_ARG
    assert "nmax" in lib().pmc_last_error().decode()
    assert np.all(disk == 7.0) and np.all(n == 3)        # untouched
    rc = lib().pmc_snapshot_read(str(path).encode(), None, None, None, disk.ctypes.data, n.ctypes.data, st.cells)
    assert rc == -1                                       # buffers without params: refused
