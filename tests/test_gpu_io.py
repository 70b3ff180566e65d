"""GPU tests of the dump / restart path through the C ABI context wrappers:
the device state dumped as create_dump text equals the oracle's state written by the host writer,
and a run restarted from a snapshot equals the uninterrupted run bit for bit (the sweep index is
the whole RNG state of the counter-based Philox streams)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_gpu_dump_frame_equals_oracle_text(pmc, oracle, tmp_path):
    import pmc_amd.io as io
    ctx = pmc.PmcContext(16)
    ctx.init_lattice(10_000)
    ctx.start(0, 2)
    st = oracle.OracleState(oracle.make_params(cps=16))
    st.init_lattice(10_000)
    st.run(0, 2)
    got = tmp_path / "gpu.txt"
    ctx.dump_frame(got, 2, append=False)
    ctx.dump_frame(got, 3, append=True)
    want = tmp_path / "orc.txt"
    r = io.disk_to_r(st.disk, st.n, st.nmax)
    io.write_dump(want, 2, r, (-20, -20, -20), (20, 20, 20), append=False)
    io.write_dump(want, 3, r, (-20, -20, -20), (20, 20, 20), append=True)
    assert got.read_bytes() == want.read_bytes()
    ts, r1, _, _ = io.read_dump(got, 1)
    assert ts == 3 and r1.shape == (3, 10_000)


def test_gpu_snapshot_restart_bitwise(pmc, oracle, tmp_path):
    full = pmc.PmcContext(16)
    full.init_lattice(10_000)
    full.start(0, 4)
    a = pmc.PmcContext(16)
    a.init_lattice(10_000)
    a.start(0, 2)
    path = tmp_path / "run.pmcsnap"
    a.save_snapshot(path, 2)
    b = pmc.PmcContext(16)                 # fresh context, state only from the file
    nxt = b.load_snapshot(path)
    assert nxt == 2
    assert b.stats() == a.stats()
    b.start(nxt, 2)
    d0, n0 = full.copy_out()
    d1, n1 = b.copy_out()
    assert oracle.valid_slots_equal(d1, n1, d0, n0, 16)
    assert b.stats() == full.stats()
    # a snapshot only loads into a context with the same parameters
    c = pmc.PmcContext(16, beta=0.5)
    with pytest.raises(pmc.PmcError, match="parameters differ"):
        c.load_snapshot(path)


def test_start_driver_save_restart(pmc, tmp_path):
    """The `start` program (start.cu:169-272 main) with --save / --restart continues the same chain."""
    import subprocess
    from pmc_amd._lib import START_PATH
    snap = str(tmp_path / "s.pmcsnap")
    dump = str(tmp_path / "d.txt")
    base = [START_PATH, "--cps", "8", "--atoms", "2000", "--every", "1"]

    def run(*extra):
        out = subprocess.run(base + list(extra), check=True, capture_output=True, text=True, timeout=120).stdout
        return [ln for ln in out.splitlines() if not ln.startswith("#")]

    straight = run("--passes", "4")
    first = run("--passes", "2", "--save", snap, "--dump", dump)
    second = run("--passes", "2", "--restart", snap)
    assert first[:3] == straight[:3]
    assert second[1:] == straight[3:]            # "3: E", "4: E" identical to the straight run
    import pmc_amd.io as io
    ts, r, _, _ = io.read_dump(dump, 2)          # frames 0, 1, 2
    assert ts == 2 and r.shape == (3, 2000)


def test_gpu_slab_snapshot_restart(pmc, oracle, tmp_path):
    """The RCCL slab driver's restart (one rank: halos are local copies) on the HIP engine."""
    import torch
    from slab_legacy import SlabSimulation
    path = str(tmp_path / "slab.pmcsnap")
    a = SlabSimulation.create(cps=16, nz_local=16, rank=0, world=1, atoms_per_rank=10_000)
    a.run(0, 2)
    a.save_snapshot(path, 2)
    a.run(2, 2)
    b = SlabSimulation.create(cps=16, nz_local=16, rank=0, world=1)
    first = b.load_snapshot(path)
    b.run(first, 2)
    torch.cuda.synchronize()
    da, na = a.owned()
    db, nb = b.owned()
    assert torch.equal(na, nb)
    assert oracle.valid_slots_equal(da.cpu().numpy().reshape(-1), na.cpu().numpy().reshape(-1),
                                    db.cpu().numpy().reshape(-1), nb.cpu().numpy().reshape(-1), 16)
    assert a.ctx.stats() == b.ctx.stats()
