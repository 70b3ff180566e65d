"""The product slab driver as separate rank PROCESSES on one GPU.

Each rank is its own process (tests/mp_slab_worker.py), as on a multi-GPU node; they all use GPU 0,
so the halo transport is the IPC one (pmc_slab_init_ipc: every rank maps its peers' state buffers
and flags, exchanges are pulled by the library's copy kernels -- RCCL refuses two ranks on one
device).  The ranks' owned planes, the four counters, the energy and pmc_slab_observables' whole-box
sums must equal the C oracle's whole-box run bit for bit over sweeps that shift along x, y and z in
both directions (start.cu:237-260 is the loop being partitioned).  bench.py's own launcher
(`--gpus 2 --same-device`) runs the N > 1 bench path with real processes, parity leg included.
Tolerance: none.
"""
import json
import os
import signal
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(REPO, "tests", "mp_slab_worker.py")
VERIFY_WORKER = os.path.join(REPO, "tests", "mp_verify_worker.py")
TIMEOUT_WORKER = os.path.join(REPO, "tests", "mp_timeout_worker.py")


def _window(oracle, count):
    """First sweep s of a window [s, s+count) whose plans shift along x, y, and z both ways."""
    for s in range(0, 400):
        plans = [oracle.sweep_plan(1234, s + k, 2.5) for k in range(count)]
        fs = {f for _, f, _ in plans}
        zdirs = {d > 0 for _, f, d in plans if f == 2}
        if fs == {0, 1, 2} and zdirs == {True, False}:
            return s
    raise AssertionError("no window")


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_processes(world, argv, timeout=180, ipc_timeout_s="30"):
    """Start `world` rank processes of argv, wait; on failure or timeout kill their process groups."""
    port = str(_free_port())
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, PMC_IPC_TIMEOUT_S=ipc_timeout_s)
        procs.append(subprocess.Popen([sys.executable] + argv, env=env, start_new_session=True,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = [None] * world
    try:
        for r, p in enumerate(procs):
            outs[r], _ = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        pass
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
    codes = [p.returncode for p in procs]
    assert codes == [0] * world, "rank processes failed: " + " | ".join(
        f"rank {r} rc {c}: {(outs[r] or '')[-1500:]}" for r, c in enumerate(codes) if c != 0)
    return outs


@pytest.mark.parametrize("world,cps,cps_z,atoms,flags,halo,restart", [
    (2, 16, 16, 10_000, 0, 1, False),
    (4, 16, 16, 10_000, 0, 1, False),
    (2, 32, 32, 120_000, 0, 1, False),
    (4, 32, 32, 120_000, 0, 1, False),
    (4, 16, 16, 10_000, 1, 1, False),     # reference-like colour order: up to 8 exchanges a sweep
    (2, 16, 16, 10_000, 0, 2, False),     # two-plane halos: send buffers mapped too
    (4, 32, 32, 120_000, 0, 2, False),
    (2, 16, 16, 10_000, 0, 1, True),      # snapshot restart onto fresh drivers (new mappings)
])
def test_ipc_processes_equal_oracle(pmc, oracle, tmp_path, world, cps, cps_z, atoms, flags, halo, restart):
    count = 8
    first = _window(oracle, count)
    argv = [WORKER, str(tmp_path), str(cps), str(cps), str(cps_z), str(atoms), str(flags), str(halo), str(first),
            str(count)] + (["restart"] if restart else [])
    _run_processes(world, argv)
    st = oracle.OracleState(oracle.make_params(cps=cps, cps_z=cps_z, flags=flags))
    assert st.init_lattice(atoms) == 0
    assert st.run(first, count) == 0
    nz = cps_z // world
    plane, row = cps * cps, 3 * 16
    tot = {"de_fixed": 0, "accepted": 0, "trials": 0, "evaluated": 0}
    whole = st.stats.as_dict()
    for r in range(world):
        z = np.load(tmp_path / f"rank{r}.npz")
        with open(tmp_path / f"rank{r}.json") as f:
            j = json.load(f)
        ref = slice(r * nz * plane, (r + 1) * nz * plane)
        assert np.array_equal(z["n"], st.n[ref]), f"rank {r}: counts differ"
        assert oracle.valid_slots_equal(z["disk"], z["n"], st.disk[ref.start * row:ref.stop * row], st.n[ref], 16), \
            f"rank {r}: coordinates differ"
        assert j["flags"] == 0, j["flags"]
        for k in tot:
            tot[k] += j["stats"][k]
        # pmc_slab_observables through the IPC transport: the whole box's counters and energy
        assert j["obs"] == whole, (r, j["obs"], whole)
        assert j["e_all"] == st.energy()
    assert tot == whole     # (a restart restores the snapshot's counters: the same totals)


@pytest.mark.parametrize("world", [2, 8])
def test_bench_rank_processes_same_device(pmc, world):
    """bench.py --gpus N launches N rank processes itself; with --same-device all use GPU 0 and the
    halos go through the IPC transport (world 8: 4 planes per rank of the 32^3 box).  The N > 1 line
    carries the gathered whole-box parity leg."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["PMC_IPC_TIMEOUT_S"] = "30"
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(world), "--same-device", "--config", "4",
                        "--cps", "32", "--atoms", "120000", "--steps", "4", "--warmup", "2", "--rewarm", "2",
                        "--serial-planes", "4", "--rank-timeout", "240"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == world
    assert "IPC" in d["config"]["parallelism"], d["config"]["parallelism"]
    assert d["error_flags"] == 0
    par = d["parity"]
    assert par["state_bitwise_equal"] and par["counters_equal"], par
    assert par["energy_rel_err"] == 0.0 and par["acceptance_rel_err"] == 0.0, par
    # the parity leg covers --cpu-sweeps (3) sweeps chosen to shift along z both ways: every exchange
    # kind, the deferred z planes from above and below included
    assert par["sweeps"] == 3 and "z+" in par["shifts"] and "z-" in par["shifts"], par
    assert d["cpu_baseline"]["sample"].startswith("3 full sweeps"), d["cpu_baseline"]["sample"]
    # the whole-node HBM roofline: every rank's staged-model bytes of a step over ms_per_step, N x 8 TB/s
    node = d["roofline"]["node"]
    assert node["gpus"] == world and node["peak"] == 8000.0 * world, node
    assert node["bytes_per_step"] > 0 and 0 < node["frac"] < 1, node
    hb = d["roofline"]["achievable_peak"]
    assert 500 < hb["copy_GBs"] < 8000 and 500 < hb["read_GBs"] < 8000, hb


def test_ipc_halo_verification(pmc, tmp_path):
    """SlabDriver.verify_transport's check (every halo equals the plane its neighbour sent, digests
    gathered over gloo): true after the IPC exchange of two rank processes, false on every rank once
    one float of one halo differs, true again after the next exchange.  (bench.py --transport auto
    falls back to RCCL on every rank when it fails: IPC between distinct GPUs runs first on the
    driver's node.)"""
    _run_processes(2, [VERIFY_WORKER, str(tmp_path)])
    for r in range(2):
        with open(tmp_path / f"rank{r}.json") as f:
            j = json.load(f)
        assert j == {"transport": "ipc", "after_init": True, "after_corruption": False, "after_exchange": True}, (r, j)


def test_ipc_timeout_fails_not_copies(pmc, tmp_path):
    """a peer that stops taking part makes every IPC wait give up (PMC_IPC_TIMEOUT_S = 2 s
    here) without copying and without publishing "pulled"; error bit 9 is set and pmc_slab_finish
    reports it (PMC_ERR_HIP), within seconds, with no hang.  The silent rank stays alive, so the
    buffers its peer maps stay valid."""
    _run_processes(2, [TIMEOUT_WORKER, str(tmp_path)], timeout=150, ipc_timeout_s="2")
    with open(tmp_path / "rank0.json") as f:
        j = json.load(f)
    assert j["transport"] == "ipc"
    assert "did not arrive" in j["finish"], j
    assert j["flags"] & 512, j
    assert j["seconds"] < 90, j

