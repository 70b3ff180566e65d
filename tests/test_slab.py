"""The LEGACY per-colour slab schedule on CPU: 2-4 gloo rank processes drive the oracle through
SlabSimulation (tests/slab_legacy.py), the Python twin of round 1's schedule -- a halo exchange after every
colour phase over torch.distributed.  It is not the product's schedule: the product multi-GPU path is
the C slab driver (pmc_slab_sweep: runs of equal z parity, one exchange per run, deferred z planes),
whose rank PROCESSES are tested on the GPU against the oracle through the IPC transport
(tests/test_gpu_multiprocess.py) and whose schedule at world 1-8 through the in-process transport
(tests/test_gpu_multirank.py).  What this file pins on CPU is the decomposition itself: global-id RNG
counters, the replicated sweep plan and the halo shift rule reproduce the whole-box run bit for bit."""
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import slab_helpers


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# sweeps 0-3 shift along x/y only; 10-17 include z shifts in both directions (13-17), where each
# rank shifts one halo plane itself and receives the other from its neighbour
@pytest.mark.parametrize("world,nz,first,sweeps", [(2, 4, 0, 4), (2, 8, 10, 8), (3, 4, 10, 8), (4, 4, 12, 6)])
def test_slab_ranks_equal_whole_box(oracle, world, nz, first, sweeps):
    cps, nmax, atoms = 8, 16, 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=slab_helpers.worker, args=(r, world, port, cps, nz, nmax, atoms, sweeps, q, first))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, init, final, stats = q.get(timeout=300)
        res[rank] = (init, final, stats)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # whole box, same initial state, same sweeps
    st = slab_helpers.whole_box_from_slabs(cps, nz, world, nmax, [res[r][0][0] for r in range(world)],
                                           [res[r][0][1] for r in range(world)])
    assert int(st.n.sum()) == atoms * world
    assert st.run(first, sweeps) == 0
    got_d = np.concatenate([res[r][1][0].reshape(-1) for r in range(world)])
    got_n = np.concatenate([res[r][1][1].reshape(-1) for r in range(world)])
    assert np.array_equal(got_n, st.n)
    assert oracle.valid_slots_equal(got_d, got_n, st.disk, st.n, nmax)
    tot = {k: sum(res[r][2][k] for r in range(world)) for k in res[0][2]}
    assert tot == st.stats.as_dict()


def test_slab_single_rank_periodic(oracle):
    """world == 1 slab (halo planes filled by local copies) equals the whole box."""
    from slab_legacy import TorchP2P
    sim = slab_helpers.make_oracle_slab(8, 8, 0, 1, 16, 1500, TorchP2P(0, 1))
    d0, n0 = sim.owned()
    st = slab_helpers.whole_box_from_slabs(8, 8, 1, 16, [d0.numpy().copy()], [n0.numpy().copy()])
    sim.run(0, 3)
    st.run(0, 3)
    d1, n1 = sim.owned()
    assert np.array_equal(n1.numpy().reshape(-1), st.n)
    assert oracle.valid_slots_equal(d1.numpy().reshape(-1), n1.numpy().reshape(-1), st.disk, st.n, 16)


def test_slab_snapshot_restart(oracle, tmp_path):
    """Per-rank snapshots + halo refill: the restarted 2-rank run equals the uninterrupted one."""
    world, cps, nz, nmax, atoms = 2, 8, 4, 16, 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=slab_helpers.worker_restart, args=(r, world, port, cps, nz, nmax, atoms,
                                                                   str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    for _ in range(world):
        rank, straight, restarted = q.get(timeout=300)
        assert np.array_equal(straight[1], restarted[1])
        assert oracle.valid_slots_equal(straight[0].reshape(-1), straight[1].reshape(-1), restarted[0].reshape(-1),
                                        restarted[1].reshape(-1), nmax)
        assert straight[2] == restarted[2]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
