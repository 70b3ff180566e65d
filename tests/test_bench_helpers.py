"""CPU tests of bench.py's host helpers: the stencil counts and the SURVEY.md 8(d) staged-bytes model
that the roofline's `achieved` figure is computed from, the host-CPU description, and the slab parity
leg's sweep window that shifts along z both ways."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import bench  # noqa: E402


def _brute_stencil(n, cps):
    cx, cy, cz = cps
    g = n.reshape(cz, cy, cx)
    out = np.zeros_like(g, dtype=np.int64)
    for z in range(cz):
        for y in range(cy):
            for x in range(cx):
                out[z, y, x] = sum(int(g[(z + dz) % cz, (y + dy) % cy, (x + dx) % cx])
                                   for dz in (-1, 0, 1) for dy in (-1, 0, 1) for dx in (-1, 0, 1))
    return out.reshape(-1)


def test_stencil_counts_matches_brute_force():
    rng = np.random.default_rng(3)
    cps = (5, 4, 6)
    n = rng.integers(0, 17, size=cps[0] * cps[1] * cps[2]).astype(np.int16)
    s = bench.stencil_counts(n, cps)
    assert np.array_equal(s, _brute_stencil(n, cps))
    # every particle lies in exactly 27 stencils of a periodic box with >= 3 cells per axis
    assert s.sum() == 27 * int(n.sum())


def test_slab_stencil_counts_equal_whole_box_rows():
    """A slab whose halo planes hold the periodic images of its neighbours' boundary planes has the
    whole box's stencil counts on its owned planes."""
    rng = np.random.default_rng(5)
    cps, cz, z0, nz = 6, 8, 2, 3
    n = rng.integers(0, 9, size=cz * cps * cps).astype(np.int16)
    whole = bench.stencil_counts(n, (cps, cps, cz)).reshape(cz, cps, cps)
    g = n.reshape(cz, cps, cps)
    storage = np.stack([g[(z0 - 1 + k) % cz] for k in range(nz + 2)])
    s = bench.slab_stencil_counts(storage.reshape(-1), cps, nz)
    assert np.array_equal(s.reshape(nz, cps, cps), whole[z0:z0 + nz])


def test_staged_bytes_formula():
    n = np.array([0, 3, 1, 0, 7], np.int16)
    stencil = np.array([10, 20, 5, 4, 30], np.int64)
    # empty cells are not visited; a visited cell reads 12 B per stencil particle and 27 two-byte
    # counts and writes 12 B per own particle
    expect = (12 * 20 + 54 + 12 * 3) + (12 * 5 + 54 + 12 * 1) + (12 * 30 + 54 + 12 * 7)
    assert bench.staged_bytes(n, stencil) == float(expect)
    assert bench.staged_bytes(np.zeros(4, np.int16), np.zeros(4, np.int64)) == 0.0


def test_staged_bytes_lattice_start_per_launch():
    """The reference lattice start at config 3's density (1e7 in 128^3: 4.77 particles per cell)
    gives ~27x the per-particle read per visited cell; one colour launch visits 1/8 of the cells."""
    cps = 16
    n = np.full(cps ** 3, 5, np.int16)
    s = bench.stencil_counts(n, (cps, cps, cps))
    assert np.all(s == 135)
    total = bench.staged_bytes(n, s)
    assert total == cps ** 3 * (12 * 135 + 54 + 12 * 5)


def test_host_cpu_description():
    d = bench.host_cpu()
    for k in ("model", "logical_cpus", "affinity_cpus", "sockets", "cores_per_socket",
              "socket0_cores_allowed", "cgroup_cpu_quota", "omp_num_threads_env"):
        assert k in d
    assert d["affinity_cpus"] >= 1
    assert d["sockets"] >= 1


def test_traffic_profile_is_per_launch_json():
    t = bench.traffic_from_profile("3", False, 128)
    assert t is not None, "profiles/pmc_traffic.json is committed with the PMC traffic of the bench kernel"
    assert t["subsweep_bytes_per_launch"] > 0
    assert t["read_bytes_per_launch"] + t["write_bytes_per_launch"] > 0


def _gather_rank(rank, world, port, cps, nz, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plane, row = cps * cps, 3 * 4
    # rank r's storage: halo, nz owned planes (values encode global plane and slot), halo
    disk = np.full((nz + 2) * plane * row, -1.0, np.float32)
    n = np.full((nz + 2) * plane, -1, np.int16)
    for z in range(nz):
        zg = rank * nz + z
        disk[(z + 1) * plane * row:(z + 2) * plane * row] = zg * 1000 + np.arange(plane * row) % 997
        n[(z + 1) * plane:(z + 2) * plane] = zg
    out = bench.make_gather(world, rank, plane, nz, row)(disk, n)
    q.put((rank, out))
    dist.destroy_process_group()


def test_make_gather_world2_gloo():
    """bench.py's gather of the owned planes (the N>1 line's CPU baseline and parity leg): rank 0
    receives the whole box in global plane order, the halo planes dropped; other ranks get None."""
    import multiprocessing as mp
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, cps, nz = 2, 4, 3
    ps = [ctx.Process(target=_gather_rank, args=(r, world, port, cps, nz, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
    assert res[1] is None
    disk, n = res[0]
    plane, row = cps * cps, 12
    assert np.array_equal(n, np.repeat(np.arange(world * nz), plane).astype(np.int16))
    expect = np.concatenate([zg * 1000 + np.arange(plane * row) % 997 for zg in range(world * nz)]).astype(np.float32)
    assert np.array_equal(disk, expect)


# ---- round 6: the slab parity leg's window of sweeps that shift along z both ways
def test_z_shift_window_covers_both_z_directions(oracle):
    for seed, first, sweeps in ((1234, 5, 3), (1234, 0, 2), (99, 17, 3), (1234, 100, 4)):
        s0 = bench.z_shift_window(seed, first, sweeps)
        assert s0 >= first
        plans = [oracle.sweep_plan(seed, s, 2.5) for s in range(s0, s0 + sweeps)]
        zdirs = {d > 0 for _, f, d in plans if f == 2}
        assert zdirs == {True, False}, (seed, first, s0, plans)
        # the first such window: no earlier start in [first, s0) has both directions
        for s in range(first, s0):
            early = [oracle.sweep_plan(seed, t, 2.5) for t in range(s, s + sweeps)]
            assert {d > 0 for _, f, d in early if f == 2} != {True, False}
        assert bench.z_shifts(seed, s0, sweeps) == ["xyz"[f] + ("+" if d > 0 else "-") for _, f, d in plans]


def test_z_shift_window_single_sweep_is_first():
    assert bench.z_shift_window(1234, 7, 1) == 7
