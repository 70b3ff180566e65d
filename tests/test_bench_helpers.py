"""CPU tests of bench.py's host helpers: the stencil counts and the SURVEY.md 8(d) staged-bytes model
that the roofline's `achieved` figure is computed from, and the host-CPU description."""
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
    t = bench.traffic_from_profile()
    assert t is not None, "profiles/pmc_traffic.json is committed with the PMC traffic of the bench kernel"
    assert t["subsweep_bytes_per_launch"] > 0
    assert t["read_bytes_per_launch"] + t["write_bytes_per_launch"] > 0
