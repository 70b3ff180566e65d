"""Helpers for the slab-decomposition tests: an oracle-backed engine with the PmcContext
phase/shift interface (TEST INFRASTRUCTURE), and a whole-box reference run."""
import ctypes as C

import numpy as np
import torch

import pmc_oracle
from pmc_amd.slab import SlabGeometry, SlabSimulation, TorchP2P


class OracleEngine:
    """phase/shift on torch CPU buffers through the C oracle (halo = 1 slab)."""

    def __init__(self, params, disk, n):
        self.p = params
        self.d = [t.numpy().reshape(-1) for t in disk]
        self.nn = [t.numpy().reshape(-1) for t in n]
        self.cur = 0
        self.stats = pmc_oracle.Stats()

    def phase(self, colour, sweep):
        o = pmc_oracle.colour_offset(colour)
        pmc_oracle.lib().orc_subsweep(C.byref(self.p), self.d[self.cur], self.nn[self.cur], o[0], o[1], o[2],
                                      sweep, C.byref(self.stats))

    def phase_range(self, colour, sweep, zl_begin, zl_end):
        o = pmc_oracle.colour_offset(colour)
        pmc_oracle.lib().orc_subsweep_range(C.byref(self.p), self.d[self.cur], self.nn[self.cur], o[0], o[1],
                                            o[2], sweep, zl_begin, zl_end, C.byref(self.stats))

    def shift(self, sweep):
        _, f, d = pmc_oracle.sweep_plan(self.p.seed, sweep, self.p.w)
        over = pmc_oracle.lib().orc_shift_cells(C.byref(self.p), self.d[self.cur], self.nn[self.cur],
                                                self.d[1 - self.cur], self.nn[1 - self.cur], f, d)
        assert over == 0
        self.cur ^= 1


def make_oracle_slab(cps, nz, rank, world, nmax, atoms_per_rank, transport):
    g = SlabGeometry(cps, nz, rank, world, nmax)
    p = pmc_oracle.make_params(cps=cps, cps_z=g.cps_z, nz_local=nz, z0=g.z0, halo=1, nmax=nmax)
    assert pmc_oracle.lib().orc_params_check(C.byref(p)) == 0
    shape = (nz + 2, cps, cps, 3, nmax)
    disk = [torch.zeros(shape, dtype=torch.float32) for _ in range(2)]
    n = [torch.zeros(shape[:3], dtype=torch.int16) for _ in range(2)]
    eng = OracleEngine(p, disk, n)
    r = np.zeros(3 * atoms_per_rank, np.float32)
    pmc_oracle.lib().orc_init_r(C.byref(p), atoms_per_rank, r)
    assert pmc_oracle.lib().orc_assign(C.byref(p), r, atoms_per_rank, eng.d[0], eng.nn[0]) == 0
    sim = SlabSimulation(eng, g, disk, n, transport, seed=p.seed, w=p.w, plan_fn=pmc_oracle.sweep_plan)
    sim.exchange_full()
    return sim


def whole_box_from_slabs(cps, nz, world, nmax, owned_disks, owned_ns):
    """Whole-box oracle state assembled from the slabs' owned planes (z-major storage)."""
    st = pmc_oracle.OracleState(pmc_oracle.make_params(cps=cps, cps_z=nz * world, nmax=nmax))
    st.disk[:] = np.concatenate([d.reshape(-1) for d in owned_disks])
    st.n[:] = np.concatenate([x.reshape(-1) for x in owned_ns])
    return st


def worker(rank, world, port, cps, nz, nmax, atoms, sweeps, out_q):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sim = make_oracle_slab(cps, nz, rank, world, nmax, atoms, TorchP2P(rank, world))
        d0, n0 = sim.owned()
        init = (d0.numpy().copy(), n0.numpy().copy())
        sim.run(0, sweeps)
        d1, n1 = sim.owned()
        out_q.put((rank, init, (d1.numpy().copy(), n1.numpy().copy()), sim.engine.stats.as_dict()))
    finally:
        dist.destroy_process_group()
