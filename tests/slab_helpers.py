"""Helpers for the slab-decomposition tests: an oracle-backed engine with the PmcContext
phase/shift interface (TEST INFRASTRUCTURE), and a whole-box reference run."""
import ctypes as C

import numpy as np
import torch

import pmc_oracle
from pmc_amd.slab import SlabGeometry
from slab_legacy import SlabSimulation, TorchP2P


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

    def shift_slab(self, sweep):
        """pmc_shift_slab's rule on the oracle: owned planes plus the locally computable halo
        planes; returns the halo still to receive (0, +1 top, -1 bottom)."""
        _, f, d = pmc_oracle.sweep_plan(self.p.seed, sweep, self.p.w)
        nz = self.p.nz_local
        recv = 0 if f != 2 else (1 if d > 0 else -1)
        zl0, zl1 = (-1 if recv >= 0 else 0), (nz + 1 if recv <= 0 else nz)
        over = pmc_oracle.lib().orc_shift_cells_planes(C.byref(self.p), self.d[self.cur], self.nn[self.cur],
                                                       self.d[1 - self.cur], self.nn[1 - self.cur], f, d, zl0, zl1)
        assert over == 0
        self.cur ^= 1
        return recv


    # restart hooks (the HIP engine's are PmcContext.save_snapshot / load_snapshot)
    def _owned(self):
        plane = self.p.cps_x * self.p.cps_y
        return slice(plane, plane * (1 + self.p.nz_local))

    def save_snapshot(self, path, next_sweep):
        import pmc_amd.io as io
        sl = self._owned()
        nm = self.p.nmax
        io.write_snapshot(path, self.p, next_sweep, self.stats.as_dict(),
                          self.d[self.cur][sl.start * 3 * nm:sl.stop * 3 * nm], self.nn[self.cur][sl])

    def load_snapshot(self, path):
        import pmc_amd.io as io
        sl = self._owned()
        nm = self.p.nmax
        q, sweep, stats, disk, n = io.read_snapshot(path, cells=sl.stop - sl.start)
        assert (q.z0, q.nz_local, q.seed) == (self.p.z0, self.p.nz_local, self.p.seed)
        self.d[self.cur][:] = 0
        self.nn[self.cur][:] = 0
        self.d[self.cur][sl.start * 3 * nm:sl.stop * 3 * nm] = disk
        self.nn[self.cur][sl] = n
        for k, v in stats.items():
            setattr(self.stats, k, v)
        return sweep


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


def worker(rank, world, port, cps, nz, nmax, atoms, sweeps, out_q, first=0):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sim = make_oracle_slab(cps, nz, rank, world, nmax, atoms, TorchP2P(rank, world))
        d0, n0 = sim.owned()
        init = (d0.numpy().copy(), n0.numpy().copy())
        sim.run(first, sweeps)
        d1, n1 = sim.owned()
        out_q.put((rank, init, (d1.numpy().copy(), n1.numpy().copy()), sim.engine.stats.as_dict()))
    finally:
        dist.destroy_process_group()


def worker_restart(rank, world, port, cps, nz, nmax, atoms, snapdir, out_q):
    """2 sweeps, per-rank snapshot, 2 more sweeps; then fresh slabs restored from the snapshots
    run the same 2 sweeps: both final states go back for comparison."""
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        path = os.path.join(snapdir, f"rank{rank}.pmcsnap")
        sim = make_oracle_slab(cps, nz, rank, world, nmax, atoms, TorchP2P(rank, world))
        sim.run(0, 2)
        sim.save_snapshot(path, 2)
        sim.run(2, 2)
        d1, n1 = sim.owned()
        straight = (d1.numpy().copy(), n1.numpy().copy(), sim.engine.stats.as_dict())
        sim2 = make_oracle_slab(cps, nz, rank, world, nmax, 0, TorchP2P(rank, world))
        first = sim2.load_snapshot(path)
        sim2.run(first, 2)
        d2, n2 = sim2.owned()
        out_q.put((rank, straight, (d2.numpy().copy(), n2.numpy().copy(), sim2.engine.stats.as_dict())))
    finally:
        dist.destroy_process_group()
