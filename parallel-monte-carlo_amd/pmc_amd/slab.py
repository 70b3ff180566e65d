"""z-slab domain decomposition over ranks (one process per GPU); halo planes over the IPC transport
(peer buffers mapped over xGMI, pulled by the library's copy kernels) or RCCL.

The reference is single-GPU (start.cu:169-272); this is the build's multi-GPU path (SURVEY.md
section 8e).  Rank r owns global cell planes z in [r*nz, (r+1)*nz) of a cps x cps x (world*nz)
periodic box and stores one halo plane below and above (pmc_params.halo = 1).  Every rank runs
every colour phase on its slab; the checkerboard guarantees that a phase only READS the halo
planes, and only the boundary plane of the phase's z-parity changes:

  * after a phase with oz = 0 the owned plane 0 changed  -> it becomes the top halo of rank r-1;
  * after a phase with oz = 1 the owned plane nz-1 changed -> the bottom halo of rank r+1;
  * after shiftCells every plane (and the counts) may change: the halo planes computable from the
    rank's own copies are shifted with the owned ones (along x/y both, along z the one on the -dir
    side), the other z halo receives the neighbour's new plane (pmc_shift_slab, as the C driver).

The sweep plan (colour order, f, d) is a pure function of (seed, sweep) that every rank derives
itself, and the RNG counters use GLOBAL cell ids, so the result is bit-identical to the
whole-box run for any number of ranks (tests/test_slab.py checks 2 ranks against 1).

The driver is SlabDriver, the product path (the C slab driver, pmc_slab_*; its schedule groups the
phases into runs of equal z parity and exchanges once per run).  The legacy per-colour schedule in
Python over torch.distributed (SlabSimulation, round 1) lives in tests/slab_legacy.py: the CPU tests
drive it with the C oracle and gloo.
"""
from __future__ import annotations

from dataclasses import dataclass
import os
from typing import Optional

@dataclass
class SlabGeometry:
    cps: int          # cells along x and y
    nz: int           # owned planes per rank (even)
    rank: int
    world: int
    nmax: int

    @property
    def cps_z(self) -> int:
        return self.nz * self.world

    @property
    def z0(self) -> int:
        return self.rank * self.nz

    @property
    def below(self) -> int:
        return (self.rank - 1) % self.world

    @property
    def above(self) -> int:
        return (self.rank + 1) % self.world


def _all_gather_bytes(data: bytes, world: int, group=None) -> list:
    """Every rank's `data` (equal lengths) in rank order, over the torch.distributed group (gloo:
    CPU tensors, nccl: device tensors)."""
    if world == 1:
        return [data]
    import numpy as np
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    mine = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).to(dev)
    out = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(out, mine, group=group)
    return [bytes(t.cpu().numpy().tobytes()) for t in out]


def _all_ok(ok: bool, world: int, group=None) -> bool:
    if world == 1:
        return ok
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


TRANSPORTS = ("ipc", "rccl", "local", "auto")


def _rccl_lib_path() -> Optional[str]:
    """The librccl torch already loaded (same soname: dlopen in C shares that instance)."""
    import torch
    cand = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return cand if os.path.exists(cand) else None


class SlabDriver:
    """The product multi-GPU path: the C slab driver (pmc_slab_*), one process per GPU.

    The sweep schedule runs in C (pmc_slab_sweep): the 8 colour phases form two
    runs of equal z parity; per run the interior planes go in 1-3 launch chains on their own streams
    (PMC_SLAB_CHAINS) and the run's boundary plane on the exchange stream, which then sends that whole
    plane to the neighbour holding it as a halo and receives the opposite halo (one RCCL send/recv
    each way per run); after shiftCells only a z shift needs one more plane.  With halo=2 (two halo
    planes per side; PMC_SLAB_HALO=2 sets the default) the first run also visits the neighbour's
    boundary plane redundantly and a sweep needs ONE exchange, after shiftCells.
    The host issues a sweep in a few dozen HIP calls.  Transports: IPC (default for world > 1: one
    process per rank, the peers' buffers mapped, exchanges pulled by the library's copy kernels), RCCL,
    local copies (one rank), or the in-process group (W ranks as threads of one process).
    """

    def __init__(self, cps: int, nz_local: int, rank: int, world: int, stream=None, atoms_per_rank: int = 0,
                 atoms_total: int = 0, nmax: int = 16, n_moves: int = 10, seed: int = 1234,
                 use_rccl: Optional[bool] = None, group=None, local_group=None, cps_y: int = 0,
                 flags: int = 0, lattice_cps_z: int = 0, halo: int = 0, transport: Optional[str] = None):
        """local_group: a pmc_amd.engine.LocalGroup -- the in-process transport (this rank is one of
        local_group.world slab contexts of this process; construct and drive each rank from its
        own thread: the exchanges are collective).  flags: pmc_params.flags (PMC_FLAG_FULL_SHUFFLE:
        the reference-like colour order, up to 8 runs and exchanges per sweep).  lattice_cps_z with
        atoms_total: the lattice of atoms_total particles over a box lattice_cps_z cells tall
        (pmc_init_lattice_planes; the config-5 weak-scaling start), else over this box.  halo: halo
        planes per side, 1 or 2 (0: PMC_SLAB_HALO, default 1; the reference-like colour order always
        uses 1).  transport (one process per rank): "ipc" -- the peers' buffers mapped with
        hipIpcOpenMemHandle, exchanges pulled by the library's own copy kernels (pmc_slab_init_ipc; also
        several rank processes on ONE GPU, which RCCL refuses); "rccl"; "local" (world 1: periodic
        halos by local copies); "auto" -- IPC, or RCCL on every rank if any rank cannot map its peers.
        Default: PMC_SLAB_TRANSPORT, else "ipc" for world > 1, "local" for one rank (use_rccl=True:
        "rccl", the one-rank RCCL rehearsal)."""
        from .engine import PmcContext, comm_unique_id
        self.g = SlabGeometry(cps, nz_local, rank, world, nmax)
        if stream is None and local_group is None:
            import torch
            stream = torch.cuda.Stream()
        self.stream = stream
        if not halo:
            halo = int(os.environ.get("PMC_SLAB_HALO", "1") or 1)
        if flags & 7:            # FULL_SHUFFLE (up to 8 runs a sweep) or quirks R1/R2: one-plane halos
            halo = 1
        self.halo = halo
        self.ctx = PmcContext(cps, cps_y=cps_y, cps_z=self.g.cps_z, nz_local=nz_local, z0=self.g.z0, halo=halo,
                              nmax=nmax, n_moves=n_moves, seed=seed, flags=flags,
                              stream=stream.cuda_stream if stream is not None else None)
        self.cps_y = cps_y or cps
        self._rank, self._world, self._group = rank, world, group
        self._requested = transport
        if local_group is not None:
            if local_group.world != world:
                raise ValueError("local_group.world != world")
            self.ctx.slab_init_local(rank, local_group)
            self.transport = "in-process"
        else:
            if transport is None:
                transport = ("rccl" if use_rccl else
                             os.environ.get("PMC_SLAB_TRANSPORT") or ("ipc" if world > 1 else "local"))
            if transport not in TRANSPORTS:
                raise ValueError(f"transport must be one of {TRANSPORTS}")
            if transport == "local" and world > 1:
                raise ValueError("transport 'local' is a one-rank slab")
            if transport in ("ipc", "auto"):
                ok, err = True, None
                try:
                    blobs = _all_gather_bytes(self.ctx.slab_ipc_handle(), world, group)
                    self.ctx.slab_init_ipc(rank, world, blobs)
                except Exception as e:      # (collective below: every rank learns of a failure)
                    ok, err = False, e
                if _all_ok(ok, world, group):
                    transport = "ipc"
                elif transport == "ipc":
                    raise RuntimeError(f"IPC halo transport unavailable on rank {rank}: {err!r}") if err \
                        else RuntimeError("IPC halo transport unavailable on another rank")
                else:
                    transport = "rccl"      # auto: every rank falls back together
            self.transport = transport
            if transport != "ipc":
                self._init_messages(transport)
        if atoms_total and lattice_cps_z:
            self.ctx.init_lattice_planes(atoms_total, lattice_cps_z)
        elif atoms_total:
            self.ctx.init_lattice_global(atoms_total)
        elif atoms_per_rank:
            self.ctx.init_lattice(atoms_per_rank)
        if atoms_total or atoms_per_rank:
            self.ctx.slab_exchange()
            self.verify_transport()

    def verify_transport(self) -> None:
        """Right after a full exchange (pmc_slab_exchange) of a non-trivial state: with the IPC transport
        at world > 1, check every halo against the plane its neighbour sent (IPC between distinct GPUs
        has only run on the driver's node); on a mismatch or a timed-out wait, "auto" falls back to RCCL
        on every rank (and exchanges again), "ipc" raises.  PMC_IPC_VERIFY=0 skips it.  Collective."""
        if self.transport != "ipc" or self._world == 1 or os.environ.get("PMC_IPC_VERIFY", "1") == "0":
            return
        if self._halos_verified():
            return
        if self._requested != "auto":
            raise RuntimeError("IPC halo transport: the first exchange delivered wrong halos")
        self.transport = "rccl"
        self._init_messages("rccl")   # (pmc_slab_init re-attaches: the IPC slab is dropped)
        self.ctx.synchronize()
        self.ctx.error_flags(reset=True)   # the failed transport's timeout bit, not the state's
        self.ctx.slab_exchange()

    def _init_messages(self, transport: str) -> None:
        """pmc_slab_init with RCCL (a communicator from a unique id broadcast over the group) or, for
        one rank, local copies.  Collective over the ranks."""
        from .engine import comm_unique_id
        rank, world, group = self._rank, self._world, self._group
        uid = None
        if transport == "rccl":
            import torch
            lib_path = _rccl_lib_path()
            if lib_path and not os.environ.get("PMC_RCCL_LIB"):
                os.environ["PMC_RCCL_LIB"] = lib_path
            buf = torch.zeros(128, dtype=torch.uint8)
            if rank == 0:
                buf = torch.tensor(list(comm_unique_id()), dtype=torch.uint8)
            if world > 1:
                import torch.distributed as dist
                on = buf.cuda() if dist.get_backend(group) == "nccl" else buf
                dist.broadcast(on, src=0, group=group)
                buf = on.cpu()
            uid = bytes(buf.numpy().tobytes())
        self.ctx.slab_init(rank, world, uid)  # RCCL communicator: collective over the ranks

    def _halos_verified(self) -> bool:
        """After an exchange: every rank's halo planes equal the planes its neighbours sent (digests
        gathered over the group) and no transfer wait timed out (error bit 512).  Collective."""
        import hashlib
        self.ctx.synchronize()
        timed_out = bool(self.ctx.error_flags() & (512 | 1024))
        d, n = self.ctx.copy_out()
        plane, row, h, nz = self.g.cps * self.cps_y, 3 * self.g.nmax, self.halo, self.g.nz

        def digest(z):   # local plane z (halo planes: -h..-1, nz..nz+h-1)
            a = (z + h) * plane
            return hashlib.sha1(d[a * row:(a + plane) * row].tobytes() + n[a:a + plane].tobytes()).digest()[:16]
        # every halo plane of both sides (h of them), against the planes the neighbours sent: the
        # bottom h planes [0, h) go up as the lower neighbour's halos above, the top h planes
        # [nz-h, nz) go down as the upper neighbour's halos below
        groups = ([digest(k) for k in range(h)], [digest(nz - h + k) for k in range(h)],
                  [digest(-h + k) for k in range(h)], [digest(nz + k) for k in range(h)])
        mine = b"".join(b"".join(g) for g in groups)
        allv = _all_gather_bytes(mine, self._world, self._group)
        w = self._world

        def part(r, g):   # rank r's group g (0 bottom, 1 top, 2 halos below, 3 halos above)
            return allv[r][16 * h * g:16 * h * (g + 1)]
        ok = not timed_out and all(part(r, 3) == part((r + 1) % w, 0) and part(r, 2) == part((r - 1) % w, 1)
                                   for r in range(w))
        return _all_ok(ok, w, self._group)

    def sweep(self, s: int) -> None:
        self.ctx.slab_sweep(s)

    def finish(self) -> None:
        self.ctx.slab_finish()

    def run(self, first: int, count: int) -> None:
        for k in range(count):
            self.sweep(first + k)
        self.finish()

    def load_state(self, disk, n) -> None:
        """Owned planes from host arrays ((nz, cps, cps, 3, nmax) floats, (nz, cps, cps) int16);
        halos refilled from the neighbours."""
        import numpy as np
        full_d, full_n = self.ctx.copy_out()
        plane = self.g.cps * self.cps_y
        row = 3 * self.g.nmax
        h = self.halo
        full_d[h * plane * row:(self.g.nz + h) * plane * row] = np.asarray(disk, np.float32).reshape(-1)
        full_n[h * plane:(self.g.nz + h) * plane] = np.asarray(n, np.int16).reshape(-1)
        self.ctx.copy_in(full_d, full_n)
        self.ctx.slab_exchange()

    def owned(self):
        """(disk, n) of the owned planes as host arrays (after finish())."""
        d, n = self.ctx.copy_out()
        plane = self.g.cps * self.cps_y
        row = 3 * self.g.nmax
        h = self.halo
        return d[h * plane * row:(self.g.nz + h) * plane * row], n[h * plane:(self.g.nz + h) * plane]
