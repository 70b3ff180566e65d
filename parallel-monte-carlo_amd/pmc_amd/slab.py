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

Two drivers: SlabDriver, the product path (the C slab driver, pmc_slab_*; its schedule groups the
phases into runs of equal z parity and exchanges once per run), and SlabSimulation, the legacy
per-colour schedule above in Python over torch.distributed, whose engine and transport are injected
so the CPU tests drive it with the C oracle and gloo.
"""
from __future__ import annotations

from dataclasses import dataclass
import os
from typing import Callable, List, Optional, Tuple

from .plan import sweep_plan


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


class TorchP2P:
    """Halo transport over torch.distributed point-to-point (nccl/RCCL or gloo)."""

    def __init__(self, rank: int, world: int, group=None, self_p2p: bool = False):
        self.rank = rank
        self.world = world
        self.group = group
        # world == 1 normally copies locally; self_p2p sends to itself through torch.distributed
        # (a one-rank RCCL group: the multi-GPU transport path, rehearsed on one GPU)
        self.self_p2p = self_p2p

    def start(self, sends: List[Tuple[object, int]], recvs: List[Tuple[object, int]]):
        """Issue the exchange; returns a handle for wait().  sends/recvs: (tensor, peer).  Every rank
        issues its sends and receives in the same logical order (down-plane first, then up-plane),
        which fixes the pairwise matching."""
        import torch.distributed as dist
        if self.world == 1 and not self.self_p2p:
            # periodic single-rank slab: each receive takes the send with the same role
            for (dst, _), (src, _) in zip(recvs, sends_for_self(sends, recvs)):
                dst.copy_(src)
            return []
        ops = [dist.P2POp(dist.isend, t, p, group=self.group) for t, p in sends]
        ops += [dist.P2POp(dist.irecv, t, p, group=self.group) for t, p in recvs]
        return dist.batch_isend_irecv(ops)

    @staticmethod
    def wait(handle) -> None:
        for w in handle or []:
            w.wait()

    def exchange(self, sends, recvs) -> None:
        self.wait(self.start(sends, recvs))


def sends_for_self(sends, recvs):
    """world == 1: the i-th receive is filled from the matching send (same order contract)."""
    return sends[: len(recvs)]


class SlabSimulation:
    """LEGACY per-colour schedule (round 1), kept as the CPU-testable twin of the decomposition:
    checkerboard sweeps on one z-slab with a halo exchange after every phase and shift, in Python over
    torch.distributed (tests/test_slab.py drives it with the oracle and gloo).  The product multi-GPU
    path is SlabDriver below (the C slab driver, pmc_slab_sweep).

    engine: object with phase(colour, sweep) and shift(sweep) acting on buffer `cur`, flipping
            `cur` in shift (PmcContext with attached state, or the test's oracle engine).
    disk/n: the two state buffers [buf0, buf1] as tensors of shape (nz+2, cps, cps, 3, nmax)
            and (nz+2, cps, cps) (storage plane 0 is the bottom halo, plane nz+1 the top halo).
    """

    def __init__(self, engine, geom: SlabGeometry, disk: list, n: list, transport, seed: int = 1234,
                 w: float = 2.5, plan_fn: Optional[Callable] = None):
        self.engine = engine
        self.g = geom
        self.disk = disk
        self.n = n
        self.tp = transport
        self.seed = seed
        self.w = w
        self.cur = 0
        self.plan_fn = plan_fn or sweep_plan

    # ---- construction of the product path -------------------------------------------------
    @classmethod
    def create(cls, cps: int, nz_local: int, rank: int, world: int, stream=None, atoms_per_rank: int = 0,
               nmax: int = 16, n_moves: int = 10, seed: int = 1234, group=None, atoms_total: int = 0, **kw):
        """HIP engine on the current device; state in torch device tensors; RCCL transport.
        atoms_per_rank: a lattice inside every slab (weak scaling); atoms_total: one lattice over
        the whole box, each rank keeping its planes (strong scaling; equals a 1-GPU run's state)."""
        import torch
        from .engine import PmcContext
        g = SlabGeometry(cps, nz_local, rank, world, nmax)
        if stream is None:                 # kernels and halo copies must share ONE stream
            stream = torch.cuda.Stream()
        ctx = PmcContext(cps, cps_z=g.cps_z, nz_local=nz_local, z0=g.z0, halo=1, nmax=nmax, n_moves=n_moves,
                         seed=seed, stream=stream.cuda_stream, **kw)
        dev = torch.device("cuda", torch.cuda.current_device())
        shape = (nz_local + 2, cps, cps, 3, nmax)
        disk = [torch.zeros(shape, dtype=torch.float32, device=dev) for _ in range(2)]
        n = [torch.zeros(shape[:3], dtype=torch.int16, device=dev) for _ in range(2)]
        torch.cuda.synchronize()
        ctx.attach_state(disk[0], n[0], disk[1], n[1])
        sim = cls(ctx, g, disk, n, TorchP2P(rank, world, group), seed=seed)
        sim.stream = stream
        sim.bstream = torch.cuda.Stream()  # boundary planes, concurrent with the interior
        if world > 1:
            import torch.distributed as dist
            dist.barrier(group=group)      # a collective first, then point-to-point (NCCL rule)
        if atoms_total:
            ctx.init_lattice_global(atoms_total)
            sim.exchange_full()
        elif atoms_per_rank:
            ctx.init_lattice(atoms_per_rank)
            sim.exchange_full()
        return sim

    @property
    def ctx(self):
        return self.engine

    # ---- halo exchange ------------------------------------------------------------------
    def _plane(self, z_local: int, with_n: bool):
        import torch
        d = self.disk[self.cur][z_local + 1]
        if not with_n:
            return d, None
        # counts travel as bytes: NCCL/RCCL has no 16-bit integer type
        return d, self.n[self.cur][z_local + 1].view(torch.uint8)

    @staticmethod
    def _colour_cells(plane, colour: int):
        """The cells of `colour` (x % 2 == ox, y % 2 == oy; itoa, start.cu:153-157) of one plane
        (cps_y, cps_x, 3, nmax), as a strided view: the only cells a phase changes."""
        ox, oy = (colour // 4) % 2, (colour // 2) % 2
        cy, cx = plane.shape[0], plane.shape[1]
        return plane.reshape(cy // 2, 2, cx // 2, 2, -1)[:, oy, :, ox]

    def _buf(self, key, like):
        """Persistent contiguous staging buffer for a packed colour plane (per role)."""
        bufs = self.__dict__.setdefault("_bufs", {})
        b = bufs.get(key)
        if b is None or b.shape != like.shape or b.device != like.device:
            import torch
            b = bufs[key] = torch.empty(like.shape, dtype=like.dtype, device=like.device)
        return b

    def _exchange(self, send_down: bool, send_up: bool, with_n: bool, wait: bool = True, stream=None,
                  colour=None):
        """Send the boundary plane(s), receive the halo(s).  With `colour` (a phase exchange) only
        that colour's quarter of the plane travels: packed into a staging buffer on the current
        stream, unpacked into the halo when the exchange is completed (_complete)."""
        g = self.g
        sends, recvs, unpack = [], [], []
        local = self.tp.world == 1 and not getattr(self.tp, "self_p2p", False)

        def add(src_z, dst_z, peer_to, peer_from, role):
            d, nn = self._plane(src_z, with_n)
            rd, rn = self._plane(dst_z, with_n)
            if colour is not None:
                sv, rv = self._colour_cells(d, colour), self._colour_cells(rd, colour)
                if local:                       # periodic single rank: one strided copy
                    unpack.append((rv, sv))
                    return
                sb = self._buf(("s", role), sv)
                sb.copy_(sv)
                rb = self._buf(("r", role), rv)
                sends.append((sb, peer_to))
                recvs.append((rb, peer_from))
                unpack.append((rv, rb))
                return
            sends.append((d, peer_to))
            recvs.append((rd, peer_from))
            if with_n:
                sends.append((nn, peer_to))
                recvs.append((rn, peer_from))

        with self._on_stream(stream):
            if send_down:   # my plane 0 -> top halo of the rank below; my top halo <- plane 0 of above
                add(0, g.nz, g.below, g.above, "down")
            if send_up:     # my plane nz-1 -> bottom halo of the rank above; my bottom halo <- below
                add(g.nz - 1, -1, g.above, g.below, "up")
            works = self.tp.start(sends, recvs) if sends else []
            handle = (works, unpack)
            if wait:
                self._complete(handle)
                return None
        return handle

    def _complete(self, handle) -> None:
        """Finish an exchange on the current stream: wait for the transport, unpack the halos."""
        if not handle:
            return
        works, unpack = handle
        self.tp.wait(works)
        for dst, src in unpack:
            dst.copy_(src)

    def _wait(self, handle) -> None:
        if handle:
            with self._on_stream():
                self._complete(handle)

    def _on_stream(self, stream=None):
        import contextlib
        stream = stream if stream is not None else getattr(self, "stream", None)
        if stream is None:
            return contextlib.nullcontext()
        import torch
        return torch.cuda.stream(stream)

    def exchange_after_phase(self, colour: int) -> None:
        oz = colour % 2          # itoa (start.cu:153-157): offset[2] = colour % 2
        self._exchange(send_down=(oz == 0), send_up=(oz == 1), with_n=False, colour=colour)

    def exchange_after_shift(self) -> None:
        self._exchange(True, True, with_n=True)

    def exchange_full(self) -> None:
        self.exchange_after_shift()

    def _shift_and_exchange(self, s: int, run, stream=None):
        """shiftCells after the 8 phases, C-driver rule (pmc_shift_slab): the engine also shifts
        the halo planes it can compute from its own copies, so along x/y nothing travels and along z
        one plane (with counts) goes one way.  Engines without shift_slab refresh both halos.
        Returns the pending exchange."""
        if not hasattr(self.engine, "shift_slab"):
            run("shift", lambda: self.engine.shift(s), *([stream] if stream is not None else []))
            self.cur ^= 1
            return self._exchange(True, True, with_n=True, wait=False)
        box = {}
        run("shift", lambda: box.__setitem__("recv", self.engine.shift_slab(s)),
            *([stream] if stream is not None else []))
        self.cur ^= 1
        recv = box["recv"]
        if recv == 0:
            return None
        # +1: my top halo <- plane 0 of the rank above (each rank sends plane 0 down);
        # -1: my bottom halo <- top plane of the rank below (each rank sends plane nz-1 up)
        return self._exchange(send_down=recv > 0, send_up=recv < 0, with_n=True, wait=False)

    # ---- driver (start.cu:237-260 per slab) -------------------------------------------------
    def phase_only(self, colour: int, sweep: int) -> None:
        self.engine.phase(colour, sweep)

    def shift_only(self, sweep: int) -> None:
        self.engine.shift(sweep)
        self.cur ^= 1

    def sweep(self, s: int, timer=None) -> None:
        if getattr(self, "bstream", None) is not None and hasattr(self.engine, "phase_range_on"):
            return self._sweep_two_streams(s, timer)
        return self._sweep_one_stream(s, timer)

    def _sweep_two_streams(self, s: int, timer=None) -> None:
        """One sweep, boundary planes on a second stream beside the interior (GPU path).

        Per colour k, with S the context stream and T the boundary stream:
          S: wait B(k-1) -> interior I(k) (planes [1, nz-1): no halo read) -> record I(k)
          T: wait I(k-1) and the halo exchange of k-1 -> boundary B(k) (planes 0 and nz-1)
             -> record B(k) -> start the exchange of k (the NCCL stream waits on T)
        so I(k) and B(k) run together, and the exchange of k overlaps I(k+1).  I(k) never touches
        the boundary planes an exchange sends nor the halos it receives; B(k) waits for the
        exchange of k-1 to complete (send and receive).  Cells of one colour are independent, so
        the result equals the sequential schedule bit for bit.  shiftCells (S) waits for both
        streams and the last exchange; its own exchange overlaps the next sweep's first interior.
        `timer(kind, fn, stream)` wraps each launch.
        """
        import torch
        run = timer or (lambda kind, fn, stream=None: fn())
        nz = self.g.nz
        S, T = self.stream, self.bstream
        order, _, _ = self.plan_fn(self.seed, s, self.w)
        pending = getattr(self, "_pending", None)
        ev_b = None
        ev_i = torch.cuda.Event()        # "I(-1)": everything issued on S before this sweep
        ev_i.record(S)
        for colour in order:
            if ev_b is not None:
                S.wait_event(ev_b)
            if nz > 2:
                run("phase", lambda: self.engine.phase_range(colour, s, 1, nz - 1), S)
            ev_prev_i = ev_i
            ev_i = torch.cuda.Event()
            ev_i.record(S)
            with torch.cuda.stream(T):
                T.wait_event(ev_prev_i)
                self._complete(pending)
                run("phase", lambda: self.engine.phase_range_on(colour, s, 0, 1, T.cuda_stream), T)
                if nz > 1:
                    run("phase", lambda: self.engine.phase_range_on(colour, s, nz - 1, nz, T.cuda_stream), T)
                ev_b = torch.cuda.Event()
                ev_b.record(T)
                oz = colour % 2
                pending = self._exchange(send_down=(oz == 0), send_up=(oz == 1), with_n=False, wait=False,
                                         stream=T, colour=colour)
        S.wait_event(ev_i)
        S.wait_event(ev_b)
        self._wait(pending)
        self._pending = self._shift_and_exchange(s, run, S)

    def _sweep_one_stream(self, s: int, timer=None) -> None:
        """One sweep with communication hidden behind the halo-free interior.

        Per colour: (1) the interior planes [1, nz-1) -- they read no halo -- run while the
        previous exchange is in flight; (2) wait for it; (3) the two boundary planes; (4) start
        sending the changed boundary plane without waiting.  shiftCells reads the halos, so it
        waits; its own exchange overlaps the next sweep's first interior.  Cells of a colour are
        independent, so the split does not change the result.  `timer(kind, fn)` wraps each launch
        (kind "phase" or "shift").
        """
        run = timer or (lambda kind, fn: fn())
        nz = self.g.nz
        order, _, _ = self.plan_fn(self.seed, s, self.w)
        pending = getattr(self, "_pending", None)
        for colour in order:
            run("phase", lambda: self.engine.phase_range(colour, s, 1, nz - 1))
            self._wait(pending)
            run("phase", lambda: self.engine.phase_range(colour, s, 0, 1))
            if nz > 1:
                run("phase", lambda: self.engine.phase_range(colour, s, nz - 1, nz))
            oz = colour % 2
            pending = self._exchange(send_down=(oz == 0), send_up=(oz == 1), with_n=False, wait=False,
                                     colour=colour)
        self._wait(pending)
        self._pending = self._shift_and_exchange(s, run)

    def finish(self) -> None:
        """Complete the outstanding halo exchange (call before reading the halos or the state)."""
        self._wait(getattr(self, "_pending", None))
        self._pending = None

    # ---- restart (per-rank PMCSNAP1 files of the owned planes) ----------
    def save_snapshot(self, path: str, next_sweep: int) -> None:
        """Write this rank's owned planes, stats and the next sweep index (the RNG state)."""
        self.finish()
        self.engine.save_snapshot(path, next_sweep)

    def load_snapshot(self, path: str) -> int:
        """Restore this rank's planes from save_snapshot's file, refill the halos from the
        neighbours (collective over the ranks), return the sweep index to continue from."""
        self.finish()
        sweep = self.engine.load_snapshot(path)
        self.exchange_full()
        return sweep

    def run(self, first: int, count: int) -> None:
        for k in range(count):
            self.sweep(first + k)
        self.finish()

    # ---- views ------------------------------------------------------------------------
    def owned(self):
        """(disk, n) of the owned planes of the current buffer; disk as (..., 3, nmax) in the reference
        order whatever the state layout (a packed state is viewed transposed)."""
        d = self.disk[self.cur][1:-1]
        if getattr(self.engine, "state_layout", None) and self.engine.state_layout() == 1:
            d = d.reshape(*d.shape[:-2], d.shape[-1], d.shape[-2]).transpose(-1, -2)
        return d, self.n[self.cur][1:-1]


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
    SlabSimulation above is the legacy per-colour schedule in Python over torch.distributed; the CPU
    tests drive it with the oracle and gloo.
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
        if flags & 1:            # PMC_FLAG_FULL_SHUFFLE: up to 8 runs a sweep, one-plane halos
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
        timed_out = bool(self.ctx.error_flags() & 512)
        d, n = self.ctx.copy_out()
        plane, row, h, nz = self.g.cps * self.cps_y, 3 * self.g.nmax, self.halo, self.g.nz

        def digest(z):   # local plane z (halo planes: -1, nz)
            a = (z + h) * plane
            return hashlib.sha1(d[a * row:(a + plane) * row].tobytes() + n[a:a + plane].tobytes()).digest()[:16]
        mine = digest(0) + digest(nz - 1) + digest(-1) + digest(nz)
        allv = _all_gather_bytes(mine, self._world, self._group)
        w = self._world
        part = [[b[16 * i:16 * (i + 1)] for i in range(4)] for b in allv]   # bottom, top, halo below, halo above
        ok = not timed_out and all(part[r][3] == part[(r + 1) % w][0] and part[r][2] == part[(r - 1) % w][1]
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
