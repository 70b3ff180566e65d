"""LEGACY per-colour slab schedule (round 1), moved out of the product package: the
Python twin of the z-slab decomposition over torch.distributed, whose engine and transport are
injected so the CPU tests drive it with the C oracle and gloo (tests/test_slab.py), and two GPU
tests drive it over the HIP engine.  The product multi-GPU path is pmc_amd.slab.SlabDriver (the C
slab driver, pmc_slab_*).  Reference: the per-slab form of start.cu:237-260.
"""
from __future__ import annotations

import os
import sys
from typing import Callable, List, Optional, Tuple

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "parallel-monte-carlo_amd"))

from pmc_amd.plan import sweep_plan  # noqa: E402
from pmc_amd.slab import SlabGeometry  # noqa: E402


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
        from pmc_amd.engine import PmcContext
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
