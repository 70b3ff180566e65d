"""Host-side mirror of the reference call surface over the C ABI (include/pmc.h).

Reference entry points (qingye3/parallel-monte-carlo):
  init_r(float* r, int N_cube)                     start.cu:47   -> PmcContext.init_r
  assign(float* r, float* disk, short* n)          start.cu:87   -> PmcContext.assign
  subsweep_kernel(float* disk, short* n, int* off) subsweep.h:240 -> PmcContext.subsweep_kernel
  shiftCells(float* disk, short* n, int f, float d) shiftCells.h:28 -> PmcContext.shiftCells
  main (the `start` program)                       start.cu:169  -> PmcContext.start

Buffers passed to the reference-kernel methods are device pointers (ints) or torch CUDA tensors
in the reference layout; the driver methods act on the context-owned state.  With torch tensors
the launch is ordered after torch's current stream and torch's current stream after the launch
(stream waits, no host sync), so tensors can be produced and consumed with ordinary torch ops.
Every call goes to the HIP library -- there is no CPU path.
"""
from __future__ import annotations

import contextlib
import ctypes as C
from typing import Optional

import numpy as np

from ._lib import PMC_IPC_HANDLE_BYTES, Params, Result, Stats, check, lib

FIX_SCALE = 2.0 ** 32


def _ptr(x) -> int:
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        if not x.is_cuda:
            raise ValueError("device buffer expected (torch CUDA tensor or device pointer)")
        return int(x.data_ptr())
    raise TypeError(f"cannot take a device pointer of {type(x)!r}")


def colour_offset(colour: int):
    """itoa (start.cu:153-157): colour id -> (ox, oy, oz)."""
    return ((colour // 4) % 2, (colour // 2) % 2, colour % 2)


class PmcContext:
    """One simulation box (or z-slab of one) on the current HIP device."""

    def __init__(self, cps: int = 4, *, cps_y: int = 0, cps_z: int = 0, nz_local: int = 0, z0: int = 0,
                 halo: int = 0, nmax: int = 16, n_moves: int = 10, w: float = 2.5, beta: float = 0.3,
                 sigma: float = 0.5, seed: int = 1234, stream: Optional[int] = None, flags: int = 0):
        self.params = Params(cps, cps_y, cps_z, nz_local, z0, halo, nmax, n_moves, w, beta, sigma, flags, seed)
        h = C.c_void_p()
        check("pmc_create", lib().pmc_create(C.byref(self.params), C.byref(h)))
        self._h = h
        self.cps_x = cps
        self.cps_y = cps_y or cps
        self.cps_z = cps_z or cps
        self.nz_local = nz_local or self.cps_z
        self.z0 = z0
        self.halo = halo
        self.nmax = nmax
        self.n_moves = n_moves
        self.w = w
        self.flags = flags
        self.cells = int(lib().pmc_storage_cells(self._h))
        if stream is not None:
            self.set_stream(stream)

    # ---- lifecycle ----------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            lib().pmc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_stream(self, stream: int):
        check("pmc_set_stream", lib().pmc_set_stream(self._h, C.c_void_p(stream)))

    def stream(self) -> int:
        st = C.c_void_p()
        check("pmc_get_stream", lib().pmc_get_stream(self._h, C.byref(st)))
        return st.value or 0

    @contextlib.contextmanager
    def _torch_ordered(self, *bufs):
        """Order a launch on the context stream between torch's current-stream work that
        produced `bufs` and the torch work that consumes them (device-side stream waits)."""
        if not any(hasattr(b, "data_ptr") for b in bufs):
            yield
            return
        import torch
        ours = torch.cuda.ExternalStream(self.stream())
        theirs = torch.cuda.current_stream()
        if ours.cuda_stream == theirs.cuda_stream:
            yield
            return
        ours.wait_stream(theirs)
        yield
        theirs.wait_stream(ours)

    def attach_state(self, disk0, n0, disk1, n1):
        check("pmc_attach_state", lib().pmc_attach_state(self._h, _ptr(disk0), _ptr(n0), _ptr(disk1), _ptr(n1)))

    def state_layout(self) -> int:
        """Layout of the state buffers (pmc_state_layout): 0 the reference rows (slot s of dimension d
        at d*nmax + s), 1 packed (3*s + d).  Host copies and snapshots are always the reference layout."""
        v = C.c_int(0)
        check("pmc_state_layout", lib().pmc_state_layout(self._h, C.byref(v)))
        return v.value

    def state_ptrs(self):
        d, n = C.c_void_p(), C.c_void_p()
        check("pmc_state", lib().pmc_state(self._h, C.byref(d), C.byref(n)))
        return d.value, n.value

    # ---- reference kernels -------------------------------------------------------------
    def init_r(self, n_atoms: int, r) -> None:
        with self._torch_ordered(r):
            check("pmc_init_r", lib().pmc_init_r(self._h, n_atoms, _ptr(r)))

    def assign(self, r, n_atoms: int, disk, n) -> None:
        with self._torch_ordered(r, disk, n):
            check("pmc_assign", lib().pmc_assign(self._h, _ptr(r), n_atoms, _ptr(disk), _ptr(n)))

    def subsweep_kernel(self, disk, n, offset, sweep: int) -> None:
        off = (C.c_int * 3)(*[int(v) for v in offset])
        with self._torch_ordered(disk, n):
            check("pmc_subsweep", lib().pmc_subsweep(self._h, _ptr(disk), _ptr(n), C.byref(off), sweep))

    def shiftCells(self, disk_in, n_in, disk_out, n_out, f: int, d: float) -> None:  # noqa: N802
        with self._torch_ordered(disk_in, n_in, disk_out, n_out):
            check("pmc_shift_cells", lib().pmc_shift_cells(self._h, _ptr(disk_in), _ptr(n_in), _ptr(disk_out),
                                                           _ptr(n_out), f, d))

    # ---- driver ------------------------------------------------------------------------
    def init_lattice(self, n_atoms: int) -> None:
        check("pmc_init_lattice", lib().pmc_init_lattice(self._h, n_atoms))

    def init_lattice_global(self, n_atoms_total: int) -> None:
        """Strong-scaling start: the whole box's lattice, this slab's planes (pmc_init_lattice_global)."""
        check("pmc_init_lattice_global", lib().pmc_init_lattice_global(self._h, n_atoms_total))

    def init_lattice_planes(self, n_atoms_lattice: int, lattice_cps_z: int) -> None:
        """The lattice of a taller box (cps x cps x lattice_cps_z cells), bottom-aligned; this slab's
        planes of it (pmc_init_lattice_planes; the config-5 weak-scaling start)."""
        check("pmc_init_lattice_planes", lib().pmc_init_lattice_planes(self._h, n_atoms_lattice, lattice_cps_z))

    def sweep(self, s: int) -> None:
        check("pmc_sweep", lib().pmc_sweep(self._h, s))

    def phase(self, colour: int, s: int) -> None:
        check("pmc_phase", lib().pmc_phase(self._h, colour, s))

    def phase_range(self, colour: int, s: int, zl_begin: int, zl_end: int) -> None:
        check("pmc_phase_range", lib().pmc_phase_range(self._h, colour, s, zl_begin, zl_end))

    def phase_range_on(self, colour: int, s: int, zl_begin: int, zl_end: int, stream: int) -> None:
        """phase_range on another HIP stream (own overflow queue): concurrent with the context
        stream's launches of the same colour on other planes; the caller orders the streams."""
        check("pmc_phase_range_on", lib().pmc_phase_range_on(self._h, colour, s, zl_begin, zl_end,
                                                             C.c_void_p(stream)))

    # ---- multi-GPU slab driver (pmc_slab_*: schedule + RCCL in C) ---------------------------
    def slab_init(self, rank: int, world: int, unique_id: Optional[bytes]) -> None:
        uid = None if unique_id is None else (C.c_ubyte * 128).from_buffer_copy(unique_id)
        check("pmc_slab_init", lib().pmc_slab_init(self._h, rank, world, uid))

    def slab_init_local(self, rank: int, group: "LocalGroup") -> None:
        """pmc_slab_init with the in-process transport (W slabs of one process, a thread per rank)."""
        check("pmc_slab_init_local", lib().pmc_slab_init_local(self._h, rank, group.handle))

    def slab_ipc_handle(self) -> bytes:
        """This rank's IPC blob (pmc_slab_ipc_handle): its symmetric buffers and flags, to gather
        in rank order and hand to every rank's slab_init_ipc."""
        buf = (C.c_ubyte * PMC_IPC_HANDLE_BYTES)()
        check("pmc_slab_ipc_handle", lib().pmc_slab_ipc_handle(self._h, buf))
        return bytes(buf)

    def slab_init_ipc(self, rank: int, world: int, blobs: list) -> None:
        """pmc_slab_init with the IPC transport (one process per rank; blobs[r] = rank r's handle)."""
        if len(blobs) != world or any(len(b) != PMC_IPC_HANDLE_BYTES for b in blobs):
            raise ValueError("slab_init_ipc: one PMC_IPC_HANDLE_BYTES blob per rank expected")
        raw = (C.c_ubyte * (PMC_IPC_HANDLE_BYTES * world)).from_buffer_copy(b"".join(blobs))
        check("pmc_slab_init_ipc", lib().pmc_slab_init_ipc(self._h, rank, world, raw))

    def slab_exchange(self) -> None:
        check("pmc_slab_exchange", lib().pmc_slab_exchange(self._h))

    def slab_sweep(self, s: int) -> None:
        check("pmc_slab_sweep", lib().pmc_slab_sweep(self._h, s))

    def slab_layout(self) -> list:
        """The interior chains of pmc_slab_sweep as (first plane, end plane) pairs."""
        n = C.c_int(0)
        b = (C.c_int * 4)()
        check("pmc_slab_layout", lib().pmc_slab_layout(self._h, C.byref(n), b))
        return [(b[j], b[j + 1]) for j in range(n.value)]

    def slab_finish(self) -> None:
        check("pmc_slab_finish", lib().pmc_slab_finish(self._h))

    def slab_observables(self, with_energy: bool = True) -> tuple:
        """Whole-box counters (and energy) summed over the ranks in fixed point, collectively
        (pmc_slab_observables): (stats dict, energy or None)."""
        st = Stats()
        e = C.c_double(0.0)
        check("pmc_slab_observables", lib().pmc_slab_observables(self._h, 1 if with_energy else 0, C.byref(st),
                                                                 C.byref(e)))
        d = {"de_fixed": st.de_fixed, "accepted": st.accepted, "trials": st.trials, "evaluated": st.evaluated}
        return d, (e.value if with_energy else None)

    def _timing(self, fn: str, enable: bool) -> dict:
        a, b = C.c_double(), C.c_double()
        na, nb = C.c_int(), C.c_int()
        check(fn, getattr(lib(), fn)(self._h, int(enable), C.byref(a), C.byref(na), C.byref(b), C.byref(nb)))
        return {"subsweep_ms": a.value, "n_subsweep": na.value, "shift_ms": b.value, "n_shift": nb.value}

    def timing(self, enable: bool) -> dict:
        """Summed kernel durations (dispatch-packet HIP events) of the subsweep / shift launches
        since the last call; then per-launch timing on or off (pmc_timing)."""
        return self._timing("pmc_timing", enable)

    def timing_kinds(self, enable: bool) -> dict:
        """Per-kind kernel durations (pmc_timing_kinds): context-stream subsweep launches, shift
        launches, other-stream (slab boundary) subsweep launches."""
        ms, cnt = (C.c_double * 3)(), (C.c_int * 3)()
        check("pmc_timing_kinds", lib().pmc_timing_kinds(self._h, int(enable), C.byref(ms), C.byref(cnt)))
        return {"subsweep_ms": ms[0], "n_subsweep": cnt[0], "shift_ms": ms[1], "n_shift": cnt[1],
                "boundary_ms": ms[2], "n_boundary": cnt[2]}

    def phase_spans(self) -> tuple:
        """(summed span ms, phases) of the colour phases pmc_sweep split over plane chains, from the last
        timing()/timing_kinds() call (pmc_timing_phase_spans)."""
        ms, n = C.c_double(0.0), C.c_int(0)
        check("pmc_timing_phase_spans", lib().pmc_timing_phase_spans(self._h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def sweep_layout(self) -> list:
        """pmc_sweep's plane chains as (first plane, end plane) pairs (pmc_sweep_layout)."""
        n = C.c_int(0)
        b = (C.c_int * 5)()   # PMC_SWEEP_MAX_CHAINS + 1
        check("pmc_sweep_layout", lib().pmc_sweep_layout(self._h, C.byref(n), C.byref(b)))
        return [(b[j], b[j + 1]) for j in range(n.value)]

    def timing_pause(self, paused: bool) -> None:
        """Per-launch events off (paused) or back on without collecting them (pmc_timing_pause)."""
        check("pmc_timing_pause", lib().pmc_timing_pause(self._h, int(paused)))

    def slab_timing(self, enable: bool) -> dict:
        return self._timing("pmc_slab_timing", enable)

    def shift(self, s: int) -> None:
        check("pmc_shift", lib().pmc_shift(self._h, s))

    def shift_slab(self, s: int) -> int:
        """Slab shiftCells incl. the locally computable halo planes (pmc_shift_slab); returns the
        halo still to receive: 0 none, +1 top (from above's plane 0), -1 bottom (below's top plane)."""
        h = C.c_int(0)
        check("pmc_shift_slab", lib().pmc_shift_slab(self._h, s, C.byref(h)))
        return h.value

    def start(self, first: int, passes: int) -> dict:
        r = Result()
        check("pmc_start", lib().pmc_start(self._h, first, passes, C.byref(r)))
        out = r.stats.as_dict()
        out.update(e_initial=r.e_initial, e_final=r.e_final, seconds=r.seconds, sweeps=int(r.sweeps))
        return out

    def run_small(self, first: int, count: int) -> None:
        """pmc_run_small: whole sweeps of a small box in one launch on one XCD."""
        check("pmc_run_small", lib().pmc_run_small(self._h, first, count))

    def run_graph(self, first: int, count: int) -> None:
        check("pmc_run_graph", lib().pmc_run_graph(self._h, first, count))

    # ---- observables / mirrors ---------------------------------------------------------
    def energy(self) -> float:
        e = C.c_double()
        check("pmc_energy", lib().pmc_energy(self._h, C.byref(e)))
        return e.value

    def stats(self, reset: bool = False) -> dict:
        s = Stats()
        check("pmc_stats_read", lib().pmc_stats_read(self._h, C.byref(s), int(reset)))
        return s.as_dict()

    def error_flags(self, reset: bool = False) -> int:
        f = C.c_uint32()
        check("pmc_error_flags", lib().pmc_error_flags(self._h, C.byref(f), int(reset)))
        return f.value

    def synchronize(self) -> None:
        check("pmc_synchronize", lib().pmc_synchronize(self._h))

    def copy_out(self):
        disk = np.empty(self.cells * 3 * self.nmax, np.float32)
        n = np.empty(self.cells, np.int16)
        check("pmc_copy_out", lib().pmc_copy_out(self._h, disk.ctypes.data, n.ctypes.data))
        return disk, n

    def copy_in(self, disk: np.ndarray, n: np.ndarray) -> None:
        disk = np.ascontiguousarray(disk, np.float32)
        n = np.ascontiguousarray(n, np.int16)
        assert disk.size == self.cells * 3 * self.nmax and n.size == self.cells
        check("pmc_copy_in", lib().pmc_copy_in(self._h, disk.ctypes.data, n.ctypes.data))

    # ---- trajectory dump / restart (kernel.cu:497-536; pmc_amd.io for the host formats) ----
    def get_params(self) -> Params:
        p = Params()
        check("pmc_get_params", lib().pmc_get_params(self._h, C.byref(p)))
        return p

    def set_stats(self, stats: dict) -> None:
        s = Stats(**{k: int(v) for k, v in stats.items()})
        check("pmc_stats_write", lib().pmc_stats_write(self._h, C.byref(s)))

    def dump_frame(self, path: str, timestep: int, append: bool = True) -> None:
        """Append (or write) the current state as one create_dump frame (kernel.cu:510-536)."""
        check("pmc_dump_frame", lib().pmc_dump_frame(self._h, str(path).encode(), int(append), timestep))

    def save_snapshot(self, path: str, next_sweep: int) -> None:
        """Binary snapshot: parameters, next sweep index (the RNG state), stats, exact coordinates."""
        check("pmc_save_snapshot", lib().pmc_save_snapshot(self._h, str(path).encode(), next_sweep))

    def load_snapshot(self, path: str) -> int:
        """Restore a snapshot written by save_snapshot; returns the sweep index to continue from."""
        sw = C.c_uint32()
        check("pmc_load_snapshot", lib().pmc_load_snapshot(self._h, str(path).encode(), C.byref(sw)))
        return sw.value

    def plane_span(self, z_local: int):
        a, b, c, d = C.c_size_t(), C.c_size_t(), C.c_size_t(), C.c_size_t()
        check("pmc_plane_span", lib().pmc_plane_span(self._h, z_local, C.byref(a), C.byref(b), C.byref(c),
                                                     C.byref(d)))
        return a.value, b.value, c.value, d.value


class LocalGroup:
    """pmc_local_group: the in-process halo transport shared by `world` slab contexts of this
    process.  Close (or drop) the contexts before the group."""

    def __init__(self, world: int):
        h = C.c_void_p()
        check("pmc_local_group_create", lib().pmc_local_group_create(world, C.byref(h)))
        self.handle = h
        self.world = world

    def close(self):
        if getattr(self, "handle", None):
            lib().pmc_local_group_destroy(self.handle)
            self.handle = None


def device_count() -> int:
    """HIP devices visible to this process (pmc_device_count); PmcError PMC_ERR_NODEV if none."""
    n = C.c_int(0)
    check("pmc_device_count", lib().pmc_device_count(C.byref(n)))
    return n.value


def comm_unique_id() -> bytes:
    """A fresh RCCL unique id (rank 0 of a slab run broadcasts it)."""
    buf = (C.c_ubyte * 128)()
    check("pmc_comm_unique_id", lib().pmc_comm_unique_id(buf))
    return bytes(buf)


def selftest_detmath(words: np.ndarray):
    """Device evaluation of pmc_detmath.h on Philox word quadruples (diagnostic)."""
    words = np.ascontiguousarray(words, np.uint32).reshape(-1, 4)
    cnt = words.shape[0]
    out_f = np.empty(4 * cnt, np.float32)
    out_d = np.empty(2 * cnt, np.float64)
    check("pmc_selftest_detmath", lib().pmc_selftest_detmath(words.ctypes.data, cnt, out_f.ctypes.data,
                                                             out_d.ctypes.data))
    return out_f.reshape(cnt, 4), out_d.reshape(cnt, 2)


def hbm_probe(nbytes: int = 1 << 30, reps: int = 10) -> tuple:
    """(read GB/s, copy GB/s): the library's streaming read and copy kernels over `nbytes`, best of
    `reps` (pmc_hbm_probe; SURVEY.md Appendix D's achievable peak beside the 8 TB/s spec)."""
    r = C.c_double()
    cp = C.c_double()
    check("pmc_hbm_probe", lib().pmc_hbm_probe(nbytes, reps, C.byref(r), C.byref(cp)))
    return r.value, cp.value
