"""ctypes wrapper of the CPU oracle (oracle/build/liborc.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the product package.  Array layouts are the reference's:
``disk`` float32[cells*3*nmax] (cell c: x[nmax], y[nmax], z[nmax]) and ``n`` int16[cells]
(start.cu:186-188).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liborc.so")


class Params(C.Structure):
    """Mirror of ``pmc_params`` (include/pmc.h)."""

    _fields_ = [
        ("cps_x", C.c_int32), ("cps_y", C.c_int32), ("cps_z", C.c_int32),
        ("nz_local", C.c_int32), ("z0", C.c_int32), ("halo", C.c_int32),
        ("nmax", C.c_int32), ("n_moves", C.c_int32),
        ("w", C.c_float), ("beta", C.c_float), ("sigma", C.c_float),
        ("flags", C.c_uint32), ("seed", C.c_uint64),
    ]


class Stats(C.Structure):
    _fields_ = [("de_fixed", C.c_int64), ("accepted", C.c_int64),
                ("trials", C.c_int64), ("evaluated", C.c_int64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


def make_params(cps=4, cps_y=0, cps_z=0, nz_local=0, z0=0, halo=0, nmax=16, n_moves=10,
                w=2.5, beta=0.3, sigma=0.5, seed=1234, flags=0) -> Params:
    p = Params(cps, cps_y, cps_z, nz_local, z0, halo, nmax, n_moves, w, beta, sigma, flags, seed)
    return p


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", HERE], check=True, capture_output=True)
    return LIB_PATH


def use_native() -> str:
    """Switch this process to the -march=native build of the same source (bench.py's timed CPU
    baseline), compiled on the host that runs it (make native: a few seconds).  Must precede the
    first lib() call.  Returns the flags used; raises if gcc fails (the caller keeps the portable
    build then)."""
    global LIB_PATH
    if _lib is not None:
        raise RuntimeError("the oracle library is already loaded")
    path = os.path.join(HERE, "build", "liborc_native.so")
    # rebuilt every time: a native build from another host must not be reused
    subprocess.run(["make", "-C", HERE, "-B", "native"], check=True, capture_output=True)
    LIB_PATH = path
    return "-O3 -march=native -ffp-contract=off -fopenmp"


_lib = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_i16p = np.ctypeslib.ndpointer(np.int16, flags="C_CONTIGUOUS")


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER(Params)
        L.orc_params_check.argtypes = [P]
        L.orc_storage_cells.argtypes = [P]
        L.orc_storage_cells.restype = C.c_int64
        L.orc_cutoff_r2.argtypes = [C.c_float]
        L.orc_cutoff_r2.restype = C.c_float
        L.orc_set_threads.argtypes = [C.c_int]
        L.orc_init_r.argtypes = [P, C.c_int64, _f32p]
        L.orc_assign.argtypes = [P, _f32p, C.c_int64, _f32p, _i16p]
        L.orc_subsweep.argtypes = [P, _f32p, _i16p, C.c_int, C.c_int, C.c_int, C.c_uint32,
                                   C.POINTER(Stats)]
        L.orc_subsweep.restype = None
        L.orc_subsweep_range.argtypes = [P, _f32p, _i16p, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_int,
                                         C.c_int, C.POINTER(Stats)]
        L.orc_subsweep_range.restype = None
        L.orc_shift_cells.argtypes = [P, _f32p, _i16p, _f32p, _i16p, C.c_int, C.c_float]
        L.orc_shift_cells_planes.argtypes = [P, _f32p, _i16p, _f32p, _i16p, C.c_int, C.c_float, C.c_int, C.c_int]
        L.orc_energy.argtypes = [P, _f32p, _i16p]
        L.orc_energy.restype = C.c_double
        L.orc_run.argtypes = [P, _f32p, _i16p, _f32p, _i16p, C.c_uint32, C.c_int, C.POINTER(Stats)]
        L.orc_run_trace.argtypes = [P, _f32p, _i16p, _f32p, _i16p, C.c_uint32, C.c_int, C.c_int,
                                    np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS"), C.POINTER(Stats)]
        L.orc_philox.argtypes = [C.POINTER(C.c_uint32 * 4), C.POINTER(C.c_uint32 * 2),
                                 C.POINTER(C.c_uint32 * 4)]
        L.orc_philox.restype = None
        L.orc_logf.argtypes = [C.c_float]
        L.orc_logf.restype = C.c_float
        L.orc_recip.argtypes = [C.c_float]
        L.orc_recip.restype = C.c_float
        L.orc_det_sincos_2pi.argtypes = [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.orc_det_sincos_2pi.restype = None
        L.orc_move_normals.argtypes = [C.POINTER(C.c_uint32 * 4), C.POINTER(C.c_float * 3)]
        L.orc_move_normals.restype = None
        L.orc_pair_energy.argtypes = [C.c_float] * 4
        L.orc_pair_energy.restype = C.c_float
        L.orc_sweep_plan.argtypes = [C.c_uint64, C.c_uint32, C.c_float, C.POINTER(C.c_int * 8),
                                     C.POINTER(C.c_int), C.POINTER(C.c_float)]
        L.orc_sweep_plan.restype = None
        L.orc_sweep_plan_ex.argtypes = [C.c_uint64, C.c_uint32, C.c_float, C.c_uint32, C.POINTER(C.c_int * 8),
                                        C.POINTER(C.c_int), C.POINTER(C.c_float)]
        L.orc_sweep_plan_ex.restype = None
        L.orc_to_fixed.argtypes = [C.c_double]
        L.orc_to_fixed.restype = C.c_int64
        L.orc_to_fixed_f32.argtypes = [C.c_float]
        L.orc_to_fixed_f32.restype = C.c_int64
        _lib = L
    return _lib


def set_threads(n: int) -> int:
    return lib().orc_set_threads(n)


class OracleState:
    """A box (or slab) held in host arrays, driven by the oracle."""

    def __init__(self, params: Params):
        self.p = Params.from_buffer_copy(params)
        rc = lib().orc_params_check(C.byref(self.p))
        if rc != 0:
            raise ValueError(f"invalid params (rc={rc})")
        self.cells = int(lib().orc_storage_cells(C.byref(self.p)))
        self.nmax = self.p.nmax
        self.disk = np.zeros(self.cells * 3 * self.nmax, np.float32)
        self.n = np.zeros(self.cells, np.int16)
        self.stats = Stats()

    # --- reference kernels -------------------------------------------------------------
    def init_r(self, n_atoms: int) -> np.ndarray:
        r = np.zeros(3 * n_atoms, np.float32)
        lib().orc_init_r(C.byref(self.p), n_atoms, r)
        return r

    def assign(self, r: np.ndarray) -> int:
        r = np.ascontiguousarray(r, np.float32)
        return lib().orc_assign(C.byref(self.p), r, r.size // 3, self.disk, self.n)

    def init_lattice(self, n_atoms: int) -> int:
        return self.assign(self.init_r(n_atoms))

    def subsweep(self, offset, sweep: int):
        lib().orc_subsweep(C.byref(self.p), self.disk, self.n, int(offset[0]), int(offset[1]),
                           int(offset[2]), sweep, C.byref(self.stats))

    def shift_cells(self, f: int, d: float) -> int:
        dout = self.disk.copy()
        nout = self.n.copy()
        over = lib().orc_shift_cells(C.byref(self.p), self.disk, self.n, dout, nout, f, d)
        self.disk, self.n = dout, nout
        return over

    def energy(self) -> float:
        return lib().orc_energy(C.byref(self.p), self.disk, self.n)

    def run(self, first: int, nsweeps: int) -> int:
        sd = self.disk.copy()
        sn = self.n.copy()
        return lib().orc_run(C.byref(self.p), self.disk, self.n, sd, sn, first, nsweeps,
                             C.byref(self.stats))

    def run_trace(self, first: int, nsweeps: int, every: int) -> np.ndarray:
        """run(first, nsweeps) recording the energy after every `every`-th sweep (one C call)."""
        sd = self.disk.copy()
        sn = self.n.copy()
        tr = np.zeros(nsweeps // every, np.float64)
        rc = lib().orc_run_trace(C.byref(self.p), self.disk, self.n, sd, sn, first, nsweeps, every, tr,
                                 C.byref(self.stats))
        if rc:
            raise RuntimeError(f"orc_run_trace: rc={rc}")
        return tr

    # --- views --------------------------------------------------------------------------
    def disk3(self) -> np.ndarray:
        return self.disk.reshape(self.cells, 3, self.nmax)

    def positions(self) -> np.ndarray:
        """(N,3) array of the owned cells' particles in storage order."""
        return positions_from(self.disk, self.n, self.nmax, self.owned_slice())

    def owned_slice(self) -> slice:
        plane = self.p.cps_x * self.p.cps_y
        lo = plane * self.p.halo
        return slice(lo, lo + plane * self.p.nz_local)


def positions_from(disk: np.ndarray, n: np.ndarray, nmax: int, sl: slice | None = None) -> np.ndarray:
    d3 = disk.reshape(-1, 3, nmax)
    nn = n.astype(np.int64)
    if sl is not None:
        d3 = d3[sl]
        nn = nn[sl]
    mask = np.arange(nmax)[None, :] < nn[:, None]
    return np.stack([d3[:, k, :][mask] for k in range(3)], axis=1)


def valid_slots_equal(disk_a, n_a, disk_b, n_b, nmax, sl=None) -> bool:
    """Bitwise equality of n and of every occupied slot (padding slots are don't-care)."""
    if sl is None:
        sl = slice(None)
    if not np.array_equal(n_a[sl], n_b[sl]):
        return False
    a = disk_a.reshape(-1, 3, nmax)[sl]
    b = disk_b.reshape(-1, 3, nmax)[sl]
    mask = (np.arange(nmax)[None, :] < n_a[sl].astype(np.int64)[:, None])
    mask3 = np.broadcast_to(mask[:, None, :], a.shape)
    return np.array_equal(a.view(np.uint32)[mask3], b.view(np.uint32)[mask3])


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().orc_philox(C.byref(c), C.byref(k), C.byref(o))
    return list(o)


def logf(x: float) -> float:
    return lib().orc_logf(x)


def recip(x: float) -> float:
    return lib().orc_recip(x)


def det_sincos_2pi(u: float):
    s, c = C.c_float(), C.c_float()
    lib().orc_det_sincos_2pi(u, C.byref(s), C.byref(c))
    return s.value, c.value


def sweep_plan(seed: int, sweep: int, w: float = 2.5, flags: int = 0):
    order = (C.c_int * 8)()
    f = C.c_int()
    d = C.c_float()
    lib().orc_sweep_plan_ex(seed, sweep, w, flags, C.byref(order), C.byref(f), C.byref(d))
    return list(order), f.value, d.value


def pair_energy(dx, dy, dz, rc2=None):
    if rc2 is None:
        rc2 = lib().orc_cutoff_r2(2.5)
    return lib().orc_pair_energy(dx, dy, dz, rc2)


def cutoff_r2(w: float = 2.5) -> float:
    return lib().orc_cutoff_r2(w)


def colour_offset(colour: int):
    return ((colour // 4) % 2, (colour // 2) % 2, colour % 2)
