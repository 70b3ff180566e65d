"""Trajectory dump / restart formats (host side, no GPU needed) over the C ABI (include/pmc.h).

Reference: disk_to_r + create_dump (CUDA-Parallel-MC/CUDA-Parallel-MC/kernel.cu:497-536), the
LAMMPS-style text frames the reference writes for OVITO (its data file dumpR3.txt is one).  The
reference has no reader and no checkpoint: read_dump and the PMCSNAP1 binary snapshot are the
restart path of this build.  Device contexts dump / save / load through PmcContext.dump_frame,
save_snapshot and load_snapshot.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import Params, Stats, check, lib


def disk_to_r(disk: np.ndarray, n: np.ndarray, nmax: int) -> np.ndarray:
    """Positions (3, N) in cell order, then slot order (disk_to_r, kernel.cu:500-510)."""
    disk = np.ascontiguousarray(disk, np.float32)
    n = np.ascontiguousarray(n, np.int16)
    cnt = C.c_int64()
    check("pmc_disk_to_r", lib().pmc_disk_to_r(disk.ctypes.data, n.ctypes.data, n.size, nmax, None, 0, C.byref(cnt)))
    r = np.empty((3, cnt.value), np.float32)
    check("pmc_disk_to_r", lib().pmc_disk_to_r(disk.ctypes.data, n.ctypes.data, n.size, nmax, r.ctypes.data,
                                               cnt.value, C.byref(cnt)))
    return r


def write_dump(path: str, timestep: int, r: np.ndarray, box_lo, box_hi, append: bool = True) -> None:
    """One create_dump frame (kernel.cu:521-535) of positions r (3, N)."""
    r = np.ascontiguousarray(r, np.float32).reshape(3, -1)
    lo = (C.c_float * 3)(*[float(v) for v in box_lo])
    hi = (C.c_float * 3)(*[float(v) for v in box_hi])
    check("pmc_write_dump", lib().pmc_write_dump(str(path).encode(), int(append), timestep, r.ctypes.data,
                                                 r.shape[1], r.shape[1], C.byref(lo), C.byref(hi)))


def read_dump(path: str, frame: int = 0):
    """Frame `frame` (0-based) of a dump file -> (timestep, r (3, N) float32, box_lo, box_hi)."""
    ts, na = C.c_int64(), C.c_int64()
    lo, hi = (C.c_float * 3)(), (C.c_float * 3)()
    check("pmc_read_dump", lib().pmc_read_dump(str(path).encode(), frame, C.byref(ts), None, 0, C.byref(na),
                                               C.byref(lo), C.byref(hi)))
    r = np.empty((3, na.value), np.float32)
    check("pmc_read_dump", lib().pmc_read_dump(str(path).encode(), frame, C.byref(ts), r.ctypes.data, na.value,
                                               C.byref(na), C.byref(lo), C.byref(hi)))
    return ts.value, r, tuple(lo), tuple(hi)


def write_snapshot(path: str, params: Params, next_sweep: int, stats: dict, disk: np.ndarray, n: np.ndarray) -> None:
    """PMCSNAP1 snapshot of host arrays (`n.size` cells in the reference layout)."""
    if not isinstance(params, Params):          # any ctypes pmc_params mirror (same layout)
        params = Params.from_buffer_copy(params)
    disk = np.ascontiguousarray(disk, np.float32)
    n = np.ascontiguousarray(n, np.int16)
    st = Stats(**{k: int(stats.get(k, 0)) for k, _ in Stats._fields_})
    check("pmc_snapshot_write", lib().pmc_snapshot_write(str(path).encode(), C.byref(params), next_sweep,
                                                         C.byref(st), disk.ctypes.data, n.ctypes.data, n.size))


def read_snapshot(path: str, cells: int | None = None):
    """-> (params, next_sweep, stats dict, disk, n); header only when cells == 0."""
    p, sw, st = Params(), C.c_uint32(), Stats()
    check("pmc_snapshot_read", lib().pmc_snapshot_read(str(path).encode(), C.byref(p), C.byref(sw), C.byref(st),
                                                       None, None, 0))
    if cells == 0:
        return p, sw.value, st.as_dict(), None, None
    if cells is None:
        raise ValueError("cells: the number of cells stored (owned cells of the writer)")
    disk = np.empty(cells * 3 * p.nmax, np.float32)
    n = np.empty(cells, np.int16)
    q = Params()
    q.nmax = p.nmax          # the buffers' nmax (the reader refuses any other)
    check("pmc_snapshot_read", lib().pmc_snapshot_read(str(path).encode(), C.byref(q), None, None, disk.ctypes.data,
                                                       n.ctypes.data, cells))
    return p, sw.value, st.as_dict(), disk, n
