"""ctypes binding of build/libpmc.so (the C ABI in include/pmc.h).

The product path has no CPU fallback: if the HIP library is missing or cannot be loaded,
``lib()`` raises.  ``build()`` compiles it with hipcc for gfx950 (works without a GPU).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # parallel-monte-carlo_amd/
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.environ.get("PMC_LIB_PATH") or os.path.join(PKG_DIR, "build", "libpmc.so")
START_PATH = os.path.join(PKG_DIR, "build", "start")
HEADER = os.path.join(REPO_DIR, "include", "pmc.h")


class Params(C.Structure):
    """``pmc_params`` (include/pmc.h)."""

    _fields_ = [
        ("cps_x", C.c_int32), ("cps_y", C.c_int32), ("cps_z", C.c_int32),
        ("nz_local", C.c_int32), ("z0", C.c_int32), ("halo", C.c_int32),
        ("nmax", C.c_int32), ("n_moves", C.c_int32),
        ("w", C.c_float), ("beta", C.c_float), ("sigma", C.c_float),
        ("flags", C.c_uint32), ("seed", C.c_uint64),
    ]


class Stats(C.Structure):
    """``pmc_stats``."""

    _fields_ = [("de_fixed", C.c_int64), ("accepted", C.c_int64),
                ("trials", C.c_int64), ("evaluated", C.c_int64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class Result(C.Structure):
    """``pmc_result``."""

    _fields_ = [("stats", Stats), ("e_initial", C.c_double), ("e_final", C.c_double),
                ("seconds", C.c_double), ("sweeps", C.c_int64)]


PMC_FLAG_FULL_SHUFFLE = 1
PMC_FLAG_QUIRK_R1, PMC_FLAG_QUIRK_R2, PMC_FLAG_QUIRK_S1 = 2, 4, 8     # reference quirks (include/pmc.h)
PMC_OK, PMC_ERR_ARG, PMC_ERR_HIP, PMC_ERR_OVERFLOW, PMC_ERR_RANGE, PMC_ERR_NODEV = 0, -1, -2, -3, -4, -5
PMC_IPC_HANDLE_BYTES = 1024     # include/pmc.h
PMC_LAYOUT_REFERENCE, PMC_LAYOUT_PACKED = 0, 1


class PmcError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} -> {code}: {msg}")
        self.code = code


def build(force: bool = False) -> str:
    """Compile the HIP library for gfx950 (hipcc cross-compiles without a GPU)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", PKG_DIR, "-j4"], check=True, capture_output=True)
    return LIB_PATH


_lib = None
_vp = C.c_void_p


def _sig(L, name, res, *args):
    if os.environ.get("PMC_LIB_PATH") and not hasattr(L, name):
        return   # analysis builds of older revisions (tools/ab_variants.sh) may lack newer symbols
    f = getattr(L, name)
    f.restype = res
    f.argtypes = list(args)


def lib():
    """Load libpmc.so; raises if it is absent (no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP extension missing: {LIB_PATH} (run __graft_entry__.build())")
        # PyTorch-ROCm bundles its own libamdhip64 (SONAME libamdhip64.so.7).  Loading torch first
        # makes libpmc.so bind to that same runtime, so one process has ONE HIP runtime and torch
        # streams/tensors can be handed to the C ABI.  (Loading libpmc first would pull in
        # /opt/rocm's copy next to torch's and the second runtime finds no GPU.)
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        P = C.POINTER(Params)
        i64, i32, u32 = C.c_int64, C.c_int, C.c_uint32
        _sig(L, "pmc_last_error", C.c_char_p)
        _sig(L, "pmc_create", i32, P, C.POINTER(_vp))
        _sig(L, "pmc_destroy", None, _vp)
        _sig(L, "pmc_set_stream", i32, _vp, _vp)
        _sig(L, "pmc_get_stream", i32, _vp, C.POINTER(_vp))
        _sig(L, "pmc_attach_state", i32, _vp, _vp, _vp, _vp, _vp)
        _sig(L, "pmc_state", i32, _vp, C.POINTER(_vp), C.POINTER(_vp))
        _sig(L, "pmc_storage_cells", i64, _vp)
        _sig(L, "pmc_state_layout", i32, _vp, C.POINTER(C.c_int))
        _sig(L, "pmc_init_r", i32, _vp, i64, _vp)
        _sig(L, "pmc_assign", i32, _vp, _vp, i64, _vp, _vp)
        _sig(L, "pmc_subsweep", i32, _vp, _vp, _vp, C.POINTER(C.c_int * 3), u32)
        _sig(L, "pmc_shift_cells", i32, _vp, _vp, _vp, _vp, _vp, i32, C.c_float)
        _sig(L, "pmc_init_lattice", i32, _vp, i64)
        _sig(L, "pmc_init_lattice_global", i32, _vp, i64)
        _sig(L, "pmc_init_lattice_planes", i32, _vp, i64, i32)
        _sig(L, "pmc_sweep", i32, _vp, u32)
        _sig(L, "pmc_phase", i32, _vp, i32, u32)
        _sig(L, "pmc_phase_range", i32, _vp, i32, u32, i32, i32)
        _sig(L, "pmc_phase_range_on", i32, _vp, i32, u32, i32, i32, _vp)
        _sig(L, "pmc_comm_unique_id", i32, _vp)
        _sig(L, "pmc_slab_init", i32, _vp, i32, i32, _vp)
        _sig(L, "pmc_local_group_create", i32, i32, C.POINTER(_vp))
        _sig(L, "pmc_local_group_destroy", None, _vp)
        _sig(L, "pmc_slab_init_local", i32, _vp, i32, _vp)
        _sig(L, "pmc_slab_ipc_handle", i32, _vp, _vp)
        _sig(L, "pmc_slab_init_ipc", i32, _vp, i32, i32, _vp)
        _sig(L, "pmc_device_count", i32, C.POINTER(C.c_int))
        _sig(L, "pmc_slab_exchange", i32, _vp)
        _sig(L, "pmc_slab_sweep", i32, _vp, u32)
        _sig(L, "pmc_slab_finish", i32, _vp)
        _sig(L, "pmc_slab_layout", i32, _vp, _vp, _vp)
        _sig(L, "pmc_slab_observables", i32, _vp, i32, C.POINTER(Stats), C.POINTER(C.c_double))
        _sig(L, "pmc_slab_timing", i32, _vp, i32, _vp, _vp, _vp, _vp)
        _sig(L, "pmc_timing", i32, _vp, i32, _vp, _vp, _vp, _vp)
        _sig(L, "pmc_timing_kinds", i32, _vp, i32, C.POINTER(C.c_double * 3), C.POINTER(C.c_int * 3))
        _sig(L, "pmc_timing_pause", i32, _vp, i32)
        _sig(L, "pmc_timing_phase_spans", i32, _vp, C.POINTER(C.c_double), C.POINTER(C.c_int))
        _sig(L, "pmc_sweep_layout", i32, _vp, C.POINTER(C.c_int), C.POINTER(C.c_int * 5))
        _sig(L, "pmc_subsweep_range", i32, _vp, _vp, _vp, C.POINTER(C.c_int * 3), u32, i32, i32)
        _sig(L, "pmc_shift", i32, _vp, u32)
        _sig(L, "pmc_shift_slab", i32, _vp, u32, _vp)
        _sig(L, "pmc_start", i32, _vp, u32, i32, C.POINTER(Result))
        _sig(L, "pmc_start_ex", i32, _vp, u32, i32, i32, C.POINTER(Result))
        _sig(L, "pmc_run_graph", i32, _vp, u32, i32)
        _sig(L, "pmc_run_small", i32, _vp, u32, i32)
        _sig(L, "pmc_sweep_plan", i32, C.c_uint64, u32, C.c_float, C.POINTER(C.c_int * 8), C.POINTER(C.c_int),
             C.POINTER(C.c_float))
        _sig(L, "pmc_sweep_plan_ex", i32, C.c_uint64, u32, C.c_float, u32, C.POINTER(C.c_int * 8),
             C.POINTER(C.c_int), C.POINTER(C.c_float))
        _sig(L, "pmc_energy", i32, _vp, C.POINTER(C.c_double))
        _sig(L, "pmc_stats_read", i32, _vp, C.POINTER(Stats), i32)
        _sig(L, "pmc_error_flags", i32, _vp, C.POINTER(C.c_uint32), i32)
        _sig(L, "pmc_copy_out", i32, _vp, _vp, _vp)
        _sig(L, "pmc_copy_in", i32, _vp, _vp, _vp)
        _sig(L, "pmc_synchronize", i32, _vp)
        _sig(L, "pmc_plane_span", i32, _vp, i32, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t),
             C.POINTER(C.c_size_t), C.POINTER(C.c_size_t))
        _sig(L, "pmc_selftest_detmath", i32, _vp, i32, _vp, _vp)
        _sig(L, "pmc_hbm_probe", i32, C.c_uint64, i32, _vp, _vp)
        # trajectory dump / restart (host formats need no GPU)
        cp, f3 = C.c_char_p, C.POINTER(C.c_float * 3)
        _sig(L, "pmc_disk_to_r", i32, _vp, _vp, i64, i32, _vp, i64, C.POINTER(i64))
        _sig(L, "pmc_write_dump", i32, cp, i32, i64, _vp, i64, i64, f3, f3)
        _sig(L, "pmc_read_dump", i32, cp, i64, C.POINTER(i64), _vp, i64, C.POINTER(i64), f3, f3)
        _sig(L, "pmc_snapshot_write", i32, cp, P, u32, C.POINTER(Stats), _vp, _vp, i64)
        _sig(L, "pmc_snapshot_read", i32, cp, P, C.POINTER(u32), C.POINTER(Stats), _vp, _vp, i64)
        _sig(L, "pmc_get_params", i32, _vp, P)
        _sig(L, "pmc_stats_write", i32, _vp, C.POINTER(Stats))
        _sig(L, "pmc_dump_frame", i32, _vp, cp, i32, i64)
        _sig(L, "pmc_save_snapshot", i32, _vp, cp, u32)
        _sig(L, "pmc_load_snapshot", i32, _vp, cp, C.POINTER(u32))
        _lib = L
    return _lib


def check(fn: str, rc: int) -> None:
    if rc != 0:
        raise PmcError(fn, rc, lib().pmc_last_error().decode(errors="replace"))
