"""bench.py -- MC trial-moves/s of the checkerboard Metropolis hot path on MI355X.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5|5box]
  torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU, z-slab decomposition)

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py launches the N rank processes
itself (launch_ranks: fresh child processes with RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*, started
before anything touches a GPU; the parent forwards their output, fails as soon as one rank fails
and kills the rest), so `python bench.py --gpus 8` and the torchrun form run the same ranks.
The ranks' control collectives (barriers, the max-over-ranks time, the gather of the box for the
parity leg) run over gloo; the halo planes travel through the slab driver's transport (--transport:
IPC pulls over xGMI by default, RCCL as the alternative).

A "step" is one full MC sweep (8 checkerboard colour phases + shiftCells) with the state resident
in HBM; w=rc=2.5, beta=0.3, sigma=0.5, n_M=10, nmax=16, Philox seed 1234, reference lattice start
(kernel.cu:78-89).  The workloads are BASELINE.json's configs:

  2                       64^3 cells, 1e6 particles, 1 GPU, single-colour sweep: a step is ONE colour
                          phase (step k: colour k % 8 at sweep index k // 8, no shiftCells).
  3     (default at N=1)  128^3 cells, 1e7 particles, 1 GPU, whole periodic box.
  4     (default at N>1)  the SAME 128^3 / 1e7 box split into N z-slabs of 128/N planes (strong
                          scaling; the C slab driver, halo planes over RCCL).  N=1 runs config 3.
  5                       weak scaling: per GPU a 256x256x32 slab of the 256^3 / 8e7 box (its planes
                          of the 8e7 lattice), box 256x256x(32N); at N=8 exactly config 5.  At N=1
                          the halos travel through a one-rank RCCL communicator (rehearsal).
  5box                    the whole 256^3 / 8e7 box on one GPU.

Rank 0 prints ONE JSON line: value = trial moves per second over all ranks; the roofline of the
dominant kernel (subsweep: algorithmic bytes per launch / HIP-event launch time vs 8 TB/s); the
CPU baseline (the C oracle: serial on one core and OpenMP over the cells of a colour on one
socket's cores, bounded samples, host CPU described); and the parity leg (the CPU sample's sweep
rerun on the GPU and compared with the oracle bit for bit).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "parallel-monte-carlo_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3   # MI355X vector FP32 (no MFMA on this path)

CONFIG_NAMES = {
    "2": "BASELINE config 2: 64^3 cells, 1e6 particles, 1 MI355X, single-colour sweep (a step is one colour "
         "phase: colour k % 8 at sweep index k // 8, no shiftCells)",
    "3": "BASELINE config 3: 128^3 cells, 1e7 particles, 1 MI355X, full checkerboard + shiftCells",
    "4": "BASELINE config 4: 128^3 cells, 1e7 particles, {n} MI355X, checkerboard domain decomposition "
         "+ RCCL halo (strong scaling: {n} z-slabs of {nz} planes)",
    "5": "BASELINE config 5: 256^3 cells, 8e7 particles, 8 MI355X weak-scaling -- per GPU a 256x256x32 "
         "slab with its 1e7 particles of the 8e7 lattice; box 256x256x{cz} at {n} GPU(s)",
    "5box": "256^3 cells, 8e7 particles (the config-5 box) whole on 1 MI355X",
}


def stencil_counts(n: np.ndarray, cps: tuple[int, int, int]) -> np.ndarray:
    """S_c = particles in the 27-cell periodic stencil of every cell (whole box)."""
    cx, cy, cz = cps
    g = n.reshape(cz, cy, cx).astype(np.int64)
    s = np.zeros_like(g)
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                s += np.roll(g, shift=(-dz, -dy, -dx), axis=(0, 1, 2))
    return s.reshape(-1)


def slab_stencil_counts(n_storage: np.ndarray, cps: int, nz: int, halo: int = 1) -> np.ndarray:
    """S_c of the owned cells of a slab (storage planes [0, halo) and [nz+halo, nz+2*halo) are the
    halos)."""
    g = n_storage.astype(np.int64).reshape(nz + 2 * halo, cps, cps)
    s = np.zeros((nz, cps, cps), np.int64)
    for dz in (-1, 0, 1):
        sub = g[halo + dz:halo + dz + nz]
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                s += np.roll(sub, shift=(-dy, -dx), axis=(1, 2))
    return s.reshape(-1)


def staged_bytes(n_cells: np.ndarray, stencil: np.ndarray) -> float:
    """SURVEY.md 8(d) staged model for a set of cell visits: per visited (non-empty) cell read its
    27-cell stencil (12 B per particle), 27 counts (2 B each) and write its own particles (12 B each)."""
    ne = n_cells > 0
    return float(np.sum(12 * stencil[ne] + 54 + 12 * n_cells[ne]))


# ---- host CPU description (nproc, model, sockets, cores used) ------------------
def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def host_cpu() -> dict:
    model = None
    txt = _read("/proc/cpuinfo") or ""
    for line in txt.splitlines():
        if line.startswith("model name"):
            model = line.split(":", 1)[1].strip()
            break
    allowed = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    topo = {}
    for cpu_dir in glob.glob("/sys/devices/system/cpu/cpu[0-9]*"):
        cpu = int(cpu_dir.rsplit("cpu", 1)[1])
        pkg = _read(f"{cpu_dir}/topology/physical_package_id")
        core = _read(f"{cpu_dir}/topology/core_id")
        if pkg is not None and core is not None:
            topo[cpu] = (int(pkg), int(core))
    sockets = sorted({p for p, _ in topo.values()}) or [0]
    cores_per_socket = {s: len({c for p, c in topo.values() if p == s}) for s in sockets}
    # one logical CPU per physical core of socket 0 among the CPUs this process may run on
    first_socket = sockets[0]
    seen, socket0_cpus = set(), []
    for cpu in allowed:
        key = topo.get(cpu)
        if key and key[0] == first_socket and key not in seen:
            seen.add(key)
            socket0_cpus.append(cpu)
    quota = None
    cm = _read("/sys/fs/cgroup/cpu.max")
    if cm and not cm.startswith("max"):
        q, per = cm.split()[:2]
        quota = float(q) / float(per)
    return {"model": model, "logical_cpus": os.cpu_count(), "affinity_cpus": len(allowed),
            "sockets": len(sockets), "cores_per_socket": cores_per_socket.get(first_socket),
            "socket0_cores_allowed": len(socket0_cpus), "cgroup_cpu_quota": quota,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(disk, n, cps: int, sweep0: int, serial_planes: int, cps_z: int = 0,
                 phase: tuple[int, int] | None = None, sweeps: int = 1) -> tuple[dict, object]:
    """The C oracle (the reference has no CPU path: SURVEY.md 0/8c) timed on this host:
    (i) serial, one core: one colour phase over planes [0, serial_planes);
    (ii) OpenMP over the cells of a colour on the cores of one socket (one thread per physical
    core, limited by the CPUs/cgroup quota this process may use): `sweeps` full sweeps from the GPU
    state, or with phase = (colour, sweep index) that one colour phase of the whole box (config 2).
    Returns the JSON object and the oracle state after (ii) for the parity leg."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pmc_oracle  # test infrastructure: timed CPU baseline only
    try:
        build_flags = pmc_oracle.use_native()     # compiled for this host (-march=native)
    except Exception as e:
        pmc_oracle.build()
        build_flags = f"-O3 -march=x86-64-v3 -ffp-contract=off -fopenmp (native build failed: {e!r})"
    host = host_cpu()
    cps_z = cps_z or cps
    box = f"{cps}^3" if cps_z == cps else f"{cps}x{cps}x{cps_z}"
    serial_planes = min(serial_planes, cps_z)
    # (i) serial
    st1 = pmc_oracle.OracleState(pmc_oracle.make_params(cps=cps, cps_z=cps_z))
    st1.disk[:] = disk
    st1.n[:] = n
    pmc_oracle.set_threads(1)
    import ctypes as C
    o1 = pmc_oracle.colour_offset(phase[0]) if phase else (0, 0, 0)
    s1 = phase[1] if phase else sweep0
    t0 = time.perf_counter()
    pmc_oracle.lib().orc_subsweep_range(C.byref(st1.p), st1.disk, st1.n, o1[0], o1[1], o1[2], s1, 0, serial_planes,
                                        C.byref(st1.stats))
    dt1 = time.perf_counter() - t0
    serial = st1.stats.trials / dt1
    del st1
    # (ii) one socket
    threads = host["socket0_cores_allowed"] or 1
    limited_by = "socket cores"
    if host["cgroup_cpu_quota"] and host["cgroup_cpu_quota"] < threads:
        threads = max(1, int(host["cgroup_cpu_quota"]))
        limited_by = "cgroup CPU quota"
    st = pmc_oracle.OracleState(pmc_oracle.make_params(cps=cps, cps_z=cps_z))
    st.disk[:] = disk
    st.n[:] = n
    used = pmc_oracle.set_threads(threads)
    t0 = time.perf_counter()
    if phase:
        st.subsweep(pmc_oracle.colour_offset(phase[0]), phase[1])
    else:
        st.run(sweep0, sweeps)
    dt = time.perf_counter() - t0
    par = st.stats.trials / dt
    cores_socket = host["cores_per_socket"] or threads
    what = (f"one colour phase {phase[0]} (sweep index {phase[1]})" if phase else
            ("one full sweep" if sweeps == 1 else f"{sweeps} full sweeps"))
    out = {"value": par, "unit": "trial-moves/s", "cores": threads, "kind": "port",
           "sample": f"{what} of the {box} box from the GPU state, C oracle, OpenMP over the cells "
                     f"of a colour on {threads} threads (one per physical core of socket 0; limited by "
                     f"{limited_by}), {dt:.2f} s",
           "serial": {"value": serial, "cores": 1,
                      "sample": f"one colour phase over planes [0,{serial_planes}) of the {box} box, 1 thread, "
                                f"{dt1:.2f} s"},
           "parallel_efficiency": par / (serial * threads),
           "socket_cores": cores_socket,
           "socket_estimate": (par * cores_socket / threads) if threads < cores_socket else par,
           "socket_estimate_note": ("measured" if threads >= cores_socket else
                                    f"linear extrapolation of the measured {threads}-thread rate to the "
                                    f"{cores_socket} cores of one socket (upper bound)"),
           "omp_threads_reported": used, "host": host, "build": build_flags}
    return out, st


def parity_leg(sim, one_sweep, disk0, n0, sweep0: int, sweeps: int, e0: float, ost) -> dict:
    """The metric's "+ mean-energy error vs reference": rerun the CPU sample's sweeps on the GPU
    from the same state (disk0/n0 at sweep index sweep0) and compare with the oracle's result:
    energy (GPU cell-list energy vs oracle energy), acceptance ratio, and every occupied slot."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pmc_oracle  # test infrastructure: the checker, never the measured path
    sim.copy_in(disk0, n0)
    sim.stats(reset=True)
    for k in range(sweeps):
        one_sweep(sweep0 + k)
    sim.synchronize()
    g = sim.stats()
    e_gpu = sim.energy()
    disk_g, n_g = sim.copy_out()
    c = ost.stats.as_dict()
    e_cpu = ost.energy()
    same = bool(np.array_equal(n_g, ost.n)) and pmc_oracle.valid_slots_equal(disk_g, n_g, ost.disk, ost.n, ost.nmax)
    acc_g = g["accepted"] / g["trials"] if g["trials"] else 0.0
    acc_c = c["accepted"] / c["trials"] if c["trials"] else 0.0
    rel = lambda a, b: abs(a - b) / abs(b) if b else abs(a - b)  # noqa: E731
    return {"reference": "C oracle (corrected-mode restatement of subsweep.h / shiftCells.h)",
            "sweeps": sweeps, "first_sweep": sweep0, "energy_start": e0,
            "energy_gpu": e_gpu, "energy_cpu": e_cpu, "energy_rel_err": rel(e_gpu, e_cpu),
            "acceptance_gpu": acc_g, "acceptance_cpu": acc_c, "acceptance_rel_err": rel(acc_g, acc_c),
            "counters_equal": g == c, "state_bitwise_equal": same}


def z_shift_window(seed: int, first: int, sweeps: int, w: float = 2.5, search: int = 4096) -> int:
    """The first sweep index s0 >= first whose `sweeps` consecutive sweeps shift along z in both
    directions (kernel.cu:683-684's f, d from the per-sweep plan): a slab parity leg over that window
    checks every exchange kind on the node -- the run boundaries' planes, a z shift's deferred plane
    from above and from below.  `first` itself when sweeps < 2 or no window is found."""
    if sweeps < 2:
        return first
    from pmc_amd.plan import sweep_plan
    sign = []
    for s in range(first, first + search + sweeps):
        _, f, d = sweep_plan(seed, s, w)
        sign.append(0 if f != 2 else (1 if d > 0 else -1))
    for k in range(search):
        win = sign[k:k + sweeps]
        if 1 in win and -1 in win:
            return first + k
    return first


def z_shifts(seed: int, s0: int, sweeps: int, w: float = 2.5) -> list:
    from pmc_amd.plan import sweep_plan
    out = []
    for s in range(s0, s0 + sweeps):
        _, f, d = sweep_plan(seed, s, w)
        out.append("xyz"[f] + ("+" if d > 0 else "-"))
    return out


def achievable_hbm(nbytes: int = 1 << 30, reps: int = 10) -> dict:
    """the HBM rate this box actually delivers, beside the 8 TB/s spec -- the
    library's streaming kernels (pmc_hbm_probe: 16-B loads, 16 workgroups of 256 per CU) over 1 GiB
    buffers, HIP events, best of `reps`: a read-only pass and a copy (read + write counted)."""
    import pmc_amd
    read, copy = pmc_amd.hbm_probe(nbytes, reps)
    return {"read_GBs": read, "copy_GBs": copy, "bytes": nbytes, "reps": reps,
            "method": "pmc_hbm_probe: streaming read of 1 GiB (16-B loads) and copy of 1 GiB (read + write "
                      "counted), HIP events, best of reps"}


def parity_leg_slab(ctx, one_sweep, finish, disk_s, n_s, sweep0: int, e0: float, gather, ost, rank: int,
                    sweeps: int = 1) -> dict | None:
    """parity_leg for the slab driver, collective over the ranks: every rank restores its storage
    (owned planes and halos) at the timed start, reruns the CPU sample's sweeps, the whole box's
    counters and energy come from pmc_slab_observables (fixed-point sums over the ranks), the owned
    planes are gathered on rank 0 and compared with the oracle's whole-box result there."""
    ctx.copy_in(disk_s, n_s)
    ctx.slab_exchange()
    ctx.stats(reset=True)
    for k in range(sweeps):
        one_sweep(sweep0 + k)
    finish()
    ctx.synchronize()
    g, e_gpu = ctx.slab_observables(True)
    d, n = ctx.copy_out()
    whole = gather(d, n)
    if rank != 0:
        return None
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pmc_oracle  # test infrastructure: the checker, never the measured path
    disk_g, n_g = whole
    c = ost.stats.as_dict()
    e_cpu = ost.energy()
    same = bool(np.array_equal(n_g, ost.n)) and pmc_oracle.valid_slots_equal(disk_g, n_g, ost.disk, ost.n, ost.nmax)
    acc_g = g["accepted"] / g["trials"] if g["trials"] else 0.0
    acc_c = c["accepted"] / c["trials"] if c["trials"] else 0.0
    rel = lambda a, b: abs(a - b) / abs(b) if b else abs(a - b)  # noqa: E731
    return {"reference": "C oracle (corrected-mode restatement of subsweep.h / shiftCells.h), whole box",
            "sweeps": sweeps, "first_sweep": sweep0, "shifts": z_shifts(ctx.params.seed, sweep0, sweeps),
            "energy_start": e0,
            "energy_gpu": e_gpu, "energy_cpu": e_cpu, "energy_rel_err": rel(e_gpu, e_cpu),
            "acceptance_gpu": acc_g, "acceptance_cpu": acc_c, "acceptance_rel_err": rel(acc_g, acc_c),
            "counters_equal": g == c, "state_bitwise_equal": same,
            "gpu_side": "all ranks (slab driver), owned planes gathered on rank 0"}


def make_gather(world: int, rank: int, plane: int, nz: int, row: int, halo: int = 1):
    """gather(disk_storage, n_storage) -> (disk, n) of the whole box on rank 0 (None elsewhere): the
    owned planes of every rank in rank order (rank r owns global planes [r*nz, (r+1)*nz)).
    Collective; counts travel as bytes (RCCL has no 16-bit integer type)."""
    def gather(disk_s, n_s):
        own_d = np.ascontiguousarray(disk_s[halo * plane * row:(nz + halo) * plane * row])
        own_n = np.ascontiguousarray(n_s[halo * plane:(nz + halo) * plane])
        if world == 1:
            return own_d, own_n
        import torch
        import torch.distributed as dist
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"     # (gloo: the CPU tests)
        td = torch.from_numpy(own_d).to(dev)
        tn = torch.from_numpy(own_n.view(np.uint8)).to(dev)
        ld = [torch.empty_like(td) for _ in range(world)] if rank == 0 else None
        ln = [torch.empty_like(tn) for _ in range(world)] if rank == 0 else None
        dist.gather(td, ld, dst=0)
        dist.gather(tn, ln, dst=0)
        if rank != 0:
            return None
        disk = np.concatenate([t.cpu().numpy() for t in ld])
        n = np.concatenate([t.cpu().numpy() for t in ln]).view(np.int16)
        return disk, n
    return gather


def traffic_from_profile(config: str, slab: bool, nz_local: int) -> dict | None:
    """Measured memory-side traffic per dominant-kernel launch (profiles/pmc_traffic.json, from
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes): the whole box at top level, slab launch shapes under
    "slab" keyed "<config>:<planes per rank>" (tools/slab_traffic.sh)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            t = json.load(f)
    except Exception:
        return None
    if not slab:
        # the top level is the config-3 whole box (128^3/1e7); other whole boxes under "box"
        return t if config == "3" else (t.get("box") or {}).get(config)
    return (t.get("slab") or {}).get(f"{config}:{nz_local}")



def valu_from_profile() -> dict | None:
    """The dominant kernel's VALU-issue roof from its committed SQ counters (profiles/pmc_valu.json,
    tools/valu_roof.py): issue cycles per SIMD at the measured per-class costs against the launch's
    cycles -- the roof that binds this kernel."""
    path = os.path.join(REPO, "profiles", "pmc_valu.json")
    try:
        with open(path) as f:
            return json.load(f)
    except Exception:
        return None


def _hip_d2d(dst: int, src: int, nbytes: int, stream: int) -> None:
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")          # the HIP runtime torch has loaded
    hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
    rc = hip.hipMemcpyAsync(C.c_void_p(dst), C.c_void_p(src), C.c_size_t(nbytes), 3, C.c_void_p(stream))
    if rc != 0:
        raise RuntimeError(f"hipMemcpyAsync D2D failed: {rc}")


def rewarm(sim, one_sweep, finish, first: int, count: int, relink=None) -> None:
    """Run `count` sweeps (sweep indices first.., the timed ones) and restore the state they
    started from with device copies on the context stream: GPU clock warm-up with the hot-path
    kernels themselves, no host gap before the timed region, no change to what is timed."""
    import torch
    cells = sim.cells
    disk_b, n_b = cells * 3 * sim.nmax * 4, cells * 2
    save = torch.empty(disk_b + n_b, dtype=torch.uint8, device="cuda")
    st = sim.stream()
    finish()
    d, n = sim.state_ptrs()
    _hip_d2d(save.data_ptr(), d, disk_b, st)
    _hip_d2d(save.data_ptr() + disk_b, n, n_b, st)
    if relink is not None:
        relink()        # slab: the other streams' next launches wait for the copies above
    for k in range(count):
        one_sweep(first + k)
    finish()
    d, n = sim.state_ptrs()                 # the current buffer of the ping-pong pair now
    _hip_d2d(d, save.data_ptr(), disk_b, st)
    _hip_d2d(n, save.data_ptr() + disk_b, n_b, st)
    if relink is not None:
        relink()                            # slab: order the driver's streams after the restore
    sim.synchronize()
    sim.stats(reset=True)
    del save

def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list, timeout_s: float) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT in their environment) and wait for them.  The parent
    touches no GPU (no torch, no libpmc: a process that initialised the GPU must never start or replace
    programs); the ranks inherit stdout/stderr, so rank 0's JSON line is this command's output.  As soon
    as one rank fails, or the time limit passes, the others are killed (their own process groups) and
    the parent exits non-zero."""
    import signal
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []

    def kill_all():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except OSError:
                    pass
        t_end = time.time() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except OSError:
                    pass
                p.wait()

    def on_signal(signum, _frame):
        kill_all()
        sys.exit(128 + signum)

    signal.signal(signal.SIGTERM, on_signal)
    signal.signal(signal.SIGINT, on_signal)
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      start_new_session=True))
    print(f"bench.py: launched {n} rank processes (MASTER_PORT {port})", file=sys.stderr, flush=True)
    t0 = time.time()
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            r, c = bad[0]
            print(f"bench.py: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr, flush=True)
            rc = c if c > 0 else 128 - c
            break
        if all(c == 0 for c in codes):
            break
        if time.time() - t0 > timeout_s:
            print(f"bench.py: ranks still running after {timeout_s:.0f} s; stopping them", file=sys.stderr, flush=True)
            rc = 124
            break
        time.sleep(0.2)
    kill_all()
    return rc


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["2", "3", "4", "5", "5box"], default=None,
                    help="BASELINE config (default: 3 at N=1, 4 at N>1)")
    ap.add_argument("--strong", action="store_true", help="alias of --config 4")
    ap.add_argument("--cps", type=int, default=None, help="override cells per side (configs 3/4)")
    ap.add_argument("--atoms", type=int, default=None, help="override the particle count (configs 3/4)")
    ap.add_argument("--serial-planes", type=int, default=None,
                    help="planes of the serial CPU sample's colour phase (default: the whole box up to 128)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", action="store_true", help="replay the timed sweeps as one hipGraph")
    ap.add_argument("--cpu-sweeps", type=int, default=3,
                    help="whole-box CPU baseline: full sweeps the OpenMP oracle times (and the parity leg reruns "
                         "on the GPU from the same state)")
    ap.add_argument("--no-events", action="store_true",
                    help="no per-launch HIP events in the timed region (no roofline; overhead check)")
    ap.add_argument("--rewarm", type=int, default=12,
                    help="sweeps run on the timed start state right before the timed region, which is "
                         "then restored on the device (the GPU comes out of the host analysis idle "
                         "and needs ~10 sweeps to reach its steady clock; 0: off)")
    ap.add_argument("--timing-every", type=int, default=0,
                    help="per-launch HIP events on the launches of every k-th timed sweep (the roofline's "
                         "kernel times).  Default: 4 for a whole box (events on every launch cost ~1.3%% of "
                         "its sweep); ceil(steps/2) (>= 4) for the slab driver, whose 0.38 ms sweep at 8 "
                         "ranks is host-issue-bound while events ride on its launches (a timed sweep "
                         "+55 us; every 4th: +3.5%%, every 20th: +0.3%%, profiles/r06s_event_every_ab.txt)")
    ap.add_argument("--slab", action="store_true", help="config 3 through the z-slab driver with one rank")
    ap.add_argument("--self-rccl", action="store_true",
                    help="one slab rank: halos through a one-rank RCCL communicator (default for config 5)")
    ap.add_argument("--local-halo", action="store_true", help="config 5 at N=1: local halo copies, no RCCL")
    ap.add_argument("--emulate-ranks", type=int, default=0,
                    help="config 4 at N=1: one rank's slab of an R-rank run (the bottom 128/R planes of the "
                         "1e7 lattice as a periodic slab) -- the per-rank launch shapes, for rocprof")
    ap.add_argument("--xfer-delay-us", type=float, default=0.0,
                    help="slab rehearsals: hold the exchange stream busy this long after every halo exchange "
                         "(PMC_XFER_DELAY_US: the xGMI time and RCCL latency a one-GPU run does not pay)")
    ap.add_argument("--halo", type=int, default=0, choices=(0, 1, 2),
                    help="slab halo planes per side: 2 = one exchange per sweep, the neighbour's boundary plane "
                         "visited redundantly (0: PMC_SLAB_HALO, default 1)")
    ap.add_argument("--transport", choices=("auto", "ipc", "rccl", "local"), default=None,
                    help="slab halo transport: ipc (peer buffers mapped over xGMI, pulled by the library's copy "
                         "kernels), rccl, local (one rank: periodic halos by local copies), auto (ipc, else rccl on "
                         "every rank).  Default: auto at N > 1, local for one-rank slabs (config 5: rccl)")
    ap.add_argument("--same-device", action="store_true",
                    help="all ranks on GPU 0 (a multi-process correctness run on one GPU; needs the ipc transport)")
    ap.add_argument("--no-hbm-probe", action="store_true",
                    help="skip the achievable-HBM copy/read measurement (roofline.achievable_peak)")
    ap.add_argument("--rank-timeout", type=float, default=1500.0,
                    help="--gpus N without a launcher: stop the ranks after this many seconds")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, sys.argv[1:], args.rank_timeout)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        print(f"bench.py rank {os.environ.get('RANK', '0')}/{os.environ['WORLD_SIZE']}: starting", file=sys.stderr,
              flush=True)
    if args.xfer_delay_us > 0:
        os.environ["PMC_XFER_DELAY_US"] = str(args.xfer_delay_us)   # read by libpmc at its first exchange

    import pmc_amd
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} != --gpus {args.gpus}", file=sys.stderr)
    if world > 1:
        # fail before any GPU call when this rank has no device (pmc_device_count: PMC_ERR_NODEV)
        try:
            ndev = pmc_amd.device_count()
        except pmc_amd.PmcError as e:
            print(f"bench.py rank {rank}/{world}: {e}", file=sys.stderr, flush=True)
            return 3
        if not args.same_device and local >= ndev:
            print(f"bench.py rank {rank}/{world}: LOCAL_RANK {local} but {ndev} GPU(s) visible", file=sys.stderr)
            return 3
    config = args.config or ("4" if args.strong else ("3" if world == 1 else "4"))
    if args.emulate_ranks:
        if config != "4" or world != 1:
            raise SystemExit("--emulate-ranks is a one-process rehearsal of config 4")
        args.slab = True
    if config == "4" and world == 1 and not args.slab:
        config = "3"          # the 1-GPU point of the config-4 strong-scaling curve is config 3
    if config in ("2", "5box") and world > 1:
        raise SystemExit(f"--config {config} is a single-GPU configuration")
    torch.cuda.set_device(0 if args.same_device else local)
    if world > 1:
        # control collectives on the host (gloo); the halo data path is the slab driver's transport
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
    stream = torch.cuda.Stream()

    def barrier():
        if world > 1:
            dist.barrier()

    if config == "2":
        cps = args.cps or 64
        atoms = args.atoms or 1_000_000
    elif config in ("3", "4"):
        cps = args.cps or 128
        atoms = args.atoms or 10_000_000
    else:
        cps, atoms = 256, 80_000_000
    slab = config in ("4", "5") or args.slab
    if args.emulate_ranks:
        nz_local = cps // args.emulate_ranks
        box_z = nz_local
    elif config == "4" or (config == "3" and slab):
        nz_local = cps // world
        box_z = cps
    elif config == "5":
        nz_local = 32
        box_z = 32 * world
    else:
        nz_local = box_z = cps
    if slab and (nz_local % 2 or nz_local < 2 or (config == "4" and cps % world)):
        raise SystemExit(f"slab thickness {nz_local} must be even and >= 2")

    if not slab:
        sim = pmc_amd.PmcContext(cps, stream=stream.cuda_stream)
        sim.init_lattice(atoms)

        if config == "2":
            def one_sweep(s):       # config 2's step: ONE colour phase, colour s % 8 at sweep s // 8
                sim.phase(s % 8, s // 8)
        else:
            def one_sweep(s):   # pmc_sweep: 8 colour phases (in plane chains) + shiftCells, all in C
                sim.sweep(s)

        def finish():
            pass
        transport = "single GPU"
    else:
        # the product multi-GPU path: sweep schedule + RCCL halo exchange in C (pmc_slab_*)
        from pmc_amd.slab import SlabDriver
        tp = args.transport
        if tp is None:
            tp = ("auto" if world > 1 else
                  "rccl" if (args.self_rccl or (config == "5" and not args.local_halo)) else "local")
        if args.same_device and tp not in ("ipc", "auto"):
            raise SystemExit("--same-device needs the ipc transport (RCCL refuses two ranks on one GPU)")
        drv = SlabDriver(cps=cps, nz_local=nz_local, rank=rank, world=world, stream=stream, transport=tp,
                         halo=args.halo)
        if config == "5" or args.emulate_ranks:
            drv.ctx.init_lattice_planes(atoms, cps)     # this rank's planes of the 256^3 / 8e7 (128^3 / 1e7) lattice
        else:
            drv.ctx.init_lattice_global(atoms)         # this rank's planes of the one 128^3 box
        drv.ctx.slab_exchange()
        drv.verify_transport()                         # IPC at N > 1: halos checked, "auto" may fall back to RCCL
        sim = drv.ctx

        def one_sweep(s):
            drv.sweep(s)

        finish = drv.finish
        tp_name = {"rccl": "RCCL", "ipc": "IPC pulls (pmc_slab_init_ipc: peer buffers mapped, copy kernels)",
                   "local": "local copies"}[drv.transport]
        transport = (f"z-slab x{world}, {nz_local} planes per rank, "
                     + ("two halo planes per side (one exchange per sweep), " if drv.halo == 2 else "")
                     + f"halo planes over {tp_name} (C slab driver)"
                     + (", all ranks on GPU 0" if args.same_device else ""))

    # warmup
    for s in range(args.warmup):
        one_sweep(s)
    finish()
    torch.cuda.synchronize()
    sim.stats(reset=True)
    # algorithmic bytes from the state at the start of the timed region
    disk_h, n_h = sim.copy_out()
    plane = cps * cps
    if config == "2":
        # the timed steps' colours (no shiftCells: the counts, hence the bytes, stay fixed)
        n_owned = n_h.astype(np.int64)
        stencil = stencil_counts(n_owned, (cps, cps, cps))
        idx = np.arange(cps ** 3)
        cx, cy, cz = idx % cps, (idx // cps) % cps, idx // (cps * cps)
        per_colour = []
        for colour in range(8):
            o = (colour // 4) % 2, (colour // 2) % 2, colour % 2     # itoa, start.cu:153-157
            m = (cx % 2 == o[0]) & (cy % 2 == o[1]) & (cz % 2 == o[2])
            per_colour.append(staged_bytes(n_owned[m], stencil[m]))
        timed = [per_colour[(args.warmup + k) % 8] for k in range(args.steps)]
        sub_launch_bytes = float(np.mean(timed))
        roof_kernel = "k_subsweep<16,16,true> (one colour phase of the 64^3 box; mean over the timed steps' colours)"
    elif not slab:
        n_owned = n_h.astype(np.int64)
        stencil = stencil_counts(n_owned, (cps, cps, cps))
        phase_bytes = staged_bytes(n_owned, stencil) / 8.0
        # pmc_sweep's plane chains (pmc_sweep_layout): each colour phase is one launch per chain, the
        # chains' launches concurrent and a chain's next phase overlapping the others' tails; the
        # roofline is per PHASE: a timed sweep's subsweep span (first launch start to last stop, HIP
        # events on the dispatch packets; gaps included, shiftCells not) / 8, launch_ms the per-launch mean
        sweep_chains = sim.sweep_layout()
        per_chain = [staged_bytes(n_owned[a * plane:b * plane], stencil[a * plane:b * plane]) / 8.0
                     for a, b in sweep_chains]
        sub_launch_bytes = sum(per_chain) / len(per_chain)
        roof_kernel = ("k_subsweep<16,16,true> (one colour phase of the whole box" +
                       (f" as {len(sweep_chains)} concurrent launches, plane chains " +
                        " and ".join(f"[{a},{b})" for a, b in sweep_chains) +
                        "; achieved/frac per phase: a sweep's subsweep span / 8" if len(sweep_chains) > 1 else "") + ")")
    else:
        n_owned = n_h[plane * drv.halo:plane * (nz_local + drv.halo)].astype(np.int64)
        stencil = slab_stencil_counts(n_h, cps, nz_local, drv.halo)
        # kind-0 launches: the interior chains (pmc_slab_layout: 1-3 chains, PMC_SLAB_CHAINS), one
        # launch per chain and colour phase; the roofline's bytes per launch are their mean (the
        # chains run concurrently)
        chains = [(a, b) for a, b in drv.ctx.slab_layout() if b > a]
        per_chain = [staged_bytes(n_owned[a * plane:b * plane], stencil[a * plane:b * plane]) / 8.0
                     for a, b in chains]
        sub_launch_bytes = sum(per_chain) / len(per_chain) if per_chain else 0.0
        roof_kernel = ("k_subsweep<16,16,true> (a slab colour phase's interior launches, planes "
                       + " and ".join(f"[{a},{b})" for a, b in chains) + ", mean bytes per launch; "
                       "per CHAIN: the chains run concurrently and share HBM, so achieved/frac describe "
                       "one chain's launch, not the chip's rate)")
    e_start = sim.energy()      # cell-list energy of the state the timed region starts from
    # The host analysis above leaves the GPU idle, and an idle MI355X comes back at a lower clock:
    # after a 0.5 s gap the first sweeps take 3.0-3.3 ms and the rate settles at 2.53 ms only
    # after ~10 sweeps, even when the gap is filled with other GPU work (energy evaluations:
    # first sweep 2.71 ms, same ramp; profiles/r02s2_clock_ramp.txt).  So the hot path itself runs
    # `rewarm` sweeps on the timed start state right before the timed region, and the state is
    # then restored by device-to-device copies: the timed region starts from exactly the state
    # analysed above, at the steady clock.  The counters of the re-warm sweeps are discarded.
    if args.rewarm > 0:
        rewarm(sim, one_sweep, finish, first=args.warmup, count=args.rewarm,
               relink=(lambda: drv.ctx.slab_exchange()) if slab else None)

    sim.timing_kinds(not args.no_events and not args.graph)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    first = args.warmup
    t_issue = None
    if args.graph and not slab:
        sim.run_graph(first, args.steps)
    else:
        timed = not args.no_events
        every = args.timing_every if args.timing_every > 0 else (max(4, -(-args.steps // 2)) if slab else 4)
        for k in range(args.steps):
            if timed and every > 1:
                sim.timing_pause(k % every != 0)   # events on sweeps 0, every, 2*every, ...
            one_sweep(first + k)
        t_issue = time.perf_counter() - t0     # host time to issue the K steps (the GPU may still run)
        finish()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    st = sim.stats()
    tm = sim.timing_kinds(False)
    span_ms, span_n = sim.phase_spans() if (not slab and config == "3") else (0.0, 0)
    trials_local = st["trials"]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tr = torch.tensor([trials_local, st["accepted"]], dtype=torch.int64)
        dist.all_reduce(tr)
        trials_total, accepted_total = (int(v) for v in tr.tolist())
    else:
        trials_total, accepted_total = trials_local, st["accepted"]
    flags = sim.error_flags()
    value = trials_total / elapsed
    # energy bookkeeping over the timed sweeps: E_start + sum of accepted dE (fixed point 2^-32,
    # order-independent) against a direct cell-list evaluation of the final state
    e_end = sim.energy()
    de_timed = st["de_fixed"] / 2.0 ** 32
    if world > 1:   # slab energies count boundary pairs half on each side: the sum is the box's
        ev = torch.tensor([e_start, e_end, de_timed], dtype=torch.float64)
        dist.all_reduce(ev)
        e_start, e_end, de_timed = (float(v) for v in ev.tolist())
    particles = int(n_owned.sum())
    if world > 1:
        pt = torch.tensor([particles], dtype=torch.int64)
        dist.all_reduce(pt)
        particles = int(pt.item())
    # node roofline (north_star: "fraction of the HBM roofline at 1, 2, 4 and 8 GPUs"): the staged
    # model's bytes of one step summed over the ranks -- every owned cell's visit plus
    # shiftCells' 36 B per particle + 6 B per cell -- over the step time, against N x 8 TB/s
    if config == "2":
        step_bytes_local = sub_launch_bytes
        step_shift_local = 0.0
    else:
        step_bytes_local = staged_bytes(n_owned, stencil)
        step_shift_local = float(36 * int(n_owned.sum()) + 6 * n_owned.size)
    sb = torch.tensor([step_bytes_local, step_shift_local], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(sb)
    step_bytes, step_shift_bytes = (float(v) for v in sb.tolist())
    # the rate this box actually delivers, measured on rank 0's GPU
    hbm_meas = achievable_hbm() if (rank == 0 and not args.no_hbm_probe) else None

    if rank == 0:
        n_launch = tm["n_subsweep"]
        avg_launch_s = (tm["subsweep_ms"] / n_launch * 1e-3) if n_launch else None
        achieved = (sub_launch_bytes / avg_launch_s / 1e9) if avg_launch_s else None
        phase_s = (span_ms / span_n * 1e-3) if span_n else None
        if phase_s:   # chained whole-box phases: bytes of a phase over the phase's span
            achieved = phase_bytes / phase_s / 1e9
        traffic = traffic_from_profile(config, slab, nz_local)
        # FP32 work of the moves (14 FLOP per pair evaluation, old + new position,
        # against the S_c - 1 stencil partners of each evaluated move; the mean stencil of the
        # visited cells stands for each cell's) per launch, over the HIP-event launch time
        fp32 = None
        if avg_launch_s and not slab:
            ne = n_owned > 0
            s_mean = float(stencil[ne].mean()) if ne.any() else 0.0
            phases = args.steps * (1 if config == "2" else 8)
            flop = 28.0 * st["evaluated"] / phases * max(s_mean - 1.0, 0.0)     # per colour phase
            t_ph = phase_s or avg_launch_s
            fp32 = {"achieved": flop / t_ph / 1e12, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": flop / t_ph / 1e12 / FP32_PEAK_TFLOPS, "flop_per_phase": flop,
                    "model": "28 FLOP x (mean stencil - 1) per evaluated move (SURVEY.md 8d), per colour phase"}
        valu = valu_from_profile() if config == "3" else None   # profiled on the config-3 launch
        shift_bytes = None
        if tm["n_shift"]:
            # shiftCells (VS shiftCells.h:23-112): per output cell, read its own occupied slots and
            # those of its dir-neighbour with both counts, write the new occupied slots and count --
            # 12 B per particle read twice (own and as a neighbour) and written once, 6 B of counts
            shift_bytes = float(36 * int(n_owned.sum()) + 6 * n_owned.size)
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic.get("subsweep_bytes_per_launch") if traffic else None,
                "traffic_source": traffic.get("source") if traffic else None,
                "kernel": roof_kernel,
                "launch_ms": avg_launch_s * 1e3 if avg_launch_s else None,
                "launches_timed": n_launch,
                **({"phase_ms": phase_s * 1e3, "phases_timed": span_n,
                    "algorithmic_bytes_per_phase": phase_bytes,
                    # the per-launch view rocprofv3's kernel statistics give (half-box launches, two at once)
                    "launch_achieved": sub_launch_bytes / avg_launch_s / 1e9 if avg_launch_s else None}
                   if phase_s else {}),
                "shift_ms": tm["shift_ms"] / tm["n_shift"] if tm["n_shift"] else None,
                "shift": ({"algorithmic_bytes_per_launch": shift_bytes,
                           "achieved": shift_bytes / (tm["shift_ms"] / tm["n_shift"] * 1e-3) / 1e9,
                           "frac": shift_bytes / (tm["shift_ms"] / tm["n_shift"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                           "model": "36 B per particle + 6 B per cell (own + neighbour occupied slots read, "
                                    "new slots written, counts)"}
                          if shift_bytes and tm["n_shift"] and tm["shift_ms"] > 0 else None),
                "fp32": fp32,
                "valu": valu,
                "binding": ("valu-issue (roofline.valu.frac; HBM frac and fp32 frac are far below it)"
                            if valu else None),
                "boundary_launch_ms": tm["boundary_ms"] / tm["n_boundary"] if tm["n_boundary"] else None,
                "algorithmic_bytes_per_launch": sub_launch_bytes}
        ms_step = elapsed / args.steps
        node_ach = (step_bytes + step_shift_bytes) / ms_step / 1e9
        roof["node"] = {
            "achieved": node_ach, "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
            "frac": node_ach / (HBM_PEAK_GBS * world),
            "bytes_per_step": step_bytes + step_shift_bytes, "subsweep_bytes_per_step": step_bytes,
            "shift_bytes_per_step": step_shift_bytes, "gpus": world,
            "model": ("sum over ranks of the staged model's bytes of one step (every owned non-empty cell: "
                      "12 B x stencil particles + 54 B of counts + 12 B x own particles written; shiftCells "
                      "36 B per particle + 6 B per cell) / ms_per_step, against N x 8 TB/s")}
        if hbm_meas:
            roof["achievable_peak"] = hbm_meas
            # the subsweep reads ~25x what it writes: its achievable roof is the read rate
            roof["frac_of_achievable"] = (achieved / hbm_meas["read_GBs"]) if achieved else None
            roof["node"]["frac_of_achievable"] = node_ach / (hbm_meas["read_GBs"] * world)
    # CPU baseline and parity leg (after the timed region).  Slabs: the start state of the timed
    # region is gathered on rank 0 (the whole box), the oracle runs there while the other ranks wait,
    # then every rank reruns the sample's sweep (collective) and rank 0 compares.
    cpu = None
    parity = None
    if not args.no_cpu_baseline:
        sp = args.serial_planes or min(cps, 128)
        ost = None
        if not slab:
            if rank == 0:
                try:
                    ph = (first % 8, first // 8) if config == "2" else None
                    cs = 1 if ph else max(1, args.cpu_sweeps)
                    cpu, ost = cpu_baseline(disk_h, n_h, cps, first, sp, phase=ph, sweeps=cs)
                    parity = parity_leg(sim, one_sweep, disk_h, n_h, first, cs, e_start, ost)
                    if config == "2":
                        parity["sweeps"] = 0
                        parity["phase"] = {"colour": first % 8, "sweep_index": first // 8}
                except Exception as e:  # the baseline is reported, never the measured value
                    cpu = {"error": repr(e)}
        else:
            gather = make_gather(world, rank, plane, nz_local, 3 * 16, drv.halo)
            whole = gather(disk_h, n_h)
            # the sample: --cpu-sweeps sweeps from the timed start state, at the first sweep indices that
            # shift along z both ways (every exchange kind, the deferred z planes included, on the node)
            cs = max(1, args.cpu_sweeps)
            s0 = z_shift_window(sim.params.seed, first, cs)
            if rank == 0:
                try:
                    cpu, ost = cpu_baseline(whole[0], whole[1], cps, s0, sp, cps_z=box_z, sweeps=cs)
                    cpu["sample"] += f" (whole {cps}x{cps}x{box_z} box gathered from {world} rank(s))"
                except Exception as e:
                    cpu = {"error": repr(e)}
            del whole
            barrier()
            ok = torch.tensor([1 if (rank != 0 or ost is not None) else 0])
            if world > 1:
                dist.broadcast(ok, src=0)
            if int(ok.item()):
                parity = parity_leg_slab(sim, one_sweep, finish, disk_h, n_h, s0, e_start, gather, ost, rank,
                                         sweeps=cs)

    if rank == 0:
        sweeps_per_s = args.steps / elapsed / (8.0 if config == "2" else 1.0)
        name = CONFIG_NAMES[config].format(n=world, nz=nz_local, cz=box_z)
        if args.emulate_ranks:
            name = (f"rehearsal of BASELINE config 4 at {args.emulate_ranks} ranks on 1 MI355X: one rank's slab "
                    f"({nz_local} planes of the 128^3 / 1e7 box, periodic, halos through "
                    + {"rccl": "a one-rank RCCL communicator", "ipc": "the IPC transport's kernels (to itself)",
                       "local": "local copies"}[drv.transport] + "); value = ONE rank's rate")
        out = {
            "metric": "MC trial-moves/s (whole node)",
            "value": value,
            "unit": "trial-moves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            # host time spent issuing a step's launches (pmc_sweep / pmc_slab_sweep calls, no waits):
            # close to ms_per_step means the host, not the GPU, sets the pace
            "host_issue_ms_per_step": (t_issue / args.steps * 1e3) if t_issue is not None else None,
            **({"step": "one colour phase"} if config == "2" else {}),
            "higher_is_better": True,
            # configs 3 -> 4 are one fixed box over 1..N GPUs (strong); config 5 fixes the work per GPU
            "scaling": "weak" if config == "5" else "strong",
            # the same run's CPU baseline (one socket of the host, C oracle): BASELINE.json publishes
            # no number, so the socket estimate is the denominator
            "vs_baseline": (value / cpu["socket_estimate"]) if (cpu and cpu.get("socket_estimate")) else None,
            "vs_baseline_of": "cpu_baseline.socket_estimate" if (cpu and cpu.get("socket_estimate")) else None,
            "dtype": "f32",
            "data": "synthetic (reference simple-cubic lattice start, Philox seed 1234)",
            "config": {"workload": name, "baseline_config": config,
                       "box_cells": [cps, cps, box_z], "cells_per_gpu": cps * cps * nz_local,
                       "particles": particles, "n_moves": 10, "nmax": 16, "beta": 0.3, "sigma": 0.5,
                       "w": 2.5, "parallelism": transport,
                       **({"injected_exchange_delay_us": args.xfer_delay_us} if args.xfer_delay_us > 0 else {})},
            "sweeps_per_s": sweeps_per_s,
            "acceptance": accepted_total / trials_total if trials_total else None,
            "energy": {"start": e_start, "end": e_end, "start_plus_sum_dE": e_start + de_timed,
                       "per_particle_end": e_end / particles if particles else None,
                       "bookkeeping_rel_err": abs(e_start + de_timed - e_end) / abs(e_end) if e_end else None,
                       "particles": particles},
            "parity": parity,
            "error_flags": flags,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
