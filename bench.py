"""bench.py -- MC trial-moves/s of the checkerboard Metropolis hot path on MI355X.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--cps 128] [--atoms 10000000]
  torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU, z-slab decomposition)

A "step" is one full MC sweep (8 checkerboard colour phases + shiftCells) of BASELINE.json
config 3 (128^3 cells, 1e7 particles per GPU, w=rc=2.5, beta=0.3, sigma=0.5, n_M=10, nmax=16,
Philox seed 1234, reference lattice start) with the state resident in HBM.  With N>1 ranks every
rank owns a 128^3-cell slab of a 128x128x(128N) periodic box (weak scaling; the 8-rank point has
the per-GPU work of config 5) and exchanges halo planes with its z-neighbours over RCCL.
--strong runs BASELINE config 4 instead: ONE 128^3 box with 1e7 particles split into N slabs of
128/N planes (the 1-GPU state, plane for plane), "scaling": "strong".

Rank 0 prints ONE JSON line with value = trial moves per second over all ranks, the roofline of
the dominant kernel (subsweep; algorithmic bytes per launch / HIP-event launch time vs 8 TB/s)
and the CPU baseline (the C oracle, OpenMP over the cells of a colour, on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "parallel-monte-carlo_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


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


def algorithmic_bytes_per_sweep(n_owned: np.ndarray, stencil: np.ndarray) -> dict:
    """SURVEY.md 8(d) staged model: per visited (non-empty) cell read its 27-cell stencil
    (12 B per particle), 27 counts (2 B each) and write its own particles (12 B each)."""
    ne = n_owned > 0
    sub = float(np.sum(12 * stencil[ne] + 54 + 12 * n_owned[ne]))
    shift = float(np.sum(36 * n_owned.astype(np.int64) + 6)) * 1.0
    return {"subsweep_sweep": sub, "subsweep_launch": sub / 8.0, "shift": shift}


def cpu_baseline(disk: np.ndarray, n: np.ndarray, cps: int, sweeps: int, threads: int, sweep0: int) -> dict:
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pmc_oracle  # test infrastructure: timed CPU baseline only
    pmc_oracle.build()
    st = pmc_oracle.OracleState(pmc_oracle.make_params(cps=cps))
    st.disk[:] = disk
    st.n[:] = n
    pmc_oracle.set_threads(threads)
    t0 = time.perf_counter()
    st.run(sweep0, sweeps)
    dt = time.perf_counter() - t0
    trials = st.stats.trials
    return {"value": trials / dt, "unit": "trial-moves/s", "cores": threads, "kind": "port",
            "sample": f"{sweeps} full sweep(s) of the {cps}^3-cell box from the GPU state "
                      f"(C oracle, OpenMP over cells of a colour, {threads} threads), {dt:.2f} s"}, st


def parity_leg(sim, one_sweep, disk0, n0, sweep0: int, sweeps: int, e0: float, ost) -> dict:
    """The metric's "+ mean-energy error vs reference": rerun the CPU sample's sweeps on the GPU
    from the same state (disk0/n0 at sweep index sweep0) and compare with the oracle's result:
    energy (GPU cell-list energy vs oracle energy), acceptance ratio, and every occupied slot."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import pmc_oracle  # test infrastructure: the checker, never the measured path
    sim.copy_in(disk0, n0)
    sim.stats(reset=True)
    for k in range(sweeps):
        one_sweep(sweep0 + k, False)
    sim.synchronize()
    g = sim.stats()
    e_gpu = sim.energy()
    disk_g, n_g = sim.copy_out()
    c = ost.stats.as_dict()
    e_cpu = ost.energy()
    same = bool(np.array_equal(n_g, ost.n)) and pmc_oracle.valid_slots_equal(disk_g, n_g, ost.disk, ost.n, ost.nmax)
    acc_g = g["accepted"] / g["trials"] if g["trials"] else 0.0
    acc_c = c["accepted"] / c["trials"] if c["trials"] else 0.0
    rel = lambda a, b: abs(a - b) / abs(b) if b else abs(a - b)
    return {"reference": "C oracle (corrected-mode restatement of subsweep.h / shiftCells.h)",
            "sweeps": sweeps, "first_sweep": sweep0, "energy_start": e0,
            "energy_gpu": e_gpu, "energy_cpu": e_cpu, "energy_rel_err": rel(e_gpu, e_cpu),
            "acceptance_gpu": acc_g, "acceptance_cpu": acc_c, "acceptance_rel_err": rel(acc_g, acc_c),
            "counters_equal": g == c, "state_bitwise_equal": same}


def traffic_from_profile() -> dict | None:
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            return json.load(f)
    except Exception:
        return None


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cps", type=int, default=128)
    ap.add_argument("--atoms", type=int, default=10_000_000)
    ap.add_argument("--cpu-sweeps", type=int, default=1)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", action="store_true", help="replay the timed sweeps as one hipGraph")
    ap.add_argument("--no-events", action="store_true",
                    help="no per-launch HIP events in the timed region (no roofline; overhead check)")
    ap.add_argument("--slab", action="store_true", help="use the z-slab/halo path even with one rank")
    ap.add_argument("--slab-driver", choices=["c", "python"], default="c",
                    help="multi-GPU driver: the C slab driver with RCCL (product) or the Python schedule "
                         "over torch.distributed")
    ap.add_argument("--self-rccl", action="store_true",
                    help="one rank with --slab: halos through a one-rank RCCL communicator (rehearsal)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling (BASELINE config 4): one cps^3 box of --atoms particles split into "
                         "world z-slabs of cps/world planes (default: weak, cps^3 and --atoms per GPU)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import pmc_amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} != --gpus {args.gpus}", file=sys.stderr)
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    stream = torch.cuda.Stream()
    cps = args.cps

    def barrier():
        if world > 1:
            dist.barrier()

    slab = world > 1 or args.slab
    nz_local = cps // world if args.strong else cps
    # weak: a lattice of --atoms per cps^3 of slab; strong: ONE lattice of --atoms over the whole
    # box, each rank keeping its planes (the 1-GPU config 3 state, split)
    atoms_local = args.atoms * nz_local // cps
    if slab and (nz_local % 2 or nz_local < 2):
        raise SystemExit(f"slab thickness {nz_local} must be even and >= 2")
    events = []      # (kind, start, end) HIP events on the kernels' stream

    def timer(kind, fn, record, on=None):
        """HIP events around one launch, on the stream it is launched on (default: the kernels')."""
        if not record or args.no_events:
            return fn()
        st = on if on is not None else stream
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        events.append((kind, a, b))

    if not slab:
        sim = pmc_amd.PmcContext(cps, stream=stream.cuda_stream)
        sim.init_lattice(args.atoms)
        from pmc_amd.plan import sweep_plan
        plans = {}

        def one_sweep(s, record):
            if s not in plans:
                plans[s] = sweep_plan(1234, s, 2.5)
            for colour in plans[s][0]:
                sim.phase(colour, s)
            sim.shift(s)

        def finish():
            pass
        cps_z = cps
    elif args.slab_driver == "c":
        # the product multi-GPU path: sweep schedule + RCCL halo exchange in C (pmc_slab_*)
        from pmc_amd.slab import SlabDriver
        drv = SlabDriver(cps=cps, nz_local=nz_local, rank=rank, world=world, stream=stream,
                         atoms_per_rank=0 if args.strong else atoms_local,
                         atoms_total=args.atoms if args.strong else 0, use_rccl=world > 1 or args.self_rccl)
        sim = drv.ctx

        def one_sweep(s, record):
            drv.sweep(s)

        finish = drv.finish
        cps_z = nz_local * world
    else:
        # the same schedule in Python over torch.distributed (comparison)
        from pmc_amd.slab import SlabSimulation
        sim_s = SlabSimulation.create(cps=cps, nz_local=nz_local, rank=rank, world=world, stream=stream,
                                      atoms_per_rank=0 if args.strong else atoms_local,
                                      atoms_total=args.atoms if args.strong else 0)
        sim = sim_s.ctx

        def one_sweep(s, record):
            sim_s.sweep(s, timer=lambda kind, fn, on=None: timer(kind, fn, record, on))

        finish = sim_s.finish
        cps_z = nz_local * world
    c_slab = slab and args.slab_driver == "c"

    # warmup
    for s in range(args.warmup):
        one_sweep(s, False)
    finish()
    torch.cuda.synchronize()
    sim.stats(reset=True)
    # algorithmic bytes from the state at the start of the timed region
    disk_h, n_h = sim.copy_out()
    plane = cps * cps
    lo = plane if slab else 0
    nzl = nz_local if slab else cps
    n_owned = n_h[lo:lo + plane * nzl].astype(np.int64)
    if not slab:
        stencil = stencil_counts(n_owned, (cps, cps, cps))
    else:
        ext = n_h.astype(np.int64).reshape(nzl + 2, cps, cps)
        g = ext
        s = np.zeros((nzl, cps, cps), np.int64)
        for dz in (-1, 0, 1):
            sub = g[1 + dz:1 + dz + nzl]
            for dy in (-1, 0, 1):
                for dx in (-1, 0, 1):
                    s += np.roll(sub, shift=(-dy, -dx), axis=(1, 2))
        stencil = s.reshape(-1)
    abytes = algorithmic_bytes_per_sweep(n_owned, stencil)
    e_start = sim.energy()      # cell-list energy of the state the timed region starts from

    c_events = not slab or c_slab      # kernel launches from C: events on their dispatch packets
    if c_events:
        sim.timing(not args.no_events)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    first = args.warmup
    if args.graph and not slab:
        sim.run_graph(first, args.steps)
    else:
        for k in range(args.steps):
            one_sweep(first + k, True)
        finish()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    st = sim.stats()
    trials_local = st["trials"]
    # kernel time of one colour phase = sum of its launches (the slab path splits a phase into the
    # interior and the two boundary planes); 8 phases per sweep
    phase_total_ms = sum(a.elapsed_time(b) for kind, a, b in events if kind == "phase")
    shift_total_ms = sum(a.elapsed_time(b) for kind, a, b in events if kind == "shift")
    n_phases = 8 * args.steps if events else 0
    if c_events:
        tm = sim.timing(False)
        phase_total_ms, shift_total_ms = tm["subsweep_ms"], tm["shift_ms"]
        n_phases = 8 * args.steps if tm["n_subsweep"] else 0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tr = torch.tensor([trials_local], dtype=torch.int64, device="cuda")
        dist.all_reduce(tr)
        trials_total = int(tr.item())
    else:
        trials_total = trials_local
    flags = sim.error_flags()
    value = trials_total / elapsed
    # energy bookkeeping over the timed sweeps: E_start + sum of accepted dE (fixed point 2^-32,
    # order-independent) against a direct cell-list evaluation of the final state
    e_end = sim.energy()
    de_timed = st["de_fixed"] / 2.0 ** 32
    if world > 1:   # slab energies count boundary pairs half on each side: the sum is the box's
        ev = torch.tensor([e_start, e_end, de_timed], dtype=torch.float64, device="cuda")
        dist.all_reduce(ev)
        e_start, e_end, de_timed = (float(v) for v in ev.tolist())

    if rank == 0:
        avg_launch_s = (phase_total_ms / n_phases * 1e-3) if n_phases else None
        achieved = (abytes["subsweep_launch"] / avg_launch_s / 1e9) if avg_launch_s else None
        traffic = traffic_from_profile()
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic.get("subsweep_bytes_per_launch") if traffic else None,
                "kernel": "k_subsweep<16> (one colour phase)",
                "launch_ms": avg_launch_s * 1e3 if avg_launch_s else None,
                "shift_ms": shift_total_ms / args.steps if n_phases else None,
                "algorithmic_bytes_per_launch": abytes["subsweep_launch"]}
        cpu = None
        parity = None
        if not args.no_cpu_baseline and not slab:
            try:
                thr = max(1, min(args.cpu_threads, os.cpu_count() or 1))
                cpu, ost = cpu_baseline(disk_h, n_h, cps, args.cpu_sweeps, thr, first)
                parity = parity_leg(sim, one_sweep, disk_h, n_h, first, args.cpu_sweeps, e_start, ost)
            except Exception as e:  # the baseline is reported, never the measured value
                cpu = {"error": repr(e)}
        sweeps_per_s = args.steps / elapsed
        out = {
            "metric": "MC trial-moves/s (whole node)",
            "value": value,
            "unit": "trial-moves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (reference simple-cubic lattice start, Philox seed 1234)",
            "config": {"workload": (f"{cps}^3 cells x {args.atoms:.0e} particles in total" if args.strong else
                                    f"{cps}x{cps}x{nzl} cells x {atoms_local:.0e} particles per GPU") +
                                   f", full checkerboard sweep (8 colour phases + shiftCells), box {cps}x{cps}x{cps_z}",
                       "cells_per_gpu": cps * cps * nzl, "particles_per_gpu": atoms_local, "n_moves": 10,
                       "nmax": 16, "beta": 0.3, "sigma": 0.5, "w": 2.5,
                       "parallelism": (f"z-slab x{world}, {nzl} planes per rank, halo planes over "
                                       + ("RCCL (C driver)" if c_slab and (world > 1 or args.self_rccl) else
                                          "local copies (C driver)" if c_slab else "torch.distributed"))
                                      if slab else "single GPU"},
            "sweeps_per_s": sweeps_per_s,
            "acceptance": st["accepted"] / st["trials"] if st["trials"] else None,
            "energy": {"start": e_start, "end": e_end, "start_plus_sum_dE": e_start + de_timed,
                       "per_particle_end": e_end / (atoms_local * world),
                       "bookkeeping_rel_err": abs(e_start + de_timed - e_end) / abs(e_end) if e_end else None,
                       "particles": atoms_local * world},
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
