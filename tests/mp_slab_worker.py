"""One rank PROCESS of the product slab driver over the IPC transport (tests/test_gpu_multiprocess.py).

Started by the test with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment; every
rank uses GPU 0 (several processes on one GPU: RCCL refuses that, the IPC transport does not).
Control collectives over gloo.  Writes rank<r>.npz (owned planes, counters, energies, error flags,
the whole-box observables) into the output directory.

  python tests/mp_slab_worker.py OUTDIR CPS CPS_Y CPS_Z ATOMS FLAGS HALO FIRST COUNT [restart]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "parallel-monte-carlo_amd"))


def main() -> int:
    outdir = sys.argv[1]
    cps, cps_y, cps_z, atoms, flags, halo, first, count = (int(v) for v in sys.argv[2:10])
    restart = len(sys.argv) > 10 and sys.argv[10] == "restart"
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import numpy as np
    import pmc_amd
    import torch
    import torch.distributed as dist
    from pmc_amd.slab import SlabDriver

    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    nz = cps_z // world
    d = SlabDriver(cps=cps, cps_y=cps_y, nz_local=nz, rank=rank, world=world, atoms_total=atoms, flags=flags,
                   halo=halo, transport="ipc")
    assert d.transport == "ipc", d.transport
    if restart:
        # half the window, a per-rank snapshot, a FRESH driver (new IPC mappings) restored from it
        half = count // 2
        d.run(first, half)
        path = os.path.join(outdir, f"rank{rank}.pmcsnap")
        d.ctx.save_snapshot(path, first + half)
        d.ctx.close()
        dist.barrier()
        d = SlabDriver(cps=cps, cps_y=cps_y, nz_local=nz, rank=rank, world=world, flags=flags, halo=halo,
                       transport="ipc")
        nxt = d.ctx.load_snapshot(path)
        d.ctx.slab_exchange()
        d.run(nxt, first + count - nxt)
    else:
        d.run(first, count)
    obs, e_all = d.ctx.slab_observables(True)
    own_d, own_n = d.owned()
    st = d.ctx.stats()
    e = d.ctx.energy()
    fl = d.ctx.error_flags()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), disk=own_d, n=own_n)
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump({"stats": st, "energy": e, "flags": fl, "obs": obs, "e_all": e_all}, f)
    dist.barrier()          # no rank unmaps its buffers while a peer may still pull from them
    d.ctx.close()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
