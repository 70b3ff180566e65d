"""One rank process of tests/test_gpu_multiprocess.py::test_ipc_halo_verification: the IPC slab driver's
halo check (SlabDriver.verify_transport) passes after a real exchange, catches a halo that does not
equal the plane its neighbour sent, and passes again after the next exchange.

  python tests/mp_verify_worker.py OUTDIR
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "parallel-monte-carlo_amd"))


def main() -> int:
    outdir = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch
    import torch.distributed as dist
    from pmc_amd.slab import SlabDriver

    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    d = SlabDriver(cps=16, nz_local=16 // world, rank=rank, world=world, atoms_total=10_000, transport="ipc")
    res = {"transport": d.transport, "after_init": d._halos_verified()}
    if rank == 1:   # one wrong float in the halo above
        disk, n = d.ctx.copy_out()
        plane, row = 16 * 16, 3 * 16
        a = (d.g.nz + d.halo) * plane * row
        disk[a] = disk[a] + 1.0
        d.ctx.copy_in(disk, n)
    res["after_corruption"] = d._halos_verified()
    d.ctx.slab_exchange()
    res["after_exchange"] = d._halos_verified()
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    d.ctx.close()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
