"""One rank process of tests/test_gpu_multiprocess.py::test_ipc_timeout_fails_not_copies: rank 1 joins the
IPC slab driver and then stops taking part (it stays alive, so its mapped buffers stay valid); rank 0
sweeps.  Every wait of rank 0's exchanges gives up after PMC_IPC_TIMEOUT_S, copies nothing and sets
error bit 9, and pmc_slab_finish must report the failure instead of returning a torn state.

  python tests/mp_timeout_worker.py OUTDIR
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "parallel-monte-carlo_amd"))


def main() -> int:
    outdir = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch
    import torch.distributed as dist
    import pmc_amd
    from pmc_amd.slab import SlabDriver

    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    d = SlabDriver(cps=16, nz_local=16 // world, rank=rank, world=world, atoms_total=10_000, transport="ipc")
    d.ctx.synchronize()
    dist.barrier()
    res = {"transport": d.transport}
    if rank == 0:
        t0 = time.time()
        d.sweep(3)                      # rank 1 never publishes "ready": every wait times out
        try:
            d.finish()
            res["finish"] = "ok"
        except pmc_amd.PmcError as e:
            res["finish"] = str(e)
        res["seconds"] = time.time() - t0
        res["flags"] = d.ctx.error_flags()
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
            json.dump(res, f)
        d.ctx.close()                   # (its teardown's wait for rank 1 times out as well)
    dist.barrier()                      # rank 1 waits here, alive and mapped, until rank 0 is done
    if rank != 0:
        d.ctx.close()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
