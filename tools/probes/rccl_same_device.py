"""Probe: does RCCL accept two ranks on ONE GPU (torch.distributed nccl backend)?  And does
hipIpcGetMemHandle/hipIpcOpenMemHandle work between two processes on one device?
Run: python tools/probes/rccl_same_device.py  (spawns 2 processes itself)"""
import os
import sys
import ctypes as C


def child(rank: int, world: int, port: int, mode: str):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    if mode == "rccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
        t = torch.full((4,), float(rank + 1), device="cuda")
        try:
            dist.all_reduce(t)
            torch.cuda.synchronize()
            print(f"rank {rank}: rccl same-device all_reduce OK {t.tolist()}", flush=True)
        except Exception as e:
            print(f"rank {rank}: rccl same-device FAILED: {e!r}"[:400], flush=True)
        dist.destroy_process_group()
        return
    # ipc: gloo for the handle exchange
    dist.init_process_group("gloo")
    hip = C.CDLL("libamdhip64.so")

    class H(C.Structure):
        _fields_ = [("b", C.c_ubyte * 64)]
    hip.hipIpcGetMemHandle.argtypes = [C.POINTER(H), C.c_void_p]
    hip.hipIpcOpenMemHandle.argtypes = [C.POINTER(C.c_void_p), H, C.c_uint]
    buf = torch.full((1024,), float(rank + 10), device="cuda")
    torch.cuda.synchronize()
    h = H()
    rc = hip.hipIpcGetMemHandle(C.byref(h), C.c_void_p(buf.data_ptr()))
    print(f"rank {rank}: get rc {rc}", flush=True)
    mine = torch.tensor(list(bytes(h.b)), dtype=torch.uint8)
    allh = [torch.zeros(64, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(allh, mine)
    peer = (rank + 1) % world
    ph = H()
    ph.b = (C.c_ubyte * 64).from_buffer_copy(bytes(allh[peer].numpy().tobytes()))
    ptr = C.c_void_p()
    rc2 = hip.hipIpcOpenMemHandle(C.byref(ptr), ph, C.c_uint(1))
    print(f"rank {rank}: open rc {rc2}", flush=True)
    out = torch.zeros(1024, device="cuda")
    rc3 = -1
    if rc2 == 0:
        rc3 = hip.hipMemcpy(C.c_void_p(out.data_ptr()), ptr, C.c_size_t(4096), 3)
    torch.cuda.synchronize()
    print(f"rank {rank}: get {rc} open {rc2} copy {rc3} peer value {out[0].item()} (want {peer + 10})", flush=True)
    dist.barrier()
    if rc2 == 0:
        hip.hipIpcCloseMemHandle(ptr)
    dist.destroy_process_group()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
        sys.exit(0)
    import subprocess
    for mode, port in (("ipc", 29611),):
        ps = [subprocess.Popen([sys.executable, __file__, "child", str(r), "2", str(port), mode]) for r in range(2)]
        try:
            rcs = [p.wait(timeout=120) for p in ps]
        except subprocess.TimeoutExpired:
            for p in ps:
                p.kill()
            rcs = "timeout"
        print(f"mode {mode}: exit codes {rcs}", flush=True)
