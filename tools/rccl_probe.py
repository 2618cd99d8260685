"""Diagnose the native RCCL runtime lifecycle in isolation (one variant per process)."""
import faulthandler
import os
import sys

import torch
import torch.distributed as dist

faulthandler.enable(all_threads=True)
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
variant = sys.argv[1]
os.environ["MASTER_ADDR"] = "127.0.0.1"
os.environ["MASTER_PORT"] = str(29500 + hash(variant) % 200)
from grace_amd.ops import _native  # noqa: E402

C = _native.lib()


def log(*a):
    print(variant, *a, flush=True)


if variant == "F":  # the Python wrapper, step by step (mirrors tests/test_gpu_a_comm.py)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from grace_amd.parallel.native_comm import RcclComm

    c = RcclComm.from_process_group()
    log("wrapper up")
    t = torch.arange(10, dtype=torch.float32, device="cuda")
    w = c.all_reduce(t, async_op=True)
    log("ar issued")
    w.wait()
    log("ar waited")
    out = torch.empty(10, device="cuda")
    c.all_gather_into(out, t).wait()
    log("ag")
    c.broadcast(t, 0).wait()
    log("bc")
    torch.cuda.synchronize()
    log("synced")
    c.check()
    log("checked")
    del c, w
    log("deleted")
    dist.destroy_process_group()
    log("exiting")
    sys.exit(0)
if variant in ("A", "C", "D", "E"):
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    log("pg up")
uid = C.rccl_unique_id()
c = C.RcclComm(0, 1, uid, 0, True)
log("comm up")
if variant in ("A", "B", "D", "E"):
    t = torch.arange(10., device="cuda")
    w = c.all_reduce(t, "sum")
    w.wait()
    torch.cuda.synchronize()
    log("op ok")
    del w
if variant == "E":
    s = torch.cuda.ExternalStream(c.stream_ptr)
    t2 = torch.ones(5, device="cuda")
    t2.record_stream(s)
    del t2
    torch.cuda.synchronize()
    log("record_stream ok")
del c
log("comm destroyed")
if dist.is_initialized():
    dist.destroy_process_group()
    log("pg destroyed")
if variant == "D":
    os._exit(0)
log("exiting")
