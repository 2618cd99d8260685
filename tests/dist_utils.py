"""Run a function on W CPU ranks (gloo over 127.0.0.1) and propagate failures."""
import os
import socket
import tempfile
import traceback

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, args, errfile):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        fn(rank, world, *args)
        dist.barrier()
    except Exception:  # pragma: no cover - reported to the parent
        with open(f"{errfile}.{rank}", "w") as f:
            f.write(traceback.format_exc())
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_distributed(fn, world: int, *args, timeout: int = 240):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        errfile = os.path.join(d, "err")
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, errfile)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout)
        errs = []
        for r, p in enumerate(procs):
            if p.is_alive():
                p.kill()
                errs.append(f"rank {r} timed out")
            elif p.exitcode != 0:
                path = f"{errfile}.{r}"
                errs.append(open(path).read() if os.path.exists(path) else f"rank {r} exit {p.exitcode}")
        if errs:
            raise AssertionError("\n".join(errs))
