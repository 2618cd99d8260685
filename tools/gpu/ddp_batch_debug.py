"""Which DDP-managed weight gradients take the batched-copy path (ops/wgrad.py ddp_batched) on the
ResNet-50 DDP surface, per eager step, and why the others do not."""
import collections
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from grace_amd import grace_from_params  # noqa: E402
from grace_amd.ops import wgrad as W  # noqa: E402
from grace_amd.parallel import GraceHookState, grace_comm_hook  # noqa: E402
from grace_amd.utils.workloads import WORKLOADS, build_model  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    w = WORKLOADS["resnet50_topk"]
    model = build_model(w, dev)
    ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0], bucket_cap_mb=128,
                                                    gradient_as_bucket_view=True, broadcast_buffers=False)
    ddp.register_comm_hook(GraceHookState(grace_from_params(dict(w.grace, world_size=1)), model=ddp), grace_comm_hook)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.5)
    data = w.make_batch(w.batch, dev)
    data = (data[0].contiguous(memory_format=torch.channels_last),) + tuple(data[1:])
    stats = collections.Counter()
    real = W.ddp_batched

    def spy(d, weight):
        out = real(d, weight)
        if out is not d:
            stats["batched"] += 1
        else:
            tgt = W.grad_target(weight)
            why = ("no_ddp" if not getattr(weight, "_grace_ddp", False) else
                   "unstable" if not getattr(weight, "_grace_view_stable", False) else
                   "no_target" if tgt is None else
                   f"layout {tuple(d.shape)} {d.stride()} vs {tgt.stride()}")
            stats[why] += 1
        return out

    W.ddp_batched = spy
    for it in range(6):
        stats.clear()
        opt.zero_grad(set_to_none=True)
        w.loss(ddp, data).backward()
        opt.step()
        torch.cuda.synchronize()
        print(it, dict(stats), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
