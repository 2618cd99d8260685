"""Host-side cProfile of eager ResNet-50 Top-K steps through the DDP comm hook vs the engine."""
import cProfile
import os
import pstats
import sys

import torch
import torch.distributed as dist
import torch.nn.functional as F

sys.path.insert(0, os.getcwd())
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
from grace_amd import grace_from_params  # noqa: E402
from grace_amd.models import resnet50  # noqa: E402
from grace_amd.parallel import FusedSGD, GraceHookState, grace_comm_hook  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
torch.backends.cudnn.benchmark = True
model = resnet50().to(dev).to(memory_format=torch.channels_last)
grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.01, "memory": "residual",
                         "communicator": "allgather", "world_size": 1})
ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[0], bucket_cap_mb=128, gradient_as_bucket_view=True)
ddp.register_comm_hook(GraceHookState(grc), grace_comm_hook)
opt = FusedSGD(list(model.parameters()), lr=0.01, momentum=0.5)
x = torch.randn(32, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (32,), device=dev)


def step():
    opt.zero_grad(set_to_none=True)
    F.cross_entropy(ddp(x), y).backward()
    opt.step()


for _ in range(8):
    step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    step()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(22)
dist.destroy_process_group()
