"""Which ops issue the small FillFunctor (zero) kernels of the fp32 ResNet-50 step?  torch.profiler
over one eager step (after warm-up): every aten::fill_/zero_ with its parent op chain."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from grace_amd import grace_from_params  # noqa: E402
from grace_amd.models import resnet50  # noqa: E402
from grace_amd.parallel import DistributedOptimizer, FusedSGD  # noqa: E402

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda", 0)
m = resnet50().to(dev).to(memory_format=torch.channels_last)
grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.01, "memory": "residual",
                         "communicator": "allgather", "world_size": 1})
opt = DistributedOptimizer(FusedSGD(list(m.parameters()), lr=0.01, momentum=0.5), grc,
                           named_parameters=list(m.named_parameters()), overlap=False)
x = torch.randn(32, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (32,), device=dev)


def step():
    opt.zero_grad(set_to_none=True)
    loss = F.cross_entropy(m(x), y)
    loss.backward()
    opt.step()


for _ in range(4):
    step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
evs = prof.events()
for e in evs:
    if e.name in ("aten::fill_", "aten::zero_", "aten::zeros", "aten::zeros_like", "aten::full"):
        par = []
        p = e.cpu_parent
        while p is not None and len(par) < 5:
            par.append(p.name)
            p = p.cpu_parent
        st = [s for s in (e.stack or []) if "grace_amd" in s or "torch/autograd" in s][:3]
        print(e.name, e.input_shapes[:1], "<-", " <- ".join(par), "|", st)
