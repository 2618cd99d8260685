"""torch.profiler view of one eager ResNet-50 Top-K training step: which aten ops launch the
remaining small kernels (copies, adds, fills)."""
import os, sys, torch, torch.nn.functional as F
sys.path.insert(0, os.getcwd())
from torch.profiler import profile, ProfilerActivity
from grace_amd import grace_from_params
from grace_amd.parallel import DistributedOptimizer
from grace_amd.parallel.precision import BF16Weights
from grace_amd.models import resnet50
dev = torch.device("cuda", 0)
torch.backends.cudnn.benchmark = True
model = resnet50().to(dev).to(memory_format=torch.channels_last)
w = BF16Weights(model)
named = list(w.named_master_parameters(model))
grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.01, "memory": "residual", "communicator": "allgather", "world_size": 1})
opt = DistributedOptimizer(torch.optim.SGD([p for _, p in named], lr=0.01, momentum=0.5), grc, named_parameters=named, weights=w, overlap=False)
x = torch.randn(32, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (32,), device=dev)
def step():
    opt.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        loss = F.cross_entropy(model(x), y)
    loss.backward()
    opt.step()
for _ in range(5):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=45, max_name_column_width=40, max_shapes_column_width=70))
