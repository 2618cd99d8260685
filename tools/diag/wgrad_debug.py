"""Which part of ops/wgrad.py changes ResNet-50 gradients? side stream x dgrad autotune x sync."""
import torch
import torch.nn.functional as F

from grace_amd.models import resnet50
from grace_amd.ops import wgrad

torch.manual_seed(0)
model = resnet50().cuda().to(memory_format=torch.channels_last)
x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (4,), device="cuda")
names = [n for n, _ in model.named_parameters()]


def grads(side, dg, sync):
    wgrad.set_enabled(side)
    wgrad._DG_AUTO = dg
    for p in model.parameters():
        p.grad = None
    F.cross_entropy(model(x), y).backward()
    if sync:
        torch.cuda.synchronize()
    return [p.grad.detach().clone() for p in model.parameters()]


grads(False, False, True)
ref = grads(False, False, True)
for side, dg, sync in [(False, False, True), (False, True, True), (True, False, True), (True, False, False),
                       (True, True, True)]:
    got = grads(side, dg, sync)
    torch.cuda.synchronize()
    bad = [(n, float((a - b).abs().max() / (b.abs().max() + 1e-12))) for n, a, b in zip(names, got, ref)]
    worst = sorted(bad, key=lambda t: -t[1])[:4]
    print(f"side={side} dgrad_auto={dg} sync={sync}: worst rel {worst}", flush=True)
print("DGRAD", wgrad.dgrad_table(), flush=True)
