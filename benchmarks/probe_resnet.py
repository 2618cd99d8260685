"""Probe: ResNet-50 batch-32 training-step time on one MI355X under several execution modes.

Used to pick the compute configuration for bench.py (the framework's own gradient path is
added on top).  Prints one JSON line per variant.
"""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd.models.resnet import resnet50  # noqa: E402

torch.backends.cudnn.benchmark = True


def run(variant, steps=20, warmup=8, bs=32):
    torch.manual_seed(0)
    model = resnet50().cuda()
    cl = "cl" in variant
    amp = "bf16" in variant
    if cl:
        model = model.to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.5)
    x = torch.randn(bs, 3, 224, 224, device="cuda")
    if cl:
        x = x.to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (bs,), device="cuda")

    def step():
        opt.zero_grad(set_to_none=False)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = model(x)
            loss = F.cross_entropy(out, y)
        loss.backward()
        opt.step()

    if "graph" in variant:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        fn = g.replay
        for _ in range(3):
            fn()
    else:
        fn = step
        for _ in range(warmup):
            fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return {"variant": variant, "ms_per_step": dt * 1e3, "img_s": bs / dt}


if __name__ == "__main__":
    variants = sys.argv[1:] or ["fp32", "bf16", "bf16_cl", "fp32_cl", "bf16_cl_graph"]
    for v in variants:
        try:
            print(json.dumps(run(v)), flush=True)
        except Exception as e:  # keep probing other variants
            print(json.dumps({"variant": v, "error": repr(e)[:400]}), flush=True)
