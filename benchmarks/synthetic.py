#!/usr/bin/env python3
"""Synthetic throughput benchmark -- the grace_amd counterpart of the reference harness
/root/reference/examples/torch/pytorch_synthetic_benchmark.py (same flags, same output lines:
"Img/sec per GPU" and "Total img/sec on N GPU(s)" with a 1.96-sigma band over iterations).

Unlike the reference (which parses --compression flags it then ignores in dawn.py, and
hard-codes the GRACE object in the synthetic benchmark), every GRACE flag here is wired into
``grace_from_params``.

    python benchmarks/synthetic.py --model resnet50 --compressor topk --compress-ratio 0.01 \
        --memory residual --communicator allgather
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/synthetic.py ...
"""
import argparse
import json
import os
import sys
import timeit

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from grace_amd import grace_from_params  # noqa: E402
from grace_amd.parallel import DistributedOptimizer, broadcast_optimizer_state, broadcast_parameters  # noqa: E402
from grace_amd.parallel.launch import init_distributed  # noqa: E402
from grace_amd.utils.workloads import WORKLOADS, build_model  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--workload", default="resnet50_topk", choices=sorted(WORKLOADS))
    ap.add_argument("--model", default=None, help="override the workload's model")
    ap.add_argument("--batch-size", type=int, default=0)
    ap.add_argument("--num-warmup-batches", type=int, default=10)
    ap.add_argument("--num-batches-per-iter", type=int, default=10)
    ap.add_argument("--num-iters", type=int, default=10)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--momentum", type=float, default=0.5)
    ap.add_argument("--compressor", default=None)
    ap.add_argument("--memory", default=None)
    ap.add_argument("--communicator", default=None)
    ap.add_argument("--compress-ratio", type=float, default=None)
    ap.add_argument("--quantum-num", type=int, default=None)
    ap.add_argument("--compress-rank", type=int, default=None)
    ap.add_argument("--threshold", type=float, default=None)
    ap.add_argument("--efsgd-lr", type=float, default=None)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--fp32", action="store_true", help="disable bf16 autocast")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()

    rank, world, dev = init_distributed()
    w = WORKLOADS[a.workload]
    if a.model:
        w = type(w)(**{**w.__dict__, "model": a.model})
    params = dict(w.grace)
    for k, v in (("compressor", a.compressor), ("memory", a.memory), ("communicator", a.communicator),
                 ("compress_ratio", a.compress_ratio), ("quantum_num", a.quantum_num),
                 ("compress_rank", a.compress_rank), ("threshold", a.threshold), ("lr", a.efsgd_lr)):
        if v is not None:
            params[k] = v
    params["world_size"] = world
    torch.backends.cudnn.benchmark = True
    model = build_model(w, dev)
    batch = a.batch_size or w.batch
    opt = torch.optim.SGD(model.parameters(), lr=a.lr * world, momentum=a.momentum)
    broadcast_parameters(model.state_dict(), root_rank=0)
    broadcast_optimizer_state(opt, root_rank=0)
    opt = DistributedOptimizer(opt, grace_from_params(params), named_parameters=model.named_parameters(),
                               bucket_cap_mb=a.bucket_mb)
    data = w.make_batch(batch, dev)

    def step():
        opt.zero_grad()
        with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=not a.fp32 and dev.type == "cuda"):
            loss = w.loss(model, data)
        loss.backward()
        opt.step()
        if dev.type == "cuda":
            torch.cuda.synchronize()

    def log(s):
        if rank == 0:
            print(s, flush=True)

    log(f"Model: {w.model}  Batch size: {batch}  GRACE: {params}  Number of GPUs: {world}")
    log("Running warmup...")
    timeit.timeit(step, number=a.num_warmup_batches)
    log("Running benchmark...")
    rates = []
    for i in range(a.num_iters):
        t = timeit.timeit(step, number=a.num_batches_per_iter)
        r = w.samples_per_batch(batch) * a.num_batches_per_iter / t
        log(f"Iter #{i}: {r:.1f} {w.unit}/sec per GPU")
        rates.append(r)
    m, c = float(np.mean(rates)), 1.96 * float(np.std(rates))
    log(f"{w.unit.capitalize()}/sec per GPU: {m:.1f} +-{c:.1f}")
    log(f"Total {w.unit}/sec on {world} GPU(s): {world * m:.1f} +-{world * c:.1f}")
    if a.json and rank == 0:
        print(json.dumps({"workload": a.workload, "params": params, "per_gpu": m, "total": world * m, "ci": c}))


if __name__ == "__main__":
    main()
