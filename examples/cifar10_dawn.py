#!/usr/bin/env python3
"""CIFAR-10 DAWNBench-style training with GRACE -- counterpart of the reference's
torch.distributed example (/root/reference/examples/dist/CIFAR10-dawndist/dawn.py, core.py,
torch_backend.py): ResNet-9-style network, batch 512, 24 epochs, piecewise-linear LR, Nesterov
SGD, and the per-parameter ``grc.step(p.grad, name)`` loop of core.py:203-206.

Fixes vs the reference example: the compression flags are actually wired into
``grace_from_params`` (dawn.py:124-127 hard-codes none/none/allreduce), parameters are
broadcast from rank 0 at start (the reference never does), and data is sharded per rank.

Data: ``--data path.npz`` with arrays x_train [N,32,32,3] uint8 and y_train [N]; without it a
synthetic CIFAR-shaped set is used (no network access for the real dataset).

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/cifar10_dawn.py \
        --compressor topk --compress-ratio 0.01 --memory residual --communicator allgather
    python examples/cifar10_dawn.py --epochs 1 --synthetic-size 2048     # CPU smoke (gloo-free)
"""
import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from grace_amd import grace_from_params  # noqa: E402
from grace_amd.models.resnet9 import ResNet9  # noqa: E402
from grace_amd.parallel import DistributedOptimizer, broadcast_parameters  # noqa: E402
from grace_amd.parallel.launch import init_distributed  # noqa: E402


def piecewise_linear(knots, vals):
    return lambda t: float(np.interp([t], knots, vals)[0])


def load_data(args, rank, world):
    if args.data:
        d = np.load(args.data, allow_pickle=False)
        x, y = d["x_train"], d["y_train"]
    else:
        g = np.random.default_rng(0)
        x = g.integers(0, 256, (args.synthetic_size, 32, 32, 3), dtype=np.uint8)
        y = g.integers(0, 10, (args.synthetic_size,))
    x = x[rank::world]
    y = y[rank::world]
    mean = np.array([125.31, 122.95, 113.87], dtype=np.float32)
    std = np.array([62.99, 62.09, 66.70], dtype=np.float32)
    xt = torch.tensor((x.astype(np.float32) - mean) / std).permute(0, 3, 1, 2).contiguous()
    return xt, torch.tensor(y, dtype=torch.long)


def augment(x):
    # random crop with 4-pixel padding + horizontal flip (core.py:69-123)
    n = x.shape[0]
    xp = F.pad(x, (4, 4, 4, 4), mode="reflect")
    i, j = np.random.randint(0, 9, 2)
    x = xp[:, :, i:i + 32, j:j + 32]
    flip = torch.rand(n, device=x.device) < 0.5
    return torch.where(flip[:, None, None, None], x.flip(3), x)


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--epochs", type=int, default=24)
    ap.add_argument("--batch-size", type=int, default=512)
    ap.add_argument("--data", default="")
    ap.add_argument("--synthetic-size", type=int, default=50000)
    ap.add_argument("--compressor", default="none")
    ap.add_argument("--memory", default="none")
    ap.add_argument("--communicator", default="allreduce")
    ap.add_argument("--compress-ratio", type=float, default=0.01)
    ap.add_argument("--quantum-num", type=int, default=127)
    ap.add_argument("--threshold", type=float, default=0.01)
    ap.add_argument("--efsgd-lr", type=float, default=0.1)
    ap.add_argument("--clipping", action="store_true")
    ap.add_argument("--engine", action="store_true", help="bucketed overlapped engine instead of the per-param loop")
    ap.add_argument("--log", default="logs.tsv")
    args = ap.parse_args()

    rank, world, dev = init_distributed()
    torch.manual_seed(0)
    model = ResNet9().to(dev)
    if dev.type == "cuda":
        model = model.to(memory_format=torch.channels_last)
    broadcast_parameters(model.state_dict(), root_rank=0)
    grc = grace_from_params({"compressor": args.compressor, "memory": args.memory, "communicator": args.communicator,
                             "compress_ratio": args.compress_ratio, "quantum_num": args.quantum_num,
                             "threshold": args.threshold, "lr": args.efsgd_lr,
                             "gradient_clipping": args.clipping, "world_size": world})
    x, y = load_data(args, rank, world)
    x, y = x.to(dev), y.to(dev)
    bs = max(1, args.batch_size // world)
    steps_per_epoch = max(1, x.shape[0] // bs)
    lr_sched = piecewise_linear([0, 5, args.epochs], [0, 0.4, 0])
    base = torch.optim.SGD(model.parameters(), lr=0.0, momentum=0.9, nesterov=True, weight_decay=5e-4 * args.batch_size)
    opt = DistributedOptimizer(base, grc, named_parameters=model.named_parameters()) if args.engine else base
    names = [n for n, _ in model.named_parameters()]
    t_start = time.time()
    with open(args.log, "w") if rank == 0 else open(os.devnull, "w") as logf:
        logf.write("epoch\thours\ttrain_loss\ttrain_acc\n")
        for epoch in range(args.epochs):
            perm = torch.randperm(x.shape[0], device=dev)
            # device-side accumulation, one host read per epoch (reference StatsLogger, core.py:180-192)
            tot_loss = torch.zeros((), device=dev)
            tot_acc = torch.zeros((), device=dev)
            model.train()
            for s in range(steps_per_epoch):
                lr = lr_sched(epoch + s / steps_per_epoch) / args.batch_size
                for grp in base.param_groups:
                    grp["lr"] = lr
                idx = perm[s * bs:(s + 1) * bs]
                xb = augment(x[idx])
                if dev.type == "cuda":
                    xb = xb.contiguous(memory_format=torch.channels_last)
                with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=dev.type == "cuda"):
                    out = model(xb)
                    loss = F.cross_entropy(out.float(), y[idx], reduction="sum")
                opt.zero_grad()
                loss.backward()
                if not args.engine:
                    # per-parameter GRACE loop (reference core.py:203-206)
                    for n, p in zip(names, model.parameters()):
                        p.grad.copy_(grc.step(p.grad, n))
                opt.step()
                tot_loss += loss.detach().float()
                tot_acc += (out.argmax(1) == y[idx]).sum()
            n_seen = steps_per_epoch * bs
            tot_loss, tot_acc = float(tot_loss), float(tot_acc)
            hours = (time.time() - t_start) / 3600
            if rank == 0:
                print(f"epoch {epoch + 1:3d}  loss {tot_loss / n_seen:.4f}  acc {tot_acc / n_seen:.4f}  "
                      f"time {hours * 3600:.1f}s", flush=True)
                logf.write(f"{epoch + 1}\t{hours:.5f}\t{tot_loss / n_seen:.4f}\t{tot_acc / n_seen:.4f}\n")


if __name__ == "__main__":
    main()
