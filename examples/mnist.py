#!/usr/bin/env python3
"""MNIST with the Horovod-style optimizer wrapper -- counterpart of
/root/reference/examples/torch/pytorch_mnist.py (2-conv Net, per-rank data shards,
``DistributedOptimizer(optimizer, grace, named_parameters)``, metric averaging by all-reduce).

Data: ``--data-dir`` containing the raw IDX files (train-images-idx3-ubyte[.gz],
train-labels-idx1-ubyte[.gz]); the reference ships only the label files
(examples/torch/data-*/MNIST/raw, images are listed as missing blobs), so without the images a
synthetic MNIST-shaped set is used.

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/mnist.py --compressor topk
"""
import argparse
import gzip
import os
import struct
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from grace_amd import grace_from_params  # noqa: E402
from grace_amd.parallel import DistributedOptimizer, broadcast_optimizer_state, broadcast_parameters  # noqa: E402
from grace_amd.parallel.launch import init_distributed  # noqa: E402


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 10, 5)
        self.conv2 = nn.Conv2d(10, 20, 5)
        self.drop = nn.Dropout2d()
        self.fc1 = nn.Linear(320, 50)
        self.fc2 = nn.Linear(50, 10)

    def forward(self, x):
        x = F.relu(F.max_pool2d(self.conv1(x), 2))
        x = F.relu(F.max_pool2d(self.drop(self.conv2(x)), 2))
        x = F.dropout(F.relu(self.fc1(x.flatten(1))), training=self.training)
        return F.log_softmax(self.fc2(x), dim=1)


def _idx(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        magic = struct.unpack(">I", f.read(4))[0]
        nd = magic & 0xFF
        dims = struct.unpack(">" + "I" * nd, f.read(4 * nd))
        return np.frombuffer(f.read(), dtype=np.uint8).reshape(dims)


def load(args):
    for suffix in ("", ".gz"):
        xi = os.path.join(args.data_dir, "train-images-idx3-ubyte" + suffix)
        yi = os.path.join(args.data_dir, "train-labels-idx1-ubyte" + suffix)
        if args.data_dir and os.path.exists(xi) and os.path.exists(yi):
            return _idx(xi).astype(np.float32) / 255.0, _idx(yi).astype(np.int64)
    g = np.random.default_rng(0)
    return g.random((args.synthetic_size, 28, 28), dtype=np.float32), g.integers(0, 10, args.synthetic_size)


def metric_average(val, world):
    t = torch.tensor([val], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t.to("cuda" if torch.cuda.is_available() else "cpu"))
    return float(t.item()) / max(world, 1) if world > 1 else val


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--momentum", type=float, default=0.5)
    ap.add_argument("--data-dir", default="")
    ap.add_argument("--synthetic-size", type=int, default=6000)
    ap.add_argument("--compressor", default="none")
    ap.add_argument("--memory", default="none")
    ap.add_argument("--communicator", default="allgather")
    ap.add_argument("--compress-ratio", type=float, default=0.01)
    args = ap.parse_args()

    rank, world, dev = init_distributed()
    x, y = load(args)
    x, y = torch.tensor(x[rank::world]).unsqueeze(1).to(dev), torch.tensor(y[rank::world]).to(dev)
    torch.manual_seed(42)
    model = Net().to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr * world, momentum=args.momentum)
    broadcast_parameters(model.state_dict(), root_rank=0)
    broadcast_optimizer_state(opt, root_rank=0)
    grc = grace_from_params({"compressor": args.compressor, "memory": args.memory, "communicator": args.communicator,
                             "compress_ratio": args.compress_ratio, "world_size": world})
    opt = DistributedOptimizer(opt, grc, named_parameters=model.named_parameters())
    for epoch in range(args.epochs):
        model.train()
        perm = torch.randperm(x.shape[0], device=dev)
        for s in range(x.shape[0] // args.batch_size):
            idx = perm[s * args.batch_size:(s + 1) * args.batch_size]
            opt.zero_grad()
            loss = F.nll_loss(model(x[idx]), y[idx])
            loss.backward()
            opt.step()
        model.eval()
        with torch.no_grad():
            out = model(x[:2000])
            acc = (out.argmax(1) == y[:2000]).float().mean().item()
        acc = metric_average(acc, world)
        if rank == 0:
            print(f"epoch {epoch + 1}: loss {loss.item():.4f} accuracy {acc:.4f}", flush=True)


if __name__ == "__main__":
    main()
