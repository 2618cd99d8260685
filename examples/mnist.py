#!/usr/bin/env python3
"""MNIST with the Horovod-style optimizer wrapper -- counterpart of
/root/reference/examples/torch/pytorch_mnist.py (2-conv Net, per-rank data shards,
``DistributedOptimizer(optimizer, grace, named_parameters)``, metric averaging by all-reduce).

Data: the reference ships only the MNIST test images (examples/torch/data-*/MNIST/raw/
t10k-images-idx3-ubyte.gz + labels; the training images are missing blobs).  This example trains
on those 10 000 real images, split 8 000 train / 2 000 held-out test (a copy lives in
tests/fixtures/mnist; ``--data-dir`` points elsewhere).  See grace_amd/utils/mnist.py.

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/mnist.py --compressor topk \
        --memory residual --communicator allgather
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from grace_amd.parallel.launch import init_distributed  # noqa: E402
from grace_amd.utils.mnist import train_eval  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--epochs", type=int, default=10)  # pytorch_mnist.py:33
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--momentum", type=float, default=0.5)
    ap.add_argument("--data-dir", default=None)
    ap.add_argument("--compressor", default="none")
    ap.add_argument("--memory", default="none")
    ap.add_argument("--communicator", default="allgather")
    ap.add_argument("--compress-ratio", type=float, default=0.01)
    ap.add_argument("--quantum-num", type=int, default=127)
    ap.add_argument("--compress-rank", type=int, default=4)
    args = ap.parse_args()

    rank, world, dev = init_distributed()
    params = {"compressor": args.compressor, "memory": args.memory, "communicator": args.communicator,
              "compress_ratio": args.compress_ratio, "quantum_num": args.quantum_num,
              "compress_rank": args.compress_rank}
    log = (lambda m: print(m, flush=True)) if rank == 0 else None
    res = train_eval(params, epochs=args.epochs, batch=args.batch_size, lr=args.lr, momentum=args.momentum,
                     device=dev, data_dir=args.data_dir, log=log)
    if rank == 0:
        print(f"held-out: loss {res['loss']:.4f} accuracy {res['accuracy']:.4f} (W={world})", flush=True)


if __name__ == "__main__":
    main()
