"""MNIST convergence harness on the reference's own data fixture.

The reference's only correctness evidence for GRACE is training curves: the Horovod MNIST example
prints loss / accuracy per epoch (/root/reference/examples/torch/pytorch_mnist.py:156-160,
193-195) with the 2-conv ``Net`` of pytorch_mnist.py:86-102, SGD(lr 0.01 * W, momentum 0.5),
batch 64 and ``Normalize((0.1307,), (0.3081,))`` (pytorch_mnist.py:58-60, 110-111).  The
reference ships ONLY the MNIST *test* images (examples/torch/data-*/MNIST/raw/
t10k-images-idx3-ubyte.gz + labels; the training images are missing blobs), so the harness
splits those 10 000 images 8 000 train / 2 000 held-out test.  A copy of the two raw IDX files
lives in ``tests/fixtures/mnist`` (raw bytes parsed here -- nothing is unpickled).

``train_eval(params, ...)`` trains the Net with a GRACE pipeline (``grace_from_params`` dict)
through the Horovod-style ``DistributedOptimizer`` on every rank of the current process group
(or alone) and returns the held-out accuracy, so compressed + error-feedback runs can be
compared against ``NoneCompressor`` (tests/test_convergence.py, examples/mnist.py).
"""
from __future__ import annotations

import gzip
import os
import struct
from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FIXTURE_DIRS = (
    os.path.join(ROOT, "tests", "fixtures", "mnist"),
    "/root/reference/examples/torch/data-0/MNIST/raw",
)
MEAN, STD = 0.1307, 0.3081  # pytorch_mnist.py:58-60


class Net(nn.Module):
    """2-conv MNIST net of pytorch_mnist.py:86-102."""

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


def read_idx(path: str) -> np.ndarray:
    """Raw IDX file (optionally gzip'd) -> uint8 array."""
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        magic = struct.unpack(">I", f.read(4))[0]
        if magic >> 8 != 0x08:  # 0x00 0x00 0x08 <ndim>: unsigned bytes
            raise ValueError(f"{path}: not an unsigned-byte IDX file")
        nd = magic & 0xFF
        dims = struct.unpack(">" + "I" * nd, f.read(4 * nd))
        return np.frombuffer(f.read(), dtype=np.uint8).reshape(dims)


def find_fixture(data_dir: Optional[str] = None) -> Optional[str]:
    for d in ((data_dir,) if data_dir else ()) + FIXTURE_DIRS:
        if d and all(os.path.exists(os.path.join(d, f + s)) for f, s in
                     (("t10k-images-idx3-ubyte", ".gz"), ("t10k-labels-idx1-ubyte", ".gz"))):
            return d
    return None


def load_t10k(data_dir: Optional[str] = None, n_train: int = 8000
              ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    """(x_train, y_train, x_test, y_test): the reference's t10k set split n_train / rest,
    normalised like the reference transform; x is [N, 1, 28, 28] fp32."""
    d = find_fixture(data_dir)
    if d is None:
        raise FileNotFoundError("MNIST t10k fixture not found (tests/fixtures/mnist)")
    x = read_idx(os.path.join(d, "t10k-images-idx3-ubyte.gz")).astype(np.float32) / 255.0
    y = read_idx(os.path.join(d, "t10k-labels-idx1-ubyte.gz")).astype(np.int64)
    x = (torch.from_numpy(x).unsqueeze(1) - MEAN) / STD
    y = torch.from_numpy(y)
    return x[:n_train], y[:n_train], x[n_train:], y[n_train:]


def train_eval(params: Dict, epochs: int = 2, batch: int = 64, lr: float = 0.01, momentum: float = 0.5,
               device=None, data_dir: Optional[str] = None, seed: int = 42, n_train: int = 8000,
               log=None) -> Dict[str, float]:
    """Train the reference Net with the GRACE pipeline ``params`` on this rank's shard (rank::W,
    like DistributedSampler) and return {"accuracy", "loss"} on the held-out set (averaged
    over ranks, like metric_average in pytorch_mnist.py:163-166)."""
    from .. import grace_from_params
    from ..parallel import DistributedOptimizer, broadcast_parameters

    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    device = torch.device(device or "cpu")
    xtr, ytr, xte, yte = load_t10k(data_dir, n_train)
    xtr, ytr = xtr[rank::world].to(device), ytr[rank::world].to(device)
    xte, yte = xte.to(device), yte.to(device)
    torch.manual_seed(seed)
    model = Net().to(device)
    broadcast_parameters(model.state_dict(), root_rank=0)
    grc = grace_from_params(dict(params, world_size=world))
    opt = DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=lr * world, momentum=momentum), grc,
                               named_parameters=model.named_parameters())
    g = torch.Generator().manual_seed(seed + rank)
    loss = torch.zeros(())
    for ep in range(epochs):
        model.train()
        perm = torch.randperm(xtr.shape[0], generator=g).to(device)
        for s in range(xtr.shape[0] // batch):
            idx = perm[s * batch:(s + 1) * batch]
            opt.zero_grad()
            loss = F.nll_loss(model(xtr[idx]), ytr[idx])
            loss.backward()
            opt.step()
        if log is not None:
            log(f"epoch {ep + 1}: train loss {loss.item():.4f}")
    model.eval()
    with torch.no_grad():
        out = model(xte)
        m = torch.tensor([(out.argmax(1) == yte).float().mean().item(), F.nll_loss(out, yte).item()],
                         dtype=torch.float64)
    if world > 1:
        mm = m.to(device) if dist.get_backend() == "nccl" else m
        dist.all_reduce(mm)
        m = mm.cpu() / world
    return {"accuracy": float(m[0]), "loss": float(m[1])}
