"""The BASELINE.json benchmark configurations as runnable workloads.

Each workload = model + synthetic batch + loss + GRACE parameters + optimizer, mirroring the
reference harness (/root/reference/examples/torch/pytorch_synthetic_benchmark.py:46-55,
110-111, 151-154: batch 32/GPU, fixed random 3x224x224 input, SGD lr 0.01*W, momentum 0.5).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Callable, Dict

import torch
import torch.nn.functional as F

from ..models import MODELS


@dataclass
class Workload:
    name: str
    model: str
    batch: int
    unit: str  # what one "sample" is
    grace: Dict[str, Any]
    make_batch: Callable[[int, torch.device], Any]
    loss: Callable[[torch.nn.Module, Any], torch.Tensor]
    samples_per_batch: Callable[[int], int] = lambda b: b
    model_kw: Dict[str, Any] = field(default_factory=dict)
    channels_last: bool = False
    seq_len: int = 0


def _img_batch(res, classes):
    def make(b, dev):
        g = torch.Generator(device="cpu").manual_seed(1234)
        x = torch.randn(b, 3, res, res, generator=g).to(dev)
        y = (torch.arange(b) % classes).to(dev)
        return x, y
    return make


def _img_loss(model, batch):
    x, y = batch
    return F.cross_entropy(model(x), y)


def _lm_batch(bptt, vocab):
    def make(b, dev):
        g = torch.Generator(device="cpu").manual_seed(1234)
        tok = torch.randint(0, vocab, (bptt + 1, b), generator=g).to(dev)
        return tok[:-1], tok[1:]
    return make


def _lm_loss(model, batch):
    inp, tgt = batch
    out, _ = model(inp)
    return F.cross_entropy(out.reshape(-1, out.size(-1)).float(), tgt.reshape(-1))


def _mlm_batch(seq, vocab):
    def make(b, dev):
        g = torch.Generator(device="cpu").manual_seed(1234)
        ids = torch.randint(0, vocab, (b, seq), generator=g)
        labels = torch.full_like(ids, -100)
        m = torch.rand(b, seq, generator=g) < 0.15
        labels[m] = ids[m]
        return ids.to(dev), labels.to(dev)
    return make


def _mlm_loss(model, batch):
    ids, labels = batch
    out = model(ids)
    return F.cross_entropy(out.reshape(-1, out.size(-1)).float(), labels.reshape(-1), ignore_index=-100)


WORKLOADS: Dict[str, Workload] = {
    # headline: BASELINE.json metric / config 2
    "resnet50_topk": Workload(
        "resnet50_topk", "resnet50", 32, "images",
        {"compressor": "topk", "compress_ratio": 0.01, "memory": "residual", "communicator": "allgather"},
        _img_batch(224, 1000), _img_loss, channels_last=True),
    "resnet50_none": Workload(
        "resnet50_none", "resnet50", 32, "images",
        {"compressor": "none", "memory": "none", "communicator": "allreduce"},
        _img_batch(224, 1000), _img_loss, channels_last=True),
    # DGC 1% + DgcMemory (momentum correction) via Allgather: fixed-capacity payload, graph-capturable
    "resnet50_dgc": Workload(
        "resnet50_dgc", "resnet50", 32, "images",
        {"compressor": "dgc", "compress_ratio": 0.01, "memory": "dgc", "communicator": "allgather"},
        _img_batch(224, 1000), _img_loss, channels_last=True),
    # Threshold 0.01 + Residual via Allgather: bounded capacity payload (1/32 of the bucket with
    # error feedback, grown lagged from the gathered counts): the bytes-on-wire check
    "resnet50_threshold": Workload(
        "resnet50_threshold", "resnet50", 32, "images",
        {"compressor": "threshold", "threshold": 0.01, "memory": "residual", "communicator": "allgather"},
        _img_batch(224, 1000), _img_loss, channels_last=True),
    "resnet18_cifar_none": Workload(
        "resnet18_cifar_none", "resnet18_cifar", 128, "images",
        {"compressor": "none", "memory": "none", "communicator": "allreduce"},
        _img_batch(32, 10), _img_loss, channels_last=True),
    # the reference's only published number: cifar10-fast ResNet-9, batch 512, 24 epochs
    # (examples/dist/CIFAR10-dawndist/README.md:17, 24-26) -- uncompressed like dawn.py:124-127
    "resnet9_dawn": Workload(
        "resnet9_dawn", "resnet9", 512, "images",
        {"compressor": "none", "memory": "none", "communicator": "allreduce"},
        _img_batch(32, 10), _img_loss, channels_last=True),
    "vgg16_powersgd": Workload(
        "vgg16_powersgd", "vgg16", 32, "images",
        {"compressor": "powersgd", "compress_rank": 4, "memory": "powersgd", "communicator": "allreduce"},
        _img_batch(224, 1000), _img_loss, channels_last=True),
    "lstm_efsignsgd": Workload(
        "lstm_efsignsgd", "lstm_ptb", 20, "tokens",
        {"compressor": "efsignsgd", "lr": 0.1, "memory": "efsignsgd", "communicator": "allreduce"},
        _lm_batch(35, 10000), _lm_loss, samples_per_batch=lambda b: 35 * b, seq_len=35),
    "bert_qsgd": Workload(
        "bert_qsgd", "bert_base", 32, "sequences",
        {"compressor": "qsgd", "quantum_num": 127, "memory": "none", "communicator": "allreduce"},
        _mlm_batch(128, 30522), _mlm_loss, seq_len=128),
}

# uncompressed reference point (None + Allreduce) for every BASELINE model
for _k in ("vgg16_powersgd", "lstm_efsignsgd", "bert_qsgd"):
    _w = WORKLOADS[_k]
    _n = _k.split("_")[0] + "_none"
    WORKLOADS[_n] = Workload(_n, _w.model, _w.batch, _w.unit,
                             {"compressor": "none", "memory": "none", "communicator": "allreduce"},
                             _w.make_batch, _w.loss, _w.samples_per_batch, dict(_w.model_kw), _w.channels_last,
                             _w.seq_len)


def build_model(w: Workload, device) -> torch.nn.Module:
    m = MODELS[w.model](**w.model_kw).to(device)
    if w.channels_last and device.type == "cuda":
        m = m.to(memory_format=torch.channels_last)
    return m
