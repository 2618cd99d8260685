"""Golden-semantics oracles: tiny independent PyTorch implementations of the reference
compressors, used only by the tests.  Each takes ONE tensor (reference
per-tensor semantics) and returns the decompressed tensor of a single rank, or the aggregate.
"""
import math

import torch


def topk(x, ratio):
    f = x.flatten()
    k = max(1, int(f.numel() * ratio))
    idx = torch.topk(f.abs(), k).indices
    out = torch.zeros_like(f)
    out[idx] = f[idx]
    return out.view_as(x)


def threshold(x, thr):
    f = x.flatten()
    out = torch.where(f.abs() > thr, f, torch.zeros_like(f))
    return out.view_as(x)


def signsgd_vote(xs):
    s = sum(torch.where(x >= 0, 1.0, -1.0) for x in xs)
    return torch.where(s >= 0, 1.0, -1.0)


def efsign(x):
    return x.abs().mean() * torch.where(x >= 0, 1.0, -1.0)


def onebit(x):
    neg = x < 0
    m0 = x[neg].mean() if neg.any() else torch.tensor(0.0)
    m1 = x[~neg].mean() if (~neg).any() else torch.tensor(0.0)
    return torch.where(neg, m0, m1)


def fp16(x):
    return x.half().float()


def qsgd_bounds(x, s):
    """QSGD decode is within one quantization step of x: |dec - x| <= norm/s."""
    return x.norm() / s


def terngrad_scalar(x, c=2.5):
    std = torch.sqrt(torch.mean((x - x.mean()) ** 2))
    cl = c * std
    return torch.clamp(x, -cl, cl).abs().max()


def natural_decode_range(x):
    """natural compression rounds |x| to an adjacent power of two: 2^floor(log2|x|) or x2."""
    a = x.abs().clamp_min(1e-30)
    lo = torch.exp2(torch.floor(torch.log2(a)))
    return lo, 2 * lo


def powersgd(m, q):
    """one power iteration (W=1) from a given (already orthogonal) Q."""
    p = m @ q
    p = gram_schmidt(p)
    q2 = m.t() @ p
    return p @ q2.t()


def gram_schmidt(a):
    a = a.clone()
    for i in range(a.shape[1]):
        a[:, i] /= a[:, i].norm()
        for j in range(i + 1, a.shape[1]):
            a[:, j] -= (a[:, i] * a[:, j]).sum() * a[:, i]
    return a
