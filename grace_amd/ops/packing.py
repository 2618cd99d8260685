"""2-bit code packing helpers (4 codes per byte).

``encode_byte`` / ``decode_byte`` reproduce the reference TF helper's wire format
(/root/reference/grace_dl/tensorflow/compressor/packing.py:4-30): pad to a multiple of 4 (the
reference always pads, 4 entries when the size is already a multiple of 4, with the values
0, 1, 2, 3), split into four contiguous quarters, byte j = q0[j] + 4 q1[j] + 16 q2[j] + 64 q3[j].
Unused by the reference's compressors; kept for format compatibility.

``pack2`` / ``unpack2`` are the interleaved layout the grace_amd kernels use (element 4j+t at
bits 2t of byte j: a thread's codes land in its own bytes, no cross-quarter gather), the
format of INCEPTIONN's class codes (csrc/kernels/inceptionn.hip).  All are elementwise torch
ops, i.e. single fused elementwise kernels on the GPU.
"""
from __future__ import annotations

import torch


def encode_byte(a: torch.Tensor) -> torch.Tensor:
    a = a.reshape(-1).to(torch.int32)
    pad = 4 - a.numel() % 4
    a = torch.cat([a, torch.arange(pad, dtype=torch.int32, device=a.device)])
    q = a.view(4, -1)
    return (q[0] + 4 * q[1] + 16 * q[2] + 64 * q[3]).to(torch.uint8)


def decode_byte(encoded: torch.Tensor, real_size: int) -> torch.Tensor:
    a = encoded.to(torch.int32)
    return torch.cat([a % 4, (a // 4) % 4, (a // 16) % 4, (a // 64) % 4])[:real_size]


def pack2(codes: torch.Tensor) -> torch.Tensor:
    c = codes.reshape(-1).to(torch.int32)
    n = c.numel()
    c = torch.nn.functional.pad(c, (0, (-n) % 4)).view(-1, 4)
    return (c[:, 0] | (c[:, 1] << 2) | (c[:, 2] << 4) | (c[:, 3] << 6)).to(torch.uint8)


def unpack2(packed: torch.Tensor, n: int) -> torch.Tensor:
    p = packed.to(torch.int32).unsqueeze(1)
    sh = torch.arange(0, 8, 2, dtype=torch.int32, device=packed.device)
    return ((p >> sh) & 3).reshape(-1)[:n]
