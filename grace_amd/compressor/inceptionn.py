"""INCEPTIONN lossy floating-point codec (Li et al., MICRO 2018) -- the TF-only compressor.

Reference: /root/reference/grace_dl/tensorflow/compressor/inceptionn.py:8-188.  Elements are
classed by their biased exponent e with e_b = 127 + int(log10(error_bound / 2)),
mid = e_b + ceil((127 - e_b) / 2):
  e >= 127        -> sent as fp32
  mid <= e < 127  -> 16-bit fixed point  (sign | (1.mantissa >> (127-e))) >> 8
  e_b <= e < mid  ->  8-bit fixed point  (same) >> 16
  e < e_b         -> dropped (0)
plus a 2-bit class code per element packed 4 per byte.  Decoding recovers the exponent from
the position of the leading one (tfp find_bins over powers of two in the reference).

MI355X: csrc/kernels/inceptionn.hip -- a per-tile class count + device scan, then ONE encode
pass writes the 2-bit codes and the three order-preserving compacted streams; the decoder
recounts classes from every rank's codes and decodes + sums all W ranks in one pass (rank
order, deterministic).  One host read of the three class totals sizes the payload (the size is
data dependent, as in the reference).  The PyTorch path below is the CPU oracle (bit-identical).
The class codes are packed little-endian 4 per byte (element 4j+t at bits 2t of byte j) instead
of the reference's quarter-split layout (wire-format detail, same information).
Payload [fp32 v32 | int16 v16 | uint8 v8 | uint8 classes].  Variable size.
"""
from __future__ import annotations

import math

import torch

from ..ops import _native
from ._base import BucketCompressor


def _bits_to_f32(bits: torch.Tensor) -> torch.Tensor:
    """uint32 bit patterns held in int64 -> float32."""
    b = bits & 0xFFFFFFFF
    return torch.where(b >= 2 ** 31, b - 2 ** 32, b).to(torch.int32).view(torch.float32)


def _leading_bin(v: torch.Tensor) -> torch.Tensor:
    """floor(log2(v)) for v >= 2, 0 for v in {0, 1} (find_bins over [0, 2, 4, ...])."""
    vf = v.clamp_min(1).double()
    b = torch.floor(torch.log2(vf)).long()
    return torch.where(v >= 2, b, torch.zeros_like(b))


class INCEPTIONNCompressor(BucketCompressor):
    def __init__(self, error_bound: float = 2e-10):
        super().__init__(tensors_size_are_same=False)
        self.error_bound = error_bound
        self.e_b = 127 + int(math.log(error_bound / 2, 10))
        self.mid = self.e_b + math.ceil((127 - self.e_b) / 2)

    def _native_compress(self, x, ctx):
        C = _native.lib()
        n = x.numel()
        nt = C.inceptionn_tiles(n)
        lay = ctx.layout
        ws = lay.cached(x.device, "inceptionn_enc", lambda: {
            "cnt": torch.empty(max(1, 4 * nt), dtype=torch.int32, device=x.device),
            "tot": torch.empty(4, dtype=torch.int32, device=x.device)})
        C.inceptionn_count(x, self.e_b, self.mid, ws["cnt"], ws["tot"])
        _, n8, n16, n32 = (int(v) for v in ws["tot"].tolist())  # payload size: one host read
        a, b, c, d = self.payload(x.device, [(torch.float32, (n32,)), (torch.int16, (n16,)), (torch.uint8, (n8,)),
                                             (torch.uint8, ((n + 3) // 4,))])
        C.inceptionn_encode(x, self.e_b, self.mid, ws["cnt"], a, b, c, d)
        return [a, b, c, d]

    def compress(self, tensor, name):
        ctx = self.ctx(tensor, name)
        x = self.flat(tensor)
        if _native.use_native(x):
            return self._native_compress(x, ctx), ctx
        u = x.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
        sign = u & 0x80000000
        expo = (u >> 23) & 0xFF
        mant = u & 0x7FFFFF
        c32 = expo >= 127
        c16 = (expo >= self.mid) & (expo < 127)
        c8 = (expo >= self.e_b) & (expo < self.mid)
        shift = (127 - expo).clamp(0, 63)
        fixed = (sign >> 8) | (((mant >> 1) | 0x400000) >> shift)
        v16 = ((fixed >> 8) & 0xFFFF)[c16]
        v8 = ((fixed >> 16) & 0xFF)[c8]
        v32 = x[c32]
        code = c8.long() * 1 + c16.long() * 2 + c32.long() * 3
        n = x.numel()
        npad = (n + 3) // 4 * 4
        cp = torch.zeros(npad, dtype=torch.int64, device=x.device)
        cp[:n] = code
        packed = (cp.view(-1, 4) << torch.tensor([0, 2, 4, 6], device=x.device)).sum(1)
        a, b, c, d = self.payload(x.device, [(torch.float32, (v32.numel(),)), (torch.int16, (v16.numel(),)),
                                             (torch.uint8, (v8.numel(),)), (torch.uint8, (packed.numel(),))])
        a.copy_(v32)
        b.copy_(v16.to(torch.int32).to(torch.int16))
        c.copy_(v8.to(torch.uint8))
        d.copy_(packed.to(torch.uint8))
        return [a, b, c, d], ctx

    def _decode(self, v32, v16, v8, packed, n, device):
        codes = ((packed.to(torch.int64).unsqueeze(1) >> torch.tensor([0, 2, 4, 6], device=device)) & 3).view(-1)[:n]
        out = torch.zeros(n, dtype=torch.float32, device=device)
        # 16-bit class
        w = v16.to(torch.int64) & 0xFFFF
        s16 = (w & 0x8000) << 16
        vs = (w << 1) & 0xFFFF
        bn = _leading_bin(vs)
        nsh = 16 - bn
        e16 = (127 - (nsh - 1)) << 23
        m16 = ((vs << nsh) & 0xFFFF) << 7
        f16 = _bits_to_f32(s16 | e16 | m16)
        # 8-bit class
        w8 = v8.to(torch.int64) & 0xFF
        s8 = (w8 & 0x80) << 24
        vs8 = (w8 << 1) & 0xFF
        bn8 = _leading_bin(vs8)
        nsh8 = 8 - bn8
        e8 = (127 - (nsh8 - 1)) << 23
        m8 = ((vs8 << nsh8) & 0xFF) << 15
        f8 = _bits_to_f32(s8 | e8 | m8)
        out[codes == 3] = v32
        out[codes == 2] = f16
        out[codes == 1] = f8
        return out

    def decompress_aggregate_impl(self, per_rank, ctx, n_ranks, scale):
        dev = per_rank[0][0].device
        if _native.use_native(per_rank[0][3]):
            C = _native.lib()
            n = ctx.layout.total
            out = self.out_buffer(ctx, dev)
            ptrs = torch.tensor([t.data_ptr() for p in per_rank for t in p], dtype=torch.int64).to(dev)
            cptr = torch.tensor([p[3].data_ptr() for p in per_rank], dtype=torch.int64).to(dev)
            cnt = torch.empty(max(1, 4 * n_ranks * C.inceptionn_tiles(n)), dtype=torch.int32, device=dev)
            tot = torch.empty(4 * n_ranks, dtype=torch.int32, device=dev)
            C.inceptionn_decode(ptrs, cptr, n_ranks, cnt, tot, scale, out, False)
            return self.finish(out, ctx)
        out = self.out_buffer(ctx, dev, zero=True)
        for v32, v16, v8, packed in per_rank:
            out += self._decode(v32, v16, v8, packed, ctx.layout.total, dev)
        if scale != 1.0:
            out *= scale
        return self.finish(out, ctx)
