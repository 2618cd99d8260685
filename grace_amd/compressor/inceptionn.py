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
order, deterministic).  The payload has a FIXED capacity (ops/cappayload.py idea): an int32
header with the class totals, ONE value stream of 4 * ceil(capacity * n) bytes holding the fp32,
16-bit and 8-bit values back to back, and the codes -- no host read of a size, graph-capturable.
capacity 1.0 (the default: INCEPTIONN has no error feedback, so nothing may be dropped) always
fits (every element as fp32); below it the lowest-precision classes are dropped first when the
step's values do not fit, and the encoder counts that step in ``parallel.health.overflows()``
(also inside a replayed HIP graph).  ``capacity="auto"`` (opt-in): the value
stream starts at n bytes (1 byte per element: every element in the 8-bit class or dropped, the
common case for gradients below 2^-5; tensors <= 16K elements start at full size) and grows lagged and sync-free when a step needed more
(ops/cappayload.py AdaptiveCapacity, decided from every rank's gathered header: ranks stay in
step).  Wire bytes ~1.25 n instead of 4.25 n; on the xGMI path only the valid bytes move.  The PyTorch path below is the CPU
oracle (bit-identical).
The class codes are packed little-endian 4 per byte (element 4j+t at bits 2t of byte j) instead
of the reference's quarter-split layout (wire-format detail, same information).
Payload [int32 header (0, n8, n16, n32) | value stream | uint8 classes].
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
    AUTO_BYTES_PER_ELEMENT = 1.0

    def __init__(self, error_bound: float = 2e-10, capacity=1.0):
        super().__init__(tensors_size_are_same=True)  # fixed-capacity payload
        self.error_bound = error_bound
        self.e_b = 127 + int(math.log(error_bound / 2, 10))
        self.mid = self.e_b + math.ceil((127 - self.e_b) / 2)
        # INCEPTIONN has no error feedback: a class that does not fit is LOST, so the default is
        # the lossless capacity 1.0 (the reference's semantics); "auto" (opt-in) sizes the value
        # stream adaptively and counts every lossy step in health.overflows()
        if capacity is None or capacity == "auto":
            capacity = None
        self.capacity = capacity
        self.adaptive = (None if capacity is not None else
                         __import__("grace_amd.ops.cappayload", fromlist=["x"]).AdaptiveCapacity(
                             self.AUTO_BYTES_PER_ELEMENT))

        self._name = None

    def _cap_bytes(self, n: int) -> int:
        """Value-stream bytes: 4 * ceil(capacity * n) (1.0 = every element fits as fp32), or the
        adaptive size of the current bucket (auto)."""
        if self.adaptive is not None and self._name is not None:
            # small tensors (<= 16K elements) start at full capacity: never a dropped class
            floor = min(4 * n, 1 << 16)
            b = max(self.adaptive.get(self._name, n, 4 * n), floor)
            return 4 * max(1, (b + 3) // 4)
        cap = 1.0 if self.capacity is None else self.capacity
        return 4 * max(1, int(math.ceil(cap * n)))

    def _payload(self, dev, n):
        return self.payload(dev, [(torch.int32, (4,)), (torch.uint8, (self._cap_bytes(n),)),
                                  (torch.uint8, ((n + 3) // 4,))])

    def _native_compress(self, x, ctx):
        from ..parallel import health as _health

        _health.init_for(x)  # the overflow counter (allocated in the first, eager step)
        C = _native.lib()
        n = x.numel()
        nt = C.inceptionn_tiles(n)
        ws = ctx.layout.cached(x.device, "inceptionn_enc", lambda: torch.empty(max(1, 4 * nt), dtype=torch.int32,
                                                                              device=x.device))
        hdr, stream, codes = self._payload(x.device, n)
        C.inceptionn_count(x, self.e_b, self.mid, ws, hdr)  # class totals -> the in-band header
        C.inceptionn_encode(x, self.e_b, self.mid, ws, hdr, stream, codes)
        return [hdr, stream, codes]

    def wire_counts(self, tensors):
        # header (0, n8, n16, n32): the value stream holds n8 + 2 n16 + 4 n32 bytes
        return [None, (0, [0, 1, 2, 4]), None]

    def compress(self, tensor, name):
        ctx = self.ctx(tensor, name)
        ctx.extra["name"] = name
        self._name = name
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
        n = x.numel()
        n32, n16, n8 = int(c32.sum()), int(c16.sum()), int(c8.sum())
        cap = self._cap_bytes(n)
        # capacity plan (same as csrc/kernels/inceptionn.hip inc_plan): drop class 8, then 16,
        # then the last class-32 elements
        keep2 = 4 * n32 + 2 * n16 <= cap
        keep1 = keep2 and 4 * n32 + 2 * n16 + n8 <= cap
        cap3 = cap // 4
        if n32 > cap3:
            pos = torch.cumsum(c32.long(), 0) - 1
            c32 = c32 & (pos < cap3)
        if not keep2:
            c16 = torch.zeros_like(c16)
        if not keep1:
            c8 = torch.zeros_like(c8)
        shift = (127 - expo).clamp(0, 63)
        fixed = (sign >> 8) | (((mant >> 1) | 0x400000) >> shift)
        v16 = ((fixed >> 8) & 0xFFFF)[c16].to(torch.int32).to(torch.int16)
        v8 = ((fixed >> 16) & 0xFF)[c8].to(torch.uint8)
        v32 = x[c32]
        code = c8.long() * 1 + c16.long() * 2 + c32.long() * 3
        npad = (n + 3) // 4 * 4
        cp = torch.zeros(npad, dtype=torch.int64, device=x.device)
        cp[:n] = code
        packed = (cp.view(-1, 4) << torch.tensor([0, 2, 4, 6], device=x.device)).sum(1)
        hdr, stream, codes = self._payload(x.device, n)
        hdr.copy_(torch.tensor([0, n8, n16, n32], dtype=torch.int32))
        stream.zero_()
        body = torch.cat([v32.view(torch.uint8), v16.view(torch.uint8), v8])
        stream[: body.numel()] = body
        codes.copy_(packed.to(torch.uint8))
        return [hdr, stream, codes], ctx

    def _decode(self, stream, packed, n, device):
        codes = ((packed.to(torch.int64).unsqueeze(1) >> torch.tensor([0, 2, 4, 6], device=device)) & 3).view(-1)[:n]
        n32, n16, n8 = int((codes == 3).sum()), int((codes == 2).sum()), int((codes == 1).sum())
        v32 = stream[: 4 * n32].view(torch.float32)
        v16 = stream[4 * n32: 4 * n32 + 2 * n16].view(torch.int16)
        v8 = stream[4 * n32 + 2 * n16: 4 * n32 + 2 * n16 + n8]
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
        if self.adaptive is not None and "name" in ctx.extra:  # every rank's header (same on all ranks)
            self.adaptive.observe(ctx.extra["name"], [p[0] for p in per_rank], lambda w: w[1] + 2 * w[2] + 4 * w[3])
        dev = per_rank[0][0].device
        n = ctx.layout.total
        if _native.use_native(per_rank[0][2]):
            C = _native.lib()
            out = self.out_buffer(ctx, dev)
            base, stride, offs = self.rows(per_rank)
            ws = ctx.layout.cached(dev, f"inceptionn_dec:{n_ranks}", lambda: (
                torch.empty(max(1, 4 * n_ranks * C.inceptionn_tiles(n)), dtype=torch.int32, device=dev),
                torch.empty(4 * n_ranks, dtype=torch.int32, device=dev)))
            C.inceptionn_decode(base, stride, offs[1], offs[2], n_ranks, ws[0], ws[1], scale, out, False)
            return self.finish(out, ctx)
        out = self.out_buffer(ctx, dev, zero=True)
        for _hdr, stream, packed in per_rank:
            out += self._decode(stream, packed, n, dev)
        if scale != 1.0:
            out *= scale
        return self.finish(out, ctx)
