"""DGC compaction A/B on one 16.6 M-element bucket (a ResNet-50 64 MB bucket's size): the
compaction kernel alone (after one full dgc_select has filled the workspace), with and without
the fused u / v masking, against a plain read of the same bytes.
Usage: python tools/gpu/dgc_compact_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from grace_amd.ops import _native  # noqa: E402
from grace_amd.ops import dgc as D  # noqa: E402
from grace_amd.ops.cappayload import sparse_payload  # noqa: E402
from grace_amd.ops.layout import SegmentLayout  # noqa: E402


def timed(fn, reps=50):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    torch.manual_seed(0)
    shapes = [(2048, 512, 3, 3), (1000, 2048), (2048,), (512, 512, 3, 3), (1001,), (333, 7)]
    lay = SegmentLayout.from_tensors([torch.empty(s) for s in shapes])
    n = lay.total
    x = torch.randn(n, device="cuda")
    cap = D.dgc_capacity(lay, 0.01, 2.0)
    D.dgc_select(x, lay, 0.01, 0.01, 10, 7, cap)
    ws = lay.cached(x.device, "dgc_ws:0.01:0.01", lambda: None)
    t = lay.device_tables(x.device)
    hdr, v, i = sparse_payload(x.device, cap)
    um, vm = torch.zeros_like(x), torch.zeros_like(x)
    C = _native.lib()

    def comp(masks):
        C.dgc_compact(x, ws["thr"], v, i, hdr[:1], t["seg"], t["begin"], t["end"], ws["ccnt"], ws["fnode"], ws["coff"],
                      vm if masks else None, um if masks else None)

    print(f"bucket {n} elements ({n * 4 / 1e6:.1f} MB), {t['n_chunks']} chunks, selected {int(hdr[0])}, "
          f"uncounted segments {int((ws['fnode'] < 0).sum())}", flush=True)
    print(f"compact, u/v masks   {timed(lambda: comp(True)):8.2f} us")
    print(f"compact, no masks    {timed(lambda: comp(False)):8.2f} us")
    print(f"plain read (sum)     {timed(lambda: x.sum()):8.2f} us")


if __name__ == "__main__":
    main()
