import sys, torch
sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo")
from test_gpu_sketch import _segments
from grace_amd import compressor as Z
from grace_amd.core import register_layout
from grace_amd.ops.layout import SegmentLayout
from grace_amd.compressor.sketch import segmented_quantile_edges
q = 1500
segs = _segments(3); flat = torch.cat(segs); lay = SegmentLayout.from_tensors(segs)
register_layout("dbg", lay)
pc, _ = Z.SketchCompressor(q).compress(flat, "dbg")
pg, _ = Z.SketchCompressor(q).compress(flat.cuda(), "dbg")
a, b = pg[0].cpu(), pc[0]
bad = (a != b).nonzero().flatten()
print("mismatches", bad.numel(), "of", a.numel())
offs = lay.offsets
edges = segmented_quantile_edges(flat, lay, q)
for i in bad[:10].tolist():
    s = max(j for j in range(lay.n_seg) if offs[j] <= i)
    v = flat[i].item()
    e = edges[s]
    print(i, "seg", s, "v", repr(v), "gpu", int(a[i]), "cpu", int(b[i]), "edges around", e[max(0,int(b[i])-1):int(b[i])+3].tolist())
