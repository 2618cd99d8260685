"""Allocator history around the failing BN backward (follow-up of bn_bwd_capture.py: the error
moves with allocation patterns and survives AMD_SERIALIZE_KERNEL=3, so it is a memory-reuse
problem, not a kernel race).  The native BN backward of layer3.0.bn2 is wrapped to record its
operands' addresses ONLY (no sync, no allocation); the caching allocator's event history then shows
which later allocations reused those blocks while the backward still needed them.
Usage: python tools/gpu/bn_memtrace.py --force dgrad=mfma_t2
"""
import argparse
import copy
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import ddp_fp64_diag as D  # noqa: E402
from grace_amd.ops import _native, conv  # noqa: E402

SHAPE = (8, 256, 4, 4)


def n_events():
    tr = torch.cuda.memory._snapshot()["device_traces"]
    return len(tr[0]) if tr else 0


class Proxy:
    def __init__(self, real):
        self._real = real
        self.rec = []

    def __getattr__(self, k):
        return getattr(self._real, k)

    def _span(self, t):
        if t is None or not isinstance(t, torch.Tensor) or not t.is_cuda:
            return None
        return (t.data_ptr(), t.data_ptr() + t.numel() * t.element_size())

    def bn_act_fwd(self, x, res, *a):
        out = self._real.bn_act_fwd(x, res, *a)
        if tuple(x.shape) == SHAPE and res is not None:
            self.rec.append({"call": "fwd", "ev": n_events(), "x": self._span(x), "y": self._span(out[0]),
                             "save": self._span(out[1]), "mask": self._span(out[2])})
        return out

    def bn_act_fwd_partials(self, x, res, *a):
        out = self._real.bn_act_fwd_partials(x, res, *a)
        if tuple(x.shape) == SHAPE and res is not None:
            self.rec.append({"call": "fwdp", "ev": n_events(), "x": self._span(x), "y": self._span(out[0]),
                             "save": self._span(out[1]), "mask": self._span(out[2])})
        return out

    def bn_act_bwd(self, dy, dy2, x, mask, weight, save, *a):
        ev0 = n_events()
        out = self._real.bn_act_bwd(dy, dy2, x, mask, weight, save, *a)
        if tuple(x.shape) == SHAPE:
            self.rec.append({"call": "bwd" + ("_dual" if dy2 is not None else ""), "ev": ev0, "ev_after": n_events(),
                             "dy": self._span(dy), "dy2": self._span(dy2), "x": self._span(x),
                             "mask": self._span(mask), "save": self._span(save), "dx": self._span(out[0]),
                             "dres": self._span(out[1]), "dw": self._span(out[2]), "db": self._span(out[3])})
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", default="dgrad=mfma_t2")
    ap.add_argument("--mode", default="plain_on")
    args = ap.parse_args()
    forced = dict(kv.split("=") for kv in args.force.split(",") if kv)
    pick3, pick_bn = conv._pick3, conv._pick_bn
    conv._pick3 = lambda d, x, w, dy, s: (forced[d] if d in forced and not (d == "dgrad" and (s != 1 or w.shape[2] != 3))
                                          else pick3(d, x, w, dy, s))
    conv._pick_bn = lambda cv, bn, x, r, relu: forced.get("bn") or pick_bn(cv, bn, x, r, relu)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(D._port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    proxy = Proxy(_native.lib())
    _native._lib = proxy

    torch.manual_seed(0)
    base = D.resnet18_cifar()
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8, 3, 16, 16, generator=g)
    y = torch.randint(0, 10, (8,), generator=g)
    _, ref_g, _ = D.run(copy.deepcopy(base).double(), x.double(), y, torch.device("cpu"), False, False)
    # one untraced run (autotune decisions), then the traced one
    D.run(base, x, y, torch.device("cuda", 0), ddp=args.mode.startswith("ddp"), stream_on="_on" in args.mode)
    torch.cuda.synchronize()
    torch.cuda.memory._record_memory_history(max_entries=200000, stacks="python")
    proxy.rec.clear()
    _, gr, _ = D.run(base, x, y, torch.device("cuda", 0), ddp=args.mode.startswith("ddp"), stream_on="_on" in args.mode,
                     steps=1)
    torch.cuda.synchronize()
    snap = torch.cuda.memory._snapshot()
    torch.cuda.memory._record_memory_history(enabled=None)
    trace = snap["device_traces"][0]
    err = D.rel(gr["layer3.0.bn2.bias"], ref_g["layer3.0.bn2.bias"])
    print(json.dumps({"bn2_bias_rel_err": err, "n_events": len(trace), "calls": [r["call"] for r in proxy.rec]}),
          flush=True)

    def overlapping(span, ev_from, ev_to):
        out = []
        for i in range(ev_from, min(ev_to, len(trace))):
            e = trace[i]
            a, sz = e.get("addr"), e.get("size", 0)
            if a is None or span is None:
                continue
            if a < span[1] and a + sz > span[0]:
                fr = [f"{f.get('filename', '').split('/')[-1]}:{f.get('line')}:{f.get('name')}" for f in
                      (e.get("frames") or [])[:6]]
                out.append({"i": i, "action": e.get("action"), "addr": a, "size": sz, "frames": fr})
        return out

    # the dual BN backward (layer3.0.bn2 / layer3.1.bn2 / ...): who touched its operands between its
    # forward and its backward, and between its backward and the end of the step
    fwds = [r for r in proxy.rec if r["call"].startswith("fwd")]
    for r in proxy.rec:
        if not r["call"].startswith("bwd"):
            continue
        f = [q for q in fwds if q["save"] == r["save"]]
        rep = {"call": r["call"], "ev": r["ev"], "fwd_ev": f[0]["ev"] if f else None}
        for k in ("dy", "dy2", "x", "mask", "save"):
            if f and k in ("x", "mask", "save"):
                rep[k + "_between_fwd_and_bwd"] = overlapping(r[k], f[0]["ev"], r["ev"])
        for k in ("dx", "dres", "dw", "db", "dy", "dy2"):
            rep[k + "_after_bwd"] = overlapping(r[k], r["ev_after"], len(trace))[:12]
        print(json.dumps(rep), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
