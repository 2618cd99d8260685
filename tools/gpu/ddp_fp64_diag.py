"""Diagnose the intermittent plain-DDP gradient mismatch (VERDICT r4 Weak #1).

resnet18_cifar (the test's model, input and seed) is run under plain DDP with the side-stream
switch off and on, without DDP, and with the allocator's free blocks poisoned with NaN; every
run's parameter gradients AND every module's output gradient (tensor hooks: the graph itself is
not changed) are compared with a float64 CPU reference of the same weights through stock ops.
Prints one JSON line per mode plus the per-process autotune decisions, so a failing and a passing
process can be diffed.  Usage (GPU box): python tools/gpu/ddp_fp64_diag.py [--poison] [--modes a,b]
"""
import argparse
import copy
import json
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from grace_amd.models import resnet18_cifar  # noqa: E402
from grace_amd.ops import conv, wgrad  # noqa: E402
from grace_amd.ops import _native  # noqa: E402


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def poison_allocator(small=1500, large=24):
    """Fill free caching-allocator blocks with NaN: every later torch.empty that lands in them
    reads NaN until written, so an uninitialised read shows up as a NaN gradient."""
    keep = [torch.full((256 * 1024,), float("nan"), device="cuda") for _ in range(small)]  # 1 MB: small pool
    keep += [torch.full((8 << 20,), float("nan"), device="cuda") for _ in range(large)]  # 32 MB: large pool
    torch.cuda.synchronize()
    del keep


def hook_modules(model, store):
    hs = []

    def fwd_hook(name):
        def f(mod, inp, out):
            outs = out if isinstance(out, (tuple, list)) else (out,)
            for i, t in enumerate(outs):
                if isinstance(t, torch.Tensor) and t.requires_grad:
                    def save(g, key=f"{name}[{i}]"):
                        if g is not None:
                            store[key] = g.detach().double().cpu().clone()
                    t.register_hook(save)
        return f

    for n, m in model.named_modules():
        if n and (n.count(".") <= 1 or n.endswith(("bn1", "bn2", "conv1", "conv2"))):
            hs.append(m.register_forward_hook(fwd_hook(n)))
    return hs


def run(base, x, y, device, ddp, stream_on, steps=2, poison=False, bn_det=None):
    m = copy.deepcopy(base).to(device)
    if device.type == "cuda":
        m = m.to(memory_format=torch.channels_last)
    net = nn.parallel.DistributedDataParallel(m, device_ids=[0], broadcast_buffers=False) if ddp else m
    wgrad.set_enabled(stream_on)
    if bn_det is not None:
        _native.lib().bn_set_deterministic(bool(bn_det))
    store = {}
    try:
        for it in range(steps):
            if poison and device.type == "cuda":
                poison_allocator()
            for p in m.parameters():
                p.grad = None
            store.clear()
            hs = hook_modules(m, store) if it == steps - 1 else []
            xi = x.to(device)
            if device.type == "cuda":
                xi = xi.contiguous(memory_format=torch.channels_last)
            loss = F.cross_entropy(net(xi), y.to(device))
            loss.backward()
            loss = loss.detach()
            for h in hs:
                h.remove()
        if device.type == "cuda":
            torch.cuda.synchronize()
        grads = {n: p.grad.detach().double().cpu().clone() for n, p in m.named_parameters()}
        # a dual-output module (block output handed to two consumers): on the GPU the two aliases
        # carry the two partial gradients, on the CPU both hooks see the same full gradient
        for k in [k for k in store if k.endswith("[0]")]:
            k1 = k[:-3] + "[1]"
            if k1 in store:
                store[k[:-3] + "[full]"] = store[k] if device.type == "cpu" else store[k] + store[k1]
                del store[k], store[k1]
    finally:
        wgrad.set_enabled(True)
        if bn_det is not None:
            _native.lib().bn_set_deterministic(False)
    return float(loss), grads, dict(store)


def rel(a, b):
    d = float((a - b).abs().max())
    s = float(b.abs().max()) + 1e-30
    if a.isnan().any():
        return float("nan")
    return d / s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--poison", action="store_true")
    ap.add_argument("--modes", default="ddp_off,ddp_on,plain_on,plain_off,ddp_on_det,ddp_on_poison")
    ap.add_argument("--tag", default="")
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--force", default="", help="DIR=BACKEND[,DIR=BACKEND]: pin a conv3x3 direction "
                    "(fwd / dgrad / wgrad) or the conv->BN forward (bn=unfused|stats_tN) for every layer")
    args = ap.parse_args()
    forced = dict(kv.split("=") for kv in args.force.split(",") if kv)
    if forced:
        pick3, pick_bn = conv._pick3, conv._pick_bn

        def forced3(direction, x, w, dy, stride):
            be = forced.get(direction)
            if be is None or (direction == "dgrad" and (stride != 1 or w.shape[2] != 3)):
                return pick3(direction, x, w, dy, stride)
            return be

        def forced_bn(cv, bn, x, residual, relu):
            return forced.get("bn") or pick_bn(cv, bn, x, residual, relu)

        conv._pick3, conv._pick_bn = forced3, forced_bn

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_port())
    if args.backend == "nccl":
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group(args.backend, rank=0, world_size=1)

    torch.manual_seed(0)
    base = resnet18_cifar()  # CPU, fp32, the test's initialisation
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8, 3, 16, 16, generator=g)
    y = torch.randint(0, 10, (8,), generator=g)

    ref_loss, ref_g, ref_m = run(copy.deepcopy(base).double(), x.double(), y, torch.device("cpu"), False, False)
    names = [n for n, _ in base.named_parameters()]
    cuda = torch.device("cuda", 0)
    results = {}
    for mode in args.modes.split(","):
        kw = dict(ddp=mode.startswith("ddp"), stream_on="_on" in mode, poison=mode.endswith("poison") or args.poison,
                  bn_det=True if mode.endswith("_det") else None)
        loss, gr, mg = run(base, x, y, cuda, **kw)
        perr = {n: rel(gr[n], ref_g[n]) for n in names}
        merr = {k: rel(mg[k], ref_m[k]) for k in ref_m if k in mg}
        results[mode] = gr
        worst = sorted(perr.items(), key=lambda kv: -(kv[1] if kv[1] == kv[1] else 1e9))[:6]
        # the deepest module whose output gradient is wrong (backward order: deepest first)
        order = [k for k in ref_m]
        bad_mod = [k for k in order if k in merr and not (merr[k] <= 1e-4)]
        print(json.dumps({"tag": args.tag, "mode": mode, "loss": loss, "ref_loss": ref_loss,
                          "max_param_rel_err": max(v if v == v else 1e9 for v in perr.values()),
                          "worst_params": worst,
                          "bad_module_grads": [(k, merr[k]) for k in bad_mod][:8],
                          "n_bad_params": sum(1 for v in perr.values() if not (v <= 1e-4))}), flush=True)
    if "ddp_off" in results and "ddp_on" in results:
        a, b = results["ddp_off"], results["ddp_on"]
        diff = [n for n in names if not torch.allclose(a[n], b[n], rtol=0, atol=1e-4 * float(b[n].abs().max()) + 1e-6)]
        print(json.dumps({"tag": args.tag, "ddp_off_vs_on_differ": diff[::-1][:6], "n": len(diff)}), flush=True)
    print(json.dumps({"tag": args.tag,
                      "conv3x3_autotune": [list(map(str, r)) for r in conv.conv3x3_autotune_table()],
                      "bn_autotune": [list(map(str, r)) for r in conv.bn_autotune_table()],
                      "conv1x1_autotune": [list(map(str, r)) for r in conv.autotune_table()]}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
