#!/usr/bin/env python3
"""GRACE exchange microbenchmark: the compress -> communicate -> decompress part of one
training step, in isolation, on the real parameter shapes of a model.

The model's parameters are bucketed exactly as in training (``GraceEngine``, 128 MB buckets as in bench.py);
their gradient buckets are filled with N(0,1) data and ``engine.synchronize()`` -- every
bucket's fused error-feedback compress, the collective, and the one-pass decode into the
bucket -- is timed with HIP events (captured in a HIP graph when the pipeline is graph-safe,
so launch overhead is excluded like in the whole-step bench).  No forward/backward and no
MIOpen kernels run, which also makes this the program to hand to ``rocprofv3 --pmc``.

The "gradient GB/s" column is 4 bytes x #gradient elements / time -- the rate at which the
pipeline consumes fp32 gradients.  Each pipeline reads the gradient and the residual at least
once and writes the residual once (>= 12 B/element), so at the ~6 TB/s HBM3E rate a
single-pass kernel chain would reach ~2000 gradient GB/s; the ratio shows how far a pipeline
is from that bound (multi-pass radix select and MFMA power iterations sit lower by design).

    python benchmarks/grace_kernels.py                        # all BASELINE pipelines
    python benchmarks/grace_kernels.py --pipeline topk --model resnet50 --iters 50
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from grace_amd import grace_from_params  # noqa: E402
from grace_amd.models import MODELS  # noqa: E402
from grace_amd.parallel.engine import GraceEngine  # noqa: E402
from grace_amd.parallel.graph import graph_safe  # noqa: E402

PIPELINES = {
    # name: (model, grace params) -- the BASELINE.json configs plus the other native codecs
    "topk": ("resnet50", {"compressor": "topk", "compress_ratio": 0.01, "memory": "residual",
                          "communicator": "allgather"}),
    "powersgd": ("vgg16", {"compressor": "powersgd", "compress_rank": 4, "memory": "powersgd",
                           "communicator": "allreduce"}),
    "efsignsgd": ("lstm_ptb", {"compressor": "efsignsgd", "lr": 0.1, "memory": "efsignsgd",
                               "communicator": "allreduce"}),
    "qsgd": ("bert_base", {"compressor": "qsgd", "quantum_num": 127, "memory": "none",
                           "communicator": "allreduce"}),
    "none": ("resnet50", {"compressor": "none", "memory": "none", "communicator": "allreduce"}),
    "fp16": ("resnet50", {"compressor": "fp16", "memory": "none", "communicator": "allreduce"}),
    "randomk": ("resnet50", {"compressor": "randomk", "compress_ratio": 0.01, "memory": "residual",
                             "communicator": "allreduce"}),
    "terngrad": ("resnet50", {"compressor": "terngrad", "memory": "none", "communicator": "allreduce"}),
    "natural": ("resnet50", {"compressor": "natural", "memory": "none", "communicator": "allreduce"}),
    "signsgd": ("resnet50", {"compressor": "signsgd", "memory": "none", "communicator": "allreduce"}),
    "onebit": ("resnet50", {"compressor": "onebit", "memory": "residual", "communicator": "allreduce"}),
    "u8bit": ("resnet50", {"compressor": "u8bit", "memory": "none", "communicator": "allreduce"}),
    "sketch": ("resnet50", {"compressor": "sketch", "memory": "none", "communicator": "allreduce"}),
    "dgc": ("resnet50", {"compressor": "dgc", "compress_ratio": 0.01, "memory": "dgc", "communicator": "allgather"}),
    "threshold": ("resnet50", {"compressor": "threshold", "threshold": 0.01, "memory": "residual",
                               "communicator": "allgather"}),
}


def run(name, model_name=None, iters=20, bucket_mb=128.0, graph=True, dev=None):
    dev = dev or torch.device("cuda", 0)
    mname, params = PIPELINES[name]
    mname = model_name or mname
    torch.manual_seed(0)
    model = MODELS[mname]().to(dev)
    grc = grace_from_params(dict(params, world_size=1))
    eng = GraceEngine(list(model.named_parameters()), grc, bucket_cap_mb=bucket_mb, overlap=False)
    eng.zero_grad(set_to_none=False)
    g = torch.Generator(device=dev).manual_seed(1)
    n = 0
    for b in eng.buckets:
        b.flat.normal_(generator=g)
        n += b.flat.numel()
    saved = [b.flat.clone() for b in eng.buckets]

    def body():
        for b, s in zip(eng.buckets, saved):
            b.flat.copy_(s)  # the decode overwrites the bucket: restore the gradient
        eng.synchronize()

    def restore_only():
        for b, s in zip(eng.buckets, saved):
            b.flat.copy_(s)

    use_graph = graph and graph_safe(grc) is None
    fn, fn0 = body, restore_only
    if use_graph:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                body()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        gr, gr0 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            body()
        with torch.cuda.graph(gr0):
            restore_only()
        fn, fn0 = gr.replay, gr0.replay
    for _ in range(3):
        fn()
    torch.cuda.synchronize()

    def timed(f):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            f()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters

    t_all = timed(fn)
    t_restore = timed(fn0)
    ms = max(t_all - t_restore, 1e-6)
    return {"pipeline": name, "model": mname, "elements": n, "buckets": len(eng.buckets),
            "graph": use_graph, "ms": round(ms, 4), "gradient_GBps": round(4 * n / ms / 1e6, 1)}


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--pipeline", default="topk,powersgd,efsignsgd,qsgd,none",
                    help=f"comma list of {sorted(PIPELINES)} or 'all'")
    ap.add_argument("--model", default=None)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--bucket-mb", type=float, default=128.0,
                    help="GraceEngine bucket cap (128 MB: the training default of bench.py)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    if not torch.cuda.is_available():
        raise SystemExit("needs a GPU")
    names = sorted(PIPELINES) if a.pipeline == "all" else a.pipeline.split(",")
    if not a.json:
        print(f"{'pipeline':10s} {'model':10s} {'elements':>10s} {'bkts':>4s} {'graph':>5s} {'ms':>8s} {'grad GB/s':>9s}")
    for nm in names:
        r = run(nm, a.model, a.iters, a.bucket_mb, not a.no_graph)
        if a.json:
            print(json.dumps(r), flush=True)
        else:
            print(f"{r['pipeline']:10s} {r['model']:10s} {r['elements']:10d} {r['buckets']:4d} {str(r['graph']):>5s} "
                  f"{r['ms']:8.3f} {r['gradient_GBps']:9.1f}", flush=True)


if __name__ == "__main__":
    main()
