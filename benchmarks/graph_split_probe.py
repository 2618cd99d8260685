#!/usr/bin/env python3
"""Probe: a two-stream step as ONE forked HIP graph vs as TWO linear graphs joined by external
event nodes (fork-free wgrad concurrency without losing the graph fast path).

Pattern (ResNet-backward-shaped): a main chain of ``L`` layers of small latency-bound kernels; after
layer l the main stream records an event, and a side stream waits for it and runs an MFMA-bound
GEMM that reads layer l's output (a weight gradient).  Variants:

  forked   one capture on S1; the side stream joins it through ordinary events (torch's fork /
           join pattern): one graph with parallel branches
  split    TWO captures running at once: the main chain on S1 (graph A, linear) and the side
           GEMMs on S2 (graph B, linear); S1 records ``external`` events, S2 waits on them with
           the external flag (event-record / event-wait nodes).  Replay: A on S1, B on S2, then an
           eager join of S2 into S1
  serial   everything on S1 (linear graph, no concurrency)

Reports per variant: host issue time per replay, device time per replay (events), and a
correctness check that every side GEMM read ITS replay's layer output (a replay counter is
folded into the main chain's values).
"""
from __future__ import annotations

import argparse
import json
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=48)
    ap.add_argument("--chain", type=int, default=6, help="small kernels per layer on the main stream")
    ap.add_argument("--m", type=int, default=1024, help="side GEMM size (m x m x m fp32)")
    ap.add_argument("--elems", type=int, default=1 << 16, help="elements of each main-chain tensor")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.backends.cuda.matmul.allow_tf32 = False
    L = a.layers
    ctr = torch.zeros(1, device=dev)
    xs = [torch.zeros(a.elems, device=dev) for _ in range(L)]
    ws = [torch.randn(a.m, a.m, device=dev) / a.m ** 0.5 for _ in range(L)]
    outs = [torch.zeros(a.m, a.m, device=dev) for _ in range(L)]
    probe = torch.zeros(L, device=dev)  # side stream's copy of xs[l][0] (must equal ctr * (l + 1))
    S1, S2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def main_layer(l):
        x = xs[l]
        x.copy_(ctr.expand_as(x))
        x.mul_(l + 1)
        for _ in range(a.chain - 2):
            x.add_(0.0)

    def side_layer(l):
        probe[l].copy_(xs[l][0])
        torch.mm(ws[l], ws[(l + 1) % L], out=outs[l])

    results = {}

    def run_variant(name, replay):
        # correctness: replays bump ctr; the side stream's probe must see this replay's values
        ok = True
        for it in range(3):
            replay()
            torch.cuda.synchronize()
            c = float(ctr.item())
            want = torch.arange(1, L + 1, device=dev, dtype=torch.float32) * c
            ok &= bool(torch.equal(probe, want))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            replay()
        issue = (time.perf_counter() - t0) / a.iters * 1e3
        e1.record()
        torch.cuda.synchronize()
        dev_ms = e0.elapsed_time(e1) / a.iters
        results[name] = {"issue_ms": round(issue, 3), "device_ms": round(dev_ms, 3), "correct": ok}
        print(name, results[name], flush=True)

    # ---------------------------------------------------------------- serial
    def step_serial():
        ctr.add_(1)
        for l in range(L):
            main_layer(l)
            side_layer(l)

    for _ in range(2):
        step_serial()
    torch.cuda.synchronize()
    gs = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gs):
        step_serial()
    run_variant("serial", gs.replay)

    # ---------------------------------------------------------------- forked (one graph)
    def step_forked():
        cur = torch.cuda.current_stream()
        ctr.add_(1)
        for l in range(L):
            main_layer(l)
            ev = torch.cuda.Event()
            ev.record(cur)
            S2.wait_event(ev)
            with torch.cuda.stream(S2):
                side_layer(l)
        cur.wait_stream(S2)

    with torch.cuda.stream(S1):
        for _ in range(2):
            step_forked()
    torch.cuda.synchronize()
    gf = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gf, stream=S1):
        step_forked()
    run_variant("forked", gf.replay)

    # ---------------------------------------------------------------- split (two linear graphs)
    # PyTorch-ROCm refuses torch.cuda.Event(external=True): the native ExtEvent issues
    # hipEventRecordWithFlags(External) / hipStreamWaitEvent(WaitExternal) while capturing
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import grace_amd._C as C

    evs = [C.ExtEvent(0) for _ in range(L)]

    def main_part():
        ctr.add_(1)
        for l in range(L):
            main_layer(l)
            evs[l].record(S1.cuda_stream)

    def side_part():
        for l in range(L):
            evs[l].wait(S2.cuda_stream)
            side_layer(l)

    for _ in range(2):  # eager warm-up of the same issue pattern
        with torch.cuda.stream(S1):
            main_part()
        with torch.cuda.stream(S2):
            side_part()
        S1.wait_stream(S2)
    torch.cuda.synchronize()
    ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    err = None
    try:
        with torch.cuda.stream(S1):
            ga.capture_begin(capture_error_mode="thread_local")
        with torch.cuda.stream(S2):
            gb.capture_begin(capture_error_mode="thread_local")
        with torch.cuda.stream(S1):
            main_part()
        with torch.cuda.stream(S2):
            side_part()
        with torch.cuda.stream(S2):
            gb.capture_end()
        with torch.cuda.stream(S1):
            ga.capture_end()
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {str(e)[:300]}"
        print("split capture failed:", err, flush=True)
        for g, st in ((gb, S2), (ga, S1)):  # end any capture still open (a live one aborts at exit)
            try:
                with torch.cuda.stream(st):
                    g.capture_end()
            except Exception:  # noqa: BLE001
                pass
    if err is None:
        join_ev = torch.cuda.Event()

        def replay_split():
            cur = torch.cuda.current_stream()
            S1.wait_stream(cur)
            S2.wait_stream(cur)
            with torch.cuda.stream(S1):
                ga.replay()
            with torch.cuda.stream(S2):
                gb.replay()
            join_ev.record(S2)
            cur.wait_event(join_ev)
            cur.wait_stream(S1)

        run_variant("split", replay_split)
    else:
        results["split"] = {"error": err}

    # ---------------------------------------------------------------- split, flag-word sync
    flags = torch.zeros(L, dtype=torch.int64, device=dev)
    gen_a = torch.zeros(1, dtype=torch.int64, device=dev)
    gen_b = torch.zeros(1, dtype=torch.int64, device=dev)
    limit = 1 << 24

    def main_part_f():
        C.xs_bump(gen_a, S1.cuda_stream)
        ctr.add_(1)
        for l in range(L):
            main_layer(l)
            C.xs_signal(flags, l, gen_a, S1.cuda_stream)

    def side_part_f():
        C.xs_bump(gen_b, S2.cuda_stream)
        for l in range(L):
            C.xs_wait(flags, l, gen_b, limit, S2.cuda_stream)
            side_layer(l)

    for _ in range(2):
        with torch.cuda.stream(S1):
            main_part_f()
        with torch.cuda.stream(S2):
            side_part_f()
        S1.wait_stream(S2)
    torch.cuda.synchronize()
    fa, fb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.stream(S1):
        fa.capture_begin(capture_error_mode="thread_local")
    with torch.cuda.stream(S2):
        fb.capture_begin(capture_error_mode="thread_local")
    with torch.cuda.stream(S1):
        main_part_f()
    with torch.cuda.stream(S2):
        side_part_f()
    with torch.cuda.stream(S2):
        fb.capture_end()
    with torch.cuda.stream(S1):
        fa.capture_end()
    jev = torch.cuda.Event()

    def replay_flags():
        cur = torch.cuda.current_stream()
        S1.wait_stream(cur)
        S2.wait_stream(cur)
        with torch.cuda.stream(S1):
            fa.replay()
        with torch.cuda.stream(S2):
            fb.replay()
        jev.record(S2)
        cur.wait_event(jev)
        cur.wait_stream(S1)

    run_variant("split_flags", replay_flags)
    print(json.dumps({"probe": "graph_split", "layers": L, "chain": a.chain, "m": a.m, "results": results}))


if __name__ == "__main__":
    main()
