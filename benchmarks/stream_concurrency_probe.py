#!/usr/bin/env python3
"""Do kernels on two HIP streams of one process run concurrently on this box?  Two one-thread
spin kernels (torch.cuda._sleep) on two streams: ~1x the single time if the hardware queues run
at once, ~2x if they are serviced one at a time.  Also eager vs graph-replayed, and a small-grid
GEMM pair."""
import json
import time

import torch


def timed(fn, reps=5):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    hi = torch.cuda.Stream(dev, priority=-1)
    cyc = 20_000_000  # ~10 ms at ~2 GHz
    out = {}
    torch.cuda._sleep(1000)
    out["one_sleep_ms"] = timed(lambda: torch.cuda._sleep(cyc))

    def two(a, b):
        def f():
            cur = torch.cuda.current_stream()
            a.wait_stream(cur)
            b.wait_stream(cur)
            with torch.cuda.stream(a):
                torch.cuda._sleep(cyc)
            with torch.cuda.stream(b):
                torch.cuda._sleep(cyc)
            cur.wait_stream(a)
            cur.wait_stream(b)
        return f

    out["two_streams_ms"] = timed(two(s1, s2))
    out["two_streams_prio_ms"] = timed(two(hi, s2))
    # many small kernels on stream 1 (a chain) + one spin on stream 2
    x = torch.randn(1 << 16, device=dev)

    def chain_plus_spin():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s2):
            torch.cuda._sleep(cyc)
        with torch.cuda.stream(s1):
            for _ in range(2000):
                x.add_(1.0)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    def chain_only():
        for _ in range(2000):
            x.add_(1.0)

    out["chain_only_ms"] = timed(chain_only)
    out["chain_plus_spin_ms"] = timed(chain_plus_spin)
    # the same two-stream pattern captured in ONE forked graph and replayed
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(dev)
    with torch.cuda.stream(cs):
        f = two(s1, s2)
        f()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=cs):
            f()
    out["graph_two_streams_ms"] = timed(g.replay)
    # TWO graphs (one spin each) replayed on two streams: do separate graph launches overlap?
    ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    with torch.cuda.graph(ga, stream=s1):
        torch.cuda._sleep(cyc)
    with torch.cuda.graph(gb, stream=s2):
        torch.cuda._sleep(cyc)

    def two_graphs():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            ga.replay()
        with torch.cuda.stream(s2):
            gb.replay()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    out["two_graphs_two_streams_ms"] = timed(two_graphs)

    # a graph on s1 + an EAGER spin on s2
    def graph_plus_eager():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            ga.replay()
        with torch.cuda.stream(s2):
            torch.cuda._sleep(cyc)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    out["graph_plus_eager_ms"] = timed(graph_plus_eager)
    print(json.dumps({k: round(v, 3) for k, v in out.items()}))


if __name__ == "__main__":
    main()
