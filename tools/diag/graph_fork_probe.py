"""Does a forked branch inside a captured HIP graph run beside a latency-bound main branch?

main: 300 small elementwise kernels (latency bound, like the BN passes of a backward);
side: 30 fp32 GEMMs, one forked after every 10th main kernel (like a wgrad per conv), waiting
only for that main kernel; main joins the side at the end.  If the branches overlap, a replay
takes ~max(main, side); serialised it takes the sum."""
import time

import torch

dev = torch.device("cuda", 0)
n = 2048
a = torch.randn(n, n, device=dev)
b = torch.randn(n, n, device=dev)
x = torch.randn(1 << 20, device=dev)
outs = [torch.empty(n, n, device=dev) for _ in range(30)]
side = torch.cuda.Stream()


def main_only():
    for i in range(300):
        x.add_(1.0)


def side_only():
    for j in range(30):
        torch.mm(a, b, out=outs[j])


def forked(many=True):
    main = torch.cuda.current_stream()
    for i in range(300):
        x.add_(1.0)
        if i % 10 == 0 and (many or i == 0):
            ev = torch.cuda.Event()
            ev.record(main)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                for j in range(i // 10, i // 10 + 1) if many else range(30):
                    torch.mm(a, b, out=outs[j])
    main.wait_stream(side)


def serial():
    main_only()
    side_only()


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t = time.perf_counter()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    host = (time.perf_counter() - t) / reps * 1e3
    e.synchronize()
    return s.elapsed_time(e) / reps, host


def graphed(fn):
    g = torch.cuda.CUDAGraph()
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        with torch.cuda.graph(g):
            fn()
    torch.cuda.synchronize()
    return g.replay


cases = [("main only", main_only), ("side only", side_only), ("serial", serial),
         ("forked x30", lambda: forked(True)), ("forked x1", lambda: forked(False))]
for name, fn in cases:
    d, h = timeit(fn)
    print(f"eager {name:11s}: {d:.3f} ms/iter (host {h:.3f})", flush=True)
for name, fn in cases:
    d, h = timeit(graphed(fn))
    print(f"graph {name:11s}: {d:.3f} ms/replay (host {h:.3f})", flush=True)
