#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--kernel-trace`` CSV over the steady-state steps of a bench run.

Steps are delimited by a marker kernel (default: the last GRACE kernel of a step,
``topk_compact_kernel``); the summary covers the last ``--steps`` steps: wall time per step
(first kernel start -> last kernel end), busy GPU time per step (union of kernel intervals),
and the top kernels by time, with grace_amd kernels tagged.

    python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steps 10 --marker topk_compact
"""
import argparse
import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    if "elementwise_kernel" in name or "reduce_kernel" in name:
        # keep the functor: "vectorized_elementwise_kernel[bfloat16_copy_kernel_cuda]"
        fn = re.findall(r"([A-Za-z0-9_]+(?:_kernel_cuda|_kernel_impl|Functor[A-Za-z0-9_]*|_kernel))", name)
        base = re.sub(r"<.*", "", re.sub(r"\(.*", "", name))
        tags = [f for f in dict.fromkeys(fn) if f not in base]
        return (base + ("[" + ",".join(tags[:2]) + "]" if tags else ""))[:110]
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"<.*", "", name)
    return name[:90]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--marker", default="topk_compact_kernel")
    ap.add_argument("--per-step-markers", type=int, default=0, help="marker kernels per step (0 = auto)")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--gaps", type=int, default=0, help="also list the N largest idle gaps (kernel pairs)")
    ap.add_argument("--gap-min-us", type=float, default=5.0)
    ap.add_argument("--grid-match", default="", help="also list per-(kernel, grid) times of kernels matching this")
    args = ap.parse_args(argv)
    rows = list(csv.DictReader(open(args.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    grids = {(int(r["Start_Timestamp"]), r["Kernel_Name"]): (r.get("Grid_Size_X", "?"), r.get("Grid_Size_Y", "?"))
             for r in rows}
    marks = [i for i, k in enumerate(ks) if args.marker in k[2]]
    if not marks:
        sys.exit(f"marker {args.marker!r} not found")
    per = args.per_step_markers
    if per == 0:  # markers per step: guess from the last gaps
        per = 1
    # window: from the end of the marker that closes step (last - steps) to the last marker
    last = marks[-1]
    first_idx = len(marks) - 1 - args.steps * per
    start_t = ks[marks[first_idx]][1] if first_idx >= 0 else ks[0][0]
    end_t = ks[last][1]
    win = [k for k in ks if k[0] >= start_t and k[1] <= end_t]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    wall = end_t - start_t
    agg = collections.defaultdict(lambda: [0, 0])
    for s, e, n in win:
        a = agg[short(n)]
        a[0] += e - s
        a[1] += 1
    total = sum(v[0] for v in agg.values())
    steps = args.steps
    print(f"window: {steps} steps, wall {wall / 1e6 / steps:.3f} ms/step, GPU busy {busy / 1e6 / steps:.3f} ms/step "
          f"({100 * busy / max(1, wall):.1f}%), kernels {len(win) / steps:.0f}/step, sum of kernel time "
          f"{total / 1e6 / steps:.3f} ms/step")
    if args.grid_match:
        by = collections.defaultdict(list)
        for s_, e, n in win:
            if args.grid_match in n:
                t = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "").replace("void ", ""))[:58]
                by[(t, grids.get((s_, n), ("?", "?")))].append((e - s_) / 1e3)
        print(f"per (kernel, grid), kernels matching {args.grid_match!r}:")
        print(f"{'us/step':>8} {'n/step':>6} {'mean_us':>8}  grid  kernel")
        for (t, g), v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            print(f"{sum(v) / steps:8.1f} {len(v) / steps:6.1f} {sum(v) / len(v):8.2f}  {g[0]}x{g[1]}  {t}")
        print()
    grace = sum(v[0] for k, v in agg.items() if k.startswith("grace::") or "grace" in k)
    print(f"grace_amd kernels: {grace / 1e6 / steps:.3f} ms/step ({100 * grace / max(1, total):.1f}% of kernel time)")
    print(f"{'ms/step':>8} {'calls/step':>10}  kernel")
    for n, (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[: args.top]:
        print(f"{t / 1e6 / steps:8.3f} {c / steps:10.1f}  {n}")
    if args.gaps:
        # idle time between the end of everything launched so far and the next kernel start
        pairs = collections.defaultdict(lambda: [0, 0])
        hi, prev = None, None
        for s, e, n in win:
            if hi is not None and s - hi > args.gap_min_us * 1e3:
                g = pairs[(short(prev)[:45], short(n)[:45])]
                g[0] += s - hi
                g[1] += 1
            if hi is None or e > hi:
                hi, prev = e, n
        idle = sum(v[0] for v in pairs.values())
        print(f"\nidle gaps > {args.gap_min_us} us: {idle / 1e6 / steps:.3f} ms/step")
        print(f"{'ms/step':>8} {'n/step':>7}  after -> before")
        for (a, b), (t, c) in sorted(pairs.items(), key=lambda kv: -kv[1][0])[: args.gaps]:
            print(f"{t / 1e6 / steps:8.3f} {c / steps:7.1f}  {a} -> {b}")


if __name__ == "__main__":
    main()
