#!/usr/bin/env python3
"""The largest idle gaps of one hardware queue in a rocprofv3 ``--kernel-trace`` CSV, with the
kernel before and after each gap and the kernels of OTHER queues that ran during it (what the
queue was waiting behind).

    python tools/trace_gaps.py gpurun_out/prof_x/run_kernel_trace.csv --steps 4 --marker nll_loss_forward --top 25
"""
import argparse
import collections
import csv
import re


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"<.*", "", name)
    return name.replace("void ", "")[:48]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--marker", default="nll_loss_forward")
    ap.add_argument("--queue", default=None, help="queue / stream id (default: the one with most kernel time)")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args(argv)
    rows = list(csv.DictReader(open(a.trace)))
    qkey = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r[qkey]) for r in rows)
    marks = [i for i, k in enumerate(ks) if a.marker in k[2]]
    t0, t1 = ks[marks[-1 - a.steps]][0], ks[marks[-1]][0]
    win = [k for k in ks if t0 <= k[0] < t1]
    tot = collections.Counter()
    for s, e, _, q in win:
        tot[q] += e - s
    q = a.queue or tot.most_common(1)[0][0]
    mine = [k for k in win if k[3] == q]
    others = [k for k in win if k[3] != q]
    gaps = []
    for prev, nxt in zip(mine, mine[1:]):
        g = nxt[0] - prev[1]
        if g > 0:
            during = [o for o in others if o[0] < nxt[0] and o[1] > prev[1]]
            gaps.append((g, prev, nxt, during))
    gaps.sort(key=lambda x: -x[0])
    total = sum(g for g, *_ in gaps)
    print(f"queue {q}: {len(mine) / a.steps:.0f} kernels/step, idle {total / 1e6 / a.steps:.3f} ms/step; "
          f"top {a.top} gaps (us): gap | before -> after | other queues' kernels during the gap")
    # what the queue waits behind, summed over all its gaps > 3 us
    behind = collections.Counter()
    for g, prev, nxt, during in gaps:
        if g > 3000:
            for o in during:
                behind[short(o[2])] += min(o[1], nxt[0]) - max(o[0], prev[1])
    for g, prev, nxt, during in gaps[:a.top]:
        d = ", ".join(f"{short(o[2])}({(o[1] - o[0]) / 1e3:.0f})" for o in during[:3])
        print(f"  {g / 1e3:7.1f} | {short(prev[2])} -> {short(nxt[2])} | {d}")
    print("other queues' kernel time inside this queue's gaps > 3 us (ms/step):")
    for n, t in behind.most_common(12):
        print(f"  {t / 1e6 / a.steps:7.3f}  {n}")


if __name__ == "__main__":
    main()
