#!/usr/bin/env python3
"""Per-queue view of a rocprofv3 ``--kernel-trace`` CSV of graphed steps (several HIP streams).

For the last ``--steps`` steps (delimited by a marker kernel) prints, per hardware queue / stream
id: kernel count and summed kernel time per step; the time the queues overlap; and the timeline
of the step's last ``--tail`` kernels (start offset from the step's end, duration, queue) -- where
the end of a step waits on the side stream.

    python tools/trace_streams.py gpurun_out/prof/run_kernel_trace.csv --steps 8 --marker nll_loss_forward
"""
import argparse
import collections
import csv
import re
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"<.*", "", name)
    return name[:70]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--marker", default="nll_loss_forward")
    ap.add_argument("--tail", type=int, default=30)
    args = ap.parse_args(argv)
    rows = list(csv.DictReader(open(args.trace)))
    qkey = "Stream_Id" if "Stream_Id" in rows[0] else ("Queue_Id" if "Queue_Id" in rows[0] else None)
    if qkey is None:
        sys.exit(f"no Stream_Id / Queue_Id column: {list(rows[0])}")
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r[qkey]) for r in rows)
    marks = [i for i, k in enumerate(ks) if args.marker in k[2]]
    if len(marks) < args.steps + 1:
        sys.exit("not enough marker kernels")
    t0 = ks[marks[-1 - args.steps]][0]
    t1 = ks[marks[-1]][0]
    win = [k for k in ks if t0 <= k[0] < t1]
    per_q = collections.defaultdict(lambda: [0, 0])
    for s, e, n, q in win:
        per_q[q][0] += 1
        per_q[q][1] += e - s
    print(f"{args.steps} steps, {(t1 - t0) / 1e6 / args.steps:.3f} ms/step between markers ({qkey})")
    for q, (c, t) in sorted(per_q.items(), key=lambda kv: -kv[1][1]):
        print(f"  queue {q:>6}: {c / args.steps:6.1f} kernels/step, {t / 1e6 / args.steps:7.3f} ms/step of kernel time")
    # per queue: idle gaps between consecutive kernels (dependency waits, launch / marker latency)
    byq = collections.defaultdict(list)
    for s_, e_, _, q in win:
        byq[q].append((s_, e_))
    for q, iv in sorted(byq.items()):
        iv.sort()
        gaps = [b[0] - a[1] for a, b in zip(iv, iv[1:]) if b[0] > a[1]]
        big = [g for g in gaps if g > 3000]
        print(f"  queue {q:>6}: idle between kernels {sum(gaps) / 1e6 / args.steps:7.3f} ms/step; "
              f"{len(big) / args.steps:5.1f} gaps/step > 3 us totalling {sum(big) / 1e6 / args.steps:7.3f} ms/step")
    # union busy time and the time two or more queues run at once
    ev = []
    for s, e, _, _ in win:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    active, last, busy, multi = 0, None, 0, 0
    for t, d in ev:
        if last is not None and active > 0:
            busy += t - last
            if active > 1:
                multi += t - last
        active += d
        last = t
    print(f"busy {busy / 1e6 / args.steps:.3f} ms/step, >= 2 kernels at once {multi / 1e6 / args.steps:.3f} ms/step")
    # the last step's tail: which kernels end the step, on which queue
    s_prev = ks[marks[-2]][0]
    step = [k for k in ks if s_prev <= k[0] < t1]
    end = max(e for _, e, _, _ in step)
    print(f"\nlast step: {(t1 - s_prev) / 1e3:.1f} us between markers; its last {args.tail} kernels "
          f"(start / end relative to the step's last kernel end, us):")
    for s, e, n, q in step[-args.tail:]:
        print(f"  {(s - end) / 1e3:9.1f} {(e - end) / 1e3:9.1f}  {(e - s) / 1e3:7.1f}  q{q:>4}  {short(n)}")


if __name__ == "__main__":
    main()
