#!/usr/bin/env python3
"""Which kernels run right before / after a given kernel (rocprofv3 --kernel-trace CSV).

Answers "who launches this memset / cast?" for library-internal kernels that carry no
caller information (e.g. MIOpen's SubTensorOpWithScalar1d, HIP's fillBufferAligned).

    python tools/trace_neighbors.py run_kernel_trace.csv --match fillBufferAligned [--last 200]
"""
import argparse
import collections
import csv
import re


def short(k):
    return re.sub(r"\(.*", "", k.replace("(anonymous namespace)::", ""))[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", action="append", required=True)
    ap.add_argument("--last", type=int, default=0, help="only the last N kernels of the trace (steady state)")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    if a.last:
        rows = rows[-a.last:]
    names = [short(r["Kernel_Name"]) for r in rows]
    for m in a.match:
        prev, nxt = collections.Counter(), collections.Counter()
        for i, n in enumerate(names):
            if m in n:
                prev[names[i - 1] if i else "<start>"] += 1
                nxt[names[i + 1] if i + 1 < len(names) else "<end>"] += 1
        print(f"== {m}: {sum(prev.values())} occurrences")
        print("  before:")
        for k, c in prev.most_common(8):
            print(f"    {c:5d}  {k}")
        print("  after:")
        for k, c in nxt.most_common(8):
            print(f"    {c:5d}  {k}")


if __name__ == "__main__":
    main()
