#!/usr/bin/env python3
"""Per (kernel, grid) mean duration from a rocprofv3 --kernel-trace CSV.

    python tools/trace_by_grid.py run_kernel_trace.csv --match grace::bn_ [--top 60]
"""
import argparse
import collections
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(a.csv)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))[:60]
        if a.match not in k:
            continue
        grid = (r.get("Grid_Size_X", "?"), r.get("Grid_Size_Y", "?"))
        acc[(k, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
    print(f"{'total_us':>9} {'n':>5} {'mean_us':>8} {'min_us':>8}  grid  kernel")
    for (k, g), v in rows[: a.top]:
        print(f"{sum(v):9.1f} {len(v):5d} {sum(v) / len(v):8.2f} {min(v):8.2f}  {g[0]}x{g[1]}  {k}")


if __name__ == "__main__":
    main()
