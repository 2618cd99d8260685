#!/usr/bin/env python3
"""In-order listing of the kernels of ONE step from a rocprofv3 --kernel-trace CSV (the step
before the last ``--marker`` kernel), filtered by ``--match`` (substring of the normalised
name): duration and grid, so per-layer costs can be read in program order.

    python tools/trace_seq.py run_kernel_trace.csv --marker nll_loss_forward --match bn_
"""
import argparse
import csv
import re


def norm(k: str) -> str:
    k = k.replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", k)[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="nll_loss_forward")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    lo, hi = marks[-3], marks[-2]  # one whole step
    tot = 0.0
    print(f"{'us':>8}  grid_x x grid_y  kernel")
    for r in rows[lo:hi]:
        k = norm(r["Kernel_Name"])
        if a.match not in k:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        print(f"{d:8.2f}  {r.get('Grid_Size_X', '?')} x {r.get('Grid_Size_Y', '?')}  {k}")
    print(f"total {tot:.1f} us")


if __name__ == "__main__":
    main()
