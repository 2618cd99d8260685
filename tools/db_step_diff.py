#!/usr/bin/env python3
"""Kernel multiset of one training step (between the last two launches of a marker kernel) in two
rocprofv3 SQLite outputs, and their difference: python3 tools/db_step_diff.py A_dir B_dir [marker]"""
import collections
import glob
import sqlite3
import sys


def step_kernels(path, marker):
    db = glob.glob(path.rstrip("/") + "/**/*.db", recursive=True)[0]
    rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    a, b = idx[-3], idx[-2]  # a full step well inside the timed region
    c = collections.Counter(r[0][:100] for r in rows[a:b])
    return c, (rows[b][1] - rows[a][1]) / 1e3


def main():
    marker = sys.argv[3] if len(sys.argv) > 3 else "nll_loss_forward"
    ca, ta = step_kernels(sys.argv[1], marker)
    cb, tb = step_kernels(sys.argv[2], marker)
    print(f"step A: {sum(ca.values())} kernels {ta:.1f} us | step B: {sum(cb.values())} kernels {tb:.1f} us")
    for k in sorted(set(ca) | set(cb)):
        if ca[k] != cb[k]:
            print(f"{ca[k]:5d} {cb[k]:5d}  {k}")


if __name__ == "__main__":
    main()
