#!/usr/bin/env python3
"""Per-kernel call counts and total time from a rocprofv3 SQLite output (rocpd .db), for diffing
two configurations:  python3 tools/db_kernel_counts.py a.db [b.db]  (with two: only the kernels
whose counts differ)."""
import glob
import sqlite3
import sys


def table(path):
    db = path if path.endswith(".db") else glob.glob(path.rstrip("/") + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration) / 1000.0 from kernels group by name").fetchall()
    return {r[0][:110]: (r[1], r[2]) for r in rows}


def main():
    a = table(sys.argv[1])
    if len(sys.argv) < 3:
        for k, (n, us) in sorted(a.items(), key=lambda kv: -kv[1][1]):
            print(f"{n:7d} {us:12.1f} us  {k}")
        return
    b = table(sys.argv[2])
    for k in sorted(set(a) | set(b)):
        na, ua = a.get(k, (0, 0.0))
        nb, ub = b.get(k, (0, 0.0))
        if na != nb:
            print(f"{na:7d} {nb:7d}  {ua:10.1f} {ub:10.1f} us  {k}")


if __name__ == "__main__":
    main()
