#!/usr/bin/env python3
"""Print the top kernels of a rocprofv3 ``--stats`` kernel_stats.csv (per-call and total time).

    python tools/prof_stats.py gpurun_out/prof/run_kernel_stats.csv --top 25 [--per N]

``--per N`` divides totals by N (e.g. the number of steps the profiled process ran) to give
per-step figures.
"""
import argparse
import csv
import re


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", name)[:100]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--grace", action="store_true", help="also list every grace_amd kernel")
    a = ap.parse_args(argv)
    rows = list(csv.DictReader(open(a.stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    grace = sum(float(r["TotalDurationNs"]) for r in rows if "grace::" in r["Name"])
    print(f"total kernel time {tot / 1e6 / a.per:.3f} ms (per {a.per:g}); grace_amd kernels "
          f"{grace / 1e6 / a.per:.3f} ms ({100 * grace / max(tot, 1):.1f}%)")
    print(f"{'ms':>9} {'calls':>8} {'us/call':>9}  kernel")
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[: a.top]:
        t = float(r["TotalDurationNs"])
        c = int(r["Calls"])
        print(f"{t / 1e6 / a.per:9.3f} {c / a.per:8.1f} {t / 1e3 / max(c, 1):9.1f}  {short(r['Name'])}")
    if a.grace:
        print("grace_amd kernels:")
        for r in rows:
            if "grace::" in r["Name"]:
                t = float(r["TotalDurationNs"])
                c = int(r["Calls"])
                print(f"{t / 1e6 / a.per:9.3f} {c / a.per:8.1f} {t / 1e3 / max(c, 1):9.1f}  {short(r['Name'])}")


if __name__ == "__main__":
    main()
