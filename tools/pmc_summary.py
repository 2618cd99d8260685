#!/usr/bin/env python3
"""Pivot rocprofv3 ``--pmc`` counter_collection.csv files into one row per kernel.

    python tools/pmc_summary.py gpurun_out/pmc1/run_counter_collection.csv [more.csv ...] \
        [--grace] [--top 30]

Counters from several passes (one csv per pass) are merged by kernel name; values are the
mean per dispatch.  Derived columns when the inputs exist:

* ``MFMA%``  = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * #CU) -- share of CU cycles with the
  matrix core busy (gfx950: 256 CUs);
* ``LDSconf%`` = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE;
* ``MB rd`` / ``MB wr`` = FETCH_SIZE / WRITE_SIZE in MB (FETCH_SIZE under-counts wide
  coalesced streams by up to 2x on gfx950: MI355X_MICROARCH.md).
"""
import argparse
import collections
import csv
import re

N_CU = 256


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", name)[:90]


def load(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    disp = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName") or ""
            c = r.get("Counter_Name") or r.get("Counter-Name") or ""
            v = r.get("Counter_Value") or r.get("Counter-Value") or "0"
            d = r.get("Dispatch_Id") or r.get("Dispatch-Id") or ""
            acc[k][c].append(float(v))
            disp[k].add((p, d))
    return acc, disp


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--grace", action="store_true", help="only grace_amd kernels")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args(argv)
    acc, disp = load(a.csv)
    counters = sorted({c for k in acc.values() for c in k})
    rows = []
    for k, cs in acc.items():
        if a.grace and "grace::" not in k:
            continue
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        rows.append((k, mean, len(disp[k])))
    key = "SQ_WAVE_CYCLES" if "SQ_WAVE_CYCLES" in counters else (counters[0] if counters else "")
    rows.sort(key=lambda r: -r[1].get(key, 0))
    hdr = ["MFMA%", "LDSconf%", "MB rd", "MB wr"]
    print("counters:", ", ".join(counters))
    print(f"{'disp':>5} " + " ".join(f"{h:>9}" for h in hdr) + " " +
          " ".join(f"{c[:14]:>14}" for c in counters) + "  kernel")
    for k, m, nd in rows[: a.top]:
        mf = (100 * m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["SQ_BUSY_CYCLES"] * N_CU)
              if m.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in m else None)
        lc = (100 * m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
              if m.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in m else None)
        rd = m["FETCH_SIZE"] / 1024 if "FETCH_SIZE" in m else None
        wr = m["WRITE_SIZE"] / 1024 if "WRITE_SIZE" in m else None
        der = " ".join(f"{x:9.2f}" if x is not None else f"{'-':>9}" for x in (mf, lc, rd, wr))
        print(f"{nd:5d} {der} " + " ".join(f"{m.get(c, float('nan')):14.4g}" for c in counters) + f"  {short(k)}")


if __name__ == "__main__":
    main()
