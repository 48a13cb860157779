#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 counter runs (``--kernel-trace --pmc ... --output-format csv``).

For every run directory given: the counters summed per kernel over its dispatches, the kernel-trace time of
those dispatches, and the derived HBM read rate (FETCH_SIZE is in KiB) and occupancy (SQ_WAVE_CYCLES /
SQ_BUSY_CYCLES and SQ_LEVEL_WAVES / SQ_BUSY_CYCLES: mean resident waves, summed over the SEs / XCDs that count
them; divide by the CUs per counting unit for waves per CU). Unknown columns are skipped, so the script runs on
any pass.

  python tools/pmc_summary.py gpurun_out/pmc_head_fetch gpurun_out/pmc_head_occ
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    name = name.strip('"')
    for sep in ("(", "<"):
        i = name.find(sep)
        if i > 0:
            name = name[:i]
    return name.replace("void ", "").strip()


def find(d, suffix):
    return sorted(glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True))


def summarize(d):
    durs = defaultdict(float)
    nd = defaultdict(int)
    for f in find(d, "kernel_trace.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", "?"))
                durs[k] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
                nd[k] += 1
    ctr = defaultdict(lambda: defaultdict(float))
    for f in find(d, "counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", "?"))
                try:
                    v = float(row["Counter_Value"])
                except (KeyError, TypeError, ValueError):  # a counter the pass could not read
                    continue
                ctr[k][row["Counter_Name"]] += v
    out = []
    for k in sorted(set(durs) | set(ctr), key=lambda k: -durs.get(k, 0.0)):
        c = ctr.get(k, {})
        line = {"kernel": k, "dispatches": nd.get(k, 0), "ms": round(durs.get(k, 0.0), 3)}
        for name, v in sorted(c.items()):
            line[name] = v
        if "FETCH_SIZE" in c and durs.get(k):
            line["fetch_GB"] = round(c["FETCH_SIZE"] * 1024 / 1e9, 3)
            line["fetch_TBps"] = round(c["FETCH_SIZE"] * 1024 / (durs[k] * 1e-3) / 1e12, 3)
        if c.get("SQ_BUSY_CYCLES"):
            if "SQ_WAVE_CYCLES" in c:
                line["wave_cycles_per_busy_cycle"] = round(c["SQ_WAVE_CYCLES"] / c["SQ_BUSY_CYCLES"], 2)
            if "SQ_LEVEL_WAVES" in c:
                line["level_waves_per_busy_cycle"] = round(c["SQ_LEVEL_WAVES"] / c["SQ_BUSY_CYCLES"], 2)
        if c.get("SQ_INSTS_MFMA") and c.get("SQ_INSTS_VALU"):
            line["valu_per_mfma"] = round(c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"], 2)
        out.append(line)
    return out


def main():
    for d in sys.argv[1:]:
        if not os.path.isdir(d):
            continue
        print(f"## {d}")
        for line in summarize(d):
            if line["ms"] < 0.05 and line["dispatches"] > 0:
                continue
            print("  " + ", ".join(f"{k}={v:.6g}" if isinstance(v, float) else f"{k}={v}" for k, v in line.items()))


if __name__ == "__main__":
    main()
