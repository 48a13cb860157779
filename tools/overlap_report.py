#!/usr/bin/env python3
"""Overlap of the per-sweep all-reduce with compute, from a rocprofv3 kernel trace (CSV) of one rank.

Usage: overlap_report.py <run_kernel_trace.csv> [--out report.json]

Counts the all-reduce kernels (the one-shot P2P kernel, ``k_p2p``) and, for each, the time it ran while a
back-projection chunk of the same process (``k_mf_backproject``) was running on the compute stream. The
multi-frame engine queues the back-projection in voxel chunks and reduces chunk c on its comm stream next to
chunks c + 1 ... (csrc/engine/multiframe.cpp, MultiFrameEngine::sweep)."""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ar = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]) for r in rows if "p2p" in r["Kernel_Name"]]
    bp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]) for r in rows
          if "k_mf_backproject" in r["Kernel_Name"]]
    bp.sort()
    total = overl = 0
    n_overlapped = 0
    for s, e, _ in ar:
        total += e - s
        o = 0
        for bs, be, _ in bp:
            if be <= s:
                continue
            if bs >= e:
                break
            o += min(e, be) - max(s, bs)
        overl += min(o, e - s)
        n_overlapped += o > 0
    rep = {"allreduce_kernels": len(ar), "backproject_kernels": len(bp),
           "allreduce_streams": sorted({x[2] for x in ar}), "backproject_streams": sorted({x[2] for x in bp}),
           "allreduce_us": total / 1e3, "allreduce_us_overlapped_with_backprojection": overl / 1e3,
           "overlapped_fraction": (overl / total) if total else None, "allreduce_calls_overlapped": n_overlapped}
    print(json.dumps(rep))
    if a.out:
        json.dump(rep, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
