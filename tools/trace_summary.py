#!/usr/bin/env python3
"""Kernel-time summary of a rocprofv3 --kernel-trace run (the rocpd SQLite database, or kernel_trace.csv): per kernel
name the calls, total and mean time; and over a window bracketed by the first / last call of a marker kernel (default
k_mf_decide: the multi-frame series), the wall time, the GPU-busy time (union of kernel intervals) and the idle share.

    python tools/trace_summary.py gpurun_out/prof_sparse16 [--marker k_mf_decide] [--top 25] [--json out.json]
"""
import argparse
import csv
import glob
import json
import os
import sqlite3
from collections import defaultdict


def load(path):
    """[(name, start_ns, end_ns)] of every kernel dispatch under path (a .db, a .csv or a directory of them)."""
    files = [path] if os.path.isfile(path) else (glob.glob(os.path.join(path, "**", "*.db"), recursive=True) or
                                                  glob.glob(os.path.join(path, "**", "*kernel_trace.csv"),
                                                            recursive=True))
    out = []
    for f in files:
        if f.endswith(".db"):
            c = sqlite3.connect(f)
            out += [(n, int(s), int(e)) for n, s, e in c.execute("select name, start, end from kernels")]
        else:
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    out.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(out, key=lambda t: t[1])


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").strip()


def summarize(ks, marker="k_mf_decide", top=25):
    per = defaultdict(lambda: [0, 0])
    for n, s, e in ks:
        p = per[short(n)]
        p[0] += 1
        p[1] += e - s
    rows = sorted(per.items(), key=lambda kv: -kv[1][1])
    res = {"kernels": [{"name": k, "calls": v[0], "total_ms": v[1] / 1e6, "mean_us": v[1] / v[0] / 1e3}
                       for k, v in rows[:top]]}
    idx = [i for i, (n, _, _) in enumerate(ks) if short(n).endswith(marker)]
    if idx:
        w = ks[idx[0]:idx[-1] + 1]
        t0, t1 = w[0][1], w[-1][2]
        busy, cur_s, cur_e = 0, None, None
        for _, s, e in w:  # union of the intervals (kernels of one stream do not overlap; a second stream may)
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        res["window"] = {"marker": marker, "calls": len(idx), "wall_ms": (t1 - t0) / 1e6, "busy_ms": busy / 1e6,
                         "idle_share": 1.0 - busy / max(1, t1 - t0),
                         "per_marker_us": (t1 - t0) / 1e3 / max(1, len(idx))}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--marker", default="k_mf_decide")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--json")
    a = ap.parse_args()
    res = summarize(load(a.path), a.marker, a.top)
    for k in res["kernels"]:
        print(f"{k['calls']:8d} {k['total_ms']:10.3f} ms {k['mean_us']:9.2f} us  {k['name']}")
    if "window" in res:
        print(json.dumps(res["window"]))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
