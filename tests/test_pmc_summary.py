"""tools/pmc_summary.py (the per-kernel summary of rocprofv3 counter runs committed under profiles/): counters summed per
kernel over its dispatches, joined with the kernel-trace times, and the derived read rate and occupancy ratios."""
import csv
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load():
    spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(ROOT, "tools", "pmc_summary.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _write(path, rows):
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)


def test_summary_joins_counters_and_trace(tmp_path):
    d = tmp_path / "pmc_x" / "host"
    d.mkdir(parents=True)
    k = "void sart::k_fused_sweep_rows<false, true>(float const*, long)"
    _write(d / "run_kernel_trace.csv", [
        {"Dispatch_Id": 1, "Kernel_Name": k, "Start_Timestamp": 1000, "End_Timestamp": 2_001_000},
        {"Dispatch_Id": 2, "Kernel_Name": k, "Start_Timestamp": 3_000_000, "End_Timestamp": 5_000_000},
        {"Dispatch_Id": 3, "Kernel_Name": "sart::k_tail(int)", "Start_Timestamp": 6_000_000, "End_Timestamp": 6_005_000},
    ])
    _write(d / "run_counter_collection.csv", [
        {"Dispatch_Id": 1, "Kernel_Name": k, "Counter_Name": "FETCH_SIZE", "Counter_Value": 4.0e6},
        {"Dispatch_Id": 2, "Kernel_Name": k, "Counter_Name": "FETCH_SIZE", "Counter_Value": 4.0e6},
        {"Dispatch_Id": 1, "Kernel_Name": k, "Counter_Name": "SQ_WAVE_CYCLES", "Counter_Value": 1200},
        {"Dispatch_Id": 1, "Kernel_Name": k, "Counter_Name": "SQ_BUSY_CYCLES", "Counter_Value": 100},
        {"Dispatch_Id": 3, "Kernel_Name": "sart::k_tail(int)", "Counter_Name": "FETCH_SIZE", "Counter_Value": "n/a"},
    ])
    rows = {r["kernel"]: r for r in _load().summarize(str(tmp_path / "pmc_x"))}
    r = rows["sart::k_fused_sweep_rows"]
    assert r["dispatches"] == 2 and abs(r["ms"] - 4.0) < 1e-9
    assert r["FETCH_SIZE"] == 8.0e6
    assert abs(r["fetch_GB"] - 8.192) < 1e-3  # KiB
    assert abs(r["fetch_TBps"] - 8.0e6 * 1024 / 4e-3 / 1e12) < 1e-3
    assert r["wave_cycles_per_busy_cycle"] == 12.0
    assert rows["sart::k_tail"]["dispatches"] == 1 and "FETCH_SIZE" not in rows["sart::k_tail"]
