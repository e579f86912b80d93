"""Copy one GPU session's evidence (tools/gpu_round_profile.sh) from gpurun_out/ into profiles/,
named per round, and check that rocprofv3's average table_kernel duration agrees with the
HIP-event kernel time bench.py measured in the same command.

    python tools/collect_profiles.py r01
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out")
DST = os.path.join(ROOT, "profiles")


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    os.makedirs(os.path.join(DST, f"{rnd}_pmc"), exist_ok=True)
    copies = {
        "bench.json": f"{rnd}_bench.json",
        "prof_bench.json": f"{rnd}_bench_under_rocprof.json",
        "pmc/pmc_summary.json": "pmc_summary.json",
        "pmc/bench_pmc.json": f"{rnd}_pmc/bench_pmc.json",
        "pmc/opweights_pmc.json": f"{rnd}_pmc/opweights_pmc.json",
    }
    for s, d in copies.items():
        shutil.copy(os.path.join(SRC, s), os.path.join(DST, d))
    stats = glob.glob(os.path.join(SRC, "prof", "**", "*kernel_stats.csv"), recursive=True)
    shutil.copy(stats[0], os.path.join(DST, f"{rnd}_kernel_stats.csv"))
    with open(stats[0]) as f:
        rows = list(csv.DictReader(f))
    with open(os.path.join(SRC, "prof_bench.json")) as f:
        bench = json.loads(f.read().strip().splitlines()[-1])
    check = {}
    for r in rows:
        if "::table_kernel<" in r["Name"]:
            check["rocprof_table_kernel_avg_ms"] = float(r["AverageNs"]) / 1e6
            check["rocprof_table_kernel_calls"] = int(r["Calls"])
        if "::roots_sorted_kernel<0>" in r["Name"]:
            check["rocprof_roots_sorted_kernel_avg_ms"] = float(r["AverageNs"]) / 1e6
            check["rocprof_roots_sorted_kernel_calls"] = int(r["Calls"])
    # the stats row averages every table_kernel launch of the command (the headline's cfg2 steps,
    # the default grid, cfg4): the per-dispatch trace gives the headline grid's own average
    traces = glob.glob(os.path.join(SRC, "prof", "**", "*kernel_trace.csv"), recursive=True)
    if traces:
        shutil.copy(traces[0], os.path.join(DST, f"{rnd}_kernel_trace.csv"))
        by_grid = {}
        with open(traces[0]) as f:
            for r in csv.DictReader(f):
                if "::table_kernel<" in r["Kernel_Name"]:
                    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
                    by_grid.setdefault(int(r["Grid_Size_X"]), []).append(d)
        check["rocprof_table_kernel_by_grid"] = {
            str(g): {"launches": len(v), "avg_ms": sum(v) / len(v)} for g, v in by_grid.items()}
        g0 = max(by_grid, key=lambda g: len(by_grid[g]))  # the headline's timed steps
        check["rocprof_table_kernel_headline_avg_ms"] = sum(by_grid[g0]) / len(by_grid[g0])
    check["bench_hip_event_kernel_ms"] = bench["roofline"]["kernel_ms"]
    check["ratio"] = check.get("rocprof_table_kernel_headline_avg_ms",
                               check["rocprof_table_kernel_avg_ms"]) / check["bench_hip_event_kernel_ms"]
    mz = (bench.get("minimizer") or {}).get("roofline") or {}
    if mz.get("kernel_ms") and "rocprof_roots_sorted_kernel_avg_ms" in check:
        check["bench_hip_event_roots_kernel_ms"] = mz["kernel_ms"]
        check["roots_ratio"] = check["rocprof_roots_sorted_kernel_avg_ms"] / mz["kernel_ms"]
    with open(os.path.join(DST, f"{rnd}_timing_check.json"), "w") as f:
        json.dump(check, f, indent=1)
    print(json.dumps(check, indent=1))


if __name__ == "__main__":
    main()
