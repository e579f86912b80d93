"""Copy one GPU session's evidence (tools/gpu_profiles.sh, and tools/gpu_pmc.sh when it ran) from
gpurun_out/ into profiles/, named per round, and check every line item's kernel time against the
rocprofv3 --kernel-trace --stats summary of that workload run on its own.

    python tools/collect_profiles.py r04 [gpurun_out/prof]

Writes profiles/<round>_bench.json (the default bench line), profiles/<round>_stats_<item>.csv
(one per workload: table = the cfg2 headline, solve = cfg3, trace = cfg5, lookup, cfg4, scalar),
the bench line each profiled command printed (<round>_bench_only_<item>.json) and
profiles/<round>_timing_check.json: for each line item, the HIP-event kernel time bench.py
reported and the rocprofv3 average of the same kernel in that item's own stats file.
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DST = os.path.join(ROOT, "profiles")

# item -> (kernel name prefix in the stats file, path of the bench-reported ms in the line)
CHECKS = {
    "table": [("airice::table_kernel<false", ("roofline", "kernel_ms"))],
    "solve": [("airice::roots_kernel<0>", ("minimizer", "roots_kernel_ms")),
              ("airice::solve_out_kernel<0>", ("minimizer", "out_kernel_ms"))],
    "lookup": [("airice::lookup_kernel", ("table_lookup", "lookup_kernel_ms"))],
    "cfg4": [("airice::table_kernel<false", ("table_cfg4", "kernel_ms"))],
}


def stats_rows(path):
    with open(path) as f:
        return {r["Name"]: r for r in csv.DictReader(f)}


def line_of(path):
    with open(path) as f:
        lines = [ln for ln in f.read().splitlines() if ln.strip().startswith("{")]
    return json.loads(lines[-1]) if lines else {}


def get(d, keys):
    for k in keys:
        d = (d or {}).get(k)
    return d


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r04"
    src = os.path.join(ROOT, sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/prof")
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(DST, f"{rnd}_bench.json"))
    headline = line_of(os.path.join(src, "bench.json"))
    check = {"_source": "tools/gpu_profiles.sh: rocprofv3 --kernel-trace --stats of each workload "
                        "on its own (bench.py --only ITEM / --cfg4-only / the scalar latency "
                        "driver); ms = the stats file's AverageNs; bench_ms = the HIP-event time "
                        "the same command's bench line reported, and the default run's"}
    for item in ("table", "solve", "trace", "lookup", "cfg4", "scalar"):
        stats = glob.glob(os.path.join(src, f"prof_{item}", "**", "*kernel_stats.csv"),
                          recursive=True)
        if not stats:
            continue
        shutil.copy(stats[0], os.path.join(DST, f"{rnd}_stats_{item}.csv"))
        rows = stats_rows(stats[0])
        only = os.path.join(src, f"prof_{item}.json")
        line = line_of(only) if os.path.exists(only) else {}
        if line:
            with open(os.path.join(DST, f"{rnd}_bench_only_{item}.json"), "w") as f:
                json.dump(line, f, indent=1)
        out = {"kernels": {n: {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6}
                           for n, r in rows.items()}}
        for prefix, path in CHECKS.get(item, []):
            hit = [r for n, r in rows.items() if n.replace("void ", "", 1).startswith(prefix)]
            if not hit:
                continue
            ms = float(hit[0]["AverageNs"]) / 1e6
            bench_only = get(line, path)
            bench_default = get(headline, path)
            out[prefix] = {"rocprof_avg_ms": ms, "calls": int(hit[0]["Calls"]),
                           "bench_ms_same_command": bench_only,
                           "ratio_same_command": ms / bench_only if bench_only else None,
                           "bench_ms_default_run": bench_default,
                           "ratio_default_run": ms / bench_default if bench_default else None}
        check[item] = out
    with open(os.path.join(DST, f"{rnd}_timing_check.json"), "w") as f:
        json.dump(check, f, indent=1)
    for item, v in check.items():
        if isinstance(v, dict):
            print(item, {k: (round(x["ratio_same_command"], 4) if x["ratio_same_command"] else None)
                         for k, x in v.items() if k != "kernels"})
    pmc = os.path.join(ROOT, "gpurun_out", "pmc", "pmc_summary.json")
    if os.path.exists(pmc):
        shutil.copy(pmc, os.path.join(DST, "pmc_summary.json"))
        os.makedirs(os.path.join(DST, f"{rnd}_pmc"), exist_ok=True)
        for name in ("bench_pmc.json", "cfg4_pmc.json", "opweights_pmc.json"):
            p = os.path.join(ROOT, "gpurun_out", "pmc", name)
            if os.path.exists(p):
                shutil.copy(p, os.path.join(DST, f"{rnd}_pmc", name))


if __name__ == "__main__":
    main()
