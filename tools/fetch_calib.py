"""FETCH_SIZE calibration summary: the probes of tools/fetch_calib.hip read a
known number of bytes per dispatch in the table lookup's access patterns; this takes rocprofv3's
per-dispatch counters of those dispatches (median over a probe's dispatches, so the warm-up of the
L3-resident probe does not count) and writes, per probe, FETCH_SIZE in bytes and the factor
bytes read / FETCH_SIZE bytes.

    python tools/fetch_calib.py OUT.json TIMINGS.json PASS_DIR [PASS_DIR ...]
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

PROBE_KERNELS = {"stream16": "stream16", "wstream16": "wstream16", "rand64_big": "rand64",
                 "rand32_big": "rand32", "rand64_small": "rand64_n"}


def per_dispatch(dirs):
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> ctr -> disp
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row.get("Kernel_Name", "?").split("(")[0].strip()
                    acc[k][row["Counter_Name"]][(f, row.get("Dispatch_Id"))] += float(
                        row.get("Counter_Value", "nan"))
    return acc


def main():
    out_path, timing_path, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    with open(timing_path) as f:
        timings = {p["name"]: p for p in json.load(f)["probes"]}
    acc = per_dispatch(dirs)
    res = {"_about": __doc__.split("\n\n")[0].replace("\n", " "),
           "_source": "tools/gpu_fetch_calib.sh: tools/fetch_calib (HIP events), then rocprofv3 "
                      "--pmc passes of the same binary (FETCH_SIZE; TCC request counters)",
           "probes": {}}
    for probe, kern in PROBE_KERNELS.items():
        t = timings.get(probe)
        c = acc.get(kern, {})
        if t is None:
            continue
        med = {name: statistics.median(v.values()) for name, v in c.items()} if c else {}
        fetch = med.get("FETCH_SIZE")
        rec = {"bytes_per_launch": t["bytes_per_launch"], "ms": t["ms"], "GBps": t["GBps"],
               "dispatches": {name: len(v) for name, v in c.items()},
               "counters_median": med}
        if fetch and probe != "wstream16":  # a write probe: its FETCH_SIZE is not its bytes
            rec["fetch_bytes_raw"] = fetch * 1024
            rec["factor_bytes_per_fetch_byte"] = t["bytes_per_launch"] / (fetch * 1024)
        res["probes"][probe] = rec
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in res["probes"].items():
        print(k, {x: v.get(x) for x in ("bytes_per_launch", "fetch_bytes_raw",
                                        "factor_bytes_per_fetch_byte", "GBps")})


if __name__ == "__main__":
    main()
