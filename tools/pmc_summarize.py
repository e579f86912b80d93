"""Summarise rocprofv3 --pmc CSV passes: per kernel, mean counter value per dispatch.

usage: python tools/pmc_summarize.py OUT.json DIR [DIR ...]
Each DIR holds one pass (*counter_collection.csv).  Kernel names are shortened to the
function name (text before '(' after the last '::').
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    base = name.replace("(anonymous namespace)::", "").split("(")[0]
    base = re.sub(r"<.*>", lambda m: m.group(0), base)
    return base.split("::")[-1].strip()


def load(dirs):
    acc = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row.get("Kernel_Name", "?"))
                    c = row.get("Counter_Name")
                    v = float(row.get("Counter_Value", "nan"))
                    disp = (f, row.get("Dispatch_Id"))
                    acc[k][c][disp] = acc[k][c].get(disp, 0.0) + v
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v.values()) / max(1, len(v)) for c, v in cs.items()}
        out[k]["_dispatches"] = {c: len(v) for c, v in cs.items()}
    return out


if __name__ == "__main__":
    res = load(sys.argv[2:])
    with open(sys.argv[1], "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for k, v in res.items():
        print(k, {c: round(x, 1) for c, x in v.items() if not c.startswith("_")})
