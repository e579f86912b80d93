"""Executed FP64 VALU instructions per ocml call on gfx950, from the PMC pass over
tools/opweights_bench.hip (tools/gpu_pmc.sh):  (counter_f - counter_base) / (waves * 16).

usage: python tools/measure_opweights.py profiles/r01_pmc/opweights_pmc.json > tools/opweights.json
"""
import json
import sys

F64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
       "SQ_INSTS_VALU_TRANS_F64")

raw = json.load(open(sys.argv[1]))
base = raw["k_base"]
evals = base["SQ_WAVES"] * 16
out = {"_comment": "Executed FP64 VALU instructions (ADD+MUL+FMA+TRANS _F64 counters) per call of "
                   "each ocml function on gfx950, measured with rocprofv3 --pmc over "
                   "tools/opweights_bench.hip (arguments in the solver's ranges); 'valu_all' adds "
                   "the non-FP64 VALU instructions of the same call.  'arith' = one add/mul.",
       "source": "pmc", "arith": 1, "valu_all": {}}
for k, c in raw.items():
    if not k.startswith("k_") or k == "k_base":
        continue
    name = k[2:]
    out[name] = round(sum(c[x] - base[x] for x in F64) / evals, 2)
    out["valu_all"][name] = round((c["SQ_INSTS_VALU"] - base["SQ_INSTS_VALU"]) / evals, 2)
print(json.dumps(out, indent=1))
