"""Derive per-kernel metrics from the PMC passes (tools/gpu_pmc.sh) -> profiles/pmc_summary.json.

HBM bytes follow MI355X_MICROARCH.md §HBM: WRITE_SIZE/FETCH_SIZE are KiB (x1024); FETCH_SIZE
under-reports wide coalesced streaming reads by 2x on gfx950 -- the compute kernels here read only
kernel arguments and <=24 B per query, so FETCH is reported both raw and doubled (upper bound).
The table lookup reads random records, whose FETCH_SIZE was calibrated separately
(apply_lookup_calibration below).

Busy figures, both bounded by construction:
* fp64_pipe_busy_pct = 100 x (executed FP64 VALU instructions x 4 cycles) / (1024 SIMDs x the
  launch's cycles, GRBM_GUI_ACTIVE / 8 XCDs): a SIMD completes at most one wave64 FP64
  instruction every 4 cycles (16 FP64 lanes per clock, the FP64 vector peak), so this cannot
  exceed 100; it is the roofline fraction at the clock the launch actually ran at.
* valu_busy_pct = 100 x (4 x FP64 VALU instructions + 2 x the other VALU instructions) / (1024
  SIMDs x the launch's cycles): every VALU instruction priced at its least issue time on a gfx950
  SIMD for a wave64 (FP64: 16 lanes per clock, 4 cycles; 32-bit and narrower: 32 lanes per clock, 2
  cycles -- tools/valu_rates.hip measures these, and the transcendental forms take longer), so the
  numerator is a lower bound of the SIMDs' VALU-occupied cycles and the figure cannot exceed 100:
  north_star's "VALU busy", bounded.
* wave_cycle_shares: SQ_ACTIVE_INST_ANY (issuing), SQ_WAIT_INST_ANY (ready to issue but stalled
  on a dependency or a busy pipe) and SQ_WAIT_ANY (parked on s_waitcnt / barrier) over
  SQ_WAVE_CYCLES -- disjoint parts of every wave's lifetime (MI355X_MICROARCH.md §rocprofv3).
(The earlier VALU-busy, 100 x SQ_ACTIVE_INST_VALU x 4 / SIMDs / (GRBM_GUI_ACTIVE / XCDs), priced
every VALU instruction at 4 cycles -- the FP64 cost -- and read 100.8 % on the cfg4 launch, where
the cheaper integer / move / select instructions share the SIMD: it is not a bounded busy and is
no longer reported.)
"""
import json
import sys

SIMDS = 256 * 4
XCDS = 8

# kernel-name prefix -> (summary key, units per launch) for `bench.py --no-cpu`
UNITS = [("table_kernel", "table_kernel", 858627),
         ("roots_kernel<0>", "roots_kernel", 1000000),
         ("roots_sorted_kernel<0>", "roots_sorted_kernel", 1000000),
         ("group_count_kernel<0>", "group_count_kernel", 1000000),
         ("group_scatter_kernel<0>", "group_scatter_kernel", 1000000),
         ("solve_out_kernel<0>", "solve_out_kernel", 1000000),
         ("lookup_kernel", "lookup_kernel", 1000000)]


def derive(name, c, n_units, kernel_ns=None):
    waves = c.get("SQ_WAVES", 0.0)
    f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                       "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
    grbm = c.get("GRBM_GUI_ACTIVE", 0.0)
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    d = {
        "units_per_launch": n_units,
        "valu_insts_per_unit": c.get("SQ_INSTS_VALU", 0.0) * 64 / n_units,
        "fp64_valu_insts_per_unit": f64 * 64 / n_units,
        "fp64_fma_share": c.get("SQ_INSTS_VALU_FMA_F64", 0.0) / f64 if f64 else None,
        "fp64_pipe_busy_pct": 100 * f64 * 4 / SIMDS / (grbm / XCDS) if grbm else None,
        "valu_busy_pct": 100 * (4 * f64 + 2 * (c.get("SQ_INSTS_VALU", 0.0) - f64)) / SIMDS /
                         (grbm / XCDS) if grbm and "SQ_INSTS_VALU" in c else None,
        "wave_cycle_shares": {
            "issuing": c["SQ_ACTIVE_INST_ANY"] / wc,
            "stalled_ready": c["SQ_WAIT_INST_ANY"] / wc,
            "parked_waitcnt_barrier": c["SQ_WAIT_ANY"] / wc,
        } if wc and "SQ_ACTIVE_INST_ANY" in c and "SQ_WAIT_INST_ANY" in c and "SQ_WAIT_ANY" in c
        else None,
        "waves": waves,
        "write_bytes_per_launch": c.get("WRITE_SIZE", 0.0) * 1024,
        "fetch_bytes_per_launch_raw": c.get("FETCH_SIZE", 0.0) * 1024,
    }
    d["hbm_bytes_per_launch"] = d["write_bytes_per_launch"] + 2 * d["fetch_bytes_per_launch_raw"]
    return d


# FETCH_SIZE per access pattern (tools/fetch_calib.hip, profiles/r06_fetch_calib.json): a wide
# coalesced streaming read reports 1/2 of its bytes; a random 64-byte record (four 16-byte loads)
# reports its 64 bytes; a random 32-byte piece reports 64 (one 64-byte fabric request).  So for the
# table lookup -- streaming query inputs, then random records and record pieces -- FETCH_SIZE
# counts every random access at the 64-byte request it costs, and only the streaming inputs need
# the x2: traffic = WRITE + (FETCH - inputs / 2) + inputs.
LOOKUP_STREAM_BYTES_PER_QUERY = 24  # src, dist, depth: three doubles, coalesced
CALIB_FILE = "profiles/r06_fetch_calib.json"  # relative to the repository root
CALIB_PATH = __import__("os").path.join(
    __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))),
    CALIB_FILE)


def apply_lookup_calibration(d, calib):
    """Replace the streaming x2 of lookup_kernel's FETCH_SIZE with the calibrated model above."""
    probes = calib["probes"]
    f_stream = probes["stream16"]["factor_bytes_per_fetch_byte"]
    f_rand = probes["rand64_big"]["factor_bytes_per_fetch_byte"]
    stream = LOOKUP_STREAM_BYTES_PER_QUERY * d["units_per_launch"]
    fetch = d["fetch_bytes_per_launch_raw"]
    reads = (fetch - stream / f_stream) * f_rand + stream
    d["hbm_bytes_per_launch"] = d["write_bytes_per_launch"] + reads
    d["fetch_bytes_per_launch_corrected"] = reads
    d["fetch_factor"] = {"streaming_inputs": f_stream, "random_records": f_rand}
    d["fetch_factor_source"] = (f"{CALIB_FILE}: stream16 (x{f_stream:.3f}) for the "
                                f"{LOOKUP_STREAM_BYTES_PER_QUERY} B/query of streamed inputs, "
                                f"rand64_big (x{f_rand:.3f}) for the rest (random 64-byte records "
                                "and 32-byte row-record pieces, each one 64-byte request)")
    d["hbm_bytes_source"] = "WRITE_SIZE + FETCH_SIZE corrected per access pattern (fetch_factor)"
    d["random_64B_probe_GBps"] = {k: probes[k]["GBps"] for k in ("rand64_big", "rand64_small")
                                  if k in probes}
    d["probe_GBps"] = {k: v["GBps"] for k, v in probes.items()}
    d["stream_input_bytes_per_launch"] = stream
    return d


# the cfg4 fine table (`bench.py --cfg4-only`): 97,001 x 8,991 rays in one launch
UNITS_CFG4 = [("table_kernel", "table_kernel_cfg4", 872135991)]


if __name__ == "__main__":
    if sys.argv[1] == "--apply-calibration":
        # re-derive the lookup's traffic in an existing summary from the calibration probes
        # (python tools/make_pmc_summary.py --apply-calibration CALIB.json SUMMARY.json)
        with open(sys.argv[2]) as f:
            calib = json.load(f)
        with open(sys.argv[3]) as f:
            summ = json.load(f)
        summ["lookup_kernel"] = apply_lookup_calibration(summ["lookup_kernel"], calib)
        with open(sys.argv[3], "w") as f:
            json.dump(summ, f, indent=1)
        print(json.dumps(summ["lookup_kernel"], indent=1))
        sys.exit(0)
    src, dst = sys.argv[1], sys.argv[2]
    with open(src) as f:
        raw = json.load(f)
    out = {"_source": "rocprofv3 --pmc passes of `python bench.py --no-cpu --no-cfg4 "
                      "--no-default-grid --steps 3 --warmup 1 --solve-steps 1` and of `bench.py "
                      "--cfg4-only` (tools/gpu_pmc.sh), mean per dispatch"}
    sets = [(raw, UNITS)]
    if len(sys.argv) > 3:
        with open(sys.argv[3]) as f:
            sets.append((json.load(f), UNITS_CFG4))
    for data, units in sets:
        for k, c in data.items():
            for prefix, key, n in units:
                if k.startswith(prefix):
                    out[key] = {**derive(k, c, n), "kernel": k,
                                "raw": {a: b for a, b in c.items() if not a.startswith("_")}}
    import os
    if "lookup_kernel" in out and os.path.exists(CALIB_PATH):
        with open(CALIB_PATH) as f:
            out["lookup_kernel"] = apply_lookup_calibration(out["lookup_kernel"], json.load(f))
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1)[:3000])
