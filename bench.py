#!/usr/bin/env python3
"""bench.py -- solved air->ice rays/s of the MI355X table path (BASELINE.json metric).

Workload (N=1): BASELINE cfg2 = MakeRayTracingTable on one MI355X, TxH 100000 -> 3000 m
@ 20 m x launch angle 92 -> 180 deg @ 0.5 deg, antenna 200 m below the 3000 m ice surface:
4,851 x 177 = 858,627 rays per step.  One step = one table build, i.e.
one launch of table_kernel writing the 11 float columns of AllTableAllAntData into HBM.

N>1 (torch.distributed.run, one process per GPU), default ``--mode sharded``: the
north_star's design -- one table over the (TxH x angle) grid, split into contiguous TxH-row
slabs, one slab per GPU, assembled on rank 0 by one RCCL gather over xGMI
(airiceraytracing_amd.distributed.run_sharded_table; the reference assembles its table in the
row loop MultiRayAirIceRefraction.cc:2079-2136).  Weak scaling: the grid is cfg2 refined N-fold
in TxH (step 20/N m), so every GPU builds about one cfg2 table per step.  The gather is timed
in its own barrier bracket (``sharded.gather_ms``); ``value`` counts the steps only and
``sharded.value_incl_gather`` adds one gather per step.  ``--mode replicas``: one antenna table
per GPU, no collective (RunMultiRayCode.C:29-52).  Timing: W untimed warm-up steps, then K
steps bracketed by barrier + synchronize, max over ranks.

Also reported (rank 0): the roofline of table_kernel from executed FP64 VALU instructions
(profiles/pmc_summary.json) over the live kernel time; the minimizer (cfg3, 1e6 Air2IceRayTracing
solves) with its own roofline, CPU baseline and parity on a stride of the timed batch; the
pythonwrapper batch (cfg5, 1e7 Py_TraceIceToAir rows) with parity; the table lookup; the CPU
baseline of the table (the oracle, OpenMP on the box's host cores) and the table's parity.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# FP64 VALU peak of one MI355X: 256 CU x 64 FP64 lane-ops/clk x 2.4 GHz (= 78.6 TFLOP/s with
# FMA counted twice; MI355X spec FP64 vector rate).  Work is counted in lane-ops (one executed
# FP64 VALU instruction x 64 lanes = 64 lane-ops, FMA = 1).
PEAK_FP64_VALU_TOPS = 256 * 64 * 2.4e9 / 1e12
CFG2 = dict(depth_cm=-20000.0, ice_cm=300000.0, height_step=20.0, start_angle=92.0,
            stop_angle=180.0, angle_step=0.5)
# BASELINE cfg4: TxH 100000 -> 3000 m @ 1 m x 90.1 -> 180 deg @ 0.01 deg, antenna 200 m below the
# ice: 97,001 x 8,991 = 872,135,991 rays, 38.4 GB of float columns
CFG4 = dict(depth_cm=-20000.0, ice_cm=300000.0, height_step=1.0, start_angle=90.1,
            stop_angle=180.0, angle_step=0.01)
# survey-session probe of the real reference (8-core container Xeon, g++ -O2,
# compiled against a GSL stand-in): quoted beside the oracle's CPU baseline, never measured here
SURVEY_REFERENCE_PROBE = {
    "table_rays_per_s": {"1_thread": 2.42e5, "8_threads": 5.58e5},
    "minimizer_solves_per_s": {"1_thread": 8.80e3, "8_threads": 6.22e4},
    "py_trace_ice_to_air_ms_per_call": 12.1,
    "source": "BASELINE.md §2 (survey container, not this box)"}
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_summary.json")


class HipBackend:
    """Where the table path of the bench runs: libairice.so's kernels on this process's GPU (the
    product).  The table-path code below (headline steps, the sharded assembly, the cfg4 item)
    only calls these methods, so tests/bench_rehearsal.py can run the same multi-rank flow on CPU
    ranks over gloo with a stand-in for the kernels."""
    is_gpu = True

    def __init__(self, local_rank: int):
        import torch
        from airiceraytracing_amd import AirIceSolver
        ndev = torch.cuda.device_count()
        self.dev = torch.device(f"cuda:{local_rank % max(1, ndev)}")
        torch.cuda.set_device(self.dev)
        self.solver = AirIceSolver()
        self.stream = torch.cuda.current_stream()

    def event(self):
        import torch
        return torch.cuda.Event(enable_timing=True)

    def sync(self) -> None:
        import torch
        torch.cuda.synchronize()

    def release(self) -> None:
        import torch
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    def table(self, grid, out, row_begin: int = 0, row_count=None, ld=None) -> None:
        self.solver.table_device(grid, out, None, row_begin=row_begin, row_count=row_count, ld=ld,
                                 stream=self.stream)

    def table_to_host(self, slab, cnt: int, host, first: int) -> None:
        """host[:, first:first+cnt] = slab[:, :cnt] (airice_table_to_host: one D2H copy per
        column into page-locked rows)."""
        import ctypes
        from airiceraytracing_amd import _lib
        from airiceraytracing_amd.solver import _stream_handle
        _lib.check(_lib.lib().airice_table_to_host(
            ctypes.c_void_p(slab.data_ptr()), slab.stride(0), cnt,
            ctypes.c_void_p(host.data_ptr() + 4 * first), host.stride(0),
            _stream_handle(self.stream)), "airice_table_to_host")

    def host_register(self, ptr: int, nbytes: int) -> None:
        import ctypes
        from airiceraytracing_amd import _lib
        _lib.check(_lib.lib().airice_host_register(ctypes.c_void_p(ptr), nbytes),
                   "airice_host_register")

    def host_unregister(self, ptr: int) -> None:
        import ctypes
        from airiceraytracing_amd import _lib
        _lib.check(_lib.lib().airice_host_unregister(ctypes.c_void_p(ptr)),
                   "airice_host_unregister")


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--mode", choices=("sharded", "replicas"), default="sharded",
                   help="N>1: one table sharded by TxH rows + RCCL gather (default), or one "
                        "antenna table per GPU")
    p.add_argument("--solve-n", type=int, default=1_000_000)
    p.add_argument("--solve-steps", type=int, default=20)
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU legs (baselines, parity)")
    p.add_argument("--no-solve", action="store_true", help="skip the minimizer line item")
    p.add_argument("--no-lookup", action="store_true", help="skip the table-lookup line item")
    p.add_argument("--no-pcie", action="store_true", help="skip the table-to-host line item")
    p.add_argument("--no-multi", action="store_true",
                   help="skip the several-antenna line item (tables on concurrent streams)")
    p.add_argument("--no-scalar", action="store_true", help="skip the scalar-call latencies")
    p.add_argument("--no-cold", action="store_true",
                   help="skip the cold (one table per antenna) line item")
    p.add_argument("--no-default-grid", action="store_true",
                   help="skip the reference default grid line item (8.7M rays)")
    p.add_argument("--no-cfg4", action="store_true", help="skip the cfg4 fine-table line item")
    p.add_argument("--cfg4-only", action="store_true",
                   help="run only the cfg4 fine-table line item (PMC passes of its launch)")
    p.add_argument("--cfg4-reps", type=int, default=3)
    p.add_argument("--cfg4-host", choices=("auto", "none"), default="auto",
                   help="assemble the cfg4 table in host memory (default) or keep it in HBM")
    p.add_argument("--cfg4-host-path", default=None,
                   help="N>1: the node-shared host table's file (default: a new file in /dev/shm)")
    p.add_argument("--workload", choices=("cfg2", "cfg4"), default="cfg2",
                   help="N>1 sharded headline: the cfg2 grid refined N-fold (weak scaling, "
                        "default) or the cfg4 fine table split over the N GPUs (strong scaling)")
    p.add_argument("--height-step", type=float, default=CFG2["height_step"],
                   help="TxH step (m) of the headline cfg2 grid (BASELINE cfg2: 20)")
    p.add_argument("--cfg4-height-step", type=float, default=CFG4["height_step"],
                   help="TxH step (m) of the cfg4 fine table (BASELINE cfg4: 1)")
    p.add_argument("--lookup-n", type=int, default=1_000_000)
    p.add_argument("--trace-n", type=int, default=10_000_000)
    p.add_argument("--no-trace", action="store_true", help="skip the cfg5 pythonwrapper line item")
    p.add_argument("--cpu-threads", type=int, default=16,
                   help="host threads of the CPU legs (the GPU box's CPU share is 16 per GPU)")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="wall time of each CPU-baseline sample")
    p.add_argument("--parity-stride", type=int, default=1,
                   help="every k-th query of the timed minimizer and trace batches is checked "
                        "against the oracle (default: every query, ~15 s of the CPU legs)")
    p.add_argument("--only", choices=("table", "solve", "trace", "lookup", "multi", "cold", "pcie",
                                      "default-grid", "cfg4", "scalar"), default=None,
                   help="run the headline table steps and this one line item only, no CPU legs "
                        "(per-workload rocprofv3 summaries, tools/gpu_profiles.sh)")
    a = p.parse_args(argv)
    if a.only is not None:
        a.no_cpu = True
        for item in ("solve", "trace", "lookup", "multi", "cold", "pcie", "default-grid", "cfg4",
                     "scalar"):
            setattr(a, "no_" + item.replace("-", "_"), item != a.only)
    return a


def load_pmc() -> dict:
    try:
        with open(PMC_FILE) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def cpu_info(nthr: int) -> dict:
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count()
    return {"cpu_model": model, "threads_used": nthr, "affinity_cpus": aff,
            "compiler": "gcc -O2 -ffp-contract=off -fopenmp (oracle/Makefile)"}


def physical_cores() -> int:
    """Physical cores among this process's CPUs (unique (package, core) pairs in /proc/cpuinfo)."""
    try:
        aff = os.sched_getaffinity(0)
    except AttributeError:
        aff = set(range(os.cpu_count() or 1))
    cores, cpu, pkg = set(), None, None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                k, _, v = ln.partition(":")
                k, v = k.strip(), v.strip()
                if k == "processor":
                    cpu = int(v)
                elif k == "physical id":
                    pkg = v
                elif k == "core id" and cpu in aff:
                    cores.add((pkg, v))
    except (OSError, ValueError):
        pass
    return len(cores) or len(aff)


# what the CPU baseline is: the oracle restatement is NOT the reference's speed
PORT_VS_REFERENCE = ("the oracle's C restatement (faithful call structure and libm calls, but no "
                     "per-segment new[], no std::cout and one medium fold per call) runs about 4-5x "
                     "the reference's own per-thread speed: the survey's probe of the real reference "
                     "(compiled against a GSL stand-in) measured 2.42e5 rays/s and 8.8e3 solves/s on "
                     "one thread against this port's ~1e6 rays/s and ~4.4e4 solves/s; so this "
                     "baseline is conservative (faster than the reference), not the reference")


ALL_CORES_NOTE = ("context only: one thread per physical core of the host; on the shared GPU box "
                  "the process's CPU quota (16 CPUs per GPU) can make this lower than the "
                  "16-thread value")


def counter_roofline(kernel_key: str, units: int, kernel_ms: float, pmc: dict,
                     algorithmic_bytes_per_unit: float) -> dict:
    """Roofline of one kernel from its executed FP64 VALU instructions (PMC, per unit) over the
    live kernel time: achieved = FP64 lane-ops per launch / launch duration."""
    p = pmc.get(kernel_key, {})
    ops_per_unit = p.get("fp64_valu_insts_per_unit")
    achieved = (ops_per_unit * units / (kernel_ms * 1e-3) / 1e12
                if ops_per_unit and kernel_ms else None)
    traffic_per_unit = (p["hbm_bytes_per_launch"] / p["units_per_launch"]
                        if p.get("hbm_bytes_per_launch") and p.get("units_per_launch") else None)
    return {
        "bound": "valu",
        "kernel": p.get("kernel", kernel_key),
        "achieved": achieved, "peak": PEAK_FP64_VALU_TOPS,
        "unit": "TFLOP/s (FP64 VALU lane-ops/s x 1e-12, FMA = 1)",
        "frac": achieved / PEAK_FP64_VALU_TOPS if achieved else None,
        "traffic": traffic_per_unit * units if traffic_per_unit else None,
        "work_source": "executed FP64 VALU instructions (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 "
                       "x 64 lanes) per unit from " + os.path.relpath(PMC_FILE, ROOT),
        "fp64_lane_ops_per_unit": ops_per_unit,
        "valu_insts_per_unit": p.get("valu_insts_per_unit"),
        "fp64_pipe_busy_pct": p.get("fp64_pipe_busy_pct"),
        "valu_busy_pct": p.get("valu_busy_pct"),
        "wave_cycle_shares": p.get("wave_cycle_shares"),
        "units_per_launch": units, "kernel_ms": kernel_ms,
        "hbm_bytes_per_launch_algorithmic": algorithmic_bytes_per_unit * units,
        "hbm_GBps_algorithmic": algorithmic_bytes_per_unit * units / (kernel_ms * 1e-3) / 1e9
        if kernel_ms else None,
    }


HBM_PEAK_GBPS = 8000.0        # MI355X HBM3E, spec (MI355X_MICROARCH.md §HBM)
HBM_ACHIEVABLE_GBPS = 6300.0  # achievable streaming rate, same section
# the lookup's necessary bytes per query: inputs (3 doubles), outputs (9 doubles + ok + flags),
# and the two 64-byte pair records its interpolation reads (one per Tx height)
LOOKUP_QUERY_IO_BYTES = 24 + 72 + 2
LOOKUP_RECORD_BYTES = 2 * 64


def lookup_roofline(units: int, kernel_ms: float, pmc: dict) -> dict:
    """The lookup is memory-bound (random records; 15 % VALU busy): its traffic per launch from the
    PMC summary, with FETCH_SIZE corrected by the factor calibrated for its access pattern
    (tools/fetch_calib.hip, profiles/r06_fetch_calib.json) instead of the streaming x2, over the
    live kernel time, against the HBM peak and the achievable 6.3 TB/s."""
    p = pmc.get("lookup_kernel", {})
    per_unit = (p["hbm_bytes_per_launch"] / p["units_per_launch"]
                if p.get("hbm_bytes_per_launch") and p.get("units_per_launch") else None)
    traffic = per_unit * units if per_unit else None
    ach = traffic / (kernel_ms * 1e-3) / 1e9 if traffic and kernel_ms else None
    algo = (LOOKUP_QUERY_IO_BYTES + LOOKUP_RECORD_BYTES) * units
    # the access-pattern bound: each part of the traffic at the rate tools/fetch_calib.hip
    # measured for its pattern (random 64-byte records from an L3-resident table, streamed reads,
    # streamed writes), one after the other
    pb = None
    probes = p.get("probe_GBps") or {}
    if traffic and all(k in probes for k in ("rand64_small", "stream16", "wstream16")):
        scale = units / p["units_per_launch"]
        stream_in = p["stream_input_bytes_per_launch"] * scale
        random_rd = p["fetch_bytes_per_launch_corrected"] * scale - stream_in
        writes = p["write_bytes_per_launch"] * scale
        pb = (random_rd / probes["rand64_small"] + stream_in / probes["stream16"] +
              writes / probes["wstream16"]) / 1e9 * 1e3  # ms
    return {
        "bound": "hbm", "kernel": "lookup_kernel", "unit": "GB/s",
        "achieved": ach, "peak": HBM_PEAK_GBPS, "frac": ach / HBM_PEAK_GBPS if ach else None,
        "frac_of_achievable": ach / HBM_ACHIEVABLE_GBPS if ach else None,
        "achievable": HBM_ACHIEVABLE_GBPS,
        "traffic": traffic,
        "traffic_source": p.get("hbm_bytes_source"),
        "fetch_factor": p.get("fetch_factor"), "fetch_factor_source": p.get("fetch_factor_source"),
        "algorithmic_bytes": algo,
        "algorithmic_note": "per query: 98 B of query I/O + two 64-byte pair records",
        "algorithmic_GBps": algo / (kernel_ms * 1e-3) / 1e9 if kernel_ms else None,
        "traffic_over_algorithmic": traffic / algo if traffic else None,
        "kernel_ms": kernel_ms, "units_per_launch": units,
        "random_64B_probe_GBps": p.get("random_64B_probe_GBps"),
        "pattern_bound_ms": pb,
        "frac_of_pattern_bound": pb / kernel_ms if pb and kernel_ms else None,
        "pattern_bound_note": "random reads at rand64_small's rate, streamed inputs at "
                              "stream16's, results at wstream16's (profiles/r06_fetch_calib.json)",
    }


def ocml_priced(grid, rays: int, kernel_ms: float) -> dict:
    """Secondary figure: the algorithm's FP64 work priced at the gfx950 ocml cost of each
    function (tools/workmodel.py, tools/opweights.json).  The kernel runs cheaper forms of the
    same functions, so this is NOT a hardware fraction."""
    from tools.workmodel import ray_ops, segments_per_ray
    with open(os.path.join(ROOT, "tools", "opweights.json")) as f:
        weights = json.load(f)
    segs = segments_per_ray(grid)
    ops = ray_ops(segs, weights, rays_per_row=grid.angle_steps)
    ach = rays * ops["W"] / (kernel_ms * 1e-3) / 1e12
    return {"W_lane_ops_per_ray": ops["W"], "achieved": ach,
            "frac_of_peak": ach / PEAK_FP64_VALU_TOPS, "mean_air_segments": segs["mean_air"],
            "note": "library-priced work model, not executed instructions"}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n: int, argv, script: str | None = None, timeout: float | None = None) -> int:
    """``bench.py --gpus N`` (N > 1) started without torch.distributed.run's environment: start
    ``python -m torch.distributed.run --nproc-per-node N <script> <argv>`` as a CHILD process
    (one rank per GPU; this process never touches the GPU and never execs), relay rank 0's JSON
    line to stdout and return the child's exit status.  ``script``: the per-rank entry (bench.py
    itself; the CPU tests pass a rehearsal entry that runs the same main() on gloo ranks)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), script or os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this pool
    print(f"bench.py: --gpus {n} without RANK in the environment: launching {n} ranks: "
          + " ".join(cmd), file=sys.stderr, flush=True)
    p = subprocess.run(cmd, stdout=subprocess.PIPE, env=env, timeout=timeout)
    lines = [ln for ln in p.stdout.decode(errors="replace").splitlines() if ln.startswith("{")]
    for ln in lines[-1:]:  # exactly one JSON line, rank 0's
        sys.stdout.write(ln + "\n")
    sys.stdout.flush()
    if p.returncode == 0 and len(lines) != 1:
        print(f"bench.py: the ranks printed {len(lines)} JSON lines (want 1)", file=sys.stderr)
        return 1
    return p.returncode


def check_world(args) -> None:
    """Under torch.distributed.run (RANK set), the world must be the --gpus the caller asked for:
    a mismatch would report a line whose n_gpus differs from the request, so it is an error."""
    if "RANK" in os.environ:
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if world != args.gpus:
            print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report an "
                  f"{world}-GPU run as {args.gpus}", file=sys.stderr, flush=True)
            raise SystemExit(2)


def main(argv=None, make_backend=None, json_path=None):
    """The bench.  argv: command-line arguments (default sys.argv); make_backend(local_rank):
    where the table path runs (default HipBackend); json_path: write rank 0's JSON line there
    instead of to stdout."""
    args = parse(argv)
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "RANK" not in os.environ:
        # before torch is imported: the launching process makes no GPU call
        raise SystemExit(self_launch(args.gpus, sys.argv[1:] if argv is None else list(argv)))
    check_world(args)
    CFG2["height_step"] = args.height_step
    CFG4["height_step"] = args.cfg4_height_step
    os.environ.setdefault("NCCL_DEBUG", "WARN")
    # stdout carries exactly one JSON line (rank 0): RCCL prints its version banner to fd 1 at
    # communicator init, so fd 1 points at stderr for the whole run and the JSON line goes to the
    # saved descriptor
    sys.stdout.flush()
    json_fd = os.dup(1) if json_path is None else os.open(json_path, os.O_WRONLY | os.O_CREAT |
                                                         os.O_TRUNC, 0o644)
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = "RANK" in os.environ  # launched by torch.distributed.run (any world size)
    backend = os.environ.get("AIRICE_DIST_BACKEND", "nccl")  # gloo: rehearsal ranks sharing a GPU
    be = (make_backend or HipBackend)(local)
    dev = be.dev
    if distributed:
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=dev)
        else:
            dist.init_process_group(backend=backend)
    coll_dev = dev if backend == "nccl" else torch.device("cpu")

    from airiceraytracing_amd import AirIceSolver, make_grid
    from airiceraytracing_amd import _lib
    from airiceraytracing_amd.distributed import run_sharded_table, sharded_step_grid_step
    solver = be.solver
    pmc = load_pmc()
    stream = be.stream
    sharded = world > 1 and args.mode == "sharded"

    def barrier():
        if distributed:
            dist.barrier()

    if args.cfg4_only:
        rep = table_cfg4(args, be, world, rank, distributed, coll_dev, pmc)
        if rank == 0:
            os.write(json_fd, (json.dumps({"table_cfg4": rep}) + "\n").encode())
        if distributed:
            dist.destroy_process_group()
        return

    # ---------------------------------------------------------------- headline: table steps
    cfg4_headline = sharded and args.workload == "cfg4"
    if cfg4_headline:
        # the cfg4 fine table split over the N GPUs (strong scaling): K builds of every rank's
        # TxH-row slab, then one host assembly (table_cfg4)
        args.cfg4_reps = args.steps
        rep4 = table_cfg4(args, be, world, rank, distributed, coll_dev, pmc)
        grid = make_grid(CFG4["depth_cm"], CFG4["ice_cm"], CFG4["height_step"],
                         CFG4["start_angle"], CFG4["stop_angle"], CFG4["angle_step"])
        depth_cm = CFG4["depth_cm"]
        elapsed = elapsed_bar = rep4["ms_per_build"] * args.steps / 1e3
        total_rays = grid.n_rays * args.steps
        n_local = rep4["roofline"]["units_per_launch"]
        kern_ms = rep4["kernel_ms_rank0"]
        table = None
        shard_rep = {k: v for k, v in rep4.items() if k != "roofline"}
        args.no_cfg4 = True
    elif sharded:
        depth_cm = CFG2["depth_cm"]
        grid = make_grid(depth_cm, CFG2["ice_cm"],
                         sharded_step_grid_step(CFG2["height_step"], world), CFG2["start_angle"],
                         CFG2["stop_angle"], CFG2["angle_step"])
    else:
        depth_cm = CFG2["depth_cm"] - 1000.0 * rank  # replicas: rank r's antenna at 200 + 10 r m
        grid = make_grid(depth_cm, CFG2["ice_cm"], CFG2["height_step"], CFG2["start_angle"],
                         CFG2["stop_angle"], CFG2["angle_step"])
    ev0, ev1 = be.event(), be.event()
    if not cfg4_headline:
        shard_rep = None
    if cfg4_headline:
        pass
    elif sharded:
        def compute(begin, count, slab):
            be.table(grid, slab, row_begin=begin, row_count=count, ld=slab.shape[1])

        # the kernel time comes from a HIP-event pair around the K launches on the launch
        # stream, recorded inside compute's stream order
        state = {"i": 0}

        def timed_compute(begin, count, slab):
            if state["i"] == args.warmup:
                ev0.record(stream)
            compute(begin, count, slab)
            state["i"] += 1
            if state["i"] == args.warmup + args.steps:
                ev1.record(stream)

        r = run_sharded_table(grid, timed_compute, args.steps, args.warmup, device=dev,
                              coll_device=coll_dev, sync=be.sync, gather_reps=3)
        elapsed = elapsed_bar = r["elapsed_s"]
        n_local = r["rays_this_rank"]
        total_rays = grid.n_rays * args.steps
        table = r["slab"][:, :n_local]
        shard_rep = {
            "grid": f"TxH 100000->3000 m @{grid.height_step:g} m x 92->180 deg @0.5 deg "
                    f"({grid.height_steps} rows x {grid.angle_steps} = {grid.n_rays} rays)",
            "rows_per_rank": r["rows_per_rank"],
            "gather_ms": r["gather_s"] * 1e3,
            "gather_bytes_to_root": r["bytes_to_root"],
            "gather_GBps_root_ingress": r["bytes_to_root"] / r["gather_s"] / 1e9
            if r["gather_s"] > 0 else None,
            "value_incl_gather": grid.n_rays / (elapsed / args.steps + r["gather_s"]),
            "collective": "torch.distributed.gather (backend %s) of the row slabs to rank 0"
                          % backend}
        if rank == 0:
            # the assembled table equals the whole grid built on one GPU, bit for bit
            full = torch.empty((11, grid.n_rays), dtype=torch.float32, device=dev)
            be.table(grid, full)
            be.sync()
            shard_rep["assembled_bitwise_equal_single_gpu"] = bool(
                torch.equal(r["assembled"].to(dev).view(torch.int32), full.view(torch.int32)))
            del full
        del r
    else:
        n_local = grid.n_rays
        table = torch.empty((11, n_local), dtype=torch.float32, device=dev)

        def step():
            be.table(grid, table)

        for _ in range(args.warmup):
            step()
        be.sync()
        barrier()
        be.sync()
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(args.steps):
            step()
        ev1.record(stream)
        be.sync()
        # the clock stops when this rank's K steps are done; the trailing barrier (an RCCL
        # all-reduce, ~0.1-0.3 ms) closes the bracket but is not step work -- the max over ranks
        # below covers rank skew.  Both figures are reported.
        elapsed = time.perf_counter() - t0
        barrier()
        be.sync()
        elapsed_bar = time.perf_counter() - t0
        el = torch.tensor([elapsed, elapsed_bar], dtype=torch.float64, device=coll_dev)
        if distributed:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        elapsed, elapsed_bar = (float(x) for x in el.tolist())
        total_rays = world * n_local * args.steps
    be.sync()
    if not cfg4_headline:
        # (a rank whose slab is empty recorded no events; only rank 0 reports, and it has rows)
        kern_ms = ev0.elapsed_time(ev1) / args.steps if n_local > 0 else None
    # every rank's own kernel time (HIP events on its launch stream), gathered for the line
    kern_ms_ranks = gather_floats(kern_ms if not cfg4_headline else rep4.get("kernel_ms_this_rank"),
                                  distributed, world, coll_dev)
    value = total_rays / elapsed
    extra = {}

    # ---------------------------------------------------------------- minimizer (cfg3)
    solve = None
    if not args.no_solve:
        from tests.parity import cfg3_queries
        txh, dst, dep = cfg3_queries(args.solve_n, seed=12345 + rank)
        tq = [torch.from_numpy(a).to(dev) for a in (txh, dst, dep)]
        out = torch.empty((17, args.solve_n), dtype=torch.float64, device=dev)
        stt = torch.empty(args.solve_n, dtype=torch.uint8, device=dev)

        def solve_call():
            solver.solve_device(tq[0], tq[1], tq[2], 3000.0, out, stt, stream=stream)

        for _ in range(2):  # warm-up: code objects, scratch pool
            solve_call()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t1 = time.perf_counter()
        e0.record(stream)
        for _ in range(args.solve_steps):
            solve_call()
        e1.record(stream)
        torch.cuda.synchronize()
        se = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device=coll_dev)
        barrier()
        if distributed:
            dist.all_reduce(se, op=dist.ReduceOp.MAX)
        call_ms = e0.elapsed_time(e1) / args.solve_steps
        # per-kernel durations of the same calls: HIP-event pairs around each stage's launch on
        # the launch stream (airice_kernel_timing), separate pass so the timed calls above carry
        # no event packets between their kernels
        _lib.kernel_time("roots_kernel"), _lib.kernel_time("out_kernel")
        _lib.kernel_time("group_passes")
        _lib.kernel_timing(True)
        for _ in range(args.solve_steps):
            solve_call()
        torch.cuda.synchronize()
        _lib.kernel_timing(False)
        stage = {}
        for k in ("roots_kernel", "group_passes", "out_kernel"):
            ms, cnt = _lib.kernel_time(k)
            stage[k + "_ms"] = ms / cnt if cnt else None
        # CheckSolution (.cc:978-983) on the last batch, and the rows whose bracket set-up
        # reads uninitialised GSL state in the reference (AIRICE_SOLVE 1|2|32)
        thd = out[1].cpu().numpy()
        st_h = stt.cpu().numpy()
        err = np.abs(thd - dst)
        solved = (((err / dst < 0.01) & (dst <= 100)) | ((err < 1) & (dst > 100))) & (thd >= 0)
        solve = {
            "metric": "Air2IceRayTracing solves/s (cfg3, 1e6 random queries per GPU)",
            "value": world * args.solve_n * args.solve_steps / float(se.item()),
            "unit": "solves/s",
            "ms_per_call": call_ms, "kernel_ms": call_ms, **stage,
            "solved_fraction": float(solved.mean()),
            "unpinned_fraction": float(((st_h & 35) != 0).mean()),
            # dominant kernel: the root finder (block-local grouping, roots_kernel: the default of
            # this source since round 4); algorithmic bytes per query = 24 B of inputs, 8 B root +
            # 8 B status parked in the output slots
            "roofline": counter_roofline("roots_kernel", args.solve_n,
                                         stage.get("roots_kernel_ms"), pmc, 40.0),
        }
        out_h = out.cpu().numpy()

    # ---------------------------------------------------------------- pythonwrapper (cfg5)
    trace_h = None
    if not args.no_trace:
        # BASELINE cfg5: the pythonwrapper Py_TraceIceToAir rows (TraceIceToAir.C:5-73) for 1e7
        # queries through the batch entry (airice_trace_ice_to_air_launch), inputs in HBM
        from tests.parity import cfg5_queries
        from airiceraytracing_amd import VARIANT_PYWRAPPER
        psolver = AirIceSolver(variant=VARIANT_PYWRAPPER)
        q5 = cfg5_queries(args.trace_n, seed=777 + rank)
        q = [torch.from_numpy(a).to(dev) for a in q5]
        tout = torch.empty((args.trace_n, 10), dtype=torch.float64, device=dev)
        psolver.trace_ice_to_air_device(*q, tout, stream=stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 3
        e0.record(stream)
        for _ in range(reps):
            psolver.trace_ice_to_air_device(*q, tout, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        tms = e0.elapsed_time(e1) / reps
        extra["pywrapper_trace"] = {
            "metric": "Py_TraceIceToAir rows/s (cfg5, batch entry, 1e7 queries per GPU)",
            "value": args.trace_n / (tms * 1e-3), "unit": "queries/s", "ms": tms,
            "solved_fraction": float((tout[:, 0] != -1000).double().mean().item())}
        idx5 = np.arange(0, args.trace_n, args.parity_stride)
        trace_h = (q5, idx5, tout[torch.from_numpy(idx5).to(dev)].cpu().numpy())
        del q, tout
    lookup_h = None
    if not args.no_lookup:
        # batched GetHorizontalDistanceToIntersectionPoint_Table on this step's table (HBM
        # resident), cfg3-distributed queries (cm) for the table's own antenna
        from tests.parity import cfg3_queries
        lgrid = grid
        ltable = table
        if sharded:  # the lookup runs on a whole table: rank 0's cfg2 table
            lgrid = make_grid(CFG2["depth_cm"], CFG2["ice_cm"], CFG2["height_step"],
                              CFG2["start_angle"], CFG2["stop_angle"], CFG2["angle_step"])
            ltable = torch.empty((11, lgrid.n_rays), dtype=torch.float32, device=dev)
            solver.table_device(lgrid, ltable, None, stream=stream)
        lk_txh, lk_dst, _ = cfg3_queries(args.lookup_n, seed=4242 + rank)
        src = torch.from_numpy(lk_txh * 100).to(dev)
        dcm = torch.from_numpy(lk_dst * 100).to(dev)
        ldep = torch.full((args.lookup_n,), depth_cm, dtype=torch.float64, device=dev)
        lout = torch.empty((9, args.lookup_n), dtype=torch.float64, device=dev)
        lok = torch.empty(args.lookup_n, dtype=torch.uint8, device=dev)
        lfl = torch.empty(args.lookup_n, dtype=torch.uint8, device=dev)
        lt = solver.lookup_table(ltable, lgrid)
        # packed copy for the lookup (airice_lookup_pack, once per table; timed separately)
        solver.lookup_pack(lt, stream=stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # re-pack into the same buffer (the kernel alone; lookup_pack also allocates)
        import ctypes
        from airiceraytracing_amd import _lib
        from airiceraytracing_amd.solver import _stream_handle
        pack_times = []
        for _ in range(10):  # each pack bracketed on its own (median: a one-time setup cost)
            e0.record(stream)
            _lib.check(_lib.lib().airice_lookup_pack(ctypes.byref(lt), _lib.ptr(lt._packed),
                                                     lt._packed.numel(), _stream_handle(stream)),
                       "airice_lookup_pack")
            e1.record(stream)
            torch.cuda.synchronize()
            pack_times.append(e0.elapsed_time(e1))
        pack_ms = float(np.median(pack_times))

        def lookup():
            solver.table_lookup_device(lt, src, dcm, ldep, CFG2["ice_cm"], lout, lok, lfl,
                                       stream=stream)

        lookup()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record(stream)
        for _ in range(reps):
            lookup()
        e1.record(stream)
        torch.cuda.synchronize()
        lms = e0.elapsed_time(e1) / reps
        _lib.kernel_time("lookup_kernel")
        _lib.kernel_timing(True)
        for _ in range(reps):
            lookup()
        torch.cuda.synchronize()
        _lib.kernel_timing(False)
        lk_ms, lk_n = _lib.kernel_time("lookup_kernel")
        extra["table_lookup"] = {
            "metric": "GetHorizontalDistanceToIntersectionPoint_Table lookups/s (1e6 cfg3 "
                      "queries on the cfg2 table, incl. the minimizer fallback, solved in place)",
            "value": args.lookup_n / (lms * 1e-3), "unit": "lookups/s", "ms": lms,
            "lookup_kernel_ms": lk_ms / lk_n if lk_n else None,
            "ok_fraction": float(lok.cpu().numpy().mean()),
            "pack_ms": pack_ms, "packed": True,
            "roofline": lookup_roofline(args.lookup_n, lk_ms / lk_n if lk_n else None, pmc)}
        if rank == 0 and world == 1:
            # the last timed batch's results, checked against the oracle in the CPU legs
            lookup_h = (lk_txh * 100, lk_dst * 100, depth_cm, ltable.cpu().numpy(),
                        lout.cpu().numpy(), lok.cpu().numpy(), lfl.cpu().numpy())
        if sharded:
            del ltable
    if not args.no_multi:
        # Several antennas' cfg2 tables (MakeRayTracingTable per AntennaNumber, .cc:2019) built
        # concurrently, one HIP stream per antenna: a single table's launch ramp and drain
        # (~15 us of its 36 us) overlap the other antennas' work.  Secondary
        # line item; the headline above stays one table per step on one stream.
        multi = {}
        for n_ant in (2, 4):
            grids = [make_grid(CFG2["depth_cm"] - 1000.0 * a, CFG2["ice_cm"],
                               CFG2["height_step"], CFG2["start_angle"], CFG2["stop_angle"],
                               CFG2["angle_step"]) for a in range(n_ant)]
            tabs = [torch.empty((11, g.n_rays), dtype=torch.float32, device=dev) for g in grids]
            streams = [torch.cuda.Stream(device=dev) for _ in range(n_ant)]
            rays = sum(g.n_rays for g in grids)

            def build_all():
                for g, t, s_ in zip(grids, tabs, streams):
                    solver.table_device(g, t, None, stream=s_)

            for _ in range(3):
                build_all()
            torch.cuda.synchronize()
            reps = 50
            t1 = time.perf_counter()
            for _ in range(reps):
                build_all()
            torch.cuda.synchronize()
            sec = time.perf_counter() - t1
            # the same tables in ONE launch (airice_table_launch_multi, table_multi_kernel)
            solver.tables_device(grids, tabs, stream=stream)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                solver.tables_device(grids, tabs, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize()
            one_ms = e0.elapsed_time(e1) / reps
            multi[f"{n_ant}_antennas"] = {
                "streams_rays_per_s": rays * reps / sec, "streams_ms_per_round": sec / reps * 1e3,
                "one_launch_rays_per_s": rays / (one_ms * 1e-3), "one_launch_ms": one_ms,
                "one_launch_vs_single_table": rays / (one_ms * 1e-3) / value if world == 1
                else None}
        extra["multi_antenna_tables"] = {
            "metric": "cfg2 tables of several antennas (MakeRayTracingTable per antenna, "
                      "RunMultiRayCode.C:29-52): concurrent HIP streams, and one "
                      "airice_table_launch_multi launch (rays/s)",
            **multi}
    if not args.no_cold and not sharded:
        extra["table_cold"] = table_cold(solver, grid, table, stream, rank, kern_ms)
    if not args.no_pcie and not sharded:
        # host-buffer callers (AllTableAllAntData is host memory): table build + D2H copy of the
        # 11 float columns into pinned memory, in stream order; never the headline value
        host = torch.empty((11, n_local), dtype=torch.float32, pin_memory=True)
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        reps = 10
        solver.table_device(grid, table, None, stream=stream)
        host.copy_(table, non_blocking=True)
        torch.cuda.synchronize()
        e0.record(stream)
        for _ in range(reps):
            solver.table_device(grid, table, None, stream=stream)
            host.copy_(table, non_blocking=True)
        e1.record(stream)
        for _ in range(reps):
            host.copy_(table, non_blocking=True)
        e2.record(stream)
        torch.cuda.synchronize()
        pms = e0.elapsed_time(e1) / reps
        cms = e1.elapsed_time(e2) / reps
        extra["table_to_host"] = {
            "metric": "cfg2 table build + D2H copy to pinned host memory (PCIe-inclusive rays/s)",
            "value": n_local / (pms * 1e-3), "unit": "rays/s", "ms": pms, "d2h_ms": cms,
            "d2h_GBps": 44 * n_local / (cms * 1e-3) / 1e9}
        del host
    if not args.no_default_grid:
        # the reference's default grid (10 m x 0.1 deg, 8,730,900 rays): throughput at a size
        # where launch ramp and tail are amortised
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        gd = make_grid(depth_cm, CFG2["ice_cm"])
        td = torch.empty((11, gd.n_rays), dtype=torch.float32, device=dev)
        solver.table_device(gd, td, None, stream=stream)
        torch.cuda.synchronize()
        e0.record(stream)
        for _ in range(5):
            solver.table_device(gd, td, None, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        dms = e0.elapsed_time(e1) / 5
        extra["table_default_grid"] = {"rays": gd.n_rays, "ms": dms,
                                       "value": gd.n_rays / (dms * 1e-3), "unit": "rays/s"}
        del td
    if not args.no_cfg4:
        extra["table_cfg4"] = table_cfg4(args, be, world, rank, distributed, coll_dev, pmc)
    if rank == 0 and not args.no_scalar:
        extra["scalar_latency_us"] = scalar_latencies(args)

    # ------------------------------------------- CPU legs: baselines + parity (rank 0, N=1)
    cpu = None
    parity_rep = None
    if rank == 0 and world == 1 and not args.no_cpu:
        import oracle
        from tests import parity
        nthr = max(1, min(args.cpu_threads, len(os.sched_getaffinity(0))))
        info = cpu_info(nthr)
        om = oracle.load_atmosphere(os.path.join(ROOT, "airiceraytracing_amd", "data",
                                                 "Atmosphere.dat.gz"))
        og = oracle.grid_init(depth_cm, CFG2["ice_cm"], CFG2["height_step"], CFG2["start_angle"],
                              CFG2["stop_angle"], CFG2["angle_step"])
        # bounded sample: whole cfg2 grids, repeated until >= cpu_seconds of wall time
        c0 = time.perf_counter()
        grids = 0
        while True:
            ot = oracle.table_rows(om, og, 0, og.height_steps, nthreads=nthr)
            grids += 1
            cdt = time.perf_counter() - c0
            if cdt >= args.cpu_seconds or grids >= 2000:
                break
        # 1-thread rate on strided rows, repeated until >= cpu_seconds / 4
        rows1 = list(range(0, og.height_steps, 97))
        c1 = time.perf_counter()
        passes = 0
        while True:
            for r_ in rows1:
                oracle.table_rows(om, og, r_, r_ + 1)
            passes += 1
            c1dt = time.perf_counter() - c1
            if c1dt >= args.cpu_seconds / 4:
                break
        one = passes * len(rows1) * og.angle_steps / c1dt
        # context: whole cfg2 grids on all physical cores of the box, for about a second (the
        # process's CPU quota, not only its affinity mask, bounds what this can show)
        nall = physical_cores()
        ca = time.perf_counter()
        ga = 0
        while True:
            oracle.table_rows(om, og, 0, og.height_steps, nthreads=nall)
            ga += 1
            cadt = time.perf_counter() - ca
            if cadt >= 1.0 or ga >= 200:
                break
        all_cores = {"value": ga * og.height_steps * og.angle_steps / cadt,
                     "threads_used": nall, "sample": f"{ga} full cfg2 grids in {cadt:.1f} s",
                     "note": ALL_CORES_NOTE}
        cpu = {"value": grids * og.height_steps * og.angle_steps / cdt, "unit": "rays/s",
               "cores": nthr, "kind": "port",
               "sample": f"{grids} x the full cfg2 grid ({og.height_steps * og.angle_steps} rays "
                         f"each) in {cdt:.1f} s, oracle C restatement (faithful call structure), "
                         f"OpenMP {nthr} threads",
               "one_thread_value": one, "seconds": cdt, **info,
               "all_physical_cores": all_cores,
               "not_the_reference": PORT_VS_REFERENCE,
               "survey_reference_probe": SURVEY_REFERENCE_PROBE["table_rays_per_s"],
               "survey_reference_probe_source": SURVEY_REFERENCE_PROBE["source"]}
        gt = table.cpu().numpy()
        ulps = parity.float_ulp_diff(gt, ot)
        finite = np.isfinite(ot) & np.isfinite(gt)
        rel = np.abs(gt.astype(np.float64) - ot) / np.maximum(np.abs(ot.astype(np.float64)), 1e-30)
        parity_rep = {"table_max_float_ulps": ulps,
                      "table_max_abs": float(np.max(np.abs(gt - ot)[finite])),
                      "table_max_rel": float(np.max(rel[finite])),
                      "nan_pattern_equal": bool(np.array_equal(np.isnan(gt), np.isnan(ot)))}
        if solve is not None:
            solve["cpu_baseline"] = minimizer_cpu_baseline(args, om, txh, dst, dep, nthr, info)
            solve["parity_vs_cpu"] = minimizer_parity(args, om, txh, dst, dep, out_h, st_h, nthr)
        if trace_h is not None:
            extra["pywrapper_trace"]["parity_vs_cpu"] = trace_parity(trace_h, nthr)
        if lookup_h is not None:
            extra["table_lookup"]["parity_vs_cpu"] = lookup_parity(om, og, lookup_h, nthr)
        if isinstance(extra.get("scalar_latency_us"), dict):
            extra["scalar_latency_us"]["cpu_oracle_per_call_us"] = scalar_cpu_per_call(om, og, ot)

    roof = counter_roofline("table_kernel_cfg4" if cfg4_headline else "table_kernel", n_local,
                            kern_ms, pmc, 44.0)
    roof["ocml_priced"] = ocml_priced(grid, n_local, kern_ms) if kern_ms else None

    if rank == 0:
        if cfg4_headline:
            par = shard_rep["parallelism"]
            workload = ("MakeRayTracingTable cfg4 (BASELINE configs[3]): TxH 100000->3000 m @1 m x "
                        "90.1->180 deg @0.01 deg, one table sharded by TxH rows over %d GPUs, "
                        "assembled in host memory" % world)
        elif sharded:
            par = f"rows-sharded+gather (dp{world}: TxH-row slabs, per-column RCCL gathers to rank 0)"
            workload = ("MakeRayTracingTable cfg2 grid refined %dx in TxH (step %g m), one "
                        "table sharded by TxH rows over %d GPUs" % (world, grid.height_step, world))
        else:
            par = f"replicas{world} (one antenna table per GPU)" if world > 1 else "single GPU"
            workload = ("MakeRayTracingTable cfg2: TxH 100000->3000 m @20 m x 92->180 deg @0.5 "
                        "deg, antenna 200 m below 3000 m ice")
        line = {
            "metric": "solved air->ice rays/sec (MakeRayTracingTable rays)",
            "value": value,
            "unit": "rays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "ms_per_step_incl_trailing_barrier": elapsed_bar / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if cfg4_headline else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (BASELINE cfg4 grid, sharded over %d GPUs)" % world
                     if cfg4_headline else
                     "synthetic (BASELINE cfg2 grid refined %dx in TxH, sharded over %d GPUs)"
                     % (world, world) if sharded else
                     "synthetic (BASELINE cfg2 grid%s)" % (", one per GPU" if world > 1 else ""))
                    + " over the reference GDAS Atmosphere.dat",
            "rccl_world_size": dist.get_world_size() if distributed else 1,
            "dist_backend": backend if distributed else None,
            "kernel_ms_per_rank": kern_ms_ranks,
            "config": {"workload": workload, "rays_per_gpu_step": n_local, "table_columns": 11,
                       "store": "f32", "parallelism": par},
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity_vs_cpu": parity_rep,
            "sharded": shard_rep,
            # BASELINE cfg4 (the north_star's 8-GPU fine table), strong scaling, beside the
            # weak-scaling headline; the full record is table_cfg4
            "sharded_cfg4": ({k: extra["table_cfg4"].get(k) for k in (
                "value", "unit", "scaling", "n_gpus", "ms_per_build", "value_incl_assembly",
                "assemble", "assemble_ms", "kernel_ms_per_rank")}
                if world > 1 and isinstance(extra.get("table_cfg4"), dict) else None),
            "minimizer": solve,
            **extra,
        }
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    if distributed:
        dist.destroy_process_group()


def gather_floats(x, distributed, world, coll_dev) -> list:
    """One float (None: NaN) from every rank, in rank order (all_gather; [x] on one process)."""
    if not distributed:
        return [x]
    import torch
    import torch.distributed as dist
    t = torch.tensor([float("nan") if x is None else float(x)], dtype=torch.float64,
                     device=coll_dev)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [None if v != v else v for v in (float(q.item()) for q in parts)]


def table_cold(solver, grid, table, stream, rank, warm_kernel_ms, builds: int = 16) -> dict:
    """The table build as the reference's callers run it: RunMultiRayCode.C:29-52 builds one
    table per AntennaDepths entry (MakeRayTracingTable, MultiRayAirIceRefraction.cc:2019-2158),
    each once.  ``builds`` cfg2-sized tables back to back on one stream, each for a grid key never
    built before in this process, timed on the wall clock (host launch work included) and by HIP
    events, beside the same number of repeated (warm) builds of the headline grid timed the same
    way:

    * ``new_depths``: antennas at new depths in the ice -- the row constants of the grid are shared
      across depths (their cache key holds only what the rows read), the angle sines too;
    * ``new_grids``: every build a new ice height and angle grid, so neither per-grid cache has
      the key: each build forms its rows and sines in the kernel."""
    import torch
    from airiceraytracing_amd import _lib, make_grid

    def run(grids) -> tuple[float, float]:
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for g in grids:
            solver.table_device(g, table, None, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / len(grids) * 1e3
        return wall, e0.elapsed_time(e1) / len(grids)

    warm_wall, warm_ev = run([grid] * builds)
    base = CFG2["depth_cm"] - 100000.0 * (rank + 1)  # depths this process has not built
    new_depths = [make_grid(base - 1300.0 * a, CFG2["ice_cm"], CFG2["height_step"],
                            CFG2["start_angle"], CFG2["stop_angle"], CFG2["angle_step"])
                  for a in range(builds)]
    before = _lib.table_cache_stats()
    d_wall, d_ev = run(new_depths)
    after = _lib.table_cache_stats()
    new_grids = [make_grid(CFG2["depth_cm"], CFG2["ice_cm"] - 1.0 * (a + 1 + 100 * rank),
                           CFG2["height_step"], CFG2["start_angle"] - 1e-7 * (a + 1),
                           CFG2["stop_angle"], CFG2["angle_step"]) for a in range(builds)]
    assert all(g.n_rays == grid.n_rays for g in new_grids + new_depths)
    g_wall, g_ev = run(new_grids)
    return {
        "metric": "cfg2-sized tables, each for an antenna / grid not built before "
                  "(RunMultiRayCode.C:29-52: one MakeRayTracingTable per antenna), ms per build",
        "builds": builds, "rays_per_build": grid.n_rays,
        "warm_ms_per_build": warm_wall, "warm_event_ms_per_build": warm_ev,
        "new_depths_ms_per_build": d_wall, "new_depths_event_ms_per_build": d_ev,
        "new_depths_vs_warm": d_wall / warm_wall,
        "new_depths_row_cache_keys_added": after["rows"]["keys"] - before["rows"]["keys"],
        "new_grids_ms_per_build": g_wall, "new_grids_event_ms_per_build": g_ev,
        "new_grids_vs_warm": g_wall / warm_wall,
        "new_grids_rays_per_s": grid.n_rays / (g_wall * 1e-3),
        "headline_kernel_ms": warm_kernel_ms}


def cfg4_check_rows(height_steps: int, step: float = 1.0) -> list[int]:
    """Rows of the cfg4 table checked against the oracle: the first and last rows, the rows on
    either side of each atmosphere-layer bound the Tx heights cross (23141.75, 8363.54 and
    3217.48 m: at the 1 m step rows 76858/76859, 91636/91637, 96782/96783), and evenly spaced rows
    between."""
    rows = {0, 1, height_steps - 1}
    for bound in (23141.75, 8363.54, 3217.48):
        r = int((100000.0 - bound) // step)
        rows |= {r, r + 1}
    rows |= {int(r) for r in np.linspace(0, height_steps - 1, 6)}
    return sorted(r for r in rows if 0 <= r < height_steps)


def table_cfg4(args, be, world, rank, distributed, coll_dev, pmc) -> dict:
    """BASELINE cfg4, the fine table (872,135,991 rays, 38.4 GB): built in HBM (N=1: the whole
    grid on one GPU; N>1: contiguous TxH-row slabs, one per GPU), timed over cfg4_reps builds, then
    assembled in host memory where the reference keeps AllTableAllAntData (.cc:2079-2136): per
    GPU one strided D2H copy per column (airice_table_to_host) into page-locked host pages -- a
    private buffer at N=1, a node-shared mapping (distributed.SharedHostTable) that every rank
    fills in parallel at N>1.
    Rank 0 checks cfg4_check_rows() of the host table against the oracle."""
    import torch
    import torch.distributed as dist
    from airiceraytracing_amd import make_grid
    from airiceraytracing_amd.distributed import run_sharded_table, shard_rows
    g = make_grid(CFG4["depth_cm"], CFG4["ice_cm"], CFG4["height_step"], CFG4["start_angle"],
                  CFG4["stop_angle"], CFG4["angle_step"])
    asteps, n = g.angle_steps, g.n_rays
    begin, count, per = shard_rows(g.table_rows, world, rank)
    dev, stream = be.dev, be.stream
    ev0, ev1 = be.event(), be.event()
    st = {"i": 0}

    def compute(b, c, slab):
        if st["i"] == 1:
            ev0.record(stream)
        be.table(g, slab, row_begin=b, row_count=c, ld=slab.shape[1])
        st["i"] += 1
        if st["i"] == 1 + args.cfg4_reps:
            ev1.record(stream)

    host_copy, register, unregister = be.table_to_host, be.host_register, be.host_unregister

    want_host = args.cfg4_host != "none"
    rep = {"metric": "cfg4 fine table rays/s (BASELINE cfg4: MakeRayTracingTable TxH 100000->3000 "
                     "m @1 m x 90.1->180 deg @0.01 deg, antenna 200 m below 3000 m ice)",
           "rays": n, "rows": g.table_rows, "angles": asteps, "table_bytes": 44 * n,
           "n_gpus": world, "unit": "rays/s",
           # the same 872,135,991-ray table at every N: strong scaling across the GPUs
           "scaling": "strong"}
    host_tab = None
    if distributed:
        mode = "host" if want_host else "rccl"
        # every rank takes the same assembly path: rank 0 checks that /dev/shm can hold the shared
        # host table and broadcasts the decision with the file name (a rank failing alone inside
        # the collective sequence would leave the others waiting)
        plan = [args.cfg4_host_path or f"/dev/shm/airice_cfg4_{os.getpid()}_{int(time.time())}",
                mode, None]
        if rank == 0 and mode == "host":
            try:
                fs = os.statvfs(os.path.dirname(plan[0]) or ".")
                free = fs.f_bavail * fs.f_frsize
                if free < 44 * n * 1.05:
                    plan[1], plan[2] = "rccl", (f"{os.path.dirname(plan[0])} has "
                                                f"{free / 1e9:.1f} GB free")
            except OSError as e:
                plan[1], plan[2] = "rccl", str(e)
        dist.broadcast_object_list(plan, src=0)
        mode = plan[1]
        if plan[2] is not None:  # no room for the shared host table: assemble on the root's GPU
            rep["host_assembly_error"] = plan[2]
        r = run_sharded_table(g, compute, args.cfg4_reps, 1, device=dev, coll_device=coll_dev,
                              sync=be.sync, gather_reps=1, assemble=mode,
                              host_path=plan[0], host_copy=host_copy,
                              host_register=register, host_unregister=unregister)
        be.sync()
        mode = r["assemble"]  # "rccl" when a rank could not create or map the shared host table
        if r.get("host_assembly_error"):
            rep["host_assembly_error"] = r["host_assembly_error"]
        build_s = r["elapsed_s"] / args.cfg4_reps
        kms_rank = ev0.elapsed_time(ev1) / args.cfg4_reps if r["rays_this_rank"] > 0 else None
        rep.update({"value": n / build_s, "ms_per_build": build_s * 1e3,
                    "kernel_ms_rank0": kms_rank, "kernel_ms_this_rank": kms_rank,
                    "kernel_ms_per_rank": gather_floats(kms_rank, distributed, world, coll_dev),
                    "rows_per_rank": r["rows_per_rank"], "assemble": mode,
                    "assemble_ms": r["gather_s"] * 1e3,
                    "assemble_GBps": r["bytes_assembled"] / r["gather_s"] / 1e9
                    if r["gather_s"] > 0 else None,
                    "value_incl_assembly": n / (build_s + r["gather_s"]),
                    "parallelism": f"rows-sharded dp{world}: TxH-row slabs, "
                                   + ("per-rank D2H into one node-shared host table (no "
                                      "collective)" if mode == "host" else
                                      "per-column RCCL gathers into rank 0's HBM")})
        host_tab = r["assembled"] if rank == 0 else None
        kern_units = r["rays_this_rank"]
        slab_holder = [r]
    else:
        slab = torch.empty((11, n), dtype=torch.float32, device=dev)
        be.sync()
        t0 = time.perf_counter()
        compute(0, g.table_rows, slab)  # the grid's first build (st i: 0 -> 1), timed apart
        be.sync()
        rep["first_build_ms"] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        for _ in range(args.cfg4_reps):
            compute(0, g.table_rows, slab)
        be.sync()
        build_s = (time.perf_counter() - t0) / args.cfg4_reps
        kms = ev0.elapsed_time(ev1) / args.cfg4_reps
        rep.update({"value": n / build_s, "ms_per_build": build_s * 1e3, "kernel_ms": kms,
                    "kernel_value": n / (kms * 1e-3), "parallelism": "single GPU"})
        # one build of a grid key never built before (ice 1 cm lower, start angle 1e-7 deg lower:
        # the same 97,001 x 8,991 rays) into the same, already written slab: the cold cost of
        # the per-grid caches at cfg4 size, apart from the first touch of fresh device memory
        # that the grid's first build above also pays (RunMultiRayCode.C builds each antenna once)
        g2 = make_grid(CFG4["depth_cm"], CFG4["ice_cm"] - 1.0, CFG4["height_step"],
                       CFG4["start_angle"] - 1e-7, CFG4["stop_angle"], CFG4["angle_step"])
        if g2.n_rays == n and be.is_gpu:
            be.sync()
            t0 = time.perf_counter()
            be.table(g2, slab)
            be.sync()
            rep["new_key_build_ms"] = (time.perf_counter() - t0) * 1e3
            be.table(g, slab)  # the table the parity rows are checked in
            be.sync()
        kern_units = n
        if want_host:
            t1 = time.perf_counter()
            host_np = np.empty((11, n), dtype=np.float32)
            register(host_np.ctypes.data, host_np.nbytes)
            rep["host_alloc_register_s"] = time.perf_counter() - t1
            host_tab = torch.from_numpy(host_np)
            e2, e3 = be.event(), be.event()
            e2.record(stream)
            host_copy(slab, n, host_tab, 0)
            e3.record(stream)
            be.sync()
            d2h_ms = e2.elapsed_time(e3)
            rep.update({"assemble": "host", "assemble_ms": d2h_ms,
                        "assemble_GBps": 44 * n / (d2h_ms * 1e-3) / 1e9,
                        "value_incl_assembly": n / (build_s + d2h_ms * 1e-3)})
        else:
            host_tab = slab
        slab_holder = [slab]
    rep["roofline"] = counter_roofline("table_kernel_cfg4", kern_units,
                                       rep.get("kernel_ms") or rep.get("kernel_ms_rank0"), pmc,
                                       44.0)
    if rank == 0 and not args.no_cpu:
        import oracle
        from tests import parity
        om = oracle.load_atmosphere(os.path.join(ROOT, "airiceraytracing_amd", "data",
                                                 "Atmosphere.dat.gz"))
        og = oracle.grid_init(CFG4["depth_cm"], CFG4["ice_cm"], CFG4["height_step"],
                              CFG4["start_angle"], CFG4["stop_angle"], CFG4["angle_step"])
        rows = cfg4_check_rows(g.table_rows, CFG4["height_step"])
        worst, nan_ok = 0, True
        for r_ in rows:
            got = host_tab[:, r_ * asteps:(r_ + 1) * asteps].cpu().numpy()
            ref = oracle.table_rows(om, og, r_, r_ + 1, nthreads=min(16, args.cpu_threads))
            worst = max(worst, parity.float_ulp_diff(got, ref))
            nan_ok &= bool(np.array_equal(np.isnan(got), np.isnan(ref)))
        rep["parity_vs_cpu"] = {"rows": rows, "rays": len(rows) * asteps,
                                "checked_in": "host-assembled table" if rep.get("assemble") ==
                                "host" else "device table",
                                "max_float_ulps": int(worst), "nan_pattern_equal": nan_ok}
    # release the 38.4 GB (device slab, page-locked host table) before the next line item
    if distributed:
        r = slab_holder[0]
        if r.get("host") is not None:
            r["host"].unregister(unregister)
            r["host"].close()
    elif want_host:
        unregister(host_np.ctypes.data)
    del host_tab, slab_holder
    be.release()
    return rep


def minimizer_cpu_baseline(args, om, txh, dst, dep, nthr, info) -> dict:
    """The oracle's Air2IceRayTracing (faithful GSL-bisection restatement) over the head of the
    same cfg3 batch, OpenMP on nthr host threads, until ~cpu_seconds; plus a 1-thread sample."""
    import oracle
    n = len(txh)
    m = min(n, 20000)
    t0 = time.perf_counter()
    oracle.solve_batch(om, txh[:m], dst[:m], dep[:m], 3000.0, nthreads=nthr)
    rate = m / max(time.perf_counter() - t0, 1e-9)
    m = int(min(n, max(m, rate * args.cpu_seconds)))
    done = 0
    t0 = time.perf_counter()
    while True:
        oracle.solve_batch(om, txh[:m], dst[:m], dep[:m], 3000.0, nthreads=nthr)
        done += m
        dt = time.perf_counter() - t0
        if dt >= args.cpu_seconds / 2:
            break
    m1 = 2000
    t1 = time.perf_counter()
    oracle.solve_batch(om, txh[:m1], dst[:m1], dep[:m1], 3000.0, nthreads=1)
    one = m1 / (time.perf_counter() - t1)
    nall = physical_cores()
    ma = int(min(n, max(20000, 2 * rate * nall / max(nthr, 1))))  # ~2 s on all cores
    ta = time.perf_counter()
    oracle.solve_batch(om, txh[:ma], dst[:ma], dep[:ma], 3000.0, nthreads=nall)
    all_cores = {"value": ma / (time.perf_counter() - ta), "threads_used": nall,
                 "sample": f"the first {ma} queries", "note": ALL_CORES_NOTE}
    return {"value": done / dt, "unit": "solves/s", "cores": nthr, "kind": "port",
            "sample": f"{done} cfg3 queries (the head of the timed batch) in {dt:.1f} s, oracle "
                      f"GSL-bisection restatement, OpenMP {nthr} threads; 1-thread on {m1}",
            "one_thread_value": one, **info, "all_physical_cores": all_cores,
            "not_the_reference": PORT_VS_REFERENCE,
            "survey_reference_probe": SURVEY_REFERENCE_PROBE["minimizer_solves_per_s"]}


def stride_text(k) -> str:
    return "every query" if int(k) == 1 else f"every {int(k)}th query"


def minimizer_parity(args, om, txh, dst, dep, out_h, st_h, nthr) -> dict:
    """Every (k-th) query of the timed 1e6 batch against the oracle: per-column relative error
    (tests/parity.py rule), NaN positions, status bits on the pinned rows."""
    import oracle
    from tests import parity
    idx = np.arange(0, len(txh), args.parity_stride)
    ref, rst = oracle.solve_batch(om, txh[idx], dst[idx], dep[idx], 3000.0, nthreads=nthr)
    pinned = (rst & oracle.SOLVE_UNPINNED) == 0
    rep = parity.compare_with_root_window(out_h[:, idx], ref, parity.SOLVE_FLOORS,
                                          out_h[10, idx], ref[10], mask=pinned)
    return {"sample": f"{stride_text(args.parity_stride)} of the timed batch ({idx.size})",
            "max_rel": rep["max_rel"], "max_abs": rep["max_abs"], "n_bad": rep["n_bad"],
            "root_window_rows": rep["window_rows"],
            "nan_mask_equal": rep["nan_mismatch"] == 0 and rep["inf_mismatch"] == 0,
            "status_bits_equal": bool(np.array_equal(st_h[idx][pinned] & 0x1F,
                                                     rst[pinned] & 0x1F)),
            "masked_unpinned": int((~pinned).sum()), "ok": rep["ok"]}


def trace_parity(trace_h, nthr) -> dict:
    import oracle
    from tests import parity
    (depth, ice, txh, dist_), idx, got = trace_h
    om = oracle.load_atmosphere(os.path.join(ROOT, "airiceraytracing_amd", "data",
                                             "Atmosphere.dat.gz"), pi=oracle.PI_EXACT)
    ref = oracle.py_trace_batch(om, depth[idx], ice[idx], txh[idx], dist_[idx], nthreads=nthr)
    rep = parity.compare_with_root_window(got.T, ref.T, parity.TRACE_FLOORS, 180 - got[:, 5],
                                          180 - ref[:, 5])
    return {"sample": f"{stride_text(idx[1] - idx[0] if idx.size > 1 else 1)} of the timed "
                      f"1e7 batch ({idx.size})",
            "max_rel": rep["max_rel"], "max_abs": rep["max_abs"], "n_bad": rep["n_bad"],
            "root_window_rows": rep["window_rows"],
            "nan_mask_equal": rep["nan_mismatch"] == 0 and rep["inf_mismatch"] == 0,
            "solved_mask_equal": bool(np.array_equal(got[:, 0] != -1000, ref[:, 0] != -1000)),
            "ok": rep["ok"]}


def lookup_parity(om, og, lookup_h, nthr) -> dict:
    """Every query of the timed lookup batch against the oracle's lookup on the same table (the
    GPU's floats copied to the host): lanes without the minimizer fallback bit for bit (NaN
    positions included), fallback lanes (.cc:1418-1420) within the minimizer tolerance, rows whose
    bracket set-up reads uninitialised GSL state masked as in tests/test_gpu_lookup.py."""
    import oracle
    from tests import parity
    src, dcm, depth_cm, tab, out, ok, fl = lookup_h
    dep = np.full(src.size, depth_cm)
    rout, rok, rfl = oracle.table_lookup_batch(om, oracle.lookup_table(tab, og), src, dcm, dep,
                                               CFG2["ice_cm"], nthreads=nthr)
    fb = (rfl & oracle.LOOKUP_FALLBACK) != 0
    a, b = out[:, ~fb], rout[:, ~fb]
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    idx = np.flatnonzero(fb)
    mask = np.ones(idx.size, dtype=bool)
    for j, i in enumerate(idx):
        _, st = oracle.air2ice(om, src[i], dcm[i], CFG2["ice_cm"] / 100, dep[i])
        mask[j] = (st & oracle.SOLVE_UNPINNED) == 0
    rep = parity.compare_columns(out[:, idx], rout[:, idx], parity.HDTIP_FLOORS, mask=mask) \
        if idx.size else {"ok": True, "max_rel": 0.0}
    return {"sample": f"every query of the timed batch ({src.size})",
            "flags_equal": bool(np.array_equal(fl, rfl)),
            "non_fallback_lanes": int((~fb).sum()),
            "non_fallback_bitwise_equal": bool(same.all()),
            "non_fallback_ok_equal": bool(np.array_equal(ok[~fb], rok[~fb])),
            "fallback_lanes": int(idx.size), "fallback_masked": int((~mask).sum()),
            "fallback_max_rel": rep["max_rel"],
            "ok": bool(np.array_equal(fl, rfl) and same.all() and
                       np.array_equal(ok[~fb], rok[~fb]) and rep["ok"])}


def scalar_cpu_per_call(om, og, ot) -> dict:
    """The same scalar operations on the CPU oracle, one thread, per call (batch time / n):
    the comparison the scalar drop-in latencies are held against."""
    import oracle
    from tests.parity import cfg3_queries
    n = 400
    txh, dst, dep = cfg3_queries(n, seed=31337)
    res = {}
    t0 = time.perf_counter()
    oracle.solve_batch(om, txh, dst, dep, 3000.0, nthreads=1)
    res["Air2IceRayTracing"] = (time.perf_counter() - t0) / n * 1e6
    t0 = time.perf_counter()
    for i in range(n):
        oracle.hdtip(om, txh[i] * 100, dst[i] * 100, -20000.0, 300000.0)
    res["GetHorizontalDistanceToIntersectionPoint"] = (time.perf_counter() - t0) / n * 1e6
    lt = oracle.lookup_table(ot, og)
    src, dcm = txh * 100, dst * 100
    t0 = time.perf_counter()
    oracle.table_lookup_batch(om, lt, src, dcm, np.full(n, -20000.0), 300000.0, nthreads=1)
    res["GetHorizontalDistanceToIntersectionPoint_Table"] = (time.perf_counter() - t0) / n * 1e6
    t0 = time.perf_counter()
    rows = 8
    oracle.table_rows(om, og, 0, rows)
    res["GetRayTracingSolutions"] = (time.perf_counter() - t0) / (rows * og.angle_steps) * 1e6
    omp = oracle.load_atmosphere(os.path.join(ROOT, "airiceraytracing_amd", "data",
                                              "Atmosphere.dat.gz"), pi=oracle.PI_EXACT)
    t0 = time.perf_counter()
    oracle.py_trace_batch(omp, dep, np.full(n, 3000.0), np.minimum(txh, 20000.0), dst * 0.6,
                          nthreads=1)
    res["Py_TraceIceToAir"] = (time.perf_counter() - t0) / n * 1e6
    # RayTracingFunctions::GetAirPropagationPar (RayTracingFunctions.cc:529-659), the latency
    # driver's arguments; the oracle's per-call ctypes overhead (~1-2 us) is measured on a no-op op
    # and subtracted
    args = [[92 + float(np.fmod(dst[i], 88.0)), float(txh[i]), 3000.0] for i in range(n)]
    t0 = time.perf_counter()
    for a in args:
        oracle.rtf_eval(om, 3, a)  # AIRICE_RTF_AIR_PROPAGATION
    t_rtf = time.perf_counter() - t0
    t0 = time.perf_counter()
    for a in args:
        oracle.getnz_air(om, a[1])
    t_call = time.perf_counter() - t0
    res["RayTracingFunctions::GetAirPropagationPar"] = max(t_rtf - t_call, 0.0) / n * 1e6
    res["note"] = ("oracle restatement, 1 thread, same query distribution; Python loop overhead "
                   "included only for GetHorizontalDistanceToIntersectionPoint; the RTF figure "
                   "has a ctypes round trip (oracle.getnz_air) subtracted")
    return res


def scalar_latencies(args) -> dict | None:
    """Per-call latency of the scalar drop-in entry points (one query per call, host arguments,
    as CoREAS and TraceIceToAir.py call them), measured by tests/cpp/latency_driver (C++, linked
    against libairice.so) in a child process: with the one-query calls on the host (the library's
    default, airice_scalar_mode), and under "device" the same calls as one-wave GPU kernels
    (AIRICE_SCALAR=device)."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "cpp", "latency_driver")
    if not os.path.exists(exe):
        return None
    import gzip
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        with gzip.open(os.path.join(ROOT, "airiceraytracing_amd", "data",
                                    "Atmosphere.dat.gz")) as fz, \
                open(os.path.join(td, "Atmosphere.dat"), "wb") as fo:
            fo.write(fz.read())
        r = subprocess.run([exe], cwd=td, capture_output=True, text=True, timeout=300)
        rd = subprocess.run([exe], cwd=td, capture_output=True, text=True, timeout=300,
                            env=dict(os.environ, AIRICE_SCALAR="device"))
    if r.returncode != 0:
        return {"error": r.stderr[-500:]}
    rep = json.loads(r.stdout.strip().splitlines()[-1])
    rep["where"] = "host (one-query calls on the CPU, airice_scalar_mode default)"
    rep["device"] = (json.loads(rd.stdout.strip().splitlines()[-1]) if rd.returncode == 0
                     else {"error": rd.stderr[-500:]})
    return rep


if __name__ == "__main__":
    main()
