"""Sharding + gather of the table grid / query batches (airiceraytracing_amd/distributed.py)
over gloo with world_size 2 on CPU; the per-shard compute is the oracle (no GPU here).  The
assembled result must be bitwise equal to a single-process run."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from airiceraytracing_amd.distributed import shard_rows


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("total,world", [(4851, 2), (4851, 8), (7, 8), (9701, 3), (1, 2)])
def test_shard_rows_cover_exactly(total, world):
    seen = []
    per0 = None
    for r in range(world):
        b, c, per = shard_rows(total, world, r)
        per0 = per if per0 is None else per0
        assert per == per0 and 0 <= c <= per
        seen.extend(range(b, b + c))
    assert seen == list(range(total))


def _worker(rank, world, port, q):
    import oracle
    from airiceraytracing_amd.distributed import queries_sharded, table_sharded
    from tests.conftest import ATMOSPHERE_GZ
    from tests.parity import cfg3_queries
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = oracle.load_atmosphere(ATMOSPHERE_GZ)
    g = oracle.grid_init(-20000.0, 300000.0, 500.0, 92.0, 180.0, 2.0)

    def tcompute(begin, count, out):
        t = oracle.table_rows(m, g, begin, begin + count)
        out[:, :t.shape[1]] = torch.from_numpy(t)

    table = table_sharded(g, tcompute)
    txh, dst, dep = cfg3_queries(301, seed=99)

    def qcompute(begin, count, out):
        o, _ = oracle.solve_batch(m, txh[begin:begin + count], dst[begin:begin + count],
                                  dep[begin:begin + count], 3000.0)
        out[:, :count] = torch.from_numpy(o)

    sol = queries_sharded(301, qcompute, cols=17)
    if rank == 0:
        q.put((table.numpy(), sol.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_sharded_equals_single_process():
    import oracle
    from tests.conftest import ATMOSPHERE_GZ
    from tests.parity import cfg3_queries
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    table, sol = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    m = oracle.load_atmosphere(ATMOSPHERE_GZ)
    g = oracle.grid_init(-20000.0, 300000.0, 500.0, 92.0, 180.0, 2.0)
    ref = oracle.table_rows(m, g, 0, g.height_steps)
    assert table.shape == ref.shape
    np.testing.assert_array_equal(table, ref)
    txh, dst, dep = cfg3_queries(301, seed=99)
    refq, _ = oracle.solve_batch(m, txh, dst, dep, 3000.0)
    np.testing.assert_array_equal(sol, refq)


def _bench_sharded_worker(rank, world, port, q):
    """bench.py --mode sharded logic (run_sharded_table) with the oracle as the slab compute."""
    import oracle
    from airiceraytracing_amd.distributed import run_sharded_table, sharded_step_grid_step
    from tests.conftest import ATMOSPHERE_GZ
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = oracle.load_atmosphere(ATMOSPHERE_GZ)
    # bench's weak-scaling grid, coarsened for the CPU: base step 1000 m refined world-fold
    g = oracle.grid_init(-20000.0, 300000.0, sharded_step_grid_step(1000.0, world), 92.0, 180.0,
                         4.0)
    calls = []

    def compute(begin, count, slab):
        calls.append((begin, count))
        t = oracle.table_rows(m, g, begin, begin + count)
        slab[:, :t.shape[1]] = torch.from_numpy(t)

    r = run_sharded_table(g, compute, steps=2, warmup=1, gather_reps=2)
    if rank == 0:
        q.put((r["assembled"].numpy(), r["rows_per_rank"], r["bytes_to_root"], len(calls),
               r["gather_s"] >= 0))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_bench_sharded_mode_assembles_table_bitwise(world):
    import oracle
    from airiceraytracing_amd.distributed import sharded_step_grid_step
    from tests.conftest import ATMOSPHERE_GZ
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_sharded_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    table, per, nbytes, ncalls, gathered = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    m = oracle.load_atmosphere(ATMOSPHERE_GZ)
    g = oracle.grid_init(-20000.0, 300000.0, sharded_step_grid_step(1000.0, world), 92.0, 180.0,
                         4.0)
    ref = oracle.table_rows(m, g, 0, g.height_steps)
    assert table.shape == ref.shape
    np.testing.assert_array_equal(table.view(np.int32), ref.view(np.int32))
    assert per == -(-g.height_steps // world)
    assert ncalls == 3 and gathered
    # every rank but the root sends its rows: 11 float columns per ray
    assert nbytes == (g.height_steps - shard_rows(g.height_steps, world, 0)[1]) * g.angle_steps * 44


def _cfg4_mode_worker(rank, world, port, q, assemble, host_path, map_raises=False):
    """bench.py's cfg4 item / --workload cfg4 logic (run_sharded_table with the cfg4 angle grid,
    coarsened in TxH for the CPU) with the oracle as the slab compute: the table assembled in host
    memory (SharedHostTable, every rank writing its rows) or by per-column gathers.  map_raises:
    every non-root rank's mapping of the shared table raises a RuntimeError (not an OSError)."""
    import oracle
    from airiceraytracing_amd import distributed as D
    from airiceraytracing_amd.distributed import run_sharded_table
    from tests.conftest import ATMOSPHERE_GZ
    if map_raises and rank != 0:
        real = D.SharedHostTable

        def failing(path, cols, n, create):
            if not create:
                raise RuntimeError("injected: mapping the shared host table failed")
            return real(path, cols, n, create=create)
        D.SharedHostTable = failing
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m = oracle.load_atmosphere(ATMOSPHERE_GZ)
    g = oracle.grid_init(-20000.0, 300000.0, 997.0, 90.1, 180.0, 0.37)  # cfg4 angles, coarse

    def compute(begin, count, slab):
        t = oracle.table_rows(m, g, begin, begin + count)
        slab[:, :t.shape[1]] = torch.from_numpy(t)

    r = run_sharded_table(g, compute, steps=1, warmup=0, gather_reps=2, assemble=assemble,
                          host_path=host_path)
    if rank == 0:
        q.put((r["assembled"].clone().numpy(), r["bytes_assembled"], r["assemble"],
               r["host_assembly_error"]))
    dist.barrier()
    if r["host"] is not None:
        r["host"].close()
    dist.destroy_process_group()


@pytest.mark.parametrize("assemble,world", [("host", 2), ("host", 3), ("rccl", 3),
                                            ("host-fail", 2), ("host-map-raises", 3)])
def test_gloo_cfg4_mode_assembles_table_bitwise(tmp_path, assemble, world):
    """host-fail: the root cannot create the shared host table (its directory does not exist):
    every rank learns it and takes the gather path, instead of the others waiting in a barrier.
    host-map-raises: the non-root ranks' mappings raise a RuntimeError (only OSError /
    ValueError used to reach the agreement); the same fallback, no deadlock."""
    import oracle
    from tests.conftest import ATMOSPHERE_GZ
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    raises = assemble == "host-map-raises"
    fail = assemble == "host-fail" or raises
    assemble = "host" if fail else assemble
    host_path = str(tmp_path / ("no_such_dir" if fail and not raises else "") / "airice_host_table")
    procs = [ctx.Process(target=_cfg4_mode_worker,
                         args=(r, world, port, q, assemble, host_path, raises))
             for r in range(world)]
    for p in procs:
        p.start()
    table, nbytes, mode, err = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    m = oracle.load_atmosphere(ATMOSPHERE_GZ)
    g = oracle.grid_init(-20000.0, 300000.0, 997.0, 90.1, 180.0, 0.37)
    ref = oracle.table_rows(m, g, 0, g.height_steps)
    if fail:
        assert mode == "rccl" and err is not None
        assert ("RuntimeError" if raises else "FileNotFoundError") in err or \
            (raises and "could not map" in err), err
        assemble = "rccl"
    else:
        assert err is None
    assert mode == assemble and table.shape == ref.shape
    np.testing.assert_array_equal(table.view(np.int32), ref.view(np.int32))
    if assemble == "host":
        assert nbytes == ref.size * 4
        assert not os.path.exists(host_path)  # unlinked once every rank had it mapped


def _run_bench_ranks(world, argv, json_path, timeout=240):
    from tests.bench_rehearsal import rank_main
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=rank_main, args=(r, world, port, argv, json_path))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=timeout)
        assert p.exitcode == 0, p.exitcode
    import json
    with open(json_path) as f:
        lines = [ln for ln in f.read().splitlines() if ln.strip()]
    assert len(lines) == 1
    return json.loads(lines[0])


BENCH8 = ["--gpus", "8", "--steps", "2", "--warmup", "1", "--height-step", "400",
          "--cfg4-height-step", "2000", "--cfg4-reps", "1", "--no-cpu", "--no-solve", "--no-trace",
          "--no-lookup", "--no-multi", "--no-scalar", "--no-default-grid", "--no-cold", "--no-pcie"]


@pytest.mark.parametrize("cfg4_host", ["shared", "fail"])
def test_gloo_world8_bench_flow(tmp_path, cfg4_host):
    """The whole bench.py N>1 flow (bench.main) at world size 8 over gloo, each rank's table slabs
    from the oracle (tests/bench_rehearsal.py): one JSON line with n_gpus 8, the sharded cfg2-style
    table assembled bit for bit equal to the whole grid built on one rank, and the cfg4 item sharded
    over 8 ranks -- assembled in a node-shared host table, or, when that file cannot be created
    (``fail``: its path is an existing directory), by the gather every rank falls back to."""
    host_path = tmp_path / "cfg4_host_table"
    if cfg4_host == "fail":
        host_path.mkdir()
    line = _run_bench_ranks(8, BENCH8 + ["--cfg4-host-path", str(host_path)],
                            str(tmp_path / "bench.json"))
    assert line["n_gpus"] == 8 and line["steps"] == 2 and line["scaling"] == "weak"
    assert line["value"] > 0 and line["ms_per_step"] > 0
    assert line["sharded"]["assembled_bitwise_equal_single_gpu"] is True
    assert line["sharded"]["rows_per_rank"] == -(-1941 // 8)
    c4 = line["table_cfg4"]
    assert c4["n_gpus"] == 8 and c4["rows"] == 49 and c4["value"] > 0
    if cfg4_host == "fail":
        assert c4["assemble"] == "rccl" and "IsADirectoryError" in c4["host_assembly_error"]
    else:
        assert c4["assemble"] == "host" and "host_assembly_error" not in c4


BENCH2 = ["--gpus", "2", "--steps", "2", "--warmup", "1", "--height-step", "400",
          "--no-cfg4", "--no-cpu", "--no-solve", "--no-trace", "--no-lookup", "--no-multi",
          "--no-scalar", "--no-default-grid", "--no-cold", "--no-pcie"]


def test_bench_world_size_mismatch_exits_nonzero(monkeypatch):
    """Under torch.distributed.run, WORLD_SIZE != --gpus is refused before any rendezvous or
    device work: exit status 2, no JSON line."""
    import bench
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("LOCAL_RANK", "0")
    for gpus in ("3", "1"):
        argv = ["--gpus", gpus] + BENCH2[2:]
        with pytest.raises(SystemExit) as e:
            bench.main(argv, make_backend=lambda r: pytest.fail("backend built"))
        assert e.value.code == 2


def test_bench_self_launch_two_ranks(monkeypatch, capsys):
    """``bench.py --gpus 2`` with no RANK in the environment starts torch.distributed.run with two
    ranks as a child process (gloo here, the CPU rehearsal backend standing in for the kernels)
    and relays rank 0's single JSON line: n_gpus 2, the sharded table bitwise equal to the whole
    grid."""
    import json
    import bench
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    entry = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench_rehearsal_entry.py")
    rc = bench.self_launch(2, BENCH2, script=entry, timeout=300)
    out = capsys.readouterr().out
    assert rc == 0, out
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1, lines
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["rccl_world_size"] == 2 and line["dist_backend"] == "gloo"
    assert line["scaling"] == "weak" and line["value"] > 0
    assert line["sharded"]["assembled_bitwise_equal_single_gpu"] is True
    assert len(line["kernel_ms_per_rank"]) == 2


def test_bench_main_self_launches_without_rank(monkeypatch):
    """bench.main(--gpus 2) outside torch.distributed.run goes to self_launch before importing
    torch (no backend is built in the launching process) and exits with its status."""
    import bench
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    seen = {}

    def fake(n, argv, script=None, timeout=None):
        seen.update(n=n, argv=list(argv))
        return 0

    monkeypatch.setattr(bench, "self_launch", fake)
    with pytest.raises(SystemExit) as e:
        bench.main(BENCH2, make_backend=lambda r: pytest.fail("backend built"))
    assert e.value.code == 0 and seen == {"n": 2, "argv": BENCH2}


def test_bench_self_launch_relays_failure(tmp_path, capsys):
    """A rank that fails makes the self-launched run fail: torch.distributed.run's non-zero
    status is bench.py's, and no JSON line is printed."""
    import bench
    script = tmp_path / "fail_rank.py"
    script.write_text("import os, sys\nsys.exit(3 if os.environ.get('RANK') == '1' else 0)\n")
    rc = bench.self_launch(2, [], script=str(script), timeout=120)
    out = capsys.readouterr().out
    assert rc != 0 and not out.strip()
