"""Where roots_kernel's wave time goes (debug, GPU box): a -DAIRICE_ROOTS_STAMP=1 build records four
shader-clock stamps per wave (entry, after the block's LDS counting sort, after the sorted query's
inputs are at hand, after solve_root) through AIRICE_SOLVE_STATS; this prints, over the 1e6 cfg3 solves,
the share of wave time in each phase and the share of a block's wave slots left idle waiting for
the block's slowest wave (a CU starts its next 1,024-query block only then).

    tools/build_variant.sh airiceraytracing_amd/csrc /tmp/stamp.so -DAIRICE_ROOTS_STAMP=1 ...
    python tools/roots_stamps.py /tmp/stamp.so [n]
    (a -DAIRICE_ROOTS_STAMP=2 build with --loop: the search's time in next_point, in the
    evaluations and in the rest of the loop, per wave)
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BLOCK = 1024


def main():
    lib = os.path.abspath(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1000000
    path = "/tmp/roots_stamps.bin"
    if os.path.exists(path):
        os.remove(path)
    env = dict(os.environ, AB_LIB=lib)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "solve_stats.py"), "--child",
                    "stamp", str(n), path], env=env, check=True, timeout=300)
    if "--begin" in sys.argv:
        # a -DAIRICE_ROOTS_STAMP=3 build: the set-up's cumulative stamps per wave (longest lane)
        a = np.fromfile(path, dtype=np.int32).reshape(-1, 8).astype(np.int64)[:n]
        key = np.stack([np.arange(len(a)) // BLOCK, a[:, 0], a[:, 1]], axis=1)
        _, inv = np.unique(key, axis=0, return_inverse=True)
        inv = inv.ravel()
        nw = inv.max() + 1
        cols = {}
        for j, name in enumerate(["tx_endpoint", "ice_endpoint_rtop", "ratio", "rx_endpoint",
                                  "probe_and_bracket", "probing_lanes"]):
            v = np.zeros(nw)
            np.maximum.at(v, inv, a[:, 2 + j])
            cols[name] = v
        tot = np.zeros(nw)
        np.maximum.at(tot, inv, a[:, 1])
        rep = {"waves": int(nw), "search_cycles_mean": float(tot.mean()),
               "waves_with_a_probing_lane": float(cols["probing_lanes"].mean())}
        for name in ["tx_endpoint", "ice_endpoint_rtop", "ratio", "rx_endpoint", "probe_and_bracket"]:
            rep[name + "_cum_cycles_mean"] = float(cols[name].mean())
        pw = cols["probing_lanes"] > 0
        rep["probe_and_bracket_cycles_probing_waves"] = float(cols["probe_and_bracket"][pw].mean()) if pw.any() else 0.0
        rep["probe_and_bracket_cycles_other_waves"] = float(cols["probe_and_bracket"][~pw].mean()) if (~pw).any() else 0.0
        print(json.dumps(rep, indent=1))
        return
    if "--loop" in sys.argv:
        a = np.fromfile(path, dtype=np.int32).reshape(-1, 7).astype(np.int64)[:n]
        # a wave: the (scalar) entry stamp and search total; its longest-running lane saw every
        # trip, so the wave's eval / next_point time is the maximum over its lanes, and the mean
        # over its lanes is the time a lane spends in them (the rest: waiting for other lanes)
        key = np.stack([np.arange(len(a)) // BLOCK, a[:, 0], a[:, 1]], axis=1)
        _, inv = np.unique(key, axis=0, return_inverse=True)
        inv = inv.ravel()
        nw = inv.max() + 1
        tot = np.zeros(nw)
        ev_max = np.zeros(nw)
        nx_max = np.zeros(nw)
        up_max = np.zeros(nw)
        pre_max = np.zeros(nw)
        beg_max = np.zeros(nw)
        np.maximum.at(beg_max, inv, a[:, 6])
        np.maximum.at(tot, inv, a[:, 1])
        np.maximum.at(ev_max, inv, a[:, 2])
        np.maximum.at(nx_max, inv, a[:, 3])
        np.maximum.at(up_max, inv, a[:, 4])
        np.maximum.at(pre_max, inv, a[:, 5])
        T = tot.sum()
        rep = {"waves": int(nw), "search_cycles_mean": float(tot.mean()),
               "share_eval_wave": float(ev_max.sum() / T),
               "share_next_point_wave": float(nx_max.sum() / T),
               "share_update_wave": float(up_max.sum() / T),
               "share_before_loop_wave": float(pre_max.sum() / T),
               "share_begin_wave": float(beg_max.sum() / T),
               "share_rest_wave": float(1 - (ev_max.sum() + nx_max.sum() + up_max.sum() +
                                             pre_max.sum()) / T),
               "lane_active_eval_share": float(a[:, 2].sum() / (nw and a[:, 1].sum())),
               "lane_eval_over_wave_eval": float(a[:, 2].mean() / (ev_max[inv].mean()))}
        print(json.dumps(rep, indent=1))
        with open(os.path.join(ROOT, "gpurun_out", "roots_stamps_loop.json"), "w") as f:
            json.dump(rep, f, indent=1)
        return
    a = np.fromfile(path, dtype=np.int32).reshape(-1, 4).astype(np.int64)[:n]
    blk = np.arange(len(a)) // BLOCK
    t0 = a[:, 0] & 0xFFFFFFFF
    # one row per wave: the 64 lanes of a wave share all four (scalar) stamps
    key = np.stack([blk, t0, a[:, 1], a[:, 2], a[:, 3]], axis=1)
    w = np.unique(key, axis=0)
    wb, w0, s1, s2, s3 = w[:, 0], w[:, 1], w[:, 2], w[:, 3], w[:, 4]
    sort_c, gather_c, solve_c = s1, s2 - s1, s3 - s2
    life = s3
    # per block: entry of its first wave, end of its last (32-bit wrap within a block)
    order = np.argsort(wb, kind="stable")
    wb, w0, life = wb[order], w0[order], life[order]
    starts = np.r_[0, np.flatnonzero(np.diff(wb)) + 1]
    ends = np.r_[starts[1:], len(wb)]
    idle = span_sum = 0
    waves_per_block = []
    for s, e in zip(starts, ends):
        rel = (w0[s:e] - w0[s]) % (1 << 32)
        rel = np.where(rel >= (1 << 31), rel - (1 << 32), rel)
        b0 = rel.min()
        fin = rel + life[s:e]
        span = fin.max() - b0
        idle += (fin.max() - fin).sum()
        span_sum += span * (e - s)
        waves_per_block.append(e - s)
    tot = life.sum()
    rep = {
        "waves": int(len(w)),
        "waves_per_block_mean": float(np.mean(waves_per_block)),
        "wave_cycles_mean": float(life.mean()),
        "share_sort": float(sort_c.sum() / tot),
        "share_gather": float(gather_c.sum() / tot),
        "share_solve": float(solve_c.sum() / tot),
        "block_slot_idle_share": float(idle / span_sum),
        "sort_cycles_mean": float(sort_c.mean()),
        "gather_cycles_mean": float(gather_c.mean()),
        "solve_cycles_mean": float(solve_c.mean()),
        "solve_cycles_p50_p90_max": [float(np.percentile(solve_c, 50)),
                                     float(np.percentile(solve_c, 90)), float(solve_c.max())],
    }
    print(json.dumps(rep, indent=1))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "roots_stamps.json"), "w") as f:
        json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
