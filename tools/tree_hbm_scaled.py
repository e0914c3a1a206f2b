"""Tree-kernel HBM bytes per simulation at C3 (2,048 slots x 800 sims/move)
from three rocprofv3 counter runs that stay under the profiler's dispatch limit
(tools/r03_tree.sh; r03 finding: rocprofv3 --pmc dies in its host library
after ~8K dispatches of any run -- 300 sims x 1 move completes, 300 sims x 3
moves and every 800-sim move crash at the same point, whatever the filter,
collection range, edge-pool size or kernel-argument placement):

  REAL300  the real network, 300 sims/move (one move: ~7.9K dispatches)
  HASH300  the hash test evaluator (3 launches per sim-step), 300 sims/move
  HASH800  the hash test evaluator, 800 sims/move (one whole C3-length move)

Bytes per launch of k_mcts_backup_select = (2 FETCH_SIZE + WRITE_SIZE) x 1024
(gfx950 FETCH_SIZE correction, MI355X_MICROARCH.md). The hash evaluator's
trees are not the network's, so its bytes are not C3's; what it gives is how
the per-sim bytes grow from 300 to 800 sims/move, applied to the network's
measured 300-sim figure:  est800 = REAL300 x HASH800 / HASH300. The GB/s uses
the kernel's measured average duration in the real C3 run (kernel trace of an
800-sim move).

    python tools/tree_hbm_scaled.py REAL300_DIR HASH300_DIR HASH800_DIR C3_TRACE_DB > profiles/r03_pmc_tree_c3_2048.json
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tree_hbm import PEAK_GBPS, durations, pmc  # noqa: E402

K = "k_mcts_backup_select"
SLOTS = 2048


def per_sim(d):
    f = pmc(os.path.join(d, "pmc_fetch", "*.csv"), "FETCH_SIZE")[K]
    w = pmc(os.path.join(d, "pmc_write", "*.csv"), "WRITE_SIZE")[K]
    n = sum(1 for r in csv.DictReader(open(glob.glob(os.path.join(d, "pmc_fetch", "*counter_collection.csv"))[0]))
            if K in r["Kernel_Name"])
    return (2 * f + w) * 1024 / SLOTS, n


def main():
    real300, n_r = per_sim(sys.argv[1])
    hash300, n_h3 = per_sim(sys.argv[2])
    hash800, n_h8 = per_sim(sys.argv[3])
    dur = durations(sys.argv[4])[K]
    est = real300 * hash800 / hash300
    gbps = est * SLOTS / dur[0]
    res = {
        "slots": SLOTS, "sims_per_move": 800, "peak_GBps": PEAK_GBPS,
        "per_sim": {"bytes_per_sim": est, "GBps": gbps, "frac": gbps / PEAK_GBPS,
                    "note": "k_mcts_backup_select at C3 (one backup + one select per slot per launch); bytes/sim "
                            "= the network's measured 300-sim figure x the measured 300 -> 800-sim growth of the "
                            "same kernel under the hash test evaluator (rocprofv3 --pmc cannot run an 800-sim move "
                            "with the network: it dies after ~8K dispatches); GB/s with its measured average "
                            "duration in the real C3 run"},
        "measured": {
            "network_300_sims": {"bytes_per_sim": real300, "launches": n_r},
            "hash_evaluator_300_sims": {"bytes_per_sim": hash300, "launches": n_h3},
            "hash_evaluator_800_sims": {"bytes_per_sim": hash800, "launches": n_h8},
            "growth_300_to_800": hash800 / hash300,
            "c3_avg_duration_ns": dur[0], "c3_launches_traced": dur[1]},
        "profiler_limit": "rocprofv3 (ROCm 7.2) --pmc segfaults in its host library at a kernel launch after ~8K "
                          "dispatches of a run: reproduced with 800 sims (any edge-pool size, kernel arguments in "
                          "host or device memory, collection range [1-300] or [1-799]) and with 300 sims x 3 moves; "
                          "300 sims x 1 move (~7.9K dispatches) and the hash evaluator's 800-sim move (~2.6K) "
                          "complete -- profiles/r03_pmc_tree_crash_stack.log",
        "sources": [sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]],
    }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
