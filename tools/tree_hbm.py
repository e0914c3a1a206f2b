"""HBM traffic of the MCTS tree kernels from rocprofv3 PMC passes (separate
FETCH_SIZE and WRITE_SIZE runs) and their durations from a kernel-trace run:
bytes per launch = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE
correction, MI355X_MICROARCH.md), achieved GB/s = bytes / average duration.
Narrow (4-16 B per lane) accesses are not calibrated by the guide; treat the
absolute figure as an estimate.

    python tools/tree_hbm.py FETCH_CSV_GLOB WRITE_CSV_GLOB TRACE_DB SLOTS [SIMS_PER_MOVE [NOTE]] > profiles/rNN_pmc_tree.json
"""
import csv
import glob
import json
import sqlite3
import sys
from collections import defaultdict

KERNELS = ("k_mcts_backup_select", "k_mcts_select", "k_mcts_backup", "k_mcts_root", "k_mcts_choose", "k_movegen")
PEAK_GBPS = 8000.0


def pmc(pattern, counter):
    v = defaultdict(list)
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            for k in KERNELS:
                if "kv::" + k + "(" in r["Kernel_Name"]:
                    v[k].append(float(r["Counter_Value"]))
    return {k: sum(x) / len(x) for k, x in v.items()}


def durations(db):
    c = sqlite3.connect(db)
    out = {}
    for name, avg, n in c.execute("select name, avg(duration), count(*) from kernels group by name"):
        for k in KERNELS:
            if "kv::" + k + "(" in name:
                out[k] = (avg, n)
    return out


def main():
    fetch, write, dur = pmc(sys.argv[1], "FETCH_SIZE"), pmc(sys.argv[2], "WRITE_SIZE"), durations(sys.argv[3])
    slots = int(sys.argv[4])
    res = {"slots": slots, "peak_GBps": PEAK_GBPS, "kernels": {}}
    if len(sys.argv) > 5:
        res["sims_per_move"] = int(sys.argv[5])
    if len(sys.argv) > 6:
        res["note"] = sys.argv[6]
    for k in KERNELS:
        if k in fetch and k in write and k in dur:
            b = (2 * fetch[k] + write[k]) * 1024
            ns = dur[k][0]
            res["kernels"][k] = {"bytes_per_launch": b, "bytes_per_slot": b / slots, "avg_ns": ns,
                                 "GBps": b / ns, "frac": b / ns / PEAK_GBPS}
    fused = res["kernels"].get("k_mcts_backup_select")
    sel, bak = res["kernels"].get("k_mcts_select"), res["kernels"].get("k_mcts_backup")
    if fused:  # backup of sim-step k + select of k+1, one launch per sim-step
        res["per_sim"] = {"bytes_per_sim": fused["bytes_per_launch"] / slots, "GBps": fused["GBps"],
                          "frac": fused["frac"], "note": "k_mcts_backup_select, one backup + one select per slot per launch"}
    elif sel and bak:
        b = sel["bytes_per_launch"] + bak["bytes_per_launch"]
        ns = sel["avg_ns"] + bak["avg_ns"]
        res["per_sim"] = {"bytes_per_sim": b / slots, "GBps": b / ns, "frac": b / ns / PEAK_GBPS,
                          "note": "select + backup, one backup per slot per launch"}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
