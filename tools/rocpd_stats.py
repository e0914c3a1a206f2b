"""Kernel statistics (calls, average / total duration) from a rocprofv3 rocpd SQLite database (the
--kernel-trace output when no csv format is asked for): the same columns as --stats' kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/x/prof/run_results.db [out.csv]
"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    names = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    kd = next(n for n in names if n.startswith("rocpd_kernel_dispatch"))
    ks = next(n for n in names if n.startswith("rocpd_info_kernel_symbol"))
    rows = c.execute(f"select s.kernel_name, count(*), avg(d.end - d.start), sum(d.end - d.start) from {kd} d "
                     f"join {ks} s on d.kernel_id = s.id group by s.kernel_name order by 4 desc").fetchall()
    tot = sum(r[3] for r in rows)
    return [(n, k, a, s, 100.0 * s / tot) for n, k, a, s in rows]


if __name__ == "__main__":
    out = stats(sys.argv[1])
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "AverageNs", "TotalDurationNs", "Percentage"])
            w.writerows(out)
    for n, k, a, s, p in out:
        print(f"{n[:100]:100s} {k:6d} {a / 1e3:9.1f} us {p:6.2f} %")
