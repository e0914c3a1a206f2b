"""Per-kernel summary (calls, total/avg/min/max ns, share) from a rocprofv3
rocpd SQLite database, in the column layout of rocprofv3's kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/prof/x_results.db [out.csv]
"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [(n, k, s, a, lo, hi, 100.0 * s / tot) for n, k, s, a, lo, hi in rows]


def main():
    rows = stats(sys.argv[1])
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"]
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(hdr)
            w.writerows(rows)
    for n, k, s, a, lo, hi, p in rows[:20]:
        print(f"{p:6.2f}% {k:6d} avg {a / 1e3:9.2f} us  {n[:110]}")


if __name__ == "__main__":
    main()
