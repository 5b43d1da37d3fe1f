"""Per-kernel summary of a rocprofv3 run (its SQLite output, the default
format) in the layout of rocprofv3's own kernel_stats.csv:

    python scripts/rocpd_stats.py gpurun_out/<dir>/run_results.db > profiles/<name>_kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys


def main(path):
    con = sqlite3.connect(path)
    per = {}
    for name, dur in con.execute("select name, duration from kernels"):
        per.setdefault(name, []).append(int(dur))
    total = sum(sum(v) for v in per.values()) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC, lineterminator="\n")
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        s = sum(v)
        w.writerow([name, len(v), s, round(s / len(v), 6), round(100.0 * s / total, 2), min(v), max(v),
                    round(statistics.pstdev(v), 6) if len(v) > 1 else 0.0])


if __name__ == "__main__":
    main(sys.argv[1])
