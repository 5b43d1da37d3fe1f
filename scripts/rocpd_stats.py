"""Per-kernel stats (calls, average / total duration, share) from a rocprofv3
sqlite result (rocpd `kernels` view), printed as CSV like --stats' kernel_stats.
usage: python scripts/rocpd_stats.py <results.db> [name-filter]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, count(*), avg(duration), sum(duration), min(duration), max(duration) "
                 "from kernels group by name order by sum(duration) desc").fetchall()
tot = sum(r[3] for r in rows)
flt = sys.argv[2] if len(sys.argv) > 2 else ""
print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
for n, k, a, s, lo, hi in rows:
    if flt in n:
        print(f'"{n}",{k},{s},{a:.1f},{100.0 * s / tot:.3f},{lo},{hi}')
