"""Summarise a rocprofv3 --kernel-trace SQLite output (per kernel: calls, avg/total time)."""
import glob
import sqlite3
import sys

db = glob.glob(f'{sys.argv[1]}/**/*.db', recursive=True)[0]
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), avg(end-start)/1000.0, sum(end-start)/1e6 from kernels "
                 "group by name order by 4 desc limit 20").fetchall()
print(f"{'kernel':80s} {'calls':>6s} {'avg_us':>10s} {'total_ms':>9s}")
for r in rows:
    print(f"{r[0][:80]:80s} {r[1]:6d} {r[2]:10.1f} {r[3]:9.2f}")
