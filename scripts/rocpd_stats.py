"""Kernel statistics (name, calls, total / average / min ns) from a rocprofv3 rocpd SQLite database,
written as the --stats kernel_stats.csv columns: python scripts/rocpd_stats.py run_results.db [out.csv]."""
import csv
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
rows = con.execute(f"select {name_col}, count(*), sum(end - start), avg(end - start), min(end - start), "
                   f"max(end - start) from kernels group by {name_col} order by sum(end - start) desc").fetchall()
tot = sum(r[2] for r in rows)
out = [dict(Name=r[0], Calls=r[1], TotalDurationNs=r[2], AverageNs=r[3], Percentage=100.0 * r[2] / tot, MinNs=r[4],
            MaxNs=r[5]) for r in rows]
if len(sys.argv) > 2:
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
        w.writeheader()
        w.writerows(out)
for x in out[:18]:
    print(f'{x["Percentage"]:5.1f}% calls={x["Calls"]:>6} avg={x["AverageNs"] / 1e3:8.1f}us {x["Name"][:100]}')
print("total ms", tot / 1e6)
