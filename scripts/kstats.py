"""Summarise a rocprofv3 kernel_stats.csv: share, calls, average per kernel."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(x["TotalDurationNs"]) for x in rows)
for x in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 16]:
    print(f'{float(x["TotalDurationNs"]) / tot * 100:5.1f}% calls={x["Calls"]:>6} '
          f'avg={float(x["AverageNs"]) / 1e3:8.1f}us {x["Name"][:110]}')
print("total ms", tot / 1e6)
