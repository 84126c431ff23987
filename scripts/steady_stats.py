"""Steady-state launch statistics of one kernel from a rocprofv3 kernel trace (warm-ups excluded).

    python scripts/steady_stats.py <run_kernel_trace.csv> <kernel substring> <warmup launches> [out.json]

Reports count / mean / median / min / max (ms) over the launches after the first `warmup`, which
is what bench.py's timed region sees; rocprofv3 --stats averages include the warm-ups."""
import csv
import json
import statistics
import sys

path, pat, warm = sys.argv[1], sys.argv[2], int(sys.argv[3])
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in csv.DictReader(open(path))
        if pat in r["Kernel_Name"]]
steady = durs[warm:]
out = {"trace": path, "kernel_match": pat, "launches_total": len(durs), "warmup_excluded": warm,
       "steady_launches": len(steady), "mean_ms": statistics.mean(steady), "median_ms": statistics.median(steady),
       "min_ms": min(steady), "max_ms": max(steady), "first_launches_ms": durs[:warm]}
print(json.dumps(out, indent=1))
if len(sys.argv) > 4:
    open(sys.argv[4], "w").write(json.dumps(out, indent=1) + "\n")
