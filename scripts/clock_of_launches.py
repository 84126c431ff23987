"""Sustained clock of the headline kernel from a rocprofv3 GRBM_GUI_ACTIVE pass (round 6):
GRBM_GUI_ACTIVE summed over the 8 XCDs / 8 = GPU-busy cycles of one launch, over that launch's own
duration (End_Timestamp - Start_Timestamp, ns).

    python scripts/clock_of_launches.py gpurun_out/<tag>/pmc_clk/run_counter_collection.csv
"""
import csv
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))
        if "coupling_r16_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
mhz, dur = [], []
for r in rows:
    ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    mhz.append(float(r["Counter_Value"]) / 8 / ns * 1e3)
    dur.append(ns / 1e6)
print({"launches": len(rows), "clock_MHz_median": round(statistics.median(mhz), 1),
       "clock_MHz_min": round(min(mhz), 1), "clock_MHz_max": round(max(mhz), 1),
       "launch_ms_median": round(statistics.median(dur), 4)})
