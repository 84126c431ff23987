"""Whole-step HBM traffic of a multi-kernel step from scripts/pmc.sh passes (FETCH_SIZE in pass
1, WRITE_SIZE in pass 2): sum over every dispatch, FETCH_SIZE x 2 (gfx950 wide-read counting,
MI355X_MICROARCH.md §HBM) + WRITE_SIZE, divided by the number of steps the profiled command ran.

    python scripts/pmc_step_traffic.py gpurun_out/pmc_<TAG> <steps> profiles/traffic_config3_train.json [rows]

``rows`` (optional): the rows one step processed, recorded as ``rows_per_launch`` so bench.py scales
the figure to its own batch.
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def main():
    src, steps, dst = Path(sys.argv[1]), int(sys.argv[2]), Path(sys.argv[3])
    tot = defaultdict(float)
    per_kernel = defaultdict(float)
    for f in sorted(src.glob("p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            c = r["Counter_Name"]
            if c in ("FETCH_SIZE", "WRITE_SIZE"):
                b = float(r["Counter_Value"]) * 1024 * (2 if c == "FETCH_SIZE" else 1)
                tot[c] += b
                per_kernel[r["Kernel_Name"].split("(")[0][:90]] += b
    hbm = (tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) / steps
    top = sorted(per_kernel.items(), key=lambda kv: -kv[1])[:8]
    out = {"kernel": "whole NLL step (every dispatch)", "hbm_bytes_per_launch": hbm,
           "fetch_bytes_corrected": tot["FETCH_SIZE"] / steps, "write_bytes": tot["WRITE_SIZE"] / steps,
           "steps_profiled": steps, "source": str(src),
           "top_kernels_bytes_per_step": {k: v / steps for k, v in top},
           "correction": "FETCH_SIZE x2 (gfx950 wide-read counting, MI355X_MICROARCH.md §HBM)"}
    if len(sys.argv) > 4:
        out["rows_per_launch"] = int(sys.argv[4])
    dst.write_text(json.dumps(out, indent=1))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
