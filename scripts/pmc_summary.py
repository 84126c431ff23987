"""Summarise rocprofv3 PMC passes (scripts/pmc.sh output) for the fused coupling kernel.

    python scripts/pmc_summary.py gpurun_out/pmc_<TAG> profiles/pmc_<TAG>.json [--traffic]

Per-launch average of every counter for the kernel matching --kernel (default: the fused
coupling kernel), plus derived quantities.  HBM bytes follow MI355X_MICROARCH.md §HBM:
FETCH_SIZE (KB) is doubled for gfx950's wide streaming reads, WRITE_SIZE (KB) taken as is.
--traffic also writes profiles/traffic_config3.json, which bench.py reports as roofline.traffic.
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    pat = "coupling_x6_kernel"
    for a in sys.argv[3:]:
        if a.startswith("--kernel="):
            pat = a.split("=", 1)[1]
    vals = defaultdict(list)
    meta = {}
    for f in sorted(glob.glob(str(src / "p*" / "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta = {k: r[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                          "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Scratch_Size")}
    per = {k: sum(v) / len(v) for k, v in vals.items()}
    out = {"kernel": meta, "per_launch": per, "launches_per_counter": {k: len(v) for k, v in vals.items()}}
    d = {}
    if "FETCH_SIZE" in per:
        d["fetch_bytes_raw"] = per["FETCH_SIZE"] * 1024
        d["fetch_bytes_corrected"] = per["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in per:
        d["write_bytes"] = per["WRITE_SIZE"] * 1024
    if "fetch_bytes_corrected" in d and "write_bytes" in d:
        d["hbm_bytes_per_launch"] = d["fetch_bytes_corrected"] + d["write_bytes"]
    if "SQ_WAVES" in per and "SQ_INSTS_VALU" in per:
        d["valu_per_wave"] = per["SQ_INSTS_VALU"] / per["SQ_WAVES"]
    if "SQ_WAVES" in per and "SQ_INSTS_MFMA" in per:
        d["mfma_per_wave"] = per["SQ_INSTS_MFMA"] / per["SQ_WAVES"]
    if "GRBM_GUI_ACTIVE" in per:
        d["gpu_cycles_per_xcd"] = per["GRBM_GUI_ACTIVE"] / 8
    out["derived"] = d
    dst.parent.mkdir(parents=True, exist_ok=True)
    dst.write_text(json.dumps(out, indent=1))
    print(json.dumps(out["derived"], indent=1))
    if "--traffic" in sys.argv and "hbm_bytes_per_launch" in d:
        t = {"kernel": meta.get("Kernel_Name"), "hbm_bytes_per_launch": d["hbm_bytes_per_launch"],
             "fetch_bytes_corrected": d["fetch_bytes_corrected"], "write_bytes": d["write_bytes"],
             "rows_per_launch": 1 << 20, "algorithmic_bytes_per_launch": 196 * (1 << 20),
             "source": str(dst), "correction": "FETCH_SIZE x2 (gfx950 wide-read counting, MI355X_MICROARCH.md §HBM)"}
        mode = "f32"
        for a in sys.argv[3:]:
            if a.startswith("--mode="):
                mode = a.split("=", 1)[1]
        Path(f"profiles/traffic_config3_{mode}.json").write_text(json.dumps(t, indent=1))


if __name__ == "__main__":
    main()
