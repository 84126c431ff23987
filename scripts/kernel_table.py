"""Per-(kernel, grid) duration table from a rocprofv3 kernel-trace CSV.
    python scripts/kernel_table.py <run_kernel_trace.csv> [steps]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    agg = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"]
        n = n.replace("(anonymous namespace)::", "")
        head = n.split("(")[0] if not n.startswith("void") else n[5:].split("(")[0]
        agg[(head[-60:], r["Grid_Size_X"], r["Grid_Size_Y"])].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in agg.values())
    print(f"total {tot / 1e3:.2f} ms over {steps} step(s): {tot / 1e3 / steps:.2f} ms/step")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:25]:
        print(f"{sum(v) / 1e3 / steps:8.3f} ms/step  {len(v) / steps:5.1f} calls  avg {sum(v) / len(v):8.1f} us  {k}")


if __name__ == "__main__":
    main()
