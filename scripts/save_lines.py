"""Copy the bench JSON line of each step log of a gpu_steps.sh session into profiles/.

    python scripts/save_lines.py gpurun_out/<TAG> <prefix> step [step ...]

writes profiles/<prefix>_<step>.json (the last JSON line of gpurun_out/<TAG>/<step>.log).
"""
import json
import sys
from pathlib import Path


def main():
    src, prefix, steps = Path(sys.argv[1]), sys.argv[2], sys.argv[3:]
    for st in steps:
        lines = [ln for ln in (src / f"{st}.log").read_text().splitlines() if ln.startswith("{")]
        if not lines:
            print(f"{st}: no bench line")
            continue
        d = json.loads(lines[-1])
        out = Path("profiles") / f"{prefix}_{st}.json"
        out.write_text(json.dumps(d, indent=1) + "\n")
        print(f"{out}: {d.get('ms_per_step'):.4f} ms, {d.get('value'):.4g} {d.get('unit')}")


if __name__ == "__main__":
    main()
