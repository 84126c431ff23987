"""Per-kernel register / scratch / LDS usage of the built library's gfx950 code objects (from the
code-object metadata notes), filtered by a name substring:

    python scripts/kernel_resources.py [substring] [naz_amd/lib/libnazhip.so]
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tests.isa_ring import LLVM, code_objects  # noqa: E402


def main():
    pat = sys.argv[1] if len(sys.argv) > 1 else ""
    lib = Path(sys.argv[2]) if len(sys.argv) > 2 else Path(__file__).resolve().parents[1] / "naz_amd/lib/libnazhip.so"
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", f.name], capture_output=True,
                                   text=True).stdout
        for blk in re.split(r"\n  - \.agpr_count:", notes)[1:]:
            name = re.search(r"\n    \.name:\s+(\S+)", blk)
            dem = subprocess.run(["c++filt"], input=name.group(1), capture_output=True,
                                 text=True).stdout.strip() if name else "?"
            if pat not in dem:
                continue
            get = lambda k: (re.search(rf"\n    \.{k}:\s+(\S+)", blk) or [None, "?"])[1]  # noqa: E731
            agpr = blk.split("\n", 1)[0].strip(": ")
            print(f"vgpr={get('vgpr_count'):>4} agpr={agpr:>4} sgpr={get('sgpr_count'):>3} "
                  f"spill_v={get('vgpr_spill_count'):>3} scratch={get('private_segment_fixed_size'):>5} "
                  f"lds={get('group_segment_fixed_size'):>6}  {dem[:150]}")


if __name__ == "__main__":
    main()
