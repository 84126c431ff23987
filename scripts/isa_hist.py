"""Instruction histogram of a kernel's longest loop (the layer loop) in a built library.
    python scripts/isa_hist.py [lib] [kernel-substring]"""
import re
import sys
from collections import Counter
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tests.isa_ring import code_objects, disassemble, functions  # noqa: E402

lib = sys.argv[1] if len(sys.argv) > 1 else "naz_amd/lib/libnazhip.so"
pat = sys.argv[2] if len(sys.argv) > 2 else "coupling_r16_kernelINS_6CfgR16ILi16ELi32ELi8ELi8ELi128ELb1EEELb1ELi0EE"
for co in code_objects(Path(lib)):
    for name, (start, ins) in functions(disassemble(co)).items():
        if pat not in name:
            continue
        edges = []
        for a, t in ins:
            if t.startswith("s_branch") or t.startswith("s_cbranch"):
                m = re.search(r"\+0x([0-9a-f]+)>", t)
                if m and start + int(m.group(1), 16) < a:
                    edges.append((a - (start + int(m.group(1), 16)), start + int(m.group(1), 16), a))
        lo, hi = (max(edges)[1], max(edges)[2]) if edges else (start, ins[-1][0])
        body = [t for a, t in ins if lo <= a <= hi]
        c = Counter(t.split()[0] for t in body)
        cats = Counter()
        for op, n in c.items():
            k = ("mfma" if op.startswith("v_mfma") else "valu" if op.startswith("v_") else "lds" if op.startswith("ds_")
                 else "nop" if op == "s_nop" else "salu" if op.startswith("s_") else "vmem")
            cats[k] += n
        print(name[:90], "loop insns", len(body), dict(cats))
        for op, n in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 25):
            print(f"{n:6d} {op}")
