"""Static instruction histogram / listing of one kernel in a hipcc -S device assembly file.

    python scripts/isa_kernel.py <file.s> <symbol-substring> [--list]
"""
import sys
from collections import Counter


def main():
    path, pat = sys.argv[1], sys.argv[2]
    s = open(path).read()
    start = [ln.split(":")[0] + ":" for ln in s.split("\n") if ln.startswith("_Z") and ":" in ln and pat in ln.split(":")[0]]
    if not start:
        raise SystemExit("no such kernel")
    name = start[0][:-1]
    i = s.index(name + ":")
    j = s.index(".Lfunc_end", i)
    body = s[i:j].split("\n")
    if "--list" in sys.argv:
        print("\n".join(body))
        return
    c = Counter()
    for ln in body:
        t = ln.strip().split(" ")[0]
        if t and not t.startswith((".", ";", "_")) and not t.endswith(":"):
            c[t] += 1
    valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
    print(name)
    print("lines", len(body), "VALU (static, non-MFMA)", valu, "MFMA", sum(v for k, v in c.items() if k.startswith("v_mfma")))
    for k, v in c.most_common(70):
        print(f"{v:6d} {k}")


if __name__ == "__main__":
    main()
