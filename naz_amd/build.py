"""Build libnazhip.so in-tree (hipcc --offload-arch=gfx950), used by __graft_entry__.build().

Objects go to naz_amd/build/, the shared library to naz_amd/lib/libnazhip.so.  Each
translation unit is rebuilt only when it or a header is newer than its object.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OBJ = PKG / "build"
LIB = PKG / "lib" / "libnazhip.so"
INCLUDE = PKG.parent / "include"
ARCH = os.environ.get("NAZ_OFFLOAD_ARCH", "gfx950")
SOURCES = ["rqs.hip", "dense.hip", "gemm.hip", "elementwise.hip", "coupling.hip", "cnf.hip", "capi.cpp"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the naz_amd HIP library cannot be built")


def _headers_mtime() -> float:
    hs = list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path, obj: Path, extra: list) -> str:
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function",
           f"-I{INCLUDE}", "-c", str(src), "-o", str(obj)] + extra
    if src.suffix == ".cpp":
        cmd[1:2] = []  # host-only TU
        cmd += ["-x", "c++"] if False else []
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r.stderr


def build(verbose: bool = False, jobs: int = 4, extra: list | None = None) -> Path:
    extra = list(extra or [])
    OBJ.mkdir(exist_ok=True)
    LIB.parent.mkdir(exist_ok=True)
    hm = _headers_mtime()
    todo = []
    objs = []
    for s in SOURCES:
        src = CSRC / s
        obj = OBJ / (src.stem + ".o")
        objs.append(obj)
        if not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hm):
            todo.append((src, obj))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for (src, obj), warn in zip(todo, ex.map(lambda t: _compile(t[0], t[1], extra), todo)):
            if verbose:
                print(f"[naz_amd.build] {src.name} -> {obj.name}", file=sys.stderr)
                if warn.strip():
                    print(warn, file=sys.stderr)
    if todo or not LIB.exists() or LIB.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB)] + [str(o) for o in objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(verbose=True))
