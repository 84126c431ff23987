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
import time
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OBJ = PKG / "build"
LIB = PKG / "lib" / "libnazhip.so"
INCLUDE = PKG.parent / "include"
ARCH = os.environ.get("NAZ_OFFLOAD_ARCH", "gfx950")
# Per-source flags.  The MFMA kernels are built without the SLP vectorizer: the packed f32 VALU
# ops it forms (v_pk_add/mul/fma_f32) issue slower than scalar ones beside MFMAs, and the
# packing moves add register pressure (spills in coupling_x6_kernel with it on).
SOURCE_FLAGS = {"coupling.hip": ["-fno-slp-vectorize"], "cnf.hip": ["-fno-slp-vectorize"],
                "made.hip": ["-fno-slp-vectorize"]}
SOURCES = ["rqs.hip", "dense.hip", "gemm.hip", "gemm_rows.hip", "elementwise.hip", "made.hip", "coupling.hip", "cnf.hip", "capi.cpp"]
# sources compiled more than once with a part macro (object name suffix, extra flags): coupling.hip
# holds the coupling, the autoregressive and the autoregressive-backward kernels, ~5 min of device
# compile in one object
PARTS = {"coupling.hip": [("", ["-DNAZ_PART=1"]), ("_ar", ["-DNAZ_PART=2"]), ("_arb", ["-DNAZ_PART=3"])]}


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
           f"-I{INCLUDE}", "-c", str(src), "-o", str(obj)] + SOURCE_FLAGS.get(src.name, []) + extra
    if src.suffix == ".cpp":
        cmd[1:2] = []  # host-only TU
        cmd += ["-x", "c++"] if False else []
    started = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    # date the object at the compile's START: hipcc reads the sources once for the device pass and
    # again, minutes later, for the host pass, so a header edited meanwhile must make the object
    # stale (a device image from the old header and a host packer from the new one disagree)
    os.utime(obj, (started, started))
    return r.stderr


def build(verbose: bool = False, jobs: int = 4, extra: list | None = None, variant: str | None = None) -> Path:
    """Build the library.  `variant` (with `extra` flags, e.g. ablation -D's) builds
    naz_amd/lib/libnazhip_<variant>.so from objects in naz_amd/build/<variant>/ instead."""
    extra = list(extra or [])
    obj_dir = OBJ / variant if variant else OBJ
    lib_path = LIB.with_name(f"libnazhip_{variant}.so") if variant else LIB
    obj_dir.mkdir(parents=True, exist_ok=True)
    lib_path.parent.mkdir(exist_ok=True)
    hm = _headers_mtime()
    todo = []
    objs = []
    for s in SOURCES:
        src = CSRC / s
        for suffix, flags in PARTS.get(s, [("", [])]):
            obj = obj_dir / (src.stem + suffix + ".o")
            objs.append(obj)
            if not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hm):
                todo.append((src, obj, flags))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for (src, obj, _), warn in zip(todo, ex.map(lambda t: _compile(t[0], t[1], extra + t[2]), todo)):
            if verbose:
                print(f"[naz_amd.build] {src.name} -> {obj.name}", file=sys.stderr)
                if warn.strip():
                    print(warn, file=sys.stderr)
    if todo or not lib_path.exists() or lib_path.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib_path)] + [str(o) for o in objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return lib_path


DEBUG_LIB = LIB.with_name("libnazhip_debug.so")


def build_debug(verbose: bool = False) -> Path:
    """naz_amd/lib/libnazhip_debug.so: the library with the fused coupling kernels built with
    -DNAZ_DEBUG_NONFINITE (the first non-finite row state recorded as (workgroup, layer, stage,
    row), naz_debug_nonfinite).  Only coupling.hip's part 1 reads the flag, so the other objects
    are the default build's (built first if needed)."""
    build(verbose=verbose)
    obj_dir = OBJ / "debug"
    obj_dir.mkdir(parents=True, exist_ok=True)
    src = CSRC / "coupling.hip"
    dobj = obj_dir / "coupling.o"
    if not dobj.exists() or dobj.stat().st_mtime < max(src.stat().st_mtime, _headers_mtime()):
        _compile(src, dobj, ["-DNAZ_DEBUG_NONFINITE", "-DNAZ_PART=1"])
        if verbose:
            print(f"[naz_amd.build] coupling.hip -> debug/{dobj.name}", file=sys.stderr)
    objs = [dobj if o.name == "coupling.o" else o for o in _objects(OBJ)]
    if not DEBUG_LIB.exists() or DEBUG_LIB.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(DEBUG_LIB)] + [str(o) for o in objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return DEBUG_LIB


def _objects(obj_dir: Path) -> list:
    return [obj_dir / (CSRC.joinpath(s).stem + suffix + ".o") for s in SOURCES for suffix, _ in PARTS.get(s, [("", [])])]


if __name__ == "__main__":
    # python -m naz_amd.build [variant -DFLAG ... | debug]
    if sys.argv[1:] == ["debug"]:
        print(build_debug(verbose=True))
    elif len(sys.argv) > 1:
        print(build(verbose=True, variant=sys.argv[1], extra=sys.argv[2:]))
    else:
        print(build(verbose=True))
