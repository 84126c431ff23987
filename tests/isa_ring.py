"""Static check of the LDS-DMA ring protocol in the built gfx950 code objects (test helper).

A `global_load_lds` (or `buffer_load ... lds`) write is pending on the issuing wave's vmcnt
until it lands in LDS.  Every kernel that streams weights through an LDS ring publishes a slot
with a workgroup barrier, so every `s_barrier` that a wave can reach with such a DMA in flight
must be preceded by `s_waitcnt vmcnt(0)` on EVERY path — loop back edges included.  Round 2's
headline kernel broke this on the layer loop's back edge (an intermittent NaN at 2^20 rows).

The check: pull each gfx950 code object out of the library's `.hip_fatbin` (offload bundles),
disassemble with llvm-objdump, build a per-kernel control-flow graph from the branch targets,
and run a forward may-analysis of "a DMA may be in flight" to a fixed point.
"""
from __future__ import annotations

import re
import struct
import subprocess
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

_FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")
_ADDR = re.compile(r"//\s*([0-9A-F]+):")
_TARGET = re.compile(r"<([^<>+]+)(?:\+0x([0-9a-f]+))?>\s*$")


def code_objects(lib: Path, arch: str = "gfx950") -> list[bytes]:
    """The `arch` device code objects of every offload bundle in `lib`'s .hip_fatbin."""
    with tempfile.TemporaryDirectory() as td:
        fb = Path(td) / "fb.bin"
        subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", str(lib),
                        str(Path(td) / "junk")], check=True, capture_output=True)
        b = fb.read_bytes()
    out = []
    i = b.find(MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", b, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", b, p)
            p += 24
            triple = b[p:p + tl].decode()
            p += tl
            if triple.endswith(arch) and size:
                out.append(b[i + off:i + off + size])
        i = b.find(MAGIC, i + 1)
    return out


def disassemble(co: bytes) -> str:
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        r = subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", f.name],
                           check=True, capture_output=True, text=True)
    return r.stdout


def functions(asm: str) -> dict[str, tuple[int, list[tuple[int, str]]]]:
    """symbol -> (start address, [(address, instruction text)])."""
    funcs: dict[str, tuple[int, list]] = {}
    cur = None
    for line in asm.splitlines():
        m = _FUNC.match(line.strip())
        if m:
            cur = m.group(2)
            funcs[cur] = (int(m.group(1), 16), [])
            continue
        if cur is None or not line.startswith("\t"):
            continue
        a = _ADDR.search(line)
        if a:
            funcs[cur][1].append((int(a.group(1), 16), line.strip()))
    return funcs


def is_dma(ins: str) -> bool:
    op = ins.split(None, 1)[0]
    return op.startswith("global_load_lds") or (op.startswith("buffer_load") and " lds" in ins.split("//")[0])


def _successors(start: int, insns: list[tuple[int, str]]) -> list[list[int]]:
    index = {a: k for k, (a, _) in enumerate(insns)}
    succ: list[list[int]] = []
    for k, (a, t) in enumerate(insns):
        op = t.split(None, 1)[0]
        nxt = [k + 1] if k + 1 < len(insns) else []
        if op in ("s_endpgm", "s_endpgm_saved", "s_setpc_b64", "s_trap"):
            succ.append([])
            continue
        if op.startswith("s_branch") or op.startswith("s_cbranch"):
            m = _TARGET.search(t)
            tgt = []
            if m:
                ta = start + int(m.group(2) or "0", 16)
                if ta in index:
                    tgt = [index[ta]]
            if not tgt:
                raise AssertionError(f"unresolved branch target: {t}")
            succ.append(tgt if op.startswith("s_branch") else tgt + nxt)
            continue
        succ.append(nxt)
    return succ


def _flagged(start: int, insns: list[tuple[int, str]], sets, clears, flags) -> list[str]:
    """Instructions `flags(text)` reachable with the state set (`sets`) and not cleared (`clears`)
    on some path through the control-flow graph (loop back edges included)."""
    succ = _successors(start, insns)
    pending_in = [None] * len(insns)
    work = [(0, False)]
    bad: dict[int, str] = {}
    while work:
        k, st = work.pop()
        if pending_in[k] is not None and (pending_in[k] or not st):
            continue  # nothing new (the state only grows False -> True)
        pending_in[k] = bool(pending_in[k]) or st
        st = pending_in[k]
        a, t = insns[k]
        if st and flags(t):
            bad[a] = t
        if clears(t):
            st = False
        elif sets(t):
            st = True
        for s in succ[k]:
            work.append((s, st))
    return [f"+0x{a - start:x}: {t.split('//')[0].strip()}" for a, t in sorted(bad.items())]


def ring_violations(start: int, insns: list[tuple[int, str]]) -> list[str]:
    """Barriers reachable with an LDS-DMA in flight and no vmcnt(0) on some path."""
    if not any(is_dma(t) for _, t in insns):
        return []
    return _flagged(start, insns, sets=is_dma,
                    clears=lambda t: t.startswith("s_waitcnt") and "vmcnt(0)" in t,
                    flags=lambda t: t.split(None, 1)[0] == "s_barrier")


_LGKM = re.compile(r"lgkmcnt\((\d+)\)")


def _is_smem(t: str) -> bool:
    op = t.split(None, 1)[0]
    return op.startswith(("s_load", "s_buffer_load", "s_scratch_load", "s_dcache", "s_memtime", "s_memrealtime"))


def counted_lgkm_violations(start: int, insns: list[tuple[int, str]]) -> list[str]:
    """Counted LDS waits (s_waitcnt lgkmcnt(N), N > 0) reachable with a scalar-memory load in flight
    since the last lgkmcnt(0): LGKM also counts SMEM, which returns out of order, so such a count
    no longer proves the older LDS reads landed (the hand-counted waits of coupling_w32.h's
    untracked A-fragment reads rely on this never happening)."""
    def counted(t):
        m = _LGKM.search(t.split("//")[0])
        return t.startswith("s_waitcnt") and m is not None and int(m.group(1)) > 0
    return _flagged(start, insns, sets=_is_smem,
                    clears=lambda t: t.startswith("s_waitcnt") and "lgkmcnt(0)" in t.split("//")[0],
                    flags=counted)


_REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")
_NODEST = ("ds_write", "ds_store", "global_store", "buffer_store", "flat_store", "scratch_store", "s_", "ds_add_u32",
           "ds_add_f32", "ds_max", "ds_min")


def _regs(operands: str) -> list[tuple[str, int]]:
    out = []
    for m in _REG.finditer(operands):
        kind = m.group(1)
        if m.group(4) is not None:
            out.append((kind, int(m.group(4))))
        else:
            out.extend((kind, r) for r in range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _operands(t: str) -> tuple[str, list[str]]:
    body = t.split("//")[0].strip()
    parts = body.split(None, 1)
    if len(parts) < 2:
        return parts[0] if parts else "", []
    return parts[0], [o.strip() for o in parts[1].split(",")]


def _dst_src(op: str, ops: list[str]) -> tuple[set, set]:
    """(destination, source) vector registers of one instruction (v and a registers)."""
    if not ops:
        return set(), set()
    if op.startswith(_NODEST):
        return set(), set(_regs(", ".join(ops)))
    dst, src = set(_regs(ops[0])), set(_regs(", ".join(ops[1:])))
    if "mac" in op or "fmac" in op or op.startswith(("v_dot2c", "v_pk_fmac")):
        src |= dst  # accumulates into its destination
    return dst, src


def _is_lgkm_op(op: str) -> bool:
    return op.startswith(("ds_", "s_load", "s_buffer_load", "s_scratch_load", "s_dcache", "s_memtime", "flat_",
                          "s_sendmsg"))


def pending_lds_read_uses(start: int, insns: list[tuple[int, str]], cap: int = 24) -> list[str]:
    """Instructions that read or overwrite a destination VGPR of an LDS read which an s_waitcnt
    lgkmcnt has not yet retired on some path (loop back edges included).

    The untracked A-fragment reads (naz_device.h lds_read_b128_untracked: inline asm, so the
    compiler's waitcnt pass does not see their destinations) are safe only if nothing touches those
    registers before the hand-counted lds_wait<N> that retires them: a v_mov copy or spill of a
    prefetched fragment placed before the wait would read stale data without any error.  The
    analysis tracks the LGKM queue in issue order (LDS returns in order; `s_waitcnt lgkmcnt(N)` keeps
    the newest N entries) as a may-pending set per queue position, merging paths aligned at the
    newest entry; SMEM entries are counted as queue entries without vector destinations (a counted
    wait with SMEM in flight is counted_lgkm_violations' finding)."""
    succ = _successors(start, insns)
    state_in: list = [None] * len(insns)
    work = [(0, ())]
    bad: dict[int, str] = {}

    def merge(a, b):
        if a is None:
            return b
        n = max(len(a), len(b))
        a2 = (frozenset(),) * (n - len(a)) + a
        b2 = (frozenset(),) * (n - len(b)) + b
        return tuple(x | y for x, y in zip(a2, b2))

    while work:
        k, st = work.pop()
        new = merge(state_in[k], st)
        if new == state_in[k]:
            continue
        state_in[k] = new
        st = new
        a, t = insns[k]
        op, ops = _operands(t)
        dst, src = _dst_src(op, ops)
        pend = frozenset().union(*st) if st else frozenset()
        lds_read = op.startswith(("ds_read", "ds_load", "ds_bpermute", "ds_permute", "ds_swizzle"))
        # (a later LDS read into a pending read's registers is fine: LDS returns in issue order)
        if pend and ((src | (set() if lds_read else dst)) & pend) and not op.startswith("s_waitcnt"):
            bad[a] = t
        if op.startswith("s_waitcnt"):
            m = _LGKM.search(t.split("//")[0])
            if m is not None:
                keep = int(m.group(1))
                st = st[len(st) - keep:] if keep < len(st) else st
                if keep == 0:
                    st = ()
        elif _is_lgkm_op(op):
            st = (st + (frozenset(dst) if op.startswith(("ds_read", "ds_load", "ds_bpermute", "ds_permute",
                                                         "ds_swizzle", "flat_load")) else frozenset(),))[-cap:]
        for s2 in succ[k]:
            work.append((s2, st))
    return [f"+0x{a - start:x}: {t.split('//')[0].strip()}" for a, t in sorted(bad.items())]


def check_library(lib: Path, arch: str = "gfx950") -> tuple[int, dict[str, list[str]]]:
    """(number of DMA kernels checked, {kernel: violations})."""
    checked = 0
    out: dict[str, list[str]] = {}
    for co in code_objects(lib, arch):
        for name, (start, insns) in functions(disassemble(co)).items():
            if not any(is_dma(t) for _, t in insns):
                continue
            checked += 1
            v = ring_violations(start, insns)
            if v:
                out[name] = v
    return checked, out


if __name__ == "__main__":
    import sys
    lib = Path(sys.argv[1] if len(sys.argv) > 1 else Path(__file__).resolve().parents[1] / "naz_amd/lib/libnazhip.so")
    n, bad = check_library(lib)
    print(f"{n} LDS-DMA kernels checked, {len(bad)} with unguarded barriers")
    for k, v in bad.items():
        print(k)
        for x in v[:8]:
            print("   ", x)
