"""CPU test: every LDS-DMA ring kernel in the built library waits vmcnt(0) before each barrier
that a wave can reach with a global_load_lds in flight (tests/isa_ring.py)."""
from pathlib import Path

import pytest

from tests.isa_ring import (check_library, code_objects, counted_lgkm_violations, disassemble, functions, is_dma,
                            pending_lds_read_uses, ring_violations)

LIB = Path(__file__).resolve().parents[1] / "naz_amd" / "lib" / "libnazhip.so"
# the config-3 log_prob kernels (name prefixes: the parameter lists' mangling follows the signature)
HEADLINE = ("_ZN3naz19coupling_r16_kernelINS_6CfgR16ILi16ELi32ELi8ELi8ELi128ELb1EEELb1ELi0EE",
            "_ZN3naz19coupling_w32_kernelINS_5CfgX6ILi16ELi32ELi8ELi8ELi128ELb1ELi2EEELb1EE")


@pytest.fixture(scope="module")
def lib():
    if not LIB.exists():
        from naz_amd import build
        build.build()
    return LIB


def test_every_ring_barrier_waits_for_its_dma(lib):
    n, bad = check_library(lib)
    assert n >= 50, f"expected the coupling / AR / wgrad ring kernels, found {n} DMA kernels"
    assert not bad, "barriers reachable with an LDS-DMA in flight:\n" + "\n".join(
        f"{k}: {v[:4]}" for k, v in bad.items())


def test_headline_kernel_present_and_checked(lib):
    found = set()
    for co in code_objects(lib):
        fs = functions(disassemble(co))
        for name, (start, insns) in fs.items():
            pre = [p for p in HEADLINE if name.startswith(p)]
            if pre:
                assert any(is_dma(t) for _, t in insns)
                assert ring_violations(start, insns) == []
                found.add(pre[0])
    assert found == set(HEADLINE), f"config-3 log_prob kernels missing from the library: {set(HEADLINE) - found}"


def test_counted_lds_waits_have_no_scalar_load_in_flight(lib):
    """coupling_w32.h reads its A fragments with untracked LDS reads and waits lgkmcnt(2) by hand:
    valid only while no scalar-memory load (which LGKM also counts, returning out of order) is in
    flight at a counted wait.  Checked over every kernel, loop back edges included."""
    bad = {}
    for co in code_objects(lib):
        for name, (start, insns) in functions(disassemble(co)).items():
            v = counted_lgkm_violations(start, insns)
            if v:
                bad[name] = v
    assert not bad, "counted lgkmcnt waits with SMEM in flight:\n" + "\n".join(f"{k}: {v[:4]}" for k, v in bad.items())


def test_counted_wait_checker_flags_smem():
    s = 0x2000
    prog = [
        (s + 0x0, "ds_read_b128 v[0:3], v4 // 2000:"),
        (s + 0x4, "s_load_dwordx2 s[0:1], s[2:3], 0x0 // 2004:"),
        (s + 0x8, "ds_read_b128 v[4:7], v4 // 2008:"),
        (s + 0xc, "s_waitcnt lgkmcnt(1) // 200C:"),
        (s + 0x10, "s_endpgm // 2010:"),
    ]
    assert counted_lgkm_violations(s, prog) == ["+0xc: s_waitcnt lgkmcnt(1)"]
    ok = prog[:2] + [(s + 0x6, "s_waitcnt lgkmcnt(0) // 2006:")] + prog[2:]
    assert counted_lgkm_violations(s, ok) == []


def test_checker_flags_a_back_edge_without_wait():
    # synthetic: DMA issued at the loop tail, back edge to a barrier without vmcnt(0)
    s = 0x1000
    prog = [
        (s + 0x0, "s_waitcnt vmcnt(0) // 1000:"),
        (s + 0x4, "s_barrier // 1004:"),
        (s + 0x8, "v_mov_b32 v0, v1 // 1008:"),
        (s + 0xc, "global_load_lds_dwordx4 v[2:3], off // 100C:"),
        (s + 0x10, "s_waitcnt lgkmcnt(0) // 1010:"),
        (s + 0x14, "s_cbranch_scc1 65531 // 1014: <k+0x4>"),
        (s + 0x18, "s_endpgm // 1018:"),
    ]
    assert ring_violations(s, prog) == ["+0x4: s_barrier"]
    fixed = prog[:4] + [(s + 0x10, "s_waitcnt vmcnt(0) lgkmcnt(0) // 1010:")] + prog[5:]
    assert ring_violations(s, fixed) == []


# kernels whose A-fragment reads are untracked inline asm with hand-counted waits
UNTRACKED = ("_ZN3naz19coupling_w32_kernel", "_ZN3naz23coupling_bwd_r16_kernel", "_ZN3naz23made_ar_inv_wide_kernel",
             "_ZN3naz18made_ar_fwd_kernel")


def test_no_instruction_touches_a_pending_lds_read(lib):
    """No instruction of any kernel reads or overwrites a destination register of an LDS read that an
    s_waitcnt lgkmcnt has not retired on some path (loop back edges included): the hazard the
    untracked reads of lds_read_b128_untracked (naz_device.h) would hit if the compiler copied,
    spilled or re-used a prefetched fragment before its counted lds_wait.  Every kernel with LDS
    reads is checked; the ones built on the untracked reads must be among them."""
    bad, seen = {}, set()
    for co in code_objects(lib):
        for name, (start, insns) in functions(disassemble(co)).items():
            if not any(t.startswith("ds_read") for _, t in insns):
                continue
            for pre in UNTRACKED:
                if name.startswith(pre):
                    seen.add(pre)
            v = pending_lds_read_uses(start, insns)
            if v:
                bad[name] = v
    assert seen == set(UNTRACKED), f"untracked-read kernels missing: {set(UNTRACKED) - seen}"
    assert not bad, "registers used before their LDS read retired:\n" + "\n".join(
        f"{k}: {v[:4]}" for k, v in bad.items())


def test_pending_read_checker_flags_early_uses():
    s = 0x3000
    prog = [
        (s + 0x0, "ds_read_b128 v[0:3], v10 // 3000:"),
        (s + 0x4, "ds_read_b128 v[4:7], v10 offset:16 // 3004:"),
        (s + 0x8, "s_waitcnt lgkmcnt(1) // 3008:"),
        (s + 0xc, "v_mov_b32_e32 v20, v1 // 300C:"),  # first read retired: fine
        (s + 0x10, "v_mfma_f32_16x16x32_f16 a[0:3], v[4:7], v[4:7], a[0:3] // 3010:"),  # second still pending
        (s + 0x14, "s_waitcnt lgkmcnt(0) // 3014:"),
        (s + 0x18, "v_mov_b32_e32 v21, v5 // 3018:"),
        (s + 0x1c, "s_endpgm // 301C:"),
    ]
    assert pending_lds_read_uses(s, prog) == ["+0x10: v_mfma_f32_16x16x32_f16 a[0:3], v[4:7], v[4:7], a[0:3]"]
    # an overwrite of a pending destination (the LDS return would land after it) is flagged too
    waw = prog[:2] + [(s + 0x8, "v_mov_b32_e32 v2, 0 // 3008:")] + prog[5:]
    assert pending_lds_read_uses(s, waw) == ["+0x8: v_mov_b32_e32 v2, 0"]
    # a read issued at a loop's tail and used at its head through the back edge, no wait between
    loop = [
        (s + 0x0, "v_add_f32_e32 v8, v0, v8 // 3000:"),
        (s + 0x4, "ds_read_b32 v0, v10 // 3004:"),
        (s + 0x8, "s_cbranch_scc1 65533 // 3008: <k+0x0>"),
        (s + 0xc, "s_endpgm // 300C:"),
    ]
    assert pending_lds_read_uses(s, loop) == ["+0x0: v_add_f32_e32 v8, v0, v8"]


def test_pending_read_checker_catches_a_copy_in_the_w32_kernel(lib):
    """Mutation check on the real w32 kernel: a v_mov of the newest untracked A-fragment read's
    destination inserted just before its counted wait is flagged."""
    for co in code_objects(lib):
        for name, (start, insns) in functions(disassemble(co)).items():
            if not name.startswith(UNTRACKED[0]):
                continue
            for k, (a, t) in enumerate(insns):
                if t.startswith("s_waitcnt") and "lgkmcnt(2)" in t:
                    j = max(i for i in range(k) if insns[i][1].startswith("ds_read_b128"))
                    reg = insns[j][1].split()[1].split(",")[0]  # v[n:m]
                    first = int(reg[2:].split(":")[0])
                    mutated = insns[:k] + [(a - 2, f"v_mov_b32_e32 v255, v{first} // {a - 2:X}:")] + insns[k:]
                    assert any("v255" in x for x in pending_lds_read_uses(start, mutated))
                    return
    pytest.fail("no counted lgkmcnt(2) wait found in the w32 kernel")
