"""CPU test: every LDS-DMA ring kernel in the built library waits vmcnt(0) before each barrier
that a wave can reach with a global_load_lds in flight (tests/isa_ring.py)."""
from pathlib import Path

import pytest

from tests.isa_ring import (check_library, code_objects, counted_lgkm_violations, disassemble, functions, is_dma,
                            ring_violations)

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
