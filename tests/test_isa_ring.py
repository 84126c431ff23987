"""CPU test: every LDS-DMA ring kernel in the built library waits vmcnt(0) before each barrier
that a wave can reach with a global_load_lds in flight (tests/isa_ring.py)."""
from pathlib import Path

import pytest

from tests.isa_ring import check_library, code_objects, disassemble, functions, is_dma, ring_violations

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
