"""CPU: the C-ABI library loads and exports every symbol include/naz_hip.h declares
(no compute calls: there is no GPU here); host-side argument errors surface as messages."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "naz_hip.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(naz_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("naz_rqs_fwd", "naz_rqs_inv", "naz_linear_act", "naz_affine_ar", "naz_coupling_log_prob",
                 "naz_coupling_sample", "naz_coupling_pack", "naz_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from naz_amd import _lib
    L = _lib.lib()
    missing = [n for n in declared_functions() if not hasattr(L, n)]
    assert not missing, missing
    assert set(declared_functions()) == set(_lib.SIGNATURES), "ctypes signature table out of sync with the header"
    # 2: naz_ar_desc.flags (NAZ_AR_CLIP_ZERO_GRAD), naz_affine_ar_bwd's mode bits, and
    # naz_ar_flow_supported's 0 / 1 / 2 contract (2 = forward direction only); 3: packed-image
    # headers + registry, caller-owned workspace of the autoregressive log_prob entries
    assert L.naz_abi_version() == 3


def test_ar_flow_supported_contract():
    """naz_ar_flow_supported: 1 = both directions fused, 2 = the sampling direction only (no
    instance today), 0 = not instantiated.  The wide production MAFs (H = [512] x 5) are fused both
    ways since round 4 (made_ar_wide.h), without the pass-0-constants form."""
    from naz_amd import _lib, ops
    L = _lib.lib()
    assert L.naz_ar_flow_supported(ops.ar_flow_desc("maf", 2, 2, 150, 16, 3)) == 1
    assert L.naz_ar_flow_supported(ops.ar_flow_desc("maf", 4, 2, 150, 16, 3)) == 1  # the 4-parameter Bayesian MAF
    assert L.naz_ar_flow_supported(ops.ar_flow_desc("nsa", 16, 32, 128, 8, 2)) == 1
    wide = ops.ar_flow_desc("maf", 4, 2, 512, 18, 5)
    assert L.naz_ar_flow_supported(wide) == 1
    assert L.naz_ar_flow_packed_bytes(wide) > 0 and L.naz_ar_flow_fwd_packed_bytes(wide) > 0
    assert L.naz_ar_flow_pass0_floats(wide) < 0
    assert not ops.ar_flow_bwd_supported(wide)
    assert L.naz_ar_flow_supported(ops.ar_flow_desc("maf", 3, 2, 150, 4, 3)) == 0
    # the fused maf backward exists at both Bayesian shapes
    assert ops.ar_flow_bwd_supported(ops.ar_flow_desc("maf", 4, 2, 150, 16, 3))
    assert ops.ar_flow_bwd_supported(ops.ar_flow_desc("maf", 2, 2, 150, 16, 3))
    assert not ops.ar_flow_bwd_supported(ops.ar_flow_desc("maf", 16, 32, 128, 4, 2))


def test_host_side_errors_have_messages():
    from naz_amd import _lib
    L = _lib.lib()
    rc = L.naz_rqs_fwd(None, 0, None, 0, None, 0, None, 0, 16, 0, 8, 0, 3.0, None)  # Dt = 0
    assert rc != 0 and b"bad shape" in L.naz_last_error()
    rc = L.naz_rqs_inv(None, 0, None, 0, None, 0, None, 0, 0, 4, 2000, 0, 3.0, None)  # K*1e-3 > 1
    assert rc != 0 and b"Minimal bin width" in L.naz_last_error()
    d = _lib.CouplingDesc()
    d.D, d.C, d.S, d.K, d.L, d.H, d.act, d.has_lower, d.bound = 7, 0, 3, 8, 2, 64, 1, 1, 3.0
    assert L.naz_coupling_supported(d) == 0
    rc = L.naz_coupling_pack(d, None, None, None)
    assert rc != 0 and b"no fused instantiation" in L.naz_last_error()


def test_maf_backward_and_batched_wgrad_host_errors():
    """The fused maf backward's and the batched dW reduction's host-side checks (no GPU: every
    call below fails before a launch)."""
    import ctypes
    from naz_amd import _lib, ops
    L = _lib.lib()
    d = ops.ar_flow_desc("maf", 2, 2, 150, 4, 3)
    rc = L.naz_ar_flow_bwd_layer(d, None, None, None, 0, None, None, 0, None, None, None, None, 128, None)
    assert rc != 0 and b"null pointer" in L.naz_last_error()
    bufs = (ctypes.c_void_p * 11)(*([16] * 11))
    rc = L.naz_ar_flow_bwd_layer(d, 16, 16, 16, 4, 16, 16, 0, 16, None, bufs, 16, 128, None)  # layer == L
    assert rc != 0 and b"layer out of range" in L.naz_last_error()
    bad = ops.ar_flow_desc("maf", 16, 32, 128, 4, 2)
    rc = L.naz_ar_flow_bwd_layer(bad, 16, 16, 16, 0, 16, 16, 0, 16, None, bufs, 16, 128, None)
    assert rc != 0 and b"no fused backward" in L.naz_last_error()
    # the saved-state forward: any affine flow with a fused inverse (the wide MLE MAFs compose their
    # backward of GEMMs); a spline flow has none
    nsa = ops.ar_flow_desc("nsa", 16, 32, 128, 4, 2)
    rc = L.naz_ar_flow_log_prob_train(nsa, 16, 16, 2, 16, 2, 16, 16, 128, None, 0, None)
    assert rc != 0 and b"no fused affine inverse" in L.naz_last_error()
    wide = ops.ar_flow_desc("maf", 4, 2, 512, 18, 5)
    assert L.naz_ar_flow_log_prob_train(wide, 16, 16, 4, 16, 2, 16, 16, 0, None, 0, None) == 0  # no rows: no launch
    # one dim of the composed backward's VJP: dim range and null checks before any launch
    rc = L.naz_maf_dim_vjp(0, 16, 8, 16, 4, 16, 4, None, 16, 4, 16, 8, None, 0, 128, 4, 4, None)
    assert rc != 0 and b"outside" in L.naz_last_error()
    rc = L.naz_maf_dim_vjp(0, None, 8, 16, 4, 16, 4, None, 16, 4, 16, 8, None, 0, 128, 4, 0, None)
    assert rc != 0 and b"null pointer" in L.naz_last_error()
    assert L.naz_maf_dim_vjp(0, None, 8, None, 4, None, 4, None, None, 4, None, 8, None, 0, 0, 4, 0, None) == 0
    # batched dW: widths beyond the bf16x6 instances, misaligned rows
    rc = L.naz_wgrad_batched(1024, 160, 168, 2, 16, 160, 1 << 20, 16, 168, 1 << 20, 16, 168, 0, None, 0, None)
    assert rc != 0 and b"naz_wgrad_batched" in L.naz_last_error()
    rc = L.naz_wgrad_batched(1024, 160, 160, 2, 16, 161, 1 << 20, 16, 160, 1 << 20, 16, 160, 0, None, 0, None)
    assert rc != 0 and b"contiguous" in L.naz_last_error()
    assert L.naz_wgrad_batched(0, 160, 160, 2, 16, 160, 0, 16, 160, 0, 16, 160, 0, None, 0, None) == 0  # no rows


def test_fused_descriptor_matches_flow_parameters():
    from naz_amd import ops
    from naz_amd.flows import NormalizingFlow
    f = NormalizingFlow("nsc", None, 16, 32, [128, 128], 8, 8, 8)
    assert f.fused
    n = sum(p.numel() for p in f.parameters())
    assert ops.coupling_param_count(f._plan.desc) == n == 365440


def test_no_cpu_fallback():
    import torch
    from naz_amd import ops
    x = torch.zeros(4, 2)
    with pytest.raises(RuntimeError, match="GPU only"):
        ops.rqs(x, torch.zeros(4, 2 * 23), 8)
    from naz_amd.flows import NormalizingFlow
    f = NormalizingFlow("nsc", None, 4, 3, [64, 64], 2, 8, 2)
    with pytest.raises(RuntimeError, match="GPU only"):
        f.log_prob(torch.zeros(3, 4), condition=torch.zeros(3, 3))


def test_generic_flow_entries_dispatch_without_compute():
    """naz_flow_*: packed sizes and workspace of both fused kinds (host-only calls), and the
    documented errors (unknown kind, missing buffers)."""
    from naz_amd import _lib, ops
    L = _lib.lib()
    c = ops.coupling_desc(16, 32, 8, 8, 8, 128)
    a = ops.ar_flow_desc("maf", 2, 2, 150, 16, n_hidden=3)
    fc, fa = ops.flow_desc(c), ops.flow_desc(a)
    assert L.naz_flow_packed_bytes(fc) == L.naz_coupling_packed_bytes(c) > 0
    assert L.naz_flow_packed_bytes(fa) == L.naz_ar_flow_packed_bytes(a) > 0
    assert L.naz_workspace_bytes(fc, 1 << 20) == 0 and L.naz_workspace_bytes(fa, 1 << 20) == 0
    bad = _lib.FlowDesc()
    bad.kind = 7
    assert L.naz_flow_packed_bytes(bad) == -1
    assert L.naz_flow_log_prob(bad, None, None, 0, None, 0, None, None, None, 0, None, 0, None) != 0
    assert b"unknown flow kind" in L.naz_last_error()
    assert L.naz_flow_sample(fa, None, None, 0, None, 0, None, None, None, 0, None, 0, None) == 0  # B = 0
    assert L.naz_flow_sample(fa, None, None, 0, None, 0, None, None, None, 0, None, 1, None) != 0
    assert b"null pointer" in L.naz_last_error()
    assert L.naz_ar_flow_fwd_packed_bytes(a) > 0


def test_workspace_sizes_are_the_wide_inverse_scratch():
    """naz_ar_flow_workspace_bytes / naz_workspace_bytes (ABI 3): 0 wherever every intermediate stays
    on chip; for the wide MLE MAF (made_ar_wide.h) one 4-wave workgroup per CU (at most one per
    64-row tile and draw), 128 KiB of hidden-layer fragments per wave.  Without a GPU the CU count
    reads as 256.  No log_prob entry allocates: too little workspace is an error before any launch."""
    from naz_amd import _lib, ops
    L = _lib.lib()
    wide = ops.ar_flow_desc("maf", 4, 2, 512, 18, 5)
    per_wg = 4 * 128 * 1024
    assert L.naz_ar_flow_workspace_bytes(wide, 100, 1) == 2 * per_wg  # 2 tiles of 64 rows
    assert L.naz_ar_flow_workspace_bytes(wide, 64, 3) == 3 * per_wg  # one tile per draw
    assert L.naz_ar_flow_workspace_bytes(wide, 1 << 18, 1) == 256 * per_wg  # 128 MiB: the persistent grid
    assert L.naz_workspace_bytes(ops.flow_desc(wide), 1 << 18) == 256 * per_wg
    assert L.naz_ar_flow_workspace_bytes(wide, 0, 1) == 0 and L.naz_ar_flow_workspace_bytes(wide, -1, 1) == -1
    for narrow in (ops.ar_flow_desc("maf", 2, 2, 150, 16, 3), ops.ar_flow_desc("nsa", 16, 32, 128, 8, 2)):
        assert L.naz_ar_flow_workspace_bytes(narrow, 1 << 20, 4) == 0
    assert L.naz_ar_flow_workspace_bytes(ops.ar_flow_desc("maf", 3, 2, 150, 4, 3), 128, 1) == -1


def test_image_registry_refuses_unregistered_images():
    """Every launch entry resolves its packed image through the registry before launching (ABI 3):
    an address no packer wrote (or attached) is an error, not a launch -- checked here without a GPU
    (the registry lookup precedes every device call)."""
    from naz_amd import _lib, ops
    L = _lib.lib()
    c = ops.coupling_desc(16, 32, 8, 8, 8, 128)
    fake = 1 << 40
    rc = L.naz_coupling_log_prob(c, fake, fake, 16, fake, 32, None, None, fake, 128, None)
    assert rc != 0 and b"is not a packed image" in L.naz_last_error()
    a = ops.ar_flow_desc("nsa", 16, 32, 128, 8, 2)
    rc = L.naz_ar_flow_log_prob(a, fake, fake, 16, fake, 32, None, None, fake, 128, None, 0, None)
    assert rc != 0 and b"is not a packed image" in L.naz_last_error()
    rc = L.naz_ar_flow_sample(a, None, fake, 16, fake, 32, None, None, fake, 16, None, 128, None)
    assert rc != 0 and b"null" in L.naz_last_error()
    assert L.naz_image_release(fake) != 0
    assert L.naz_image_attach(None, 4096, None) != 0


def test_host_packed_image_headers():
    """The host packers write the 256-byte header the registry reads back (naz_image_attach): magic,
    layout version, kind (3 inverse / 4 forward), a tag that depends on the descriptor's layout fields
    only, layers, body bytes."""
    import ctypes
    import numpy as np
    from naz_amd import _lib, ops
    L = _lib.lib()

    def header(d, fwd):
        n = int((L.naz_ar_flow_fwd_packed_bytes if fwd else L.naz_ar_flow_packed_bytes)(d))
        per = (4 * 2 + 2) * 150 + 2 * (150 * 150 + 150) + 2 * 2 * 150 + 4  # D=2 | C=2, H=[150]x3 maf
        flat = np.zeros(d.L * per, np.float32)
        perm = np.tile(np.arange(2, dtype=np.int32), (d.L, 1))
        host = np.zeros(n // 4, np.float32)
        if fwd:
            ops.check(L.naz_ar_flow_pack_fwd_host(d, flat.ctypes.data, host.ctypes.data), "fwd")
        else:
            ops.check(L.naz_ar_flow_pack_host(d, flat.ctypes.data, perm.ctypes.data, host.ctypes.data), "inv")
        return n, host[:64].view(np.uint32).copy()

    d = ops.ar_flow_desc("maf", 2, 2, 150, 4, 3)
    n, h = header(d, False)
    assert (h[0], h[1], h[2], h[4], h[5]) == (0x495A414E, 3, 3, 4, 0)
    assert int(h[6]) | (int(h[7]) << 32) == n - 256
    _, hf = header(d, True)
    assert hf[2] == 4 and hf[3] != h[3]
    d2 = ops.ar_flow_desc("maf", 2, 2, 150, 7, 3)  # more layers: same layout tag, more bytes
    n2, h2 = header(d2, False)
    assert h2[3] == h[3] and h2[4] == 7 and n2 - 256 == (n - 256) // 4 * 7
    d3 = ops.ar_flow_desc("maf", 2, 2, 150, 4, 3)
    d3.flags = 1  # the backward's clip semantics do not change the layout
    assert header(d3, False)[1][3] == h[3]


def test_tuning_keys():
    """naz_tuning: the batch-row GEMM's panel split (default on), arithmetic (default exact FP32) and
    small-batch grid fill (clamped to 16), set and read back; an unknown key is an error."""
    from naz_amd import _lib
    L = _lib.lib()
    for key, default in ((b"rowgemm_split", 1), (b"rowgemm_x6", 0), (b"rowgemm_h3", 0)):
        cur = L.naz_tuning(key, -1)
        assert cur in (0, 1)
        assert L.naz_tuning(key, 1 - cur) == cur and L.naz_tuning(key, -1) == 1 - cur
        assert L.naz_tuning(key, cur) == 1 - cur and L.naz_tuning(key, -1) == cur
    cur = L.naz_tuning(b"rowgemm_fill", -1)  # workgroups per CU the small-batch narrowing aims for
    assert 0 <= cur <= 16
    assert L.naz_tuning(b"rowgemm_fill", 4) == cur and L.naz_tuning(b"rowgemm_fill", 99) == 4
    assert L.naz_tuning(b"rowgemm_fill", cur) == 16 and L.naz_tuning(b"rowgemm_fill", -1) == cur
    assert L.naz_tuning(b"no_such_key", 1) == -1 and b"unknown key" in L.naz_last_error()
