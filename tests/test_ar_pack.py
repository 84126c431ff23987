"""CPU: the fused autoregressive kernel's host side — the hidden mask indices it is compiled for
equal pyro create_mask's (torch.linspace(1, D, H).round() - 1 with a context, linspace(1, D-1, H)
without), and the host packer (naz_ar_flow_pack_host) lays weights into f16 hi/lo fragments
that decode back to the scaled weights (no GPU: host memory only)."""
import numpy as np
import pytest
import torch

from naz_amd import ops


@pytest.mark.parametrize("kind,D,C,H,NH", [("nsa", 16, 32, 128, 2), ("nsa", 16, 0, 128, 2), ("nsa", 8, 0, 128, 2),
                                           ("nsa", 4, 2, 128, 2), ("maf", 2, 2, 150, 3), ("maf", 16, 32, 128, 2),
                                           ("maf", 4, 2, 512, 5)])
def test_compiled_degrees_match_pyro_create_mask(kind, D, C, H, NH):
    d = ops.ar_flow_desc(kind, D, C, H, 1, NH)
    assert ops.ar_flow_supported(d)
    deg = ops.ar_flow_degrees(d)
    if C > 0:
        ref = (torch.linspace(1, D, H).round() - 1).int().numpy()
    else:
        ref = torch.linspace(1, D - 1, H).round().int().numpy()
    np.testing.assert_array_equal(deg, ref)


def test_unsupported_shape_reports():
    assert not ops.ar_flow_supported(ops.ar_flow_desc("nsa", 5, 3, 128, 1))
    assert not ops.ar_flow_supported(ops.ar_flow_desc("nsa", 16, 32, 128, 1, act="relu"))
    assert not ops.ar_flow_supported(ops.ar_flow_desc("nsa", 16, 32, 128, 1, n_hidden=3))
    assert not ops.ar_flow_supported(ops.ar_flow_desc("maf", 2, 2, 150, 1, n_hidden=2))
    assert not ops.ar_flow_supported(ops.ar_flow_desc("bogus", 2, 2, 150, 1, n_hidden=3))
    with pytest.raises(RuntimeError, match="no fused instantiation"):
        ops.ar_flow_degrees(ops.ar_flow_desc("maf", 3, 2, 150, 1, n_hidden=3))


@pytest.mark.parametrize("kind,D,C,H,NH", [("nsa", 16, 32, 128, 2), ("maf", 2, 2, 150, 3), ("maf", 4, 2, 512, 5)])
def test_host_pack_decodes_to_scaled_weights(kind, D, C, H, NH):
    K, L = 8, 3
    P = 2 if kind == "maf" else 3 * K - 1
    d = ops.ar_flow_desc(kind, D, C, H, L, NH, K)
    rng = np.random.default_rng(0)
    sizes = [H * (C + D), H] + [H * H, H] * (NH - 1) + [D * P * H, D * P]
    flat = rng.standard_normal(L * sum(sizes)).astype(np.float32) * 0.1
    perm = np.stack([rng.permutation(D) for _ in range(L)]).astype(np.int32)
    nbytes = int(ops.lib().naz_ar_flow_packed_bytes(d))
    host = np.empty(nbytes // 4, dtype=np.float32)
    ops.check(ops.lib().naz_ar_flow_pack_host(d, np.ascontiguousarray(flat).ctypes.data, perm.ctypes.data,
                                                host.ctypes.data), "pack")
    # the 256-byte image header (include/naz_hip.h "Packed images"), then the layers
    hdr = host[:64].view(np.uint32)
    assert hdr[0] == 0x495A414E and hdr[2] == 3 and hdr[4] == L and hdr[5] == 0
    assert int(hdr[6]) | (int(hdr[7]) << 32) == nbytes - 256 and not hdr[8:].any()
    host = host[64:]
    words = host.view(np.uint32)
    layer_floats = host.size // L
    per = sum(sizes)
    # every layer l, pass 0, first L1 fragment (block 0, k-step 0 = context): lane (m, kg) pair w
    # holds W0[m][8 kg + 2w (+1)] * kSigScale as hi | lo f16 pieces (layer l's flat rows at l * per:
    # a wrong per-layer stride reads another layer's — or no — weights)
    ks = 2.88539008177792681
    for layer in range(L):
        W0 = flat[layer * per:layer * per + H * (C + D)].reshape(H, C + D)
        base = layer * layer_floats
        for lane in (0, 5, 17, 63):
            m, kg = lane & 15, lane >> 4
            for pair in range(4):
                hi = words[base + (0 * 64 + lane) * 4 + pair]
                lo = words[base + (1 * 64 + lane) * 4 + pair]
                for e in range(2):
                    h16 = np.array([(hi >> (16 * e)) & 0xFFFF], np.uint16).view(np.float16)[0]
                    l16 = np.array([(lo >> (16 * e)) & 0xFFFF], np.uint16).view(np.float16)[0]
                    col = 8 * kg + 2 * pair + e
                    want = np.float32(ks) * W0[m, col] if col < C else np.float32(0)
                    # hi + lo carries ~22 bits; lo below f16's normal range keeps 2^-24 absolute spacing
                    assert abs((np.float32(h16) + np.float32(l16)) - want) <= 2.5e-7 * abs(want) + 3.1e-8
    # the permutation table rides in the image (last D ints before the layer padding)
    assert layer_floats * 4 * L + 256 == nbytes and layer_floats % 256 == 0
    perm_off = None
    for off in range(layer_floats - 512, layer_floats - D + 1):
        if np.array_equal(host[off:off + D].view(np.int32), perm[0]):
            perm_off = off
            break
    assert perm_off is not None


def test_fused_maf_backward_host_queries():
    """naz_ar_flow_bwd_*: the fused maf backward exists at the paper shape only, with the operand
    widths include/naz_hip.h documents; every other shape / kind reports itself unsupported."""
    d = ops.ar_flow_desc("maf", 2, 2, 150, 16, 3)
    assert ops.ar_flow_bwd_supported(d)
    assert ops.ar_flow_bwd_dims(d) == dict(n_hidden=3, HP=160, XA=160, XB=0, X0W=8, rows=128)
    per_layer = int(ops.lib().naz_ar_flow_bwd_packed_bytes(ops.ar_flow_desc("maf", 2, 2, 150, 1, 3)))
    assert per_layer > 256 and int(ops.lib().naz_ar_flow_bwd_packed_bytes(d)) - 256 == 16 * (per_layer - 256)
    for bad in (ops.ar_flow_desc("nsa", 16, 32, 128, 1), ops.ar_flow_desc("maf", 16, 32, 128, 1, 2),
                ops.ar_flow_desc("maf", 2, 2, 150, 1, 3, act="relu"), ops.ar_flow_desc("maf", 4, 2, 512, 1, 5)):
        assert not ops.ar_flow_bwd_supported(bad)
    with pytest.raises(RuntimeError, match="no fused backward"):
        ops.ar_flow_bwd_dims(ops.ar_flow_desc("maf", 16, 32, 128, 1, 2))
