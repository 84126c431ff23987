"""CPU: the fused autoregressive kernel's host side — the hidden mask indices it is compiled for
equal pyro create_mask's (torch.linspace(1, D, H).round() - 1 with a context, linspace(1, D-1, H)
without), and the host packer (naz_spline_ar_pack_host) lays weights into f16 hi/lo fragments
that decode back to the scaled weights (no GPU: host memory only)."""
import numpy as np
import pytest
import torch

from naz_amd import ops


@pytest.mark.parametrize("D,C", [(16, 32), (16, 0), (8, 0), (4, 2)])
def test_compiled_degrees_match_pyro_create_mask(D, C):
    d = ops.spline_ar_desc(D, C, 128, 8, 1)
    assert ops.spline_ar_supported(d)
    deg = ops.spline_ar_degrees(d)
    if C > 0:
        ref = (torch.linspace(1, D, 128).round() - 1).int().numpy()
    else:
        ref = torch.linspace(1, D - 1, 128).round().int().numpy()
    np.testing.assert_array_equal(deg, ref)


def test_unsupported_shape_reports():
    assert not ops.spline_ar_supported(ops.spline_ar_desc(5, 3, 128, 8, 1))
    assert not ops.spline_ar_supported(ops.spline_ar_desc(16, 32, 128, 8, 1, act="relu"))


def test_host_pack_decodes_to_scaled_weights():
    D, C, H, K, L = 16, 32, 128, 8, 2
    P = 3 * K - 1
    d = ops.spline_ar_desc(D, C, H, K, L)
    rng = np.random.default_rng(0)
    sizes = [H * (C + D), H, H * H, H, D * P * H, D * P]
    flat = rng.standard_normal(L * sum(sizes)).astype(np.float32) * 0.1
    perm = np.stack([rng.permutation(D) for _ in range(L)]).astype(np.int32)
    nbytes = int(ops.lib().naz_spline_ar_packed_bytes(d))
    host = np.empty(nbytes // 4, dtype=np.float32)
    ops.check(ops.lib().naz_spline_ar_pack_host(d, np.ascontiguousarray(flat).ctypes.data, perm.ctypes.data,
                                                host.ctypes.data), "pack")
    words = host.view(np.uint32)
    # layer 0, pass 0, first L1 fragment (block blo(0) = 0, k-step 0 = context): lane (m, kg) pair w
    # holds W0[m][8 kg + 2w (+1)] * kSigScale as hi | lo f16 pieces
    W0 = flat[:H * (C + D)].reshape(H, C + D)
    ks = 2.88539008177792681
    for lane in (0, 5, 17, 63):
        m, kg = lane & 15, lane >> 4
        for pair in range(4):
            hi = words[(0 * 64 + lane) * 4 + pair]
            lo = words[(1 * 64 + lane) * 4 + pair]
            for e in range(2):
                h16 = np.array([(hi >> (16 * e)) & 0xFFFF], np.uint16).view(np.float16)[0]
                l16 = np.array([(lo >> (16 * e)) & 0xFFFF], np.uint16).view(np.float16)[0]
                want = np.float32(ks) * W0[m, 8 * kg + 2 * pair + e]
                # hi + lo carries ~22 bits; lo below f16's normal range keeps 2^-24 absolute spacing
                assert abs((np.float32(h16) + np.float32(l16)) - want) <= 2.5e-7 * abs(want) + 3.1e-8
    # the permutation table rides in the image (last D ints before the layer padding)
    layer_floats = nbytes // 4 // L
    perm_off = None
    for off in range(layer_floats - 512, layer_floats - D + 1):
        if np.array_equal(host[off:off + D].view(np.int32), perm[0]):
            perm_off = off
            break
    assert perm_off is not None
