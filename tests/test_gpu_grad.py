"""GPU: the NLL training step's backward kernels against the oracle's
float64 torch autograd (the gradient pyro's eager transforms produce, restated in
oracle/naz_oracle.py), with the oracle's float32 autograd as the reference-precision yardstick.

Criterion: tests/parity.py median / q99 / max bounds with the gradient floor
max(|g64|, rms(g64)) and no exceedance-count bound (see tests/parity.py).
"""
import numpy as np
import pytest
import torch

from oracle import naz_oracle as O
from tests.conftest import load_golden, spec_state
from tests.parity import assert_parity, grad_floor

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _cuda(a):
    return torch.as_tensor(np.asarray(a), dtype=torch.float32, device=DEV)


def _np(t):
    return t.detach().double().cpu().numpy()


def _check(v, g64, g32, what):
    g64 = _np(g64) if torch.is_tensor(g64) else g64
    g32 = _np(g32) if torch.is_tensor(g32) else g32
    return assert_parity(_np(v), g64, g32, what=what, floor=grad_floor(g64), count_factor=None)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from naz_amd import _lib
    _lib.lib()


def _oracle_rqs_grads(x, raw, Dt, K, layout, inverse, g_out, g_ld, dtype, per_dim):
    xo = torch.as_tensor(x).to(dtype).requires_grad_(True)
    ro = torch.as_tensor(raw).to(dtype).requires_grad_(True)
    y, ld = O.rqs_from_raw(xo, ro, Dt, K, layout, inverse)
    gl = torch.as_tensor(g_ld).to(dtype)
    loss = (y * torch.as_tensor(g_out).to(dtype)).sum()
    loss = loss + ((ld * gl).sum() if per_dim else (ld.sum(-1) * gl).sum())
    gx, gr = torch.autograd.grad(loss, [xo, ro])
    return gx, gr


# ------------------------------------------------------------------ a1+a2 spline VJP
@pytest.mark.parametrize("name", ["rqs_dense_k8.npz", "rqs_arn_k5.npz", "rqs_dense_k16.npz"])
@pytest.mark.parametrize("inverse", [False, True])
@pytest.mark.parametrize("per_dim", [False, True])
def test_rqs_bwd_vs_oracle(name, inverse, per_dim):
    from naz_amd import ops
    fx = load_golden(name)
    K, Dt, layout = int(fx["K"]), int(fx["Dt"]), int(fx["layout"])
    x, raw = fx["x"], fx["raw"]
    B = x.shape[0]
    rng = np.random.default_rng(7)
    g_out = rng.standard_normal((B, Dt)).astype(np.float32)
    g_ld = rng.standard_normal((B, Dt) if per_dim else (B,)).astype(np.float32)
    gx, gr = ops.rqs_bwd(_cuda(x), _cuda(raw), K, layout, inverse, 3.0, _cuda(g_out), _cuda(g_ld))
    gx64, gr64 = _oracle_rqs_grads(x, raw, Dt, K, layout, inverse, g_out, g_ld, torch.float64, per_dim)
    gx32, gr32 = _oracle_rqs_grads(x, raw, Dt, K, layout, inverse, g_out, g_ld, torch.float32, per_dim)
    _check(gx, gx64, gx32, f"{name} inv={inverse} d/dx")
    _check(gr, gr64, gr32, f"{name} inv={inverse} d/draw")


@pytest.mark.parametrize("inverse", [False, True])
def test_rqs_bwd_broadcast_params(inverse):
    """The coupling's lower spline: ONE parameter row for every batch row (ldr = 0); the
    parameter gradient is reduced over the batch in-kernel."""
    from naz_amd import ops
    K, Dt, B = 8, 8, 3000
    rng = np.random.default_rng(3)
    x = (rng.standard_normal((B, Dt)) * 1.5).astype(np.float32)
    raw = (rng.standard_normal(Dt * (3 * K - 1)) * 0.7).astype(np.float32)
    g_out = rng.standard_normal((B, Dt)).astype(np.float32)
    g_ld = rng.standard_normal(B).astype(np.float32)
    gx, gr = ops.rqs_bwd(_cuda(x), _cuda(raw), K, O.LAYOUT_DENSE, inverse, 3.0, _cuda(g_out), _cuda(g_ld),
                         broadcast_raw=True)
    refs = []
    for dt in (torch.float64, torch.float32):
        ro = torch.as_tensor(raw).to(dt).requires_grad_(True)
        xo = torch.as_tensor(x).to(dt).requires_grad_(True)
        y, ld = O.rqs_from_raw(xo, ro.expand(B, -1), Dt, K, O.LAYOUT_DENSE, inverse)
        loss = (y * torch.as_tensor(g_out).to(dt)).sum() + (ld.sum(-1) * torch.as_tensor(g_ld).to(dt)).sum()
        refs.append(torch.autograd.grad(loss, [xo, ro]))
    _check(gx, refs[0][0], refs[1][0], "broadcast d/dx")
    _check(gr, refs[0][1], refs[1][1], "broadcast d/draw (batch-reduced)")


# ------------------------------------------------------------------ a6/a7 conditioner VJP
@pytest.mark.parametrize("act", ["identity", "tanh", "relu", "softplus", "sigmoid"])
@pytest.mark.parametrize("ctx_kind", ["none", "rows", "one_row"])
@pytest.mark.parametrize("masked", [False, True])
@pytest.mark.parametrize("M", [1000, 3000])
def test_linear_act_grad(act, ctx_kind, masked, M):
    """M = 1000 runs the generic 64x64-tile kernels, M = 3000 the batch-row kernels
    (gemm_rows.hip: rowgemm forward / dX, wgrad dW + db)."""
    from naz_amd import autograd as ag
    rng = np.random.default_rng(11)
    Kx, C, N = 24, (0 if ctx_kind == "none" else 13), 70
    x = rng.standard_normal((M, Kx)).astype(np.float32)
    W = (rng.standard_normal((N, C + Kx)) / np.sqrt(C + Kx)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32) * 0.1
    mask = (rng.random((N, C + Kx)) > 0.4).astype(np.float32) if masked else None
    ctx = None
    if ctx_kind == "rows":
        ctx = rng.standard_normal((M, C)).astype(np.float32)
    elif ctx_kind == "one_row":
        ctx = rng.standard_normal((1, C)).astype(np.float32)
    gy = rng.standard_normal((M, N)).astype(np.float32)

    def run(dev, dt, kernel):
        ts = {"x": torch.as_tensor(x, device=dev, dtype=dt), "W": torch.as_tensor(W, device=dev, dtype=dt),
              "b": torch.as_tensor(b, device=dev, dtype=dt)}
        if ctx is not None:
            ts["c"] = torch.as_tensor(ctx, device=dev, dtype=dt)
        for t in ts.values():
            t.requires_grad_(True)
        m = None if mask is None else torch.as_tensor(mask, device=dev, dtype=dt)
        if kernel:
            y = ag.linear_act(ts["x"], ts["W"], ts["b"], act, context=ts.get("c"), mask=m)
        else:
            inp = ts["x"] if ctx is None else torch.cat([ts["c"].expand(M, C), ts["x"]], 1)
            Wm = ts["W"] if m is None else ts["W"] * m
            y = O.ACTIVATIONS[act](inp @ Wm.t() + ts["b"])
        keys = list(ts)
        gs = torch.autograd.grad((y * torch.as_tensor(gy, device=dev, dtype=dt)).sum(), [ts[k] for k in keys])
        return dict(zip(keys, gs))

    got = run(DEV, torch.float32, True)
    r64 = run("cpu", torch.float64, False)
    r32 = run("cpu", torch.float32, False)
    for k in got:
        _check(got[k], r64[k], r32[k], f"linear_act[{act},{ctx_kind},mask={masked}] d/d{k}")


def test_rowgemm_config3_shapes():
    """The batch-row forward kernel at config-3 conditioner shapes (ctx 32 | x1 8 -> 128 -> 128
    -> 184), odd row count, 16-byte and unaligned row strides, and the dX GEMM with a mask."""
    from naz_amd import ops
    g = torch.Generator().manual_seed(5)
    M = 5003
    for C, Kx, N, ldx_pad in [(32, 8, 128, 8), (0, 128, 128, 0), (0, 128, 184, 3), (13, 5, 300, 1)]:
        ctx = torch.randn(M, C, generator=g)
        xfull = torch.randn(M, Kx + ldx_pad, generator=g)
        x = xfull[:, :Kx]
        W = torch.randn(N, C + Kx, generator=g) / (C + Kx) ** 0.5
        b = torch.randn(N, generator=g) * 0.1
        y = ops.linear_act(_cuda(x) if ldx_pad == 0 else _cuda(xfull)[:, :Kx], _cuda(W), _cuda(b), "tanh",
                           context=_cuda(ctx) if C else None)
        inp = torch.cat([ctx, x], 1) if C else x
        ref64 = torch.tanh(inp.double() @ W.double().t() + b.double())
        ref32 = torch.tanh(inp @ W.t() + b)
        _check(y, ref64, ref32, f"rowgemm fwd C={C} Kx={Kx} N={N}")
    G = torch.randn(M, 184, generator=g)
    W = torch.randn(184, 128, generator=g) / 13.0
    mask = (torch.rand(184, 128, generator=g) > 0.3).float()
    dx = ops.gemm(_cuda(G), _cuda(W), mask=_cuda(mask), mask_b=True)
    _check(dx, G.double() @ (W.double() * mask.double()), G @ (W * mask), "rowgemm dX masked")


@pytest.mark.parametrize("N", [168, 172, 300])
@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("arith", ["fp32", "x6", "h3", "bres"])
def test_rowgemm_panel_split(N, split, arith):
    """The batch-row kernel with the panel split on and off (naz_tuning "rowgemm_split"; default on):
    widths of 6 / 6 / 10 column blocks (an odd half-panel at 168 / 172 runs the paired epilogue's
    guard) through every epilogue -- bias + activation (linear_act), the masked dX GEMM, the chained
    act' (gemm_dact), the CNF pair VJP (gemm_jvp_bwd) -- on a ragged row count, against fp64; on both
    arithmetics (naz_tuning "rowgemm_x6" / "rowgemm_h3": exact FP32 MFMA, the bf16x6 split, or the
    f16x3 split with per-row power-of-two scales)."""
    from naz_amd import ops
    prev = ops.rowgemm_split(split)
    prev6 = ops.rowgemm_x6(arith == "x6")
    prevh = ops.rowgemm_h3(arith == "h3")
    prevb = ops.rowgemm_bres(arith == "bres")  # (B-resident f16x3: the masked dX and chained act' here)
    prevf = ops.rowgemm_fill(0)  # the panels as the split sets them (4098 rows would be narrowed)
    try:
        g = torch.Generator().manual_seed(N + 11 * split)
        M = 4098
        ctx, x = torch.randn(M, 13, generator=g), torch.randn(M, 40, generator=g)
        W = torch.randn(N, 53, generator=g) / 53 ** 0.5
        b = torch.randn(N, generator=g) * 0.1
        y = ops.linear_act(_cuda(x), _cuda(W), _cuda(b), "tanh", context=_cuda(ctx))
        inp = torch.cat([ctx, x], 1)
        _check(y, torch.tanh(inp.double() @ W.double().t() + b.double()), torch.tanh(inp @ W.t() + b),
               f"fwd N={N} split={split}")
        G = torch.randn(M, 184, generator=g)
        W2 = torch.randn(184, N, generator=g) / 13.0
        mask = (torch.rand(184, N, generator=g) > 0.3).float()
        dx = ops.gemm(_cuda(G), _cuda(W2), mask=_cuda(mask), mask_b=True)
        _check(dx, G.double() @ (W2.double() * mask.double()), G @ (W2 * mask), f"dX N={N} split={split}")
        h = torch.tanh(torch.randn(M, N, generator=g))
        da = ops.gemm_dact(_cuda(G), _cuda(W2), _cuda(h), "tanh", mask=_cuda(mask))
        ref64 = (G.double() @ (W2.double() * mask.double())) * (1 - h.double() ** 2)
        _check(da, ref64, (G @ (W2 * mask)) * (1 - h * h), f"dact N={N} split={split}")
        S = torch.tanh(torch.randn(M, N, generator=g))
        S[1::2] = torch.randn(M // 2, N, generator=g)  # tangent rows
        jv = ops.gemm_jvp_bwd(_cuda(G), _cuda(W2), _cuda(S), "tanh")
        P64 = G.double() @ W2.double()
        hv, dt = S[0::2].double(), S[1::2].double()
        r64 = torch.empty(M, N, dtype=torch.float64)
        r64[0::2] = P64[0::2] * (1 - hv ** 2) + P64[1::2] * dt * (-2 * hv)
        r64[1::2] = P64[1::2] * (1 - hv ** 2)
        P32 = G @ W2
        r32 = torch.empty(M, N)
        r32[0::2] = P32[0::2] * (1 - S[0::2] ** 2) + P32[1::2] * S[1::2] * (-2 * S[0::2])
        r32[1::2] = P32[1::2] * (1 - S[0::2] ** 2)
        _check(jv, r64, r32, f"jvp N={N} split={split}")
    finally:
        ops.rowgemm_split(prev)
        ops.rowgemm_x6(prev6)
        ops.rowgemm_h3(prevh)
        ops.rowgemm_bres(prevb)
        ops.rowgemm_fill(prevf)


@pytest.mark.parametrize("N", [64, 172])
def test_rowgemm_h3_row_scales(N):
    """The f16x3 batch-row GEMM splits every A row at its own power-of-two scale: rows spanning 10^-30
    .. 10^30 (gradients have no range), an all-zero row and a ragged row count keep fp32-grade relative
    accuracy per row in every epilogue's product, against fp64."""
    from naz_amd import ops
    g = torch.Generator().manual_seed(N)
    M, K = 4099, 200
    A = torch.randn(M, K, generator=g) * torch.pow(10.0, torch.empty(M, 1).uniform_(-30, 30, generator=g))
    A[5] = 0.0
    W = torch.randn(N, K, generator=g) / K ** 0.5
    prev = ops.rowgemm_h3(True)
    try:
        y = ops.linear_act(_cuda(A), _cuda(W), None, "identity")
        dx = ops.gemm(_cuda(A), _cuda(W.t().contiguous()))
    finally:
        ops.rowgemm_h3(prev)
    ref = A.double() @ W.double().t()
    for out, what in ((y, "linear_act"), (dx, "dX")):
        o = out.double().cpu()
        scale = ref.abs().amax(1, keepdim=True).clamp_min(1e-300)
        rel = ((o - ref).abs() / scale).amax(1)
        assert torch.isfinite(o).all(), what
        assert float(rel.max()) < 2e-6, (what, float(rel.max()))
        assert float(o[5].abs().max()) == 0.0


@pytest.mark.parametrize("M,N", [(10752, 512), (10752, 172), (1000, 300), (70000, 512)])
def test_rowgemm_fill_changes_no_bit(M, N):
    """The small-batch grid fill (naz_tuning "rowgemm_fill": column panels narrowed until the grid
    holds that many workgroups per CU) only regroups output columns into workgroups; each output's
    k-order is the same, so every epilogue -- bias + activation, the masked dX GEMM, the chained act',
    the CNF pair VJP -- is bit-identical with it off, at the default and at 16.  The first shape is the
    wide maf at naz's 10,752-row minibatch."""
    from naz_amd import ops
    g = torch.Generator().manual_seed(M + N)
    ctx, x = torch.randn(M, 2, generator=g), torch.randn(M, 40, generator=g)
    W = torch.randn(N, 42, generator=g) / 42 ** 0.5
    b = torch.randn(N, generator=g) * 0.1
    G = torch.randn(M, 184, generator=g)
    W2 = torch.randn(184, N, generator=g) / 13.0
    mask = (torch.rand(184, N, generator=g) > 0.3).float()
    h = torch.tanh(torch.randn(M, N, generator=g))
    outs = {}
    prev = ops.rowgemm_fill()
    try:
        for fill in (0, prev, 16):
            ops.rowgemm_fill(fill)
            outs[fill] = (ops.linear_act(_cuda(x), _cuda(W), _cuda(b), "tanh", context=_cuda(ctx)),
                          ops.gemm(_cuda(G), _cuda(W2), mask=_cuda(mask), mask_b=True),
                          ops.gemm_dact(_cuda(G), _cuda(W2), _cuda(h), "tanh", mask=_cuda(mask)),
                          ops.gemm_jvp_bwd(_cuda(G), _cuda(W2), _cuda(h), "tanh"))
    finally:
        ops.rowgemm_fill(prev)
    ref64 = torch.tanh(torch.cat([ctx, x], 1).double() @ W.double().t() + b.double())
    _check(outs[0][0], ref64, torch.tanh(torch.cat([ctx, x], 1) @ W.t() + b), f"fwd M={M} N={N}")
    for fill in (prev, 16):
        for name, a, c in zip(("fwd", "dX", "dact", "jvp"), outs[0], outs[fill]):
            assert torch.equal(a, c), f"{name} M={M} N={N}: fill {fill} changed bits"


@pytest.mark.parametrize("M,N,K,split", [(128, 40, 50000, None), (184, 128, 4097, 7), (3, 5, 1, None),
                                         (1000, 24, 70, None), (65, 130, 200000, None)])
def test_gemm_strided_split_k(M, N, K, split):
    """naz_gemm over transposed views (the dW = dPre^T X case) with split-K atomics."""
    from naz_amd import ops
    g = torch.Generator().manual_seed(M * 7 + N)
    a = torch.randn(K, M, generator=g)  # used transposed
    b = torch.randn(K, N, generator=g)
    mask = (torch.rand(M, N, generator=g) > 0.5).float()
    rs = torch.empty(M, device=DEV)
    out = ops.gemm(_cuda(a).t(), _cuda(b), mask=_cuda(mask), split_k=split, rowsum=rs)
    ref64 = (a.double().t() @ b.double()) * mask.double()
    ref32 = (a.t() @ b) * mask
    _check(out, ref64, ref32, f"gemm {M}x{N}x{K}")
    _check(rs, a.double().sum(0), a.sum(0), f"gemm {M}x{N}x{K} fused row sums (bias gradient)")


@pytest.mark.parametrize("M,N,K,masked,acc", [(512, 432, 65573, True, False), (172, 512, 70001, False, True),
                                                (428, 300, 2048, False, False), (100, 97, 9000, True, True),
                                                (88, 512, 65536, False, True), (84, 88, 4096, True, False)])
def test_gemm_tn128_wide_reductions(M, N, K, masked, acc):
    """The 128 x 128-tile batch reduction (gemm_tn128_kernel: dW of a 512-wide MADE's degree blocks,
    flows/maf_grad_wide.py) on strided column views of wider row-major buffers, ragged tiles and
    chunks, split-K atomics, the fused row sums, an output mask and accumulation, vs fp64."""
    from naz_amd import ops
    g = torch.Generator().manual_seed(M * 3 + N)
    ga = torch.randn(K, M + 9, generator=g)  # G = ga[:, 5:5+M] (row stride M + 9)
    xb = torch.randn(K, N + 3, generator=g)
    a, b = ga[:, 5:5 + M], xb[:, 1:1 + N]
    mask = (torch.rand(M, N, generator=g) > 0.3).float() if masked else None
    c0 = torch.randn(M, N, generator=g) if acc else torch.zeros(M, N)
    r0 = torch.randn(M, generator=g) if acc else torch.zeros(M)
    out, rs = _cuda(c0).clone(), _cuda(r0).clone()
    ops.gemm(_cuda(ga)[:, 5:5 + M].t(), _cuda(xb)[:, 1:1 + N], out=out, mask=None if mask is None else _cuda(mask),
             accumulate=acc, rowsum=rs)
    p64 = a.double().t() @ b.double()
    p32 = a.t() @ b
    if mask is not None:
        p64, p32 = p64 * mask.double(), p32 * mask
    _check(out, p64 + c0.double(), p32 + c0, f"gemm_tn128 {M}x{N}x{K}")
    _check(rs, a.double().sum(0) + r0.double(), a.sum(0) + r0, f"gemm_tn128 {M}x{N}x{K} row sums")


@pytest.mark.parametrize("N1,N2,M", [(192, 128, 70001), (128, 128, 4096), (128, 40, 33333), (184, 128, 517),
                                     (60, 20, 1000), (256, 96, 20000), (100, 52, 16), (4, 4, 9), (128, 8, 1 << 18),
                                     # the deep-ring (3-4 slot) instances: fewer chunks than slots,
                                     # a ragged last chunk, one or two chunks per workgroup, full size
                                     (192, 128, 32), (192, 128, 95), (128, 128, 33), (128, 128, 200),
                                     (128, 40, 100), (160, 8, 64), (192, 128, (1 << 20) + 77)])
def test_wgrad_t16_shapes(N1, N2, M):
    """dW = G^T X (+ column sums of G) on contiguous row-major operands: the LDS-ring reductions
    (bf16x6 with two- or deep rings, fp32 16x16x4; unmasked padding blocks, partial tail chunk) vs fp64."""
    from naz_amd import ops
    g = torch.Generator().manual_seed(N1 * 131 + N2 + M)
    a = torch.randn(M, N1, generator=g)
    b = torch.randn(M, N2, generator=g)
    rs = torch.empty(N1, device=DEV)
    out = ops.gemm(_cuda(a).t(), _cuda(b), rowsum=rs)
    _check(out, a.double().t() @ b.double(), a.t() @ b, f"wgrad {N1}x{N2} M={M}")
    _check(rs, a.double().sum(0), a.sum(0), f"wgrad {N1}x{N2} M={M} row sums")


@pytest.mark.parametrize("N1,N2", [(128, 40), (128, 128), (192, 128)])
@pytest.mark.parametrize("M", [1, 31, 32, 33, 257 * 32 + 5, (1 << 19) + 3])
def test_wgrad_nsc_shapes_masked_accumulate(N1, N2, M):
    """The nsc backward's three per-layer reductions (dPre1 x [ctx | x1], dPre2 x H1, dPre3 x H2 at
    config 3) on wgrad_x6: fewer chunks than workgroups, one partial chunk, a ragged tail, half a
    million rows; an output mask and accumulation into existing dW / db, vs fp64 (and the fp32
    reference's own error, tests/parity.py's criterion)."""
    from naz_amd import ops
    g = torch.Generator().manual_seed(N1 + 7 * N2 + M)
    a = torch.randn(M, N1, generator=g) * 1e-3  # dPre-like magnitudes
    b = torch.tanh(torch.randn(M, N2, generator=g))
    mask = (torch.rand(N1, N2, generator=g) > 0.25).float()
    c0, r0 = torch.randn(N1, N2, generator=g), torch.randn(N1, generator=g)
    out, rs = _cuda(c0).clone(), _cuda(r0).clone()
    ops.gemm(_cuda(a).t(), _cuda(b), out=out, mask=_cuda(mask), accumulate=True, rowsum=rs)
    _check(out, (a.double().t() @ b.double()) * mask.double() + c0.double(), (a.t() @ b) * mask + c0,
           f"wgrad nsc {N1}x{N2} M={M}")
    _check(rs, a.double().sum(0) + r0.double(), a.sum(0) + r0, f"wgrad nsc {N1}x{N2} M={M} row sums")


# ------------------------------------------------------------------ a5 affine step VJP
@pytest.mark.parametrize("N1,N2,M,nb", [(160, 160, 65536, 3), (160, 8, 3000, 3), (8, 160, 4097, 5), (160, 144, 517, 2),
                                        (128, 128, 70001, 1)])
def test_wgrad_batched_shapes(N1, N2, M, nb):
    """naz_wgrad_batched (the fused maf backward's dW of all layers in one launch, bf16x6): every
    reduction c[b] += G[b]^T X[b], rowsum[b] += column sums of G[b], into strided workspace views,
    vs fp64; N2 up to 160 (the maf's 150-wide hidden layers padded) and ragged row counts."""
    from naz_amd import ops
    g = torch.Generator().manual_seed(N1 * 7 + N2 + M + nb)
    a = torch.randn(nb, M, N1, generator=g)
    b = torch.randn(nb, M, N2, generator=g)
    ws = torch.zeros(nb, N1 * N2 + N1 + 4, device=DEV)  # padded workspace rows, as flows/maf_grad.py
    c = ws[:, :N1 * N2].view(nb, N1, N2)
    rs = ws[:, N1 * N2:N1 * N2 + N1]
    ops.wgrad_batched(_cuda(a), _cuda(b), c, rs)
    ops.wgrad_batched(_cuda(a), _cuda(b), c, rs)  # accumulates
    for k in range(nb):
        _check(c[k] / 2, a[k].double().t() @ b[k].double(), a[k].t() @ b[k], f"wgrad batch {k} {N1}x{N2} M={M}")
        _check(rs[k] / 2, a[k].double().sum(0), a[k].sum(0), f"wgrad batch {k} row sums")
    assert float(ws[:, -4:].abs().max()) == 0.0, "wrote past the reduction"


@pytest.mark.parametrize("inverse", [False, True])
def test_affine_ar_grad(inverse):
    from naz_amd import autograd as ag
    rng = np.random.default_rng(5)
    B, D = 2000, 5
    x = rng.standard_normal((B, D)).astype(np.float32)
    raw = (rng.standard_normal((B, 2 * D)) * 3).astype(np.float32)  # exercises both clip ends
    gy = rng.standard_normal((B, D)).astype(np.float32)
    gl = rng.standard_normal(B).astype(np.float32)

    def ref(dt):
        xo = torch.as_tensor(x, dtype=dt).requires_grad_(True)
        ro = torch.as_tensor(raw, dtype=dt).requires_grad_(True)
        mean, ls = ro[:, :D], O._clamp(ro[:, D:], -5.0, 3.0)
        y = (xo - mean) * torch.exp(-ls) if inverse else torch.exp(ls) * xo + mean
        loss = (y * torch.as_tensor(gy, dtype=dt)).sum() + (ls.sum(-1) * torch.as_tensor(gl, dtype=dt)).sum()
        return torch.autograd.grad(loss, [xo, ro])

    xg = _cuda(x).requires_grad_(True)
    rg = _cuda(raw).requires_grad_(True)
    y, ld = ag.affine_ar(xg, rg, inverse)
    gx, gr = torch.autograd.grad((y * _cuda(gy)).sum() + (ld * _cuda(gl)).sum(), [xg, rg])
    (x64, r64), (x32, r32) = ref(torch.float64), ref(torch.float32)
    _check(gx, x64, x32, f"affine inv={inverse} d/dx")
    _check(gr, r64, r32, f"affine inv={inverse} d/draw")


# ------------------------------------------------------------------ a10: whole-flow NLL gradient
def _product_flow(spec, state):
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    ft = spec["flow_type"]
    if ft == "nsc":
        f = NormalizingFlow("nsc", None, spec["D"], spec["C"], spec["hidden"], spec["L"], spec["K"], spec["split"])
    elif ft == "nsa":
        f = NormalizingFlow("nsa", None, spec["D"], spec["C"], spec["hidden"], spec["L"], spec["K"])
    else:
        f = NormalizingFlow("maf", None, spec["D"], spec["C"], spec["hidden"], spec["L"])
    fio.load_state(f, state)
    return f


def _oracle_nll_grads(spec, state, x, ctx, dt):
    st = {}
    for k, v in state.items():
        v = np.asarray(v)
        st[k] = (torch.as_tensor(v) if v.dtype.kind in "iu" else
                 torch.as_tensor(v).to(dt).requires_grad_(True))
    of = O.build_flow(spec, st, dt)
    c = None if ctx is None else torch.as_tensor(ctx).to(dt)
    lp = of.log_prob(torch.as_tensor(x).to(dt), c)
    loss = -lp.mean()
    keys = [k for k in st if st[k].requires_grad]
    gs = torch.autograd.grad(loss, [st[k] for k in keys])
    return lp.detach(), dict(zip(keys, gs))


@pytest.mark.parametrize("name", ["nsc_d16c32_l2.npz", "nsc_d8c0_l6.npz", "nsc_d6c2_small.npz", "nsa_d4c2.npz",
                                  "maf_d3c2.npz", "maf_twomoons.npz"])
def test_flow_nll_gradient_vs_oracle(name):
    """loss = -log_prob(x | ctx).mean() -> backward (naz/trainers/train_flows.py:195,208):
    every parameter's gradient against the oracle's float64 autograd."""
    from naz_amd.flows import io as fio
    fx = load_golden(name)
    spec, state = spec_state(fx)
    x, ctx = fx["x"], fx.get("ctx")
    if name == "maf_twomoons.npz":
        x = x[:512]
    f = _product_flow(spec, state)
    lp = f.log_prob(_cuda(x), condition=None if ctx is None else _cuda(ctx))
    assert lp.requires_grad, "grad mode with trainable weights must record the autograd walk"
    (-lp.mean()).backward()
    lp64, g64 = _oracle_nll_grads(spec, state, x, ctx, torch.float64)
    lp32, g32 = _oracle_nll_grads(spec, state, x, ctx, torch.float32)
    assert_parity(_np(lp), _np(lp64), _np(lp32), what=f"{name} graph-walk log_prob")
    params = fio.named_state_params(f)
    assert set(params) == set(g64), "canonical parameter sets differ"
    for k, p in params.items():
        assert p.grad is not None, f"{k}: no gradient"
        _check(p.grad, g64[k], g32[k], f"{name} d/d{k}")


def test_graph_walk_matches_fused_inference():
    """The autograd walk and the fused inference launch evaluate the same density."""
    fx = load_golden("nsc_d16c32_l2.npz")
    spec, state = spec_state(fx)
    f = _product_flow(spec, state)
    assert f.fused
    x, c = _cuda(fx["x"]), _cuda(fx["ctx"])
    lp_graph = f.log_prob(x, condition=c)
    with torch.no_grad():
        lp_fused = f.log_prob(x, condition=c)
    assert lp_graph.requires_grad and not lp_fused.requires_grad
    assert_parity(_np(lp_graph), fx["lp64"], fx["lp32"], what="graph walk")
    assert_parity(_np(lp_fused), fx["lp64"], fx["lp32"], what="fused")


@pytest.mark.parametrize("ftype,extra,C", [("nsc", (8, 8), 32), ("maf", (), 2), ("nsa", (8,), 2)])
def test_chain_node_matches_per_layer_walk(monkeypatch, ftype, extra, C):
    """The conditioner chain as one autograd node (ChainFn: act' fused into the dX GEMM
    epilogue by naz_gemm_dact) gives the per-layer LinearActFn walk's gradients."""
    from naz_amd import nn as nnmod
    from naz_amd.flows import NormalizingFlow
    D = 16 if ftype == "nsc" else 4
    torch.manual_seed(0)
    f = NormalizingFlow(ftype, None, D, C, [64, 64], 2, *extra).to(DEV)
    x = torch.randn(2048, D, device=DEV)
    c = torch.randn(2048, C, device=DEV)
    grads = {}
    for node in (True, False):
        monkeypatch.setattr(nnmod, "_CHAIN_NODE", node)
        f.zero_grad()
        (-f.log_prob(x, condition=c).mean()).backward()
        grads[node] = [p.grad.detach().clone() for p in f.parameters() if p.grad is not None]
    assert len(grads[True]) == len(grads[False]) > 0
    for a, b in zip(grads[True], grads[False]):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-7 * float(b.abs().max()) + 1e-12), (a - b).abs().max()


@pytest.mark.parametrize("D,C,hidden", [(4, 2, [64, 64]), (16, 32, [128, 128])])
def test_nsa_scheduled_differentiable_inverse_matches_d_pass(D, C, hidden):
    """nsa training walk: the degree-scheduled differentiable inverse (ARInversePlan.run_grad,
    every MADE unit once) gives pyro's D-pass gradients (degree_schedule off)."""
    from naz_amd.flows import NormalizingFlow
    torch.manual_seed(3)
    f = NormalizingFlow("nsa", None, D, C, hidden, 2, 8).to(DEV)
    x = torch.randn(1024, D, device=DEV) * 1.5
    c = torch.randn(1024, C, device=DEV)
    out = {}
    for on in (True, False):
        for net in f.nets:
            net.degree_schedule = on
        f.zero_grad()
        lp = f.log_prob(x, condition=c)
        (-lp.mean()).backward()
        out[on] = (lp.detach(), [p.grad.detach().clone() for p in f.parameters() if p.grad is not None])
    assert torch.allclose(out[True][0], out[False][0], rtol=1e-5, atol=1e-5)
    assert len(out[True][1]) == len(out[False][1]) > 0
    for a, b in zip(out[True][1], out[False][1]):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-5 * float(b.abs().max()) + 1e-12), (a - b).abs().max()
