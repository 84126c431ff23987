"""Batched-over-parameters affine MAF (naz_amd.flows.bflow_maf): the
Bayesian front end's ``make_normalizing_flow(...)["lp"]`` / ``["sampler"]`` (naz
bflow_jax_maf.py:196-225) evaluated for P weight draws at once.

CPU: the per-draw pack (gather map built from index-valued weights) reproduces the degree
schedule of the real weights, and ravel/unravel follow ``ravel_pytree`` order.
GPU: every draw's log_prob vs the numpy restatement of the reference's own JAX MAF
(oracle/jax_maf_np.py) in float64, with its float32 run as ref32 (tests/parity.py); sampler
vs the restated forward pass on the same base draws; the single-draw functions vs the
batched ones; the sample -> log_prob round trip."""
import numpy as np
import pytest
import torch

from oracle import jax_maf_np as J
from oracle import naz_oracle as O
from tests.parity import assert_parity

CASES = [
    dict(flow_type="maf", D=2, C=2, hidden=[150, 150, 150], L=3, P=6, B=700, ctx="vec"),  # paper shape
    dict(flow_type="maf", D=4, C=0, hidden=[32, 32], L=2, P=5, B=513, ctx=None),
    dict(flow_type="maf", D=3, C=5, hidden=[40, 24], L=2, P=3, B=300, ctx="rows"),
]


def _setup(spec, seed=7):
    """Base weights (the MLE flow), P perturbed draws as the Bayesian model makes them
    (params = flat * (1 + scale * u), u ~ U(-1, 1), bflow_jax_maf.py:224-226), eval rows."""
    st = {k: v.numpy() for k, v in O.random_state(spec, seed=seed).items()}
    layers = J.layers_from_state(spec, st)  # [(params64, perm, masks64)] in flow order
    rng = np.random.default_rng(seed)
    P, B, D, C = spec["P"], spec["B"], spec["D"], spec["C"]
    draws = []
    for _ in range(P):
        draws.append([[(W * (1 + 0.25 * rng.uniform(-1, 1, W.shape)), b * (1 + 0.25 * rng.uniform(-1, 1, b.shape)))
                       for (W, b) in params] for params, _, _ in layers])
    draws = [[[(W.astype(np.float32).astype(np.float64), b.astype(np.float32).astype(np.float64))
               for (W, b) in lay] for lay in d] for d in draws]
    x = (1.5 * rng.standard_normal((B, D))).astype(np.float32)
    ctx = None
    if spec["ctx"] == "vec":
        ctx = rng.standard_normal(C).astype(np.float32)
    elif spec["ctx"] == "rows":
        ctx = rng.standard_normal((B, C)).astype(np.float32)
    return layers, draws, x, ctx


def _oracle_layers(layers, draw):
    return [(draw[l], perm, masks) for l, (_, perm, masks) in enumerate(layers)]


def _batched_params(draws, dev):
    """[P] pytrees -> one pytree with a leading draw axis (what jax.vmap(unravel_fn) gives)."""
    L, n = len(draws[0]), len(draws[0][0])
    return [[(torch.tensor(np.stack([d[l][i][0] for d in draws]), dtype=torch.float32, device=dev),
              torch.tensor(np.stack([d[l][i][1] for d in draws]), dtype=torch.float32, device=dev))
             for i in range(n)] for l in range(L)]


def _flow(spec, layers, x, ctx, dev, **kw):
    from naz_amd.flows import bflow_maf as BM
    nn_spec, _, _ = BM.make_conditional_autoregressive_nn(spec["D"], spec["C"], spec["hidden"])
    tr = BM.make_masked_affine_autoregressive_transform(nn_spec, spec["D"])
    masks = [[torch.tensor(m, dtype=torch.float32) for m in ms] for _, _, ms in layers]
    perms = [torch.tensor(p) for _, p, _ in layers]
    c = None if ctx is None else torch.tensor(ctx, device=dev)
    return BM.make_normalizing_flow(tr, torch.tensor(x, device=dev), masks, [None] * len(layers), perms,
                                    context=c, **kw)


# ----------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("spec", CASES[:2], ids=lambda s: f"D{s['D']}C{s['C']}")
def test_pack_gather_map_matches_schedule(spec):
    """The gather map (schedule on index-valued weights) picks exactly the entries the degree
    schedule places when run on the real weights (naz_amd.nn.degree_schedule)."""
    from naz_amd.flows import bflow_maf as BM
    from naz_amd.nn import degree_schedule
    layers, draws, _, _ = _setup(spec)
    nn_spec, _, _ = BM.make_conditional_autoregressive_nn(spec["D"], spec["C"], spec["hidden"])
    for l, (_, perm, masks) in enumerate(layers):
        plan = BM._LayerPlan([torch.tensor(m) for m in masks], torch.tensor(perm), nn_spec)
        params = draws[0][l]
        F = torch.cat([torch.zeros(1, dtype=torch.float64)] +
                      [torch.cat((torch.tensor(W).reshape(-1), torch.tensor(b))) for (W, b) in params])
        assert F.numel() == plan.size
        widths, hidden, outs = degree_schedule(
            torch.tensor(perm), [torch.tensor(m) for m in masks], [torch.tensor(W) for W, _ in params],
            [torch.tensor(b) for _, b in params], spec["D"], spec["C"], 2)
        assert widths == plan.widths
        for g in range(spec["D"]):
            assert len(hidden[g]) == len(plan.hidden[g])
            for (li, a, b, n, wb, bb), (li2, a2, b2, n2, wi, bi) in zip(hidden[g], plan.hidden[g]):
                assert (li, a, b, n) == (li2, a2, b2, n2)
                assert torch.equal(F[wi], wb) and torch.equal(F[bi], bb)
        for (i, n, wb, bb), (i2, n2, wi, bi) in zip(outs, plan.outs):
            assert (i, n) == (i2, n2)
            assert torch.equal(F[wi], wb) and torch.equal(F[bi], bb)


def test_ravel_unravel_roundtrip():
    from naz_amd.flows import bflow_maf as BM
    spec = CASES[0]
    _, shapes, _ = BM.make_conditional_autoregressive_nn(spec["D"], spec["C"], spec["hidden"])
    shapes = [shapes] * 2
    n = sum(int(np.prod(w)) + int(np.prod(b)) for layer in shapes for (w, b) in layer)
    flat = torch.randn(3, n)
    tree = BM.unravel(flat, shapes)
    assert tree[0][0][0].shape == (3, 150, 4) and tree[1][-1][1].shape == (3, 4)
    assert torch.equal(BM.ravel(tree), flat)
    assert torch.equal(tree[0][0][0][1].reshape(-1), flat[1, :600])  # leaf order = ravel_pytree's
    with pytest.raises(ValueError):
        BM.unravel(flat[:, :-1], shapes)


def test_rejects_unbuilt_options():
    from naz_amd.flows import bflow_maf as BM
    with pytest.raises(NotImplementedError):
        BM.make_conditional_autoregressive_nn(2, 2, [8], skip_connections=True)
    with pytest.raises(NotImplementedError):
        BM.make_conditional_autoregressive_nn(2, 2, [8], param_dims=[1, 1, 1])


# ----------------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.gpu
@pytest.mark.parametrize("spec", CASES, ids=lambda s: f"D{s['D']}C{s['C']}P{s['P']}")
def test_lp_batched_vs_oracle(_gpu, spec):
    layers, draws, x, ctx = _setup(spec)
    flow = _flow(spec, layers, x, ctx, "cuda")
    lp = flow["lp_batched"](_batched_params(draws, "cuda")).cpu().numpy()
    assert lp.shape == (spec["P"], spec["B"])
    for p, d in enumerate(draws):
        ol = _oracle_layers(layers, d)
        ref64 = J.log_prob(x, ol, ctx)
        ref32 = J.log_prob(x, J.cast_layers(ol, np.float32), ctx, np.float32)
        assert_parity(lp[p], ref64, ref32, what=f"lp_batched draw {p}")


@pytest.mark.gpu
def test_lp_single_equals_batched(_gpu):
    spec = CASES[0]
    layers, draws, x, ctx = _setup(spec)
    flow = _flow(spec, layers, x, ctx, "cuda")
    batched = flow["lp_batched"](_batched_params(draws, "cuda"))
    one = _batched_params(draws[2:3], "cuda")
    single = flow["lp"]([[(w[0], b[0]) for (w, b) in layer] for layer in one])
    assert torch.equal(single, batched[2])


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [CASES[0], CASES[1]], ids=lambda s: f"D{s['D']}C{s['C']}")
def test_sampler_batched_vs_oracle(_gpu, spec):
    layers, draws, x, ctx = _setup(spec)
    flow = _flow(spec, layers, x, ctx, "cuda")
    S = 400
    z = np.random.default_rng(3).standard_normal((spec["P"], S, spec["D"])).astype(np.float32)
    y, lj = flow["sampler_batched"](_batched_params(draws, "cuda"), size=S, z=torch.tensor(z, device="cuda"))
    y, lj = y.cpu().numpy(), lj.cpu().numpy()
    for p, d in enumerate(draws):
        ol = _oracle_layers(layers, d)
        y64, lj64 = J.sample_from_z(z[p], ol, ctx)
        y32, lj32 = J.sample_from_z(z[p], J.cast_layers(ol, np.float32), ctx, np.float32)
        assert_parity(y[p], y64, y32, what=f"sampler y draw {p}")
        assert_parity(lj[p], lj64, lj32, what=f"sampler log_j draw {p}")


@pytest.mark.gpu
def test_sample_logprob_roundtrip_and_rng(_gpu):
    """log p(y) of the sampled y under the same draw = 2 base(z) - log_j (the sampler's log_j
    is base(z) + Σ ls, bflow_jax_maf.py:220); seeded sampling is reproducible."""
    spec = CASES[0]
    layers, draws, x, ctx = _setup(spec)
    flow = _flow(spec, layers, x, ctx, "cuda")
    params = _batched_params(draws, "cuda")
    S = 2048
    z = torch.randn((spec["P"], S, spec["D"]), device="cuda", generator=torch.Generator("cuda").manual_seed(5))
    y, lj = flow["sampler_batched"](params, size=S, z=z)
    base = (-0.5 * (z.double() ** 2).sum(-1) - spec["D"] / 2 * np.log(2 * np.pi))
    for p in range(spec["P"]):
        f1 = _flow(spec, layers, y[p].cpu().numpy(), ctx, "cuda")
        one = [[(w[p:p + 1], b[p:p + 1]) for (w, b) in layer] for layer in params]
        lp = f1["lp_batched"](one)[0].double()
        want = 2 * base[p] - lj[p].double()
        err = ((lp - want).abs() / want.abs().clamp(min=1)).cpu().numpy()
        assert np.quantile(err, 0.99) < 1e-4 and err.max() < 1e-3, (np.median(err), err.max())
    y1, _ = flow["sampler_batched"](params, 11, S)
    y2, _ = flow["sampler_batched"](params, 11, S)
    assert torch.equal(y1, y2) and bool(torch.isfinite(y1).all())


def _emulate_made_fwd(packed, nhid, nh, C, D, ctx, x):
    """numpy model of made.hip's lane/register mapping (v_mfma_f32_32x32x2_f32: lane l supplies
    A[l % 32][l // 32] and B[l // 32][l % 32]; D[m][n] sits in lane n + 32((m >> 2) & 1), register
    (m & 3) + 4(m >> 3)) for one wave of 32 rows; returns y and Σ clamp(ls)."""
    lane = np.arange(64)
    regs_m = lambda r, l: (r & 3) + 8 * (r >> 2) + 4 * (l >> 5)  # noqa: E731

    def mfma_steps(A, Bsteps):  # A [steps][64] values, Bsteps [steps][64] -> acc [16][64]
        acc = np.zeros((32, 32))
        for a, b in zip(A, Bsteps):
            Am = np.stack([a[:32], a[32:]], 1)  # [m][k]
            Bm = np.stack([b[:32], b[32:]], 0)  # [k][n]
            acc += Am @ Bm
        r, l = np.meshgrid(np.arange(16), lane, indexing="ij")
        return acc[regs_m(r, l), l % 32]

    s0 = ((C + D + 1) // 2 + 3) // 4 * 4
    pos = 0

    def take(n):
        nonlocal pos
        v = packed[pos:pos + n]
        pos += n
        return v
    inp = np.concatenate([np.broadcast_to(ctx, (32, C)), x], 1) if C else x
    A0 = take(nh * s0 * 64).reshape(nh, s0 // 4, 64, 4).transpose(0, 1, 3, 2).reshape(nh, s0, 64)
    B0 = np.zeros((s0, 64))
    for s in range(s0):
        k = 2 * s + lane // 32
        B0[s] = np.where(k < C + D, inp[lane % 32, np.minimum(k, C + D - 1)], 0)
    b = take(nh * 1024).reshape(nh, 16, 64)
    hv = np.tanh(np.stack([mfma_steps(A0[o], B0) for o in range(nh)]) + b)
    for _ in range(1, nhid):
        A = take(nh * nh * 1024).reshape(nh * 4, nh, 64, 4).transpose(1, 0, 3, 2).reshape(nh, nh * 16, 64)
        Bs = hv.reshape(nh * 16, 64)
        b = take(nh * 1024).reshape(nh, 16, 64)
        hv = np.tanh(np.stack([mfma_steps(A[o], Bs) for o in range(nh)]) + b)
    A = take(nh * 1024).reshape(nh * 4, 64, 4).transpose(0, 2, 1).reshape(nh * 16, 64)
    out = mfma_steps(A, hv.reshape(nh * 16, 64)) + take(1024).reshape(16, 64)
    assert pos == packed.size
    raw = np.zeros((32, 32))
    r, l = np.meshgrid(np.arange(16), lane, indexing="ij")
    raw[l % 32, regs_m(r, l)] = out
    ls = np.clip(raw[:, D:2 * D], -5, 3)
    return raw[:, :D] + x * np.exp(ls), ls.sum(1)


@pytest.mark.parametrize("spec", CASES, ids=lambda s: f"D{s['D']}C{s['C']}")
def test_made_pack_map_against_lane_model(spec):
    """The fused forward kernel's packed layout, read the way made.hip reads it (numpy model of
    the MFMA lane mapping), gives the reference's forward_fn (bflow_jax_maf.py:172-178)."""
    from naz_amd.flows import bflow_maf as BM
    layers, draws, _, _ = _setup(spec)
    nn_spec, _, _ = BM.make_conditional_autoregressive_nn(spec["D"], spec["C"], spec["hidden"])
    nh = (max(spec["hidden"]) + 31) // 32
    D, C = spec["D"], spec["C"]
    rng = np.random.default_rng(0)
    x = rng.standard_normal((32, D))
    ctx = rng.standard_normal(C) if C else None
    for l, (_, perm, masks) in enumerate(layers[:2]):
        mp = BM.made_pack_map(nn_spec, [torch.tensor(m) for m in masks], nh).numpy()
        params = draws[0][l]
        F = np.concatenate([[0.0]] + [np.concatenate((W.reshape(-1), b)) for (W, b) in params])
        y, ld = _emulate_made_fwd(F[mp], len(spec["hidden"]), nh, C, D, ctx, x)
        y64, ld64 = J.forward_fn(x, params, masks, ctx)
        np.testing.assert_allclose(y, y64, rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(ld, ld64, rtol=1e-10, atol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("D,C,hidden,ctx_rows", [(2, 2, [150, 150, 150], False), (4, 3, [64, 40], True),
                                                 (5, 0, [37], False)])
def test_naz_maf_forward_uses_fused_kernel(_gpu, D, C, hidden, ctx_rows):
    """naz_amd's NormalizingFlow("maf") forward direction (AffineAutoregressive._call, used by
    sample) runs as one naz_made_affine_fwd launch per layer under no_grad; it matches the
    per-GEMM path (naz_linear_act chain + naz_affine_ar) and the fp64 oracle layer."""
    from naz_amd import ops
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    from naz_amd.flows.transforms import _fused_made_forward
    spec = dict(flow_type="maf", D=D, C=C, hidden=hidden, L=2)
    st = {k: v.float() for k, v in O.random_state(spec, seed=3).items()}
    f = NormalizingFlow("maf", None, D, C, hidden, 2)
    fio.load_state(f, {k: v.numpy() for k, v in st.items()})
    rng = np.random.default_rng(1)
    B = 1000
    x = torch.tensor(rng.standard_normal((B, D)).astype(np.float32), device="cuda")
    ctx = None
    if C:
        ctx = torch.tensor(rng.standard_normal((B, C) if ctx_rows else (C,)).astype(np.float32), device="cuda")
    layers = J.layers_from_state(spec, {k: v.numpy() for k, v in st.items()})
    with torch.no_grad():
        for l, t in enumerate(f.transforms[:1]):
            arn = t.nn
            ld_f = torch.zeros(B, device="cuda")
            y_f = _fused_made_forward(arn, x, ctx, ld_f, ops.LD_ROWSUM_ADD)
            assert y_f is not None, "fused MADE forward not taken"
            ld_g = torch.zeros(B, device="cuda")
            y_g, _ = ops.affine_ar(x, arn.raw(x, ctx), False, ops.LD_ROWSUM_ADD, ld_g)
            assert torch.allclose(y_f, y_g, rtol=1e-5, atol=1e-5) and torch.allclose(ld_f, ld_g, rtol=1e-5, atol=1e-5)
            params, perm, masks = layers[l]
            y64, ld64 = J.forward_fn(x.cpu().double().numpy(), params, masks,
                                     None if ctx is None else ctx.cpu().double().numpy())
            assert_parity(y_f.cpu().numpy(), y64, what="fused maf forward y", strict=True)
            assert_parity(ld_f.cpu().numpy(), ld64, what="fused maf forward ld", strict=True)


def test_torch_to_jax_layout():
    """torch_to_jax (bflow_jax_maf.py:26-46) over a naz_amd maf flow: per layer (W, b) per MADE
    linear in ravel order, the masks, mask_skip and permutation; shapes = the spec's."""
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import bflow_maf as BM
    f = NormalizingFlow("maf", None, 2, 2, [150, 150, 150], 3)
    params, shapes, masks, skips, perms = BM.torch_to_jax(f)
    _, want, _ = BM.make_conditional_autoregressive_nn(2, 2, [150, 150, 150])
    assert len(params) == 3 and all(sh == [(tuple(w), tuple(b)) for (w, b) in want] for sh in shapes)
    arn = f.transforms[0].nn
    assert torch.equal(params[0][1][0], arn.layers[1].weight.detach())
    assert all(torch.equal(m, a.float()) for m, a in zip(masks[0], arn.masks))
    assert torch.equal(perms[0], arn.permutation) and skips[0].shape == (4, 4)
    assert BM.ravel(params).numel() == sum(p.numel() for p in f.parameters())


@pytest.mark.gpu
@pytest.mark.parametrize("D,C,hidden", [(2, 2, [150, 150, 150]), (4, 3, [64, 40]), (3, 5, [33, 20, 17])])
def test_lp_context_folding(_gpu, D, C, hidden):
    """One context vector: the degree-0 (context-only) MADE units evaluated once per draw and
    folded into biases give the plain degree schedule's log_prob and the oracle's."""
    spec = dict(flow_type="maf", D=D, C=C, hidden=hidden, L=2, P=4, B=600, ctx="vec")
    layers, draws, x, ctx = _setup(spec)
    params = _batched_params(draws, "cuda")
    a = _flow(spec, layers, x, ctx, "cuda", fused_ar=False)["lp_batched"](params)
    b = _flow(spec, layers, x, ctx, "cuda", fold_context=False, fused_ar=False)["lp_batched"](params)
    assert torch.allclose(a, b, rtol=2e-5, atol=2e-5), (a - b).abs().max()
    for p, d in enumerate(draws):
        ol = _oracle_layers(layers, d)
        assert_parity(a[p].cpu().numpy(), J.log_prob(x, ol, ctx),
                      J.log_prob(x, J.cast_layers(ol, np.float32), ctx, np.float32), what=f"folded lp draw {p}")


@pytest.mark.gpu
@pytest.mark.parametrize("ctx_kind", ["vec", "rows"])
def test_lp_and_grad_vs_oracle_autograd(_gpu, ctx_kind):
    """The NUTS potential Σ_rows lp(θ) and its gradient (bflow_jax_maf.py:233-235) from the HIP
    training walk vs the fp64 oracle's torch autograd (and its fp32 run as ref32)."""
    from naz_amd.flows import bflow_maf as BM
    spec = dict(flow_type="maf", D=2, C=2, hidden=[48, 48], L=3, P=2, B=1500, ctx=ctx_kind, clip_grad="zero")
    layers, draws, x, ctx = _setup(spec)
    flow = _flow(spec, layers, x, ctx, "cuda")
    d = draws[0]
    params = [[(torch.tensor(W, dtype=torch.float32, device="cuda"), torch.tensor(b, dtype=torch.float32,
                                                                                   device="cuda"))
               for (W, b) in lay] for lay in d]
    total, grad = flow["lp_and_grad"](params)
    total2, grad2 = flow["lp_and_grad"](BM.ravel(params))  # flat draw, second call reuses the flow
    # the dW reductions accumulate with fp32 atomics: equal up to summation order
    assert torch.equal(total, total2) and torch.allclose(grad, grad2, rtol=1e-5, atol=1e-6 * float(grad.abs().max()))
    assert "graph" in flow["grad_state"], "the gradient step was not captured as a HIP graph"
    total3, grad3 = flow["lp_and_grad"](params, use_graph=False)  # eager launches
    assert torch.allclose(total, total3, rtol=1e-6) and torch.allclose(grad, grad3, rtol=1e-5,
                                                                        atol=1e-6 * float(grad.abs().max()))
    d2 = draws[1] if len(draws) > 1 else d  # replay with new weights follows them
    p2 = BM.ravel([[(torch.tensor(W, dtype=torch.float32, device="cuda"), torch.tensor(b, dtype=torch.float32,
                                                                                        device="cuda"))
                    for (W, b) in lay] for lay in d2])
    t_g, g_g = flow["lp_and_grad"](p2)
    t_e, g_e = flow["lp_and_grad"](p2, use_graph=False)
    assert torch.allclose(t_g, t_e, rtol=1e-6) and torch.allclose(g_g, g_e, rtol=1e-5, atol=1e-6 * float(g_e.abs().max()))

    def oracle(dtype):
        st = {}
        for l, lay in enumerate(d):
            for i, (W, b) in enumerate(lay):
                st[f"layers.{l}.nn.layers.{i}.weight"] = torch.tensor(W, dtype=dtype, requires_grad=True)
                st[f"layers.{l}.nn.layers.{i}.bias"] = torch.tensor(b, dtype=dtype, requires_grad=True)
            st[f"layers.{l}.nn.permutation"] = torch.tensor(layers[l][1])
        f = O.build_flow(spec, st, dtype)
        xc = torch.tensor(x, dtype=dtype)
        cc = torch.tensor(ctx, dtype=dtype)
        cc = cc.expand(len(x), -1) if cc.dim() == 1 else cc
        lp = f.log_prob(xc, cc).sum()
        lp.backward()
        g = torch.cat([t.grad.reshape(-1) for l in range(len(d)) for i in range(len(d[0]))
                       for t in (st[f"layers.{l}.nn.layers.{i}.weight"], st[f"layers.{l}.nn.layers.{i}.bias"])])
        return lp.item(), g.numpy()
    lp64, g64 = oracle(torch.float64)
    lp32, g32 = oracle(torch.float32)
    assert abs(total.item() - lp64) / abs(lp64) < 1e-5
    from tests.parity import grad_floor
    assert_parity(grad.cpu().numpy(), g64, g32, what="NUTS potential gradient", floor=grad_floor(g64),
                  count_factor=None)


@pytest.mark.gpu
def test_lp_layer_batched_constants():
    """D = 2, one context vector: the per-draw constants / packs of all layers in single
    launches (_lp_chunk_const2) give the per-layer folded path's log_prob."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    spec = dict(flow_type="maf", D=2, C=2, hidden=[150, 150, 150], L=4, P=5, B=700, ctx="vec")
    layers, draws, x, ctx = _setup(spec)
    params = _batched_params(draws, "cuda")
    a = _flow(spec, layers, x, ctx, "cuda", fused_ar=False)["lp_batched"](params)
    b = _flow(spec, layers, x, ctx, "cuda", batch_layers=False, fused_ar=False)["lp_batched"](params)
    assert torch.allclose(a, b, rtol=1e-5, atol=1e-5), (a - b).abs().max()
    for p, d in enumerate(draws):
        ol = _oracle_layers(layers, d)
        assert_parity(a[p].cpu().numpy(), J.log_prob(x, ol, ctx),
                      J.log_prob(x, J.cast_layers(ol, np.float32), ctx, np.float32), what=f"layer-batched lp {p}")


@pytest.mark.gpu
def test_lp_layer_batched_many_draws_few_rows():
    """L x P beyond the batched launches' grid-z limit (65535) with few rows: the
    layer-batched constants path caps its draw chunks at 65535 // L and budgets the per-draw
    packs; the result equals the per-layer path draw for draw."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    spec = dict(flow_type="maf", D=2, C=2, hidden=[32, 32], L=4, P=1, B=8, ctx="vec")
    layers, draws, x, ctx = _setup(spec)
    base = _batched_params(draws, "cuda")
    P = 16500  # L * P = 66000 > 65535
    g = torch.Generator(device="cuda").manual_seed(0)

    def jitter(t):
        return t.expand(P, *t.shape[1:]) * (1 + 0.1 * (2 * torch.rand((P,) + tuple(t.shape[1:]), device="cuda",
                                                                      generator=g) - 1))
    params = [[(jitter(W), jitter(b)) for (W, b) in lay] for lay in base]
    a = _flow(spec, layers, x, ctx, "cuda")["lp_batched"](params)
    b = _flow(spec, layers, x, ctx, "cuda", batch_layers=False)["lp_batched"](params)
    assert a.shape == (P, spec["B"]) and bool(torch.isfinite(a).all())
    assert torch.allclose(a, b, rtol=1e-5, atol=1e-5), (a - b).abs().max()


@pytest.mark.gpu
@pytest.mark.parametrize("D", [2, 4])
def test_sampler_batched_fused_ar_paper_shape(_gpu, D):
    """At the paper shape (D=2 | C=2, H=[150]*3) and the 4-parameter Bayesian MAF (D=4,
    calibrate_4p.py:75) the batched sampler runs the whole flow for every draw in ONE
    naz_ar_flow_sample_batched launch (weights packed on the device per draw); against the numpy
    restatement of the reference's JAX sampler and the per-layer fused-MADE path."""
    spec = dict(D=D, C=2, hidden=[150, 150, 150], L=4, P=5, B=64, ctx="vec", flow_type="maf")
    layers, draws, x, ctx = _setup(spec)
    S = 700
    z = np.random.default_rng(4).standard_normal((spec["P"], S, spec["D"])).astype(np.float32)
    params = _batched_params(draws, "cuda")
    flow = _flow(spec, layers, x, ctx, "cuda")
    calls = []
    from naz_amd.flows import bflow_maf as BM
    orig = BM.ops.ar_flow_sample_batched
    BM.ops.ar_flow_sample_batched = lambda *a, **k: calls.append(1) or orig(*a, **k)
    try:
        y, lj = flow["sampler_batched"](params, size=S, z=torch.tensor(z, device="cuda"))
    finally:
        BM.ops.ar_flow_sample_batched = orig
    assert calls, "the fused batched AR sampler was not used"
    flow_made = _flow(spec, layers, x, ctx, "cuda", fused_ar=False)
    y_m, lj_m = flow_made["sampler_batched"](params, size=S, z=torch.tensor(z, device="cuda"))
    y, lj = y.cpu().numpy(), lj.cpu().numpy()
    for p, d in enumerate(draws):
        ol = _oracle_layers(layers, d)
        y64, lj64 = J.sample_from_z(z[p], ol, ctx)
        y32, lj32 = J.sample_from_z(z[p], J.cast_layers(ol, np.float32), ctx, np.float32)
        assert_parity(y[p], y64, y32, what=f"fused-AR sampler y draw {p}")
        assert_parity(lj[p], lj64, lj32, what=f"fused-AR sampler log_j draw {p}", count_factor=3.0)
    np.testing.assert_allclose(y, y_m.cpu().numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("D,P,B", [(2, 5, 700), (2, 3, 1), (4, 4, 900)])
def test_lp_batched_fused_ar_paper_shape(_gpu, D, P, B):
    """At the paper shape the batched log-density packs every draw's inverse image on the device
    (naz_ar_flow_pack) and runs the whole flow for all draws in ONE naz_ar_flow_log_prob_batched
    launch; against the numpy restatement of the reference's JAX log_prob, the layer-batched
    MADE path, and a flow whose masks are not pyro's create_mask (must not take the fused path)."""
    from naz_amd.flows import bflow_maf as BM
    spec = dict(D=D, C=2, hidden=[150, 150, 150], L=5, P=P, B=B, ctx="vec", flow_type="maf")
    layers, draws, x, ctx = _setup(spec)
    params = _batched_params(draws, "cuda")
    calls = []
    orig = BM.ops.ar_flow_log_prob_batched
    BM.ops.ar_flow_log_prob_batched = lambda *a, **k: calls.append(1) or orig(*a, **k)
    try:
        lp = _flow(spec, layers, x, ctx, "cuda")["lp_batched"](params)
        assert calls, "the fused batched AR log_prob was not used"
        # a mask that is not create_mask's for the permutation: the degree passes do not apply
        bad = [(p_, perm, [m.copy() for m in ms]) for (p_, perm, ms) in layers]
        bad[0][2][0][0, 0] = 0.0  # a context input of a degree-0 unit
        calls.clear()
        _flow(spec, bad, x, ctx, "cuda")["lp_batched"](params)
        assert not calls
    finally:
        BM.ops.ar_flow_log_prob_batched = orig
    ref = _flow(spec, layers, x, ctx, "cuda", fused_ar=False)["lp_batched"](params)
    assert torch.allclose(lp, ref, rtol=1e-4, atol=1e-4), (lp - ref).abs().max()
    # the same draws as unravel()'s views of one [P, n] buffer (the packers read it in place)
    flat_draws = BM.ravel(params)
    assert torch.equal(_flow(spec, layers, x, ctx, "cuda")["lp_batched"](BM.unravel(flat_draws, [
        [tuple(t.shape[1:] for t in wb) for wb in layer] for layer in params])), lp)
    # fold_context=False: the first degree pass computed per row instead of packed as constants
    lp_rows = _flow(spec, layers, x, ctx, "cuda", fold_context=False)["lp_batched"](params)
    assert torch.allclose(lp, lp_rows, rtol=1e-4, atol=1e-4), (lp - lp_rows).abs().max()
    lp = lp.cpu().numpy()
    for p, d in enumerate(draws):
        ol = _oracle_layers(layers, d)
        assert_parity(lp[p], J.log_prob(x, ol, ctx), J.log_prob(x, J.cast_layers(ol, np.float32), ctx, np.float32),
                      what=f"fused-AR lp draw {p}")


@pytest.mark.gpu
@pytest.mark.parametrize("D,ctx_kind,B", [(2, "rows", 1500), (2, "vec", 700), (2, "rows", 64), (4, "rows", 1300),
                                          (4, "vec", 64)])
def test_lp_and_grad_fused_maf_backward_vs_oracle(_gpu, D, ctx_kind, B):
    """The NUTS potential's gradient on the fused maf backward (maf_grad.py: the inverse kernel
    with saved states, made_ar_bwd_kernel per layer, batch-reduction dW) at the paper shape (D=2 |
    C=2, H=[150]x3) and the 4-parameter Bayesian MAF (D=4, calibrate_4p.py:75, hmc_maf_exact.py:
    101-133) vs the fp64 oracle's torch autograd with jnp.clip's gradient (ref32 = its fp32 run),
    vs the training walk, graph replay vs eager, and new weights through the replay; ragged rows."""
    from naz_amd.flows import bflow_maf as BM
    spec = dict(flow_type="maf", D=D, C=2, hidden=[150, 150, 150], L=3, P=2, B=B, ctx=ctx_kind, clip_grad="zero")
    layers, draws, x, ctx = _setup(spec, seed=11)
    flow = _flow(spec, layers, x, ctx, "cuda")
    assert flow["grad_fused"], "the paper shape must take the fused maf backward"
    walk = _flow(spec, layers, x, ctx, "cuda", fused_grad=False)
    assert not walk["grad_fused"]

    def flat_of(d):
        return BM.ravel([[(torch.tensor(W, dtype=torch.float32, device="cuda"),
                           torch.tensor(b, dtype=torch.float32, device="cuda")) for (W, b) in lay] for lay in d])
    p1 = flat_of(draws[0])
    total, grad = flow["lp_and_grad"](p1)
    assert "graph" in flow["grad_state"] and "mafgrad" in flow["grad_state"]
    t_e, g_e = flow["lp_and_grad"](p1, use_graph=False)
    assert torch.allclose(total, t_e, rtol=1e-6) and torch.allclose(grad, g_e, rtol=1e-5,
                                                                     atol=1e-6 * float(g_e.abs().max()))
    t_w, g_w = walk["lp_and_grad"](p1, use_graph=False)
    assert abs(total.item() - t_w.item()) <= 1e-5 * abs(t_w.item())
    assert torch.allclose(grad, g_w, rtol=1e-3, atol=1e-4 * float(g_w.abs().max())), \
        float((grad - g_w).abs().max() / g_w.abs().max())
    p2 = flat_of(draws[1])  # the replay follows new weights
    t_g, g_g = flow["lp_and_grad"](p2)
    t_e2, g_e2 = flow["lp_and_grad"](p2, use_graph=False)
    # the dW reductions add per-workgroup partials with fp32 atomics: equal up to summation order
    err = float((g_g - g_e2).abs().max() / g_e2.abs().max())
    assert torch.allclose(t_g, t_e2, rtol=1e-6) and err < 1e-5, err
    assert not torch.allclose(g_g, grad, rtol=1e-3), "the replay must follow the new weights"
    d = draws[0]

    def oracle(dtype):
        st = {}
        for l, lay in enumerate(d):
            for i, (W, b) in enumerate(lay):
                st[f"layers.{l}.nn.layers.{i}.weight"] = torch.tensor(W, dtype=dtype, requires_grad=True)
                st[f"layers.{l}.nn.layers.{i}.bias"] = torch.tensor(b, dtype=dtype, requires_grad=True)
            st[f"layers.{l}.nn.permutation"] = torch.tensor(layers[l][1])
        f = O.build_flow(spec, st, dtype)
        xc = torch.tensor(x, dtype=dtype)
        cc = torch.tensor(ctx, dtype=dtype)
        cc = cc.expand(len(x), -1) if cc.dim() == 1 else cc
        lp = f.log_prob(xc, cc).sum()
        lp.backward()
        g = torch.cat([t.grad.reshape(-1) for l in range(len(d)) for i in range(len(d[0]))
                       for t in (st[f"layers.{l}.nn.layers.{i}.weight"], st[f"layers.{l}.nn.layers.{i}.bias"])])
        return lp.item(), g.numpy()
    lp64, g64 = oracle(torch.float64)
    lp32, g32 = oracle(torch.float32)
    assert abs(total.item() - lp64) / abs(lp64) < 1e-5
    from tests.parity import grad_floor
    assert_parity(grad.cpu().numpy(), g64, g32, what="fused NUTS potential gradient", floor=grad_floor(g64),
                  count_factor=None)


@pytest.mark.gpu
@pytest.mark.parametrize("D", [2, 4])
def test_lp_and_grad_fused_full_size_properties(_gpu, D):
    """The §8f rank-1 workload (paper shape D=2 and the 4-parameter Bayesian MAF D=4, L=16, 2^16
    training rows, per-row contexts): the fused potential and gradient are finite, the potential
    bitwise reproducible, the gradient equal up to the dW reductions' summation order, and the
    potential equals the fused log-density's sum."""
    from naz_amd.flows import bflow_maf as BM
    spec = dict(flow_type="maf", D=D, C=2, hidden=[150, 150, 150], L=16, P=1, B=1 << 16, ctx="rows")
    layers, draws, x, ctx = _setup(spec, seed=5)
    flow = _flow(spec, layers, x, ctx, "cuda")
    assert flow["grad_fused"]
    p = BM.ravel([[(torch.tensor(W, dtype=torch.float32, device="cuda"),
                    torch.tensor(b, dtype=torch.float32, device="cuda")) for (W, b) in lay] for lay in draws[0]])
    t1, g1 = flow["lp_and_grad"](p)
    t2, g2 = flow["lp_and_grad"](p)
    assert bool(torch.isfinite(t1)) and bool(torch.isfinite(g1).all())
    assert torch.equal(t1, t2)
    assert torch.allclose(g1, g2, rtol=1e-5, atol=1e-6 * float(g1.abs().max()))
    mg = flow["grad_state"]["mafgrad"]
    lp_rows = mg._buffers(spec["B"])["lp"].clone()
    from naz_amd import ops
    xd, cd = torch.tensor(x, device="cuda"), torch.tensor(ctx, device="cuda")
    ref = ops.ar_flow_log_prob(mg.desc, ops.ar_flow_pack_batched(mg.desc, p[None], mg.perms, mask=mg.mask)[0],
                               xd, cd)
    assert torch.equal(lp_rows, ref), "the training forward must be the log_prob kernel's arithmetic"


def _oracle_grad(spec, layers, d, x, ctx, dtype, clip_grad):
    """Σ_rows log p and its gradient (ravel order) from the oracle's torch autograd."""
    st = {}
    for l, lay in enumerate(d):
        for i, (W, b) in enumerate(lay):
            st[f"layers.{l}.nn.layers.{i}.weight"] = torch.tensor(W, dtype=dtype, requires_grad=True)
            st[f"layers.{l}.nn.layers.{i}.bias"] = torch.tensor(b, dtype=dtype, requires_grad=True)
        st[f"layers.{l}.nn.permutation"] = torch.tensor(layers[l][1])
    f = O.build_flow(dict(spec, clip_grad=clip_grad), st, dtype)
    cc = torch.tensor(ctx, dtype=dtype)
    cc = cc.expand(len(x), -1) if cc.dim() == 1 else cc
    lp = f.log_prob(torch.tensor(x, dtype=dtype), cc).sum()
    lp.backward()
    g = torch.cat([t.grad.reshape(-1) for l in range(len(d)) for i in range(len(d[0]))
                   for t in (st[f"layers.{l}.nn.layers.{i}.weight"], st[f"layers.{l}.nn.layers.{i}.bias"])])
    return lp.item(), g.numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("D", [2, 4])
def test_lp_and_grad_clip_gradient_is_jnp_clip(_gpu, D):
    """the reference's JAX MAF clips log_scale with jnp.clip (bflow_jax_maf.py:177,188,
    192), whose gradient is ZERO outside [-5, 3]; pyro's clamp_preserve_gradients (naz's torch maf)
    passes it through.  Weights that drive many log_scales past the clip: the NUTS gradient (fused
    and walk) follows jnp.clip, and differs from the pass-through gradient; NormalizingFlow's maf
    NLL gradient keeps pyro's semantics."""
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import bflow_maf as BM
    from naz_amd.flows import io as fio
    from tests.parity import grad_floor
    spec = dict(flow_type="maf", D=D, C=2, hidden=[150, 150, 150], L=3, P=1, B=900, ctx="rows")
    layers, draws, x, ctx = _setup(spec, seed=13)
    d = [[(W, b) for (W, b) in lay] for lay in draws[0]]
    for lay in d:  # log_scale rows (D..2D-1) of the output layer: large weights and biases
        W, b = lay[-1]
        W, b = W.copy(), b.copy()
        W[D:] *= 40.0
        b[D:] += np.where(np.arange(D) % 2 == 0, 4.0, -5.5)
        lay[-1] = (W, b)
    flat = BM.ravel([[(torch.tensor(W, dtype=torch.float32, device="cuda"),
                       torch.tensor(b, dtype=torch.float32, device="cuda")) for (W, b) in lay] for lay in d])
    flow = _flow(spec, layers, x, ctx, "cuda")
    assert flow["grad_fused"]
    total, grad = flow["lp_and_grad"](flat, use_graph=False)
    walk = _flow(spec, layers, x, ctx, "cuda", fused_grad=False)
    t_w, g_w = walk["lp_and_grad"](flat, use_graph=False)
    lp64, g64 = _oracle_grad(spec, layers, d, x, ctx, torch.float64, "zero")
    lp32, g32 = _oracle_grad(spec, layers, d, x, ctx, torch.float32, "zero")
    _, gp64 = _oracle_grad(spec, layers, d, x, ctx, torch.float64, "preserve")
    # the case is exercised: the two clip semantics give visibly different gradients
    assert np.abs(g64 - gp64).max() > 1e-2 * np.abs(g64).max()
    assert abs(total.item() - lp64) / abs(lp64) < 1e-5
    assert_parity(grad.cpu().numpy(), g64, g32, what="fused NUTS gradient (jnp.clip)", floor=grad_floor(g64),
                  count_factor=None)
    assert_parity(g_w.cpu().numpy(), g64, g32, what="walk NUTS gradient (jnp.clip)", floor=grad_floor(g64),
                  count_factor=None)
    # naz's torch maf (train's loss) keeps clamp_preserve_gradients
    nf = NormalizingFlow("maf", None, D, 2, [150, 150, 150], spec["L"])
    st = {}
    for l, lay in enumerate(d):
        for i, (W, b) in enumerate(lay):
            st[f"layers.{l}.nn.layers.{i}.weight"] = W.astype(np.float32)
            st[f"layers.{l}.nn.layers.{i}.bias"] = b.astype(np.float32)
        st[f"layers.{l}.nn.permutation"] = np.asarray(layers[l][1])
    fio.load_state(nf, st)
    nf = nf.to("cuda")
    lp = nf.log_prob(torch.tensor(x, device="cuda"), condition=torch.tensor(ctx, device="cuda")).sum()
    lp.backward()
    gn = torch.cat([t.grad.reshape(-1) for tr in nf.flow_dist.transforms for lin in tr.nn.layers
                    for t in (lin.weight, lin.bias)]).cpu().numpy()
    mask = torch.cat([t.reshape(-1) for tr in nf.flow_dist.transforms for lin in tr.nn.layers
                      for t in (lin.mask, torch.ones_like(lin.bias))]).cpu().numpy()
    _, gp32 = _oracle_grad(spec, layers, d, x, ctx, torch.float32, "preserve")
    assert_parity(gn * mask, gp64, gp32, what="NormalizingFlow maf NLL gradient (pyro clamp)",
                  floor=grad_floor(gp64), count_factor=None)
