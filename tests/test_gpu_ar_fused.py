"""GPU: the fused autoregressive-inverse flow kernel (naz_ar_flow_log_prob, csrc/made_ar_r16.h) —
naz nsa NormalizingFlow.log_prob (pyro ConditionedSplineAutoregressive._inverse, the D-pass loop
of naz/flows/transforms.py:165-198, over L layers) as one launch.

Checked against the float64 oracle (pyro's D full passes per layer) with tests/parity.py's
criterion, against this library's per-layer path on the same weights, and on the edge cases the
kernel has: ragged batches, one broadcast context row, the bounding map, an empty batch, and
inputs outside the fp16 split range (which must route to the per-layer path)."""
import numpy as np
import pytest
import torch

from oracle import naz_oracle as O
from tests.parity import assert_parity

pytestmark = pytest.mark.gpu

DEV = "cuda"

CASES = [
    dict(flow_type="nsa", D=16, C=32, hidden=[128, 128], L=8, K=8, n=512),  # SURVEY §8d AR variant
    dict(flow_type="nsa", D=16, C=0, hidden=[128, 128], L=3, K=8, n=1000),
    dict(flow_type="nsa", D=8, C=0, hidden=[128, 128], L=2, K=8, n=1500),
    dict(flow_type="nsa", D=4, C=2, hidden=[128, 128], L=3, K=8, n=1200),  # bench --flow nsa
    dict(flow_type="maf", D=2, C=2, hidden=[150, 150, 150], L=16, n=3000),  # the maf paper shape
    dict(flow_type="maf", D=16, C=32, hidden=[128, 128], L=4, n=700),
    # the 4-parameter Bayesian MAF (calibrate_4p.py:75,90-96)
    dict(flow_type="maf", D=4, C=2, hidden=[150, 150, 150], L=16, n=2500),
    # naz's 4-parameter MLE MAF (train_mle_all_data_4param.py:87-92): the wide inverse (made_ar_wide.h)
    dict(flow_type="maf", D=4, C=2, hidden=[512] * 5, L=18, n=900),
]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _id(spec):
    return f"{spec['flow_type']}D{spec['D']}C{spec['C']}L{spec['L']}"


def _flow(spec, bounds=None):
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    state = {k: v.float() for k, v in O.random_state(spec, seed=11).items()}
    extra = (spec["K"],) if spec["flow_type"] == "nsa" else ()
    f = NormalizingFlow(spec["flow_type"], bounds, spec["D"], spec["C"], spec["hidden"], spec["L"], *extra)
    fio.load_state(f, {k: v.numpy() for k, v in state.items()})
    return f.to(DEV), state


@pytest.mark.parametrize("spec", CASES, ids=_id)
def test_fused_ar_vs_oracle_and_per_layer(spec):
    f, state = _flow(spec)
    assert f.fused, "the fused autoregressive kernel must be selected for this shape"
    n = spec["n"]
    x = torch.as_tensor(O.gaussian_mixture(n, spec["D"], seed=5))
    c = torch.as_tensor(O.context_normal(n, spec["C"], seed=6)) if spec["C"] else None
    cd = None if c is None else c.to(DEV)
    with torch.no_grad():
        lp = f.log_prob(x.to(DEV), condition=cd).cpu().numpy()
        f.set_fused(False)
        lp_walk = f.log_prob(x.to(DEV), condition=cd).cpu().numpy()
        f.set_fused(True)
    lp64 = O.build_flow(spec, state, torch.float64).log_prob(x.double(), None if c is None else c.double()).numpy()
    lp32 = O.build_flow(spec, state, torch.float32).log_prob(x, c).numpy()
    st = assert_parity(lp, lp64, lp32, what=f"fused {_id(spec)}")
    assert_parity(lp_walk, lp64, lp32, what=f"per-layer {_id(spec)}")
    print(_id(spec), st, "max |fused - walk|", float(np.abs(lp - lp_walk).max()))


@pytest.mark.parametrize("spec", [dict(flow_type="nsa", D=16, C=32, hidden=[128, 128], L=2, K=8),
                                  dict(flow_type="maf", D=2, C=2, hidden=[150, 150, 150], L=5)], ids=_id)
def test_fused_ar_broadcast_context_bounds_ragged_empty(spec):
    D, C = spec["D"], spec["C"]
    lo, hi = np.full(D, -9.0, np.float32), np.full(D, 9.5, np.float32)
    f, _ = _flow(spec, bounds={"low": lo, "high": hi})
    assert f.fused
    g = torch.Generator().manual_seed(3)
    x = (torch.rand(777, D, generator=g) * 17.0 - 8.0).to(DEV)
    c1 = torch.randn(C, generator=g).to(DEV)
    with torch.no_grad():
        lp = f.log_prob(x, condition=c1)
        f.set_fused(False)
        ref = f.log_prob(x, condition=c1)
        f.set_fused(True)
        empty = f.log_prob(x[:0], condition=c1)
    assert empty.shape == (0,)
    assert torch.isfinite(lp).all()
    np.testing.assert_allclose(lp.cpu().numpy(), ref.cpu().numpy(), rtol=2e-5, atol=2e-4)


def test_fused_ar_out_of_fp16_range_routes_to_per_layer():
    spec = dict(flow_type="nsa", D=16, C=32, hidden=[128, 128], L=2, K=8)
    f, _ = _flow(spec)
    x = torch.randn(300, 16, device=DEV)
    x[7, 3] = 1e6  # outside the kernel's f16x3 input split: identity in every spline
    c = torch.randn(300, 32, device=DEV)
    with torch.no_grad():
        lp = f.log_prob(x, condition=c)
        f.set_fused(False)
        ref = f.log_prob(x, condition=c)
    np.testing.assert_allclose(lp.cpu().numpy(), ref.cpu().numpy(), rtol=0, atol=0)


SAMPLE_CASES = [
    dict(flow_type="nsa", D=16, C=32, hidden=[128, 128], L=4, K=8),
    dict(flow_type="nsa", D=16, C=0, hidden=[128, 128], L=2, K=8),
    dict(flow_type="nsa", D=4, C=2, hidden=[128, 128], L=3, K=8),
    dict(flow_type="maf", D=2, C=2, hidden=[150, 150, 150], L=16),
    dict(flow_type="maf", D=16, C=32, hidden=[128, 128], L=3),
    dict(flow_type="maf", D=4, C=2, hidden=[150, 150, 150], L=16),  # the 4-parameter Bayesian MAF
    # naz's 4-parameter MLE MAF (train_mle_all_data_4param.py:87-92): the wide instance
    dict(flow_type="maf", D=4, C=2, hidden=[512] * 5, L=18),
]


@pytest.mark.parametrize("spec", SAMPLE_CASES, ids=_id)
def test_fused_ar_sample_vs_oracle_and_per_layer(spec):
    """sample direction (pyro *Autoregressive._call over all layers, naz flow.py:94-129) in one
    naz_ar_flow_sample launch: y and the summed forward log-det against the fp64 oracle's
    forward_with_logdet and against the per-layer kernels."""
    from naz_amd import ops
    f, state = _flow(spec)
    assert f.fused
    g = torch.Generator().manual_seed(5)
    n, D, C = 1500, spec["D"], spec["C"]
    z = torch.randn(n, D, generator=g)
    c = torch.randn(n, C, generator=g) if C else None
    plan = f._plan
    y, ld = ops.ar_flow_sample(plan.desc, plan.packed_fwd(), z.to(DEV), None if c is None else c.to(DEV),
                               with_logdet=True)
    of64 = O.build_flow(spec, state, torch.float64)
    y64, ld64 = of64.forward_with_logdet(z.double(), None if c is None else c.double())
    of32 = O.build_flow(spec, state, torch.float32)
    y32, ld32 = of32.forward_with_logdet(z, c)
    assert_parity(y.detach().double().cpu().numpy(), y64.numpy(), y32.numpy(), what=f"fused sample y {_id(spec)}")
    # the forward log-det sums L x D select-first spline log-dets on the hardware transcendentals:
    # median / q99 / max at the reference fp32's level, the count of rows above 1e-5 up to ~2.2x
    # (measured nsa D4C2L3: 24 vs the reference fp32's 10 of 1500): 3x headroom on the count
    assert_parity(ld.detach().double().cpu().numpy(), ld64.numpy(), ld32.numpy(), what=f"fused sample ld {_id(spec)}",
                  count_factor=3.0)
    # the NormalizingFlow API takes the fused launch (z drawn inside: compare through fixed z)
    with torch.no_grad():
        f.set_fused(False)
        from naz_amd.flows.distributions import TransformedDistribution  # noqa: F401
        pdf = f._pdf(None if c is None else c.to(DEV))
        y_walk = pdf._transform_z(z.to(DEV))
        f.set_fused(True)
        pdf = f._pdf(None if c is None else c.to(DEV))
        y_api = pdf._transform_z(z.to(DEV))
    assert torch.equal(y_api, y)
    np.testing.assert_allclose(y.cpu().numpy(), y_walk.cpu().numpy(), rtol=1e-4, atol=1e-4)


def test_fused_ar_sample_broadcast_context_bounds_ragged():
    spec = dict(flow_type="nsa", D=16, C=32, hidden=[128, 128], L=2, K=8)
    lo, hi = np.full(16, -9.0, np.float32), np.full(16, 9.5, np.float32)
    f, _ = _flow(spec, bounds={"low": lo, "high": hi})
    c1 = torch.randn(32, device=DEV)
    with torch.no_grad():
        s = f.sample([333], condition=c1)
        assert s.shape == (333, 16) and torch.isfinite(s).all()
        assert bool(((s > -9.0) & (s < 9.5)).all())
        torch.manual_seed(0)
        a = f.sample([1000], condition=c1)
        f.set_fused(False)
        torch.manual_seed(0)
        b = f.sample([1000], condition=c1)
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-4, atol=1e-4)


def test_fused_ar_inverse_growing_values_stay_finite():
    """maf inverse with log-scales at the -5 clamp: every layer multiplies by e^5, so the values
    pass the f16 range inside the launch (the input check cannot see it); the per-row scaling of
    the hidden-layer-1 split keeps the fused result equal to the fp32 per-layer walk."""
    spec = dict(flow_type="maf", D=16, C=32, hidden=[128, 128], L=4)
    f, _ = _flow(spec)
    D = spec["D"]
    with torch.no_grad():
        for t in f.flow_dist.transforms:
            last = t.nn.layers[-1]
            last.weight.mul_(1e-3)
            last.bias[D:].fill_(-10.0)  # clamped to -5
    g = torch.Generator().manual_seed(9)
    x = (torch.randn(500, D, generator=g) * 3.0).to(DEV)
    c = torch.randn(500, 32, generator=g).to(DEV)
    with torch.no_grad():
        assert f.fused
        lp = f.log_prob(x, condition=c)
        f.set_fused(False)
        ref = f.log_prob(x, condition=c)
    assert torch.isfinite(lp).all() and torch.isfinite(ref).all()
    np.testing.assert_allclose(lp.cpu().numpy(), ref.cpu().numpy(), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("spec", [CASES[0], CASES[4]], ids=_id)
def test_fused_ar_device_pack_and_batched_draws(spec):
    """naz_ar_flow_pack (device pack of P weight draws) gives the host packer's image bit for bit,
    and naz_ar_flow_log_prob_batched (grid y = draw, one context vector) gives every draw's
    naz_ar_flow_log_prob bit for bit, for shared rows (sx = 0) and per-draw rows."""
    from naz_amd import ops
    f, _ = _flow(spec)
    plan = f._plan
    flat = plan._flat().astype(np.float32)
    perm = np.stack([n.permutation.detach().cpu().numpy() for n in plan._nets()]).astype(np.int32)
    flats = [flat, flat * np.float32(1.03), flat * np.float32(0.97)]
    dev = ops.ar_flow_pack_batched(plan.desc, torch.tensor(np.stack(flats), device=DEV), perm)
    for p, fl in enumerate(flats):
        # bit for bit, subnormal f16 lo pieces included (the maf shape's |W| 2^-11 falls below 2^-14)
        host = ops.ar_flow_pack(plan.desc, fl, perm, DEV)
        nbad = int((dev[p].view(torch.int32) != host.view(torch.int32)).sum())
        assert nbad == 0, f"draw {p} image: {nbad} words differ"
    fwd = ops.ar_flow_pack_fwd_batched(plan.desc, torch.tensor(np.stack(flats), device=DEV))  # the sampler's
    for p, fl in enumerate(flats):
        assert torch.equal(fwd[p].view(torch.int32), ops.ar_flow_pack_fwd(plan.desc, fl, DEV).view(torch.int32))
    # unmasked rows + the mask vector (the Bayesian front end's path): the packers' product equals
    # packing the rows masked beforehand, bit for bit (same fp32 multiply)
    ft = torch.tensor(np.stack(flats), device=DEV)
    mask = (ft[0] != 0).float()
    noisy = ft + torch.rand_like(ft) * (1 - mask)
    assert torch.equal(ops.ar_flow_pack_batched(plan.desc, noisy, perm, mask=mask).view(torch.int32),
                       ops.ar_flow_pack_batched(plan.desc, noisy * mask, perm).view(torch.int32))
    assert torch.equal(ops.ar_flow_pack_fwd_batched(plan.desc, noisy, mask=mask).view(torch.int32),
                       ops.ar_flow_pack_fwd_batched(plan.desc, noisy * mask).view(torch.int32))
    n, D, C = 777, spec["D"], spec["C"]
    x = torch.as_tensor(O.gaussian_mixture(n, D, seed=9)).to(DEV)
    xs = torch.stack([x, 0.9 * x, 1.1 * x])
    c1 = torch.as_tensor(O.context_normal(1, C, seed=3)).reshape(-1).to(DEV)
    shared = ops.ar_flow_log_prob_batched(plan.desc, dev, x, c1)
    per = ops.ar_flow_log_prob_batched(plan.desc, dev, xs, c1)
    for p in range(3):
        assert torch.equal(shared[p], ops.ar_flow_log_prob(plan.desc, dev[p], x, c1))
        assert torch.equal(per[p], ops.ar_flow_log_prob(plan.desc, dev[p], xs[p], c1))
    with pytest.raises(ValueError):
        ops.ar_flow_pack_batched(plan.desc, torch.tensor(np.stack(flats), device=DEV), perm[:, ::-1] * 0)


@pytest.mark.parametrize("spec", [CASES[4], CASES[3], CASES[0]], ids=_id)
def test_fused_ar_one_context_vector_pass0(spec):
    """One condition vector for every row (the density grid, naz plot.py:126-127): the
    context-only first degree pass is computed once and packed as constants (naz_ar_flow_pack
    pass0; the kernel skips the pass).  Same log_prob as the plain fused launch, and the oracle's."""
    from naz_amd import ops
    from naz_amd.flows import flow as FL
    f, state = _flow(spec)
    n, D, C = 5000, spec["D"], spec["C"]
    x = torch.as_tensor(O.gaussian_mixture(n, D, seed=21))
    c1 = torch.as_tensor(O.context_normal(1, C, seed=22)).reshape(-1)
    calls, orig = [], ops.ar_flow_log_prob_batched
    ops.ar_flow_log_prob_batched = lambda *a, **k: calls.append(k.get("pass0_const")) or orig(*a, **k)
    try:
        with torch.no_grad():
            a = f.log_prob(x.to(DEV), condition=c1.to(DEV))
            assert calls == [True], "the pass-0 path was not taken"
            FL._AR_PASS0 = False
            b = f.log_prob(x.to(DEV), condition=c1.to(DEV))
    finally:
        FL._AR_PASS0 = True
        ops.ar_flow_log_prob_batched = orig
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-4, atol=1e-4)
    cc = c1.reshape(1, -1).expand(n, -1)
    lp64 = O.build_flow(spec, state, torch.float64).log_prob(x.double(), cc.double()).numpy()
    lp32 = O.build_flow(spec, state, torch.float32).log_prob(x, cc).numpy()
    assert_parity(a.cpu().numpy(), lp64, lp32, what=f"pass0 {_id(spec)}")


def _full_size_properties(fn, x, c, what):
    """Rows are independent: the batch result must be finite, deterministic, bitwise
    permutation-equivariant and chunk-invariant (the ring kernels at full size)."""
    B = x.shape[0]
    out = fn(x, c)
    flat = out.reshape(B, -1)
    bad = torch.nonzero(~torch.isfinite(flat).all(dim=1)).reshape(-1)
    if bad.numel():
        pytest.fail(f"{what}: non-finite output in {bad.numel()} rows {bad[:8].tolist()} "
                    f"(workgroups of 192 rows: {(bad // 192).unique()[:8].tolist()})")
    assert torch.equal(out, fn(x, c)), f"{what}: not deterministic"
    g = torch.Generator(device=DEV).manual_seed(3)
    perm = torch.randperm(B, device=DEV, generator=g)
    assert torch.equal(fn(x[perm], None if c is None else c[perm]), out[perm]), f"{what}: permutation"
    step = 99991
    chunks = torch.cat([fn(x[i:i + step], None if c is None else c[i:i + step]) for i in range(0, B, step)])
    assert torch.equal(chunks, out), f"{what}: chunking"


def test_fused_ar_full_size_properties_nsa16():
    """The §8d AR variant (nsa D=16 | C=32, L=8) at BASELINE's 2^20 rows, both directions."""
    spec = dict(flow_type="nsa", D=16, C=32, hidden=[128, 128], L=8, K=8)
    f, _ = _flow(spec)
    assert f.fused
    B = 1 << 20
    x = torch.as_tensor(O.gaussian_mixture(B, 16, seed=21), device=DEV)
    c = torch.as_tensor(O.context_normal(B, 32, seed=22), device=DEV)
    with torch.no_grad():
        _full_size_properties(lambda a, b: f.log_prob(a, condition=b), x, c, "nsa16 log_prob")
        z = torch.randn(B, 16, device=DEV, generator=torch.Generator(device=DEV).manual_seed(4))
        def fwd(a, b):
            y, ld = f._plan.sample(a, b, with_logdet=True)
            return torch.cat([y, ld[:, None]], 1)
        _full_size_properties(fwd, z, c, "nsa16 sample")


@pytest.mark.parametrize("D", [2, 4])
def test_fused_ar_full_size_properties_maf_paper(D):
    """The maf paper shape (D=2 | C=2, H=[150]x3, L=16) and the 4-parameter Bayesian MAF (D=4) at
    2^20 rows, log_prob and sample."""
    spec = dict(flow_type="maf", D=D, C=2, hidden=[150, 150, 150], L=16)
    f, _ = _flow(spec)
    assert f.fused
    B = 1 << 20
    x = torch.as_tensor(O.gaussian_mixture(B, D, seed=23), device=DEV)
    c = torch.as_tensor(O.context_normal(B, 2, seed=24), device=DEV)
    with torch.no_grad():
        _full_size_properties(lambda a, b: f.log_prob(a, condition=b), x, c, f"maf D={D} log_prob")
        if D == 4:
            z = torch.randn(B, D, device=DEV, generator=torch.Generator(device=DEV).manual_seed(4))

            def fwd(a, b):
                y, ld = f._plan.sample(a, b, with_logdet=True)
                return torch.cat([y, ld[:, None]], 1)
            _full_size_properties(fwd, z, c, f"maf D={D} sample")


def test_wide_maf_fused_both_directions():
    """The production MAF shapes (D=4 | C=2, H=[512]x5; L=18 MLE, L=16 POSYDON,
    eposydon/train_maf_mle.py:84-90) take the fused wide inverse (made_ar_inv_wide_kernel) for
    log_prob and the fused sampler for sample: log_prob parity vs the fp64 oracle and vs the
    degree-scheduled per-layer path, and the sampler's y round-trips through log_prob
    (base(z) - ld(z) == log_prob(y))."""
    from naz_amd import ops
    for L in (16, 18):
        spec = dict(flow_type="maf", D=4, C=2, hidden=[512] * 5, L=L)
        f, state = _flow(spec)
        assert f.fused and f._plan.inverse and ops.ar_flow_supported(f._plan.desc)
        n = 600
        x = torch.as_tensor(O.gaussian_mixture(n, 4, seed=7))
        c = torch.as_tensor(O.context_normal(n, 2, seed=8))
        with torch.no_grad():
            lp = f.log_prob(x.to(DEV), condition=c.to(DEV)).cpu().numpy()
            f.set_fused(False)
            lp_walk = f.log_prob(x.to(DEV), condition=c.to(DEV)).cpu().numpy()
            f.set_fused(True)
        lp64 = O.build_flow(spec, state, torch.float64).log_prob(x.double(), c.double()).numpy()
        lp32 = O.build_flow(spec, state, torch.float32).log_prob(x, c).numpy()
        assert_parity(lp, lp64, lp32, what=f"wide maf L={L} log_prob (fused)")
        assert_parity(lp_walk, lp64, lp32, what=f"wide maf L={L} log_prob (per-layer path)")
        z = torch.randn(n, 4, generator=torch.Generator().manual_seed(L)).to(DEV)
        y, ld = ops.ar_flow_sample(f._plan.desc, f._plan.packed_fwd(), z, c.to(DEV), with_logdet=True)
        with torch.no_grad():
            lpy = f.log_prob(y, condition=c.to(DEV))
        rt = (lpy - (ops.base_log_prob(z) - ld)).abs() / lpy.abs().clamp_min(1.0)
        assert float(rt.max()) < 1e-4, float(rt.max())


def test_wide_maf_persistent_grid_and_draws():
    """The wide inverse's persistent grid (256 workgroups walking the (draw, 64-row tile) space,
    hidden layers 2.. through per-wave scratch): a batch of several tiles per workgroup plus a
    ragged tail against the per-layer path; one broadcast context row; an empty batch; the device
    packer's image bit-identical to the host packer's; three weight draws in one batched launch
    equal to three single-draw launches."""
    from naz_amd import ops
    spec = dict(flow_type="maf", D=4, C=2, hidden=[512] * 5, L=3)
    f, state = _flow(spec)
    plan = f._plan
    B = 256 * 64 * 2 + 77
    x = torch.as_tensor(O.gaussian_mixture(B, 4, seed=31)).to(DEV)
    c = torch.as_tensor(O.context_normal(B, 2, seed=32)).to(DEV)
    with torch.no_grad():
        lp = f.log_prob(x, condition=c)
        c1 = c[5]
        lp1 = f.log_prob(x[:3000], condition=c1)
        empty = f.log_prob(x[:0], condition=c[:0])
        f.set_fused(False)
        ref = f.log_prob(x, condition=c)
        ref1 = f.log_prob(x[:3000], condition=c1)
        f.set_fused(True)
    assert empty.shape == (0,)
    assert torch.isfinite(lp).all()
    np.testing.assert_allclose(lp.cpu().numpy(), ref.cpu().numpy(), rtol=2e-5, atol=2e-4)
    np.testing.assert_allclose(lp1.cpu().numpy(), ref1.cpu().numpy(), rtol=2e-5, atol=2e-4)
    # device packer == host packer, word for word
    flat = torch.from_numpy(plan._flat()).to(DEV)
    perm = np.stack([n.permutation.detach().cpu().numpy() for n in plan._nets()]).astype(np.int32)
    img_dev = ops.ar_flow_pack_batched(plan.desc, flat[None].contiguous(), perm)
    img_host = plan.packed()
    assert img_dev.shape[1] == img_host.numel()
    assert torch.equal(img_dev[0].view(torch.int32), img_host.view(torch.int32))
    # three draws (scaled weights) in one launch vs one launch each
    flats = torch.stack([flat * s for s in (1.0, 0.9, 1.1)]).contiguous()
    imgs = ops.ar_flow_pack_batched(plan.desc, flats, perm)
    xs = x[:5000]
    lpb = ops.ar_flow_log_prob_batched(plan.desc, imgs, xs, c1)
    for p in range(3):
        one = ops.ar_flow_log_prob(plan.desc, imgs[p].contiguous(), xs, c1)
        np.testing.assert_array_equal(lpb[p].cpu().numpy(), one.cpu().numpy())
