"""CPU: the oracle itself — known-answer tests of SURVEY.md §8c and the golden fixtures."""
import math

import numpy as np
import pytest
import torch

from oracle import jax_maf_np as J
from oracle import naz_oracle as O
from tests.conftest import load_golden, spec_state
from tests.parity import assert_parity, rel_err

torch.set_default_dtype(torch.float32)


def _rand_raw(B, Dt, K, scale=2.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(B, Dt * (3 * K - 1), generator=g, dtype=torch.float64) * scale


def test_uniform_bins_identity_interior():
    """§8c-1: w=h uniform and interior slopes exactly 1 => identity on the interior bins."""
    K, Dt, B = 8, 3, 400
    # softplus(ud) + 1e-3 == 1  <=>  ud = log(expm1(1 - 1e-3))
    ud = math.log(math.expm1(1 - 1e-3))
    raw = torch.cat([torch.zeros(B, 2 * Dt * K, dtype=torch.float64),
                     torch.full((B, Dt * (K - 1)), ud, dtype=torch.float64)], 1)
    x = torch.linspace(-2.2, 2.2, B).double()[:, None].expand(B, Dt).contiguous()  # interior bins (edges at +-2.25)
    y, ld = O.rqs_from_raw(x, raw, Dt, K, O.LAYOUT_DENSE, inverse=False)
    assert torch.allclose(y, x, atol=1e-12) and ld.abs().max() < 1e-12


def test_tails_identity():
    """§8c-2: |x| > B is the identity with zero log-det (both directions)."""
    K, Dt = 8, 4
    x = torch.tensor([[-7.0, 3.0001, -3.5, 100.0]]).double()
    raw = _rand_raw(1, Dt, K)
    for inv in (False, True):
        y, ld = O.rqs_from_raw(x, raw, Dt, K, O.LAYOUT_DENSE, inverse=inv)
        assert torch.equal(y, x) and torch.all(ld == 0)


@pytest.mark.parametrize("layout", [O.LAYOUT_DENSE, O.LAYOUT_ARN])
def test_round_trip_and_logdet_sign(layout):
    """§8c-3: inv(fwd(x)) = x; ld_inv(fwd(x)) = -ld_fwd(x); including points on knots."""
    K, Dt, B = 8, 5, 2000
    raw = _rand_raw(B, Dt, K, seed=1)
    x = (torch.rand(B, Dt, generator=torch.Generator().manual_seed(2), dtype=torch.float64) * 6 - 3)
    # put some inputs exactly on the knots
    w, h, d = O.normalize_spline_params(*O.split_raw_params(raw, Dt, K, layout))
    _, cw = O._calculate_knots(1e-3 + (1 - 1e-3 * K) * w, -3.0, 3.0)
    x[:50, :] = cw[:50, :, 3]
    y, ld = O.rqs_from_raw(x, raw, Dt, K, layout, inverse=False)
    x2, ldi = O.rqs_from_raw(y, raw, Dt, K, layout, inverse=True)
    assert (x2 - x).abs().max() < 1e-8
    assert (ld + ldi).abs().max() < 1e-8


def test_logdet_matches_jacobian():
    """§8c-4: ld equals log|det dy/dx| from float64 autograd (diagonal Jacobian)."""
    K, Dt = 8, 3
    raw = _rand_raw(1, Dt, K, seed=3)
    x = torch.tensor([[-2.5, 0.3, 1.7]], dtype=torch.float64)
    f = lambda v: O.rqs_from_raw(v, raw, Dt, K, O.LAYOUT_DENSE, False)[0]
    J_ = torch.autograd.functional.jacobian(f, x).reshape(Dt, Dt)
    _, ld = O.rqs_from_raw(x, raw, Dt, K, O.LAYOUT_DENSE, False)
    assert torch.allclose(torch.log(torch.diagonal(J_).abs()), ld[0], atol=1e-10)
    assert torch.allclose(J_ - torch.diag(torch.diagonal(J_)), torch.zeros_like(J_))


@pytest.mark.parametrize("C", [0, 3])
def test_made_masks_autoregressive(C):
    """§8c-5: the MADE output for variable perm[k] depends only on perm[:k] (and context)."""
    D, hidden, mult = 5, [16, 16], 2
    perm = torch.randperm(D, generator=torch.Generator().manual_seed(4))
    masks, _ = O.create_mask(D, C, hidden, perm, mult)
    M = masks[0]
    for m in masks[1:]:
        M = m @ M
    conn = (M[:, C:] > 0).reshape(mult, D, D)  # [param, out var, in var]
    order = {int(v): k for k, v in enumerate(perm)}
    for o in range(D):
        for i in range(D):
            if conn[:, o, i].any():
                assert order[i] < order[o]
    if C > 0:
        assert (M[:, :C] > 0).any()


def test_mask_indices_round_half_even():
    # linspace(1, 4, 7) = 1, 1.5, 2, 2.5, 3, 3.5, 4 -> torch.round is half-to-even
    assert O.sample_mask_indices(4, 7).tolist() == [1, 2, 2, 2, 3, 4, 4]


@pytest.mark.parametrize("ft", ["nsc", "nsa", "maf"])
def test_density_round_trip(ft):
    """§8c-6: log_prob(T(z)) = base(z) - sum ld_fwd(z)."""
    spec = dict(flow_type=ft, D=4, C=2, hidden=[16, 16], L=3, K=6, split=2)
    f = O.build_flow(spec, O.random_state(spec, seed=9, last_layer_scale=1.0), torch.float64)
    g = torch.Generator().manual_seed(5)
    z = torch.randn(64, 4, generator=g, dtype=torch.float64)
    c = torch.randn(64, 2, generator=g, dtype=torch.float64)
    y, ld = f.forward_with_logdet(z, c)
    assert torch.allclose(f.log_prob(y, c), O.base_log_prob(z) - ld, atol=1e-7)


def test_normalisation_2d():
    """§8c-7: config-1 shaped flow integrates to 1 over [-8, 8]^2.  Parameters are scaled by
    0.3 so the density has no spikes narrower than the quadrature grid (random sharp splines
    compose into needles that any fixed grid under-samples)."""
    spec = dict(flow_type="nsc", D=2, C=0, hidden=[16, 16], L=3, K=8, split=1)
    st = O.random_state(spec, seed=3, last_layer_scale=0.3)
    st = {k: (v * 0.3 if "lower" in k else v) for k, v in st.items()}
    f = O.build_flow(spec, st, torch.float64)
    n = 2001
    g = torch.linspace(-8, 8, n, dtype=torch.float64)
    X, Y = torch.meshgrid(g, g, indexing="ij")
    pts = torch.stack([X.reshape(-1), Y.reshape(-1)], 1)
    p = torch.exp(f.log_prob(pts)).reshape(n, n)
    dx = (g[1] - g[0]).item()
    assert abs(p.sum().item() * dx * dx - 1.0) < 1e-3


def test_affine_matches_reference_jax_restatement():
    """§8c-8: the torch oracle's affine MAF equals the numpy restatement of the reference's
    own JAX MAF (naz/flows/bflow_jax_maf.py:48-225) on random weights."""
    spec = dict(flow_type="maf", D=4, C=3, hidden=[24, 24], L=4)
    st = O.random_state(spec, seed=21)
    f = O.build_flow(spec, st, torch.float64)
    g = torch.Generator().manual_seed(6)
    x = torch.randn(128, 4, generator=g, dtype=torch.float64)
    c = torch.randn(128, 3, generator=g, dtype=torch.float64)
    a = f.log_prob(x, c).numpy()
    b = J.log_prob(x.numpy(), J.layers_from_state(spec, {k: v.numpy() for k, v in st.items()}), c.numpy())
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12)


def test_bounding_transform_semantics():
    """naz/flows/transforms.py:20-27: logit box map, its log-jacobian and its inverse."""
    low, high = torch.tensor([-1.0, 0.0]).double(), torch.tensor([2.0, 5.0]).double()
    x = torch.tensor([[0.5, 1.0], [1.9, 4.9]]).double()
    y, lj = O.bounding_transform(x, low, high)
    assert torch.allclose(O.inverse_bounding_transform(y, low, high), x)
    u = (x - low) / (high - low)
    assert torch.allclose(lj, (-(torch.log(u) + torch.log1p(-u)) - torch.log(high - low)).sum(-1))


# ------------------------------------------------------------------ golden fixtures
@pytest.mark.parametrize("name", ["rqs_dense_k8.npz", "rqs_arn_k5.npz", "rqs_dense_k16.npz"])
def test_golden_spline_fixture(name):
    fx = load_golden(name)
    K, Dt, layout = int(fx["K"]), int(fx["Dt"]), int(fx["layout"])
    x, raw = torch.as_tensor(fx["x"]).double(), torch.as_tensor(fx["raw"]).double()
    for inv, ky, kl in ((False, "y_fwd", "ld_fwd"), (True, "y_inv", "ld_inv")):
        y, ld = O.rqs_from_raw(x, raw, Dt, K, layout, inverse=inv)
        np.testing.assert_array_equal(y.numpy(), fx[ky])
        np.testing.assert_array_equal(ld.numpy(), fx[kl])


@pytest.mark.parametrize("name", ["nsc_d16c32_l2.npz", "nsc_d8c0_l6.npz", "nsc_d6c2_small.npz", "nsa_d4c2.npz",
                                  "maf_d3c2.npz", "maf_twomoons.npz"])
def test_golden_flow_fixture(name):
    fx = load_golden(name)
    spec, state = spec_state(fx)
    f = O.build_flow(spec, state, torch.float64)
    x = torch.as_tensor(fx["x"]).double()
    c = torch.as_tensor(fx["ctx"]).double() if "ctx" in fx else None
    np.testing.assert_allclose(f.log_prob(x, c).numpy(), fx["lp64"], rtol=1e-12, atol=1e-10)
    # the reference-precision (fp32) path stays close to fp64 (its deviation is the tail bound
    # the GPU is held to, tests/parity.py)
    r = rel_err(fx["lp32"], fx["lp64"])
    assert np.median(r) < 1e-6 and r.max() < 1e-3
    if "lp_jaxref" in fx:
        np.testing.assert_allclose(fx["lp64"], fx["lp_jaxref"], rtol=1e-12, atol=1e-10)


def test_synthetic_inputs_match_baseline_spec():
    x = O.gaussian_mixture(20000, 16, seed=0)
    assert x.dtype == np.float32 and x.shape == (20000, 16)
    out = np.mean(np.abs(x) > 3.0)
    assert 0.05 < out < 0.4  # a meaningful share of coordinates hits the identity tails


# ------------------------------------------------------------------ a11: CNF restatement
def _cnf_flow(spec, seed=1234, dtype=torch.float64):
    st = O.random_state(spec, seed=seed, last_layer_scale=1.0)
    return O.build_flow(spec, st, dtype)


def test_cnf_hutchinson_is_unbiased_for_the_trace():
    """naz hutch_trace (continuous_transforms.py:85-89): E_eps[eps^T J eps] = tr J."""
    spec = dict(flow_type="cnf", D=4, C=2, hidden=[32, 32], L=1)
    net = _cnf_flow(spec).layers[0].nn
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 4, generator=g, dtype=torch.float64)
    c = torch.randn(3, 2, generator=g, dtype=torch.float64)
    n = 40000
    xr, cr = x.repeat_interleave(n, 0), c.repeat_interleave(n, 0)
    eps = torch.randn(3 * n, 4, generator=g, dtype=torch.float64)
    _, neg_tr = O.hutchinson_rhs(net, xr, cr, eps)
    est = (-neg_tr).reshape(3, n)
    for r in range(3):
        J = torch.autograd.functional.jacobian(lambda v: net(v[None], c[r:r + 1])[0], x[r])
        exact = torch.trace(J)
        sem = est[r].std() / math.sqrt(n)
        assert abs(est[r].mean() - exact) < 5 * sem


def test_cnf_rk4_converges_and_inverts():
    """Pinned 8-step RK4 (odeint.py:46-52) is within RK4 error of a 128-step solve, and the
    sampling solve (t 1 -> 0) inverts the density solve (t 0 -> 1) for the same probe."""
    spec = dict(flow_type="cnf", D=4, C=2, hidden=[32, 32], L=1)
    blk = _cnf_flow(spec).layers[0]
    g = torch.Generator().manual_seed(1)
    x = torch.randn(64, 4, generator=g, dtype=torch.float64)
    c = torch.randn(64, 2, generator=g, dtype=torch.float64)
    eps = torch.randn(64, 4, generator=g, dtype=torch.float64)
    z8, a8 = O.rk4_augmented(blk.nn, x, c, eps, 0.0, 1.0, 8)
    z128, a128 = O.rk4_augmented(blk.nn, x, c, eps, 0.0, 1.0, 128)
    assert (z8 - z128).abs().max() < 1e-5 and (a8 - a128).abs().max() < 1e-5
    xb, ab = O.rk4_augmented(blk.nn, z128, c, eps, 1.0, 0.0, 128)
    assert (xb - x).abs().max() < 1e-10 and (ab + a128).abs().max() < 1e-10


def test_cnf_dopri5_global_controller_meets_tolerance():
    """torchdyn's controller (one step size for the batch, hairer_norm over [B, D + 1];
    oracle.dopri5_global): its solution is within the promised tolerance of the converged one, and
    of the kernel's per-16-row controller (oracle.dopri5_augmented), in both directions."""
    spec = dict(flow_type="cnf", D=4, C=2, hidden=[32, 32], L=1)
    blk = _cnf_flow(spec).layers[0]
    g = torch.Generator().manual_seed(2)
    x = torch.randn(96, 4, generator=g, dtype=torch.float64) * 0.8
    c = torch.randn(96, 2, generator=g, dtype=torch.float64)
    eps = torch.randn(96, 4, generator=g, dtype=torch.float64)
    atol = rtol = 1e-4
    for t0, t1 in ((0.0, 1.0), (1.0, 0.0)):
        yg, ag, nfe = O.dopri5_global(blk.nn, x, c, eps, t0, t1, atol, rtol)
        yr, ar = O.rk4_augmented(blk.nn, x, c, eps, t0, t1, 256)
        yl, al, nfes = O.dopri5_augmented(blk.nn, x, c, eps, t0, t1, atol, rtol)
        assert nfe >= max(nfes)  # the batch-global step is set by the hardest rows
        assert ((yg - yr).abs() <= 20 * (atol + rtol * yr.abs())).all()
        assert ((ag - ar).abs() <= 20 * (atol + rtol * ar.abs())).all()
        assert ((yg - yl).abs() <= 20 * (atol + rtol * yg.abs())).all()


@pytest.mark.parametrize("name", ["cnf_d4c2.npz", "cnf_d16c0.npz"])
def test_golden_cnf_fixture(name):
    fx = load_golden(name)
    spec = {k[5:]: fx[k].tolist() for k in fx if k.startswith("spec/")}
    state = {k[6:]: fx[k] for k in fx if k.startswith("state/")}
    f = O.build_flow(spec, state, torch.float64)
    c = torch.as_tensor(fx["ctx"]).double() if "ctx" in fx else None
    for l, layer in enumerate(f.layers):
        layer.eps = torch.as_tensor(fx[f"eps_l/{l}"])
    lp = f.log_prob(torch.as_tensor(fx["x"]).double(), c)
    np.testing.assert_allclose(lp.numpy(), fx["lp64"], rtol=1e-12, atol=1e-10)
    r = rel_err(fx["lp32"], fx["lp64"])
    assert np.median(r) < 1e-6 and r.max() < 1e-4
