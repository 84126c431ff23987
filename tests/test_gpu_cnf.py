"""GPU: the fused FFJORD solve against the oracle
(oracle/naz_oracle.py FFJORD: torch autograd VJP Hutchinson trace + odeint.py RK4) on the same
fp32 weights, inputs and Hutchinson probes.  Criterion: tests/parity.py."""
import numpy as np
import pytest
import torch

from oracle import naz_oracle as O
from tests.conftest import load_golden
from tests.parity import assert_parity

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _cuda(a):
    return torch.as_tensor(np.asarray(a), dtype=torch.float32, device=DEV)


def _np(t):
    return t.detach().double().cpu().numpy()


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from naz_amd import _lib
    _lib.lib()


@pytest.fixture(autouse=True)
def _inference():
    with torch.no_grad():
        yield


def _spec_state(fx):
    spec = {k[5:]: fx[k].tolist() for k in fx if k.startswith("spec/")}
    state = {k[6:]: fx[k] for k in fx if k.startswith("state/")}
    return spec, state


def _product_cnf(spec, state):
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    f = NormalizingFlow("cnf", None, spec["D"], spec["C"], spec["hidden"], spec["L"], steps=spec.get("steps", 8))
    fio.load_state(f, state)
    return f


@pytest.mark.parametrize("name", ["cnf_d4c2.npz", "cnf_d16c0.npz"])
def test_cnf_log_prob_vs_golden(name):
    fx = load_golden(name)
    spec, state = _spec_state(fx)
    f = _product_cnf(spec, state)
    for l, t in enumerate(f.transforms):
        t.noise = _cuda(fx[f"eps_l/{l}"])
    c = _cuda(fx["ctx"]) if "ctx" in fx else None
    lp = f.log_prob(_cuda(fx["x"]), condition=c)
    assert_parity(_np(lp), fx["lp64"], fx["lp32"], what=f"{name} log_prob")


@pytest.mark.parametrize("name", ["cnf_d4c2.npz", "cnf_d16c0.npz"])
def test_cnf_sample_direction_vs_golden(name):
    """naz _call (t 1 -> 0) per block, accumulated log-det (sampling direction)."""
    fx = load_golden(name)
    spec, state = _spec_state(fx)
    f = _product_cnf(spec, state)
    c = _cuda(fx["ctx"]) if "ctx" in fx else None
    y = _cuda(fx["z"])
    ld = torch.zeros(y.shape[0], device=DEV)
    for l, t in enumerate(f.transforms):
        t.noise = _cuda(fx[f"eps_s/{l}"])
        tt = t.condition(c) if c is not None else t
        y = tt._call_acc(y, ld)
    assert_parity(_np(y), fx["y_sample64"], fx["y_sample32"], what=f"{name} sample y")
    assert_parity(_np(ld), fx["ld_sample64"], fx["ld_sample32"], what=f"{name} sample ld")


def _oracle_block(D, C, hidden, act, x, c, eps, t0, t1, steps, dt, seed=3):
    spec = dict(flow_type="cnf", D=D, C=C, hidden=hidden, L=1, activation=act)
    st = {k: v.float() for k, v in O.random_state(spec, seed=seed, last_layer_scale=1.0).items()}
    net = O.build_flow(spec, st, dt).layers[0].nn
    y, a = O.rk4_augmented(net, torch.as_tensor(x).to(dt), None if c is None else torch.as_tensor(c).to(dt),
                           torch.as_tensor(eps).to(dt), t0, t1, steps)
    flat = torch.cat([st[f"layers.0.nn.layers.{i}.{n}"].reshape(-1) for i in range(len(hidden) + 1)
                      for n in ("weight", "bias")])
    return y.numpy(), a.numpy(), flat


@pytest.mark.parametrize("D,C,hidden,act", [(4, 2, [32, 32], "softplus"), (4, 2, [32, 32], "tanh"),
                                            (5, 3, [48, 32, 16, 16], "softplus"), (2, 2, [128, 64, 64], "softplus"),
                                            (16, 0, [128, 128, 128], "softplus")])
@pytest.mark.parametrize("direction", [(0.0, 1.0), (1.0, 0.0)])
@pytest.mark.parametrize("mfma", ["f32", "f16x3"])
def test_cnf_kernel_vs_oracle(D, C, hidden, act, direction, mfma):
    from naz_amd import ops
    B = 300
    rng = np.random.default_rng(D * 10 + C)
    x = (rng.standard_normal((B, D)) * 0.8).astype(np.float32)
    c = rng.standard_normal((B, C)).astype(np.float32) if C else None
    eps = rng.standard_normal((B, D)).astype(np.float32)
    t0, t1 = direction
    y64, a64, flat = _oracle_block(D, C, hidden, act, x, c, eps, t0, t1, 8, torch.float64)
    y32, a32, _ = _oracle_block(D, C, hidden, act, x, c, eps, t0, t1, 8, torch.float32)
    d = ops.cnf_desc(D, C, hidden, act, mfma)
    if mfma == "f16x3" and any(h % 32 for h in hidden):
        assert not ops.cnf_supported(d)
        pytest.skip("fp16x3 CNF needs hidden widths in multiples of 32")
    assert ops.cnf_supported(d)
    packed = ops.cnf_pack(d, _cuda(flat))
    y, a = ops.cnf_integrate(d, packed, _cuda(x), _cuda(eps), t0, t1, 8, context=None if c is None else _cuda(c))
    assert_parity(_np(y), y64, y32, what=f"cnf D{D} C{C} {hidden} {act} y")
    assert_parity(_np(a), a64, a32, what=f"cnf D{D} C{C} {hidden} {act} ld")


def test_cnf_ld_modes_broadcast_context_and_ragged_batches():
    from naz_amd import ops
    D, C, hidden = 4, 2, [32, 32]
    rng = np.random.default_rng(9)
    for B in (1, 15, 127, 129, 1000):
        x = rng.standard_normal((B, D)).astype(np.float32)
        c1 = rng.standard_normal((1, C)).astype(np.float32)
        eps = rng.standard_normal((B, D)).astype(np.float32)
        y64, a64, flat = _oracle_block(D, C, hidden, "softplus", x, np.repeat(c1, B, 0), eps, 0.0, 1.0, 8,
                                       torch.float64)
        y32, a32, _ = _oracle_block(D, C, hidden, "softplus", x, np.repeat(c1, B, 0), eps, 0.0, 1.0, 8,
                                    torch.float32)
        d = ops.cnf_desc(D, C, hidden)
        packed = ops.cnf_pack(d, _cuda(flat))
        base = torch.full((B,), 2.5, device=DEV)
        y, ld = ops.cnf_integrate(d, packed, _cuda(x), _cuda(eps), 0.0, 1.0, 8, context=_cuda(c1[0]),
                                  ld_out=base.clone(), ld_mode=ops.LD_ROWSUM_SUB)
        assert_parity(_np(y), y64, y32, what=f"B={B} y")
        assert_parity(_np(ld) - 2.5, -a64, -a32, what=f"B={B} ld SUB")
        _, ld_add = ops.cnf_integrate(d, packed, _cuda(x), _cuda(eps), 0.0, 1.0, 8, context=_cuda(c1[0]),
                                      ld_out=base.clone(), ld_mode=ops.LD_ROWSUM_ADD)
        assert torch.equal(ld_add - 2.5, -(ld - 2.5)) or np.allclose(_np(ld_add) - 2.5, a64, rtol=1e-4, atol=1e-5)


def test_cnf_full_size_exact_properties():
    """Config 5 at BASELINE's batch (2^18 rows): rows are independent, so the solve is bitwise
    deterministic, permutation-equivariant and chunk-invariant."""
    from naz_amd import ops
    D, hidden, B = 16, [128, 128, 128], 1 << 18
    g = torch.Generator().manual_seed(0)
    _, _, flat = _oracle_block(D, 0, hidden, "softplus", np.zeros((1, D), np.float32), None,
                               np.zeros((1, D), np.float32), 0.0, 1.0, 1, torch.float32)
    d = ops.cnf_desc(D, 0, hidden)
    packed = ops.cnf_pack(d, _cuda(flat))
    x = torch.randn(B, D, generator=g).to(DEV)
    eps = torch.randn(B, D, generator=g).to(DEV)
    y, a = ops.cnf_integrate(d, packed, x, eps, 0.0, 1.0, 8)
    y2, a2 = ops.cnf_integrate(d, packed, x, eps, 0.0, 1.0, 8)
    assert torch.equal(y, y2) and torch.equal(a, a2)
    perm = torch.randperm(B, generator=g).to(DEV)
    yp, ap = ops.cnf_integrate(d, packed, x[perm], eps[perm], 0.0, 1.0, 8)
    assert torch.equal(yp, y[perm]) and torch.equal(ap, a[perm])
    ys, as_ = [], []
    for i in range(0, B, 70001):
        yc, ac = ops.cnf_integrate(d, packed, x[i:i + 70001], eps[i:i + 70001], 0.0, 1.0, 8)
        ys.append(yc)
        as_.append(ac)
    assert torch.equal(torch.cat(ys), y) and torch.equal(torch.cat(as_), a)
    # spot-check a slice against the oracle
    idx = torch.arange(0, B, B // 256)
    y64, a64, _ = _oracle_block(D, 0, hidden, "softplus", x[idx].cpu().numpy(), None, eps[idx].cpu().numpy(), 0.0,
                                1.0, 8, torch.float64)
    y32, a32, _ = _oracle_block(D, 0, hidden, "softplus", x[idx].cpu().numpy(), None, eps[idx].cpu().numpy(), 0.0,
                                1.0, 8, torch.float32)
    assert_parity(_np(a[idx.to(DEV)]), a64, a32, what="full-size spot ld")


def test_cnf_flow_api():
    """naz surface: NormalizingFlow('cnf', ...) log_prob / sample, fresh probes per call."""
    from naz_amd.flows import NormalizingFlow
    f = NormalizingFlow("cnf", None, 4, 2, [32, 32], 2)
    x = torch.randn(500, 4, device=DEV)
    c = torch.randn(500, 2, device=DEV)
    lp1 = f.log_prob(x, condition=c)
    lp2 = f.log_prob(x, condition=c)
    assert lp1.shape == (500,) and bool(torch.isfinite(lp1).all())
    assert not torch.equal(lp1, lp2)  # Hutchinson probes are redrawn per solve, as torchdyn does
    s = f.sample([64], condition=c[0])
    assert s.shape == (64, 4) and bool(torch.isfinite(s).all())
    with torch.enable_grad():  # the training path: differentiable through the solve (test_gpu_cnf_grad.py)
        lp = f.log_prob(x, condition=c)
        assert lp.requires_grad
        lp.mean().backward()
        assert all(p.grad is not None and bool(torch.isfinite(p.grad).all()) for p in f.parameters())


@pytest.mark.parametrize("scale", [1.0, 3000.0])
def test_cnf_f16x3_range_guard(scale):
    """Large activations: hidden values / tangents past 2^14 take the exact power-of-two scaling
    path of the fp16x3 GEMMs (x and eps scaled so layer-1 inputs overflow fp16 unscaled)."""
    from naz_amd import ops
    D, C, hidden, act = 4, 2, [32, 32], "softplus"
    B = 256
    rng = np.random.default_rng(21)
    x = (rng.standard_normal((B, D)) * scale).astype(np.float32)
    c = (rng.standard_normal((B, C)) * scale).astype(np.float32)
    eps = (rng.standard_normal((B, D)) * scale).astype(np.float32)
    y64, a64, flat = _oracle_block(D, C, hidden, act, x, c, eps, 0.0, 1.0, 2, torch.float64)
    y32, a32, _ = _oracle_block(D, C, hidden, act, x, c, eps, 0.0, 1.0, 2, torch.float32)
    d = ops.cnf_desc(D, C, hidden, act, "f16x3")
    packed = ops.cnf_pack(d, _cuda(flat))
    y, a = ops.cnf_integrate(d, packed, _cuda(x), _cuda(eps), 0.0, 1.0, 2, context=_cuda(c))
    # at 3000 sigma the fp16 pieces' 22 bits leave the trace's tail a few times the fp32 path's
    # (measured: 10 vs 3 rows above 1e-5 of 256, max 1.6e-4 vs 1.7e-5): the guard's job is no
    # overflow and fp32-grade bulk statistics; the exceedance count gets 4x headroom here
    cf = 2.0 if scale == 1.0 else 4.0
    assert_parity(_np(y), y64, y32, what=f"range guard scale={scale} y", count_factor=cf)
    assert_parity(_np(a), a64, a32, what=f"range guard scale={scale} ld", count_factor=cf)


def _oracle_dopri5(D, C, hidden, act, x, c, eps, t0, t1, atol, rtol, seed=3):
    spec = dict(flow_type="cnf", D=D, C=C, hidden=hidden, L=1, activation=act)
    st = {k: v.float() for k, v in O.random_state(spec, seed=seed, last_layer_scale=1.0).items()}
    net = O.build_flow(spec, st, torch.float64).layers[0].nn
    ct = None if c is None else torch.as_tensor(c).double()
    y, a, nfe = O.dopri5_augmented(net, torch.as_tensor(x).double(), ct, torch.as_tensor(eps).double(), t0, t1,
                                   atol, rtol)
    yr, ar = O.rk4_augmented(net, torch.as_tensor(x).double(), ct, torch.as_tensor(eps).double(), t0, t1, 256)
    return y.numpy(), a.numpy(), nfe, yr.numpy(), ar.numpy()


def _oracle_dopri5_global(D, C, hidden, act, x, c, eps, t0, t1, atol, rtol, seed=3):
    """torchdyn's batch-global step control (oracle.dopri5_global), fp64."""
    spec = dict(flow_type="cnf", D=D, C=C, hidden=hidden, L=1, activation=act)
    st = {k: v.float() for k, v in O.random_state(spec, seed=seed, last_layer_scale=1.0).items()}
    net = O.build_flow(spec, st, torch.float64).layers[0].nn
    ct = None if c is None else torch.as_tensor(c).double()
    y, a, nfe = O.dopri5_global(net, torch.as_tensor(x).double(), ct, torch.as_tensor(eps).double(), t0, t1, atol, rtol)
    return y.numpy(), a.numpy(), nfe


@pytest.mark.parametrize("D,C,hidden,act", [(4, 2, [32, 32], "softplus"), (2, 2, [128, 64, 64], "softplus"),
                                            (16, 0, [128, 128, 128], "softplus")])
@pytest.mark.parametrize("direction", [(0.0, 1.0), (1.0, 0.0)])
@pytest.mark.parametrize("mfma", ["f32", "f16x3"])
def test_cnf_dopri5_vs_oracle(D, C, hidden, act, direction, mfma):
    """§8f rank 3: adaptive dopri5 (per-16-row step control) vs the fp64 restatement with the same
    groups and controller, and vs the converged solution (RK4, 256 steps): the error is at the
    tolerance's scale and the step counts agree with the oracle's on (almost) every group."""
    from naz_amd import ops
    B, atol, rtol = 200, 1e-4, 1e-4
    rng = np.random.default_rng(D * 10 + C + 1)
    x = (rng.standard_normal((B, D)) * 0.8).astype(np.float32)
    c = rng.standard_normal((B, C)).astype(np.float32) if C else None
    eps = rng.standard_normal((B, D)).astype(np.float32)
    t0, t1 = direction
    y64, a64, nfe64, yr, ar = _oracle_dopri5(D, C, hidden, act, x, c, eps, t0, t1, atol, rtol)
    _, _, flat = _oracle_block(D, C, hidden, act, x, c, eps, t0, t1, 1, torch.float64)
    d = ops.cnf_desc(D, C, hidden, act, mfma)
    if not ops.cnf_supported(d):
        pytest.skip("mode not available for this shape")
    packed = ops.cnf_pack(d, _cuda(flat))
    nfe = torch.zeros((B + 15) // 16, device=DEV, dtype=torch.int32)
    y, a = ops.cnf_integrate_dopri5(d, packed, _cuda(x), _cuda(eps), t0, t1, atol, rtol,
                                    context=None if c is None else _cuda(c), nfe=nfe)
    y, a, nfe = _np(y), _np(a), nfe.cpu().numpy()
    assert (nfe > 0).all(), "a group ran out of steps"
    # same step decisions on most groups (fp32 vs fp64 may flip a decision sitting at the threshold)
    assert np.mean(nfe == np.asarray(nfe64)) >= 0.75, (nfe, nfe64)
    # accuracy vs the converged solution: at the tolerance's scale
    tol_y = 20 * (atol + rtol * np.abs(yr))
    assert np.all(np.abs(y - yr) <= tol_y), np.abs(y - yr).max()
    assert np.all(np.abs(a - ar) <= 20 * (atol + rtol * np.abs(ar))), np.abs(a - ar).max()
    # vs the oracle's same-controller solve where the step sequence matched
    same = np.repeat(nfe == np.asarray(nfe64), 16)[:B]
    assert np.abs(y - y64)[same].max() <= 2e-4 and np.abs(a - a64)[same].max() <= 2e-4
    # vs torchdyn's semantics (one step size for the whole batch, hairer_norm over [B, D + 1]):
    # a different step sequence, the same solution within the solver's promised tolerance
    yg, ag, _ = _oracle_dopri5_global(D, C, hidden, act, x, c, eps, t0, t1, atol, rtol)
    assert np.all(np.abs(y - yg) <= 20 * (atol + rtol * np.abs(yg))), np.abs(y - yg).max()
    assert np.all(np.abs(a - ag) <= 20 * (atol + rtol * np.abs(ag))), np.abs(a - ag).max()


@pytest.mark.parametrize("D,C,hidden,act", [(4, 2, [32, 32], "softplus"), (2, 2, [128, 64, 64], "softplus"),
                                            (16, 0, [128, 128, 128], "softplus")])
@pytest.mark.parametrize("direction", [(0.0, 1.0), (1.0, 0.0)])
@pytest.mark.parametrize("mfma", ["f32", "f16x3"])
def test_cnf_dopri5_global_vs_oracle(D, C, hidden, act, direction, mfma):
    """torchdyn's batch-global step control (naz_cnf_integrate_dopri5_global, the reference's
    semantics: continuous_transforms.py:73-82) vs oracle.dopri5_global in fp64: the same number
    of RHS evaluations (= the same accepted/rejected step sequence), the same solution within
    atol = rtol = 1e-4 (2e-4 absolute), and within the tolerance of the converged solution."""
    from naz_amd import ops
    B, atol, rtol = 200, 1e-4, 1e-4
    rng = np.random.default_rng(D * 10 + C + 1)
    x = (rng.standard_normal((B, D)) * 0.8).astype(np.float32)
    c = rng.standard_normal((B, C)).astype(np.float32) if C else None
    eps = rng.standard_normal((B, D)).astype(np.float32)
    t0, t1 = direction
    yg, ag, nfe64 = _oracle_dopri5_global(D, C, hidden, act, x, c, eps, t0, t1, atol, rtol)
    _, _, _, yr, ar = _oracle_dopri5(D, C, hidden, act, x, c, eps, t0, t1, atol, rtol)
    _, _, flat = _oracle_block(D, C, hidden, act, x, c, eps, t0, t1, 1, torch.float64)
    d = ops.cnf_desc(D, C, hidden, act, mfma)
    if not ops.cnf_supported(d):
        pytest.skip("mode not available for this shape")
    packed = ops.cnf_pack(d, _cuda(flat))
    nfe = torch.zeros(1, device=DEV, dtype=torch.int32)
    y, a = ops.cnf_integrate_dopri5_global(d, packed, _cuda(x), _cuda(eps), t0, t1, atol, rtol,
                                           context=None if c is None else _cuda(c), nfe=nfe)
    y, a, n = _np(y), _np(a), int(nfe.item())
    assert n == nfe64, (n, nfe64)
    assert np.abs(y - yg).max() <= 2e-4 and np.abs(a - ag).max() <= 2e-4, (np.abs(y - yg).max(), np.abs(a - ag).max())
    assert np.all(np.abs(y - yr) <= 20 * (atol + rtol * np.abs(yr))), np.abs(y - yr).max()
    assert np.all(np.abs(a - ar) <= 20 * (atol + rtol * np.abs(ar))), np.abs(a - ar).max()


def test_cnf_dopri5_global_ragged_and_max_steps():
    """Batch-global control: ragged batch sizes (partial waves and workgroups) agree with the fp64
    oracle's step count; max_steps exhaustion is reported (negative count)."""
    from naz_amd import ops
    D, C, hidden, act = 4, 2, [32, 32], "softplus"
    for B in (1, 37, 1000):
        rng = np.random.default_rng(B)
        x = (rng.standard_normal((B, D)) * 0.8).astype(np.float32)
        c = rng.standard_normal((B, C)).astype(np.float32)
        eps = rng.standard_normal((B, D)).astype(np.float32)
        yg, ag, nfe64 = _oracle_dopri5_global(D, C, hidden, act, x, c, eps, 0.0, 1.0, 1e-4, 1e-4)
        _, _, flat = _oracle_block(D, C, hidden, act, x, c, eps, 0.0, 1.0, 1, torch.float64)
        d = ops.cnf_desc(D, C, hidden, act, "f32")
        packed = ops.cnf_pack(d, _cuda(flat))
        nfe = torch.zeros(1, device=DEV, dtype=torch.int32)
        y, a = ops.cnf_integrate_dopri5_global(d, packed, _cuda(x), _cuda(eps), 0.0, 1.0, context=_cuda(c), nfe=nfe)
        n = int(nfe.item())
        # with one or two rows the error norm averages 5-10 elements and the first step's estimate
        # (fp64: 8e-10) sits at fp32's cancellation floor (~2e-5: err = hh sum(e_i k_i), sum(e_i) = 0,
        # |k| ~ 4e3): the step-size factor lands below the clamp of 10 and one extra short step
        # closes the interval (measured: 20 vs 14 RHS evaluations at B = 1, 2; exact from B = 16)
        assert (n == nfe64) if B >= 16 else (nfe64 <= n <= nfe64 + 6), (B, n, nfe64)
        assert np.abs(_np(y) - yg).max() <= 2e-4, (B, np.abs(_np(y) - yg).max())
        y, a = ops.cnf_integrate_dopri5_global(d, packed, _cuda(x), _cuda(eps), 0.0, 1.0, 1e-9, 1e-9, max_steps=2,
                                               context=_cuda(c), nfe=nfe)
        assert int(nfe.item()) < 0, "max_steps exhaustion must be reported"


def test_cnf_dopri5_flow_api_and_ragged():
    """NormalizingFlow("cnf", ..., solver="dopri5", step_control="group") log_prob runs the
    per-group adaptive kernel; ragged batches (the last wave partially filled) give the same
    per-row result as a full batch.  The default (batch-global control) runs and is finite."""
    from naz_amd.flows import NormalizingFlow
    rng = np.random.default_rng(4)
    g = NormalizingFlow("cnf", None, 4, 2, [32, 32], 2, solver="dopri5").to(DEV)
    xg = _cuda(rng.standard_normal((200, 4)) * 0.8)
    assert bool(torch.isfinite(g.log_prob(xg, condition=_cuda(rng.standard_normal((200, 2))))).all())
    assert all(t.step_control == "global" for t in g.transforms)
    f = NormalizingFlow("cnf", None, 4, 2, [32, 32], 2, solver="dopri5", step_control="group").to(DEV)
    x = _cuda(rng.standard_normal((200, 4)) * 0.8)
    c = _cuda(rng.standard_normal((200, 2)))
    for t in f.transforms:
        t.noise = _cuda(rng.standard_normal((200, 4)))
    lp = f.log_prob(x, condition=c)
    assert bool(torch.isfinite(lp).all())
    nfe = f.transforms[0].last_nfe if hasattr(f.transforms[0], "last_nfe") else None
    for t in f.transforms:
        t.noise = t.noise[:37]
    lp37 = f.log_prob(x[:37], condition=c[:37])
    # rows 0..31 form the same two 16-row groups in both batches
    assert torch.equal(lp37[:32], lp[:32])
    assert nfe is None or int(nfe.min()) > 0


def test_cnf_dopri5_max_steps_raises():
    """A dopri5 solve that reaches max_steps before t1 returns a partial state; the transform
    fails loudly (strict=True, the default) instead of handing it to log_prob."""
    from naz_amd.flows import NormalizingFlow
    rng = np.random.default_rng(5)
    x = _cuda(rng.standard_normal((64, 4)) * 0.8)
    c = _cuda(rng.standard_normal((64, 2)))
    f = NormalizingFlow("cnf", None, 4, 2, [32, 32], 1, solver="dopri5", atol=1e-9, rtol=1e-9,
                        max_steps=1).to(DEV)
    with pytest.raises(RuntimeError, match="max_steps"):
        f.log_prob(x, condition=c)
    f.transforms[0].strict = False
    assert f.log_prob(x, condition=c).shape == (64,)


@pytest.mark.parametrize("mfma", ["auto", "f32"])
@pytest.mark.parametrize("name", ["cnf_refode_d4c2.npz", "cnf_refode_d16c0.npz"])
def test_cnf_kernel_vs_reference_odeint(name, mfma):
    """The HIP FFJORD block solve against the REFERENCE'S OWN solver and trace estimator (naz's
    neural_odes odeint.py RK4 + cnf.py trace_df_dz_hutchinson, run in the build container by
    oracle/gen_refode_fixtures.py): 8 RK4 steps t 0 -> 1 (log_prob) and 1 -> 0 (sample), probe
    fixed per solve; ref32 = the reference run in float32."""
    from naz_amd import ops
    fx = load_golden(name)
    spec, state = _spec_state(fx)
    f = _product_cnf(spec, state)
    t = f.transforms[0]
    t.noise = _cuda(fx["eps"])
    t._plan.set_mfma(mfma)
    c = _cuda(fx["ctx"]) if "ctx" in fx else None
    tt = t.condition(c) if c is not None else t
    for direction, (t0, t1), v in (("inv", (0.0, 1.0), fx["x"]), ("fwd", (1.0, 0.0), fx["z"])):
        y, a = tt._solve(_cuda(v), t0, t1, None, ops.LD_ROWSUM)
        assert_parity(_np(y), fx[f"{direction}_x64"], fx[f"{direction}_x32"], what=f"{name} {direction} x ({mfma})")
        assert_parity(_np(a), fx[f"{direction}_a64"], fx[f"{direction}_a32"], what=f"{name} {direction} a ({mfma})")
