"""GPU: gradients through the FFJORD solve — the CNF training step (SURVEY.md §8f rank 3;
naz trains CNFs through torchdyn's adjoint, naz/flows/continuous_transforms.py:73-89,
naz/trainers/train_flows.py:194-213).

* rk4 (the pinned config-5 solver): the discrete adjoint (flows/cnf_adjoint.py) is the exact
  gradient of the solve, so it is checked against the oracle's float64 torch autograd through the
  same RK4 steps (oracle hutchinson_rhs with create_graph, as torchdyn's hutch_trace), with the
  oracle's float32 autograd as the precision yardstick (tests/parity.py gradient criterion).
* dopri5: the continuous adjoint approximates the exact-solution gradient; checked against fp64
  autograd through a converged RK4 solve (64 steps) within a solver-scale tolerance.
"""
import numpy as np
import pytest
import torch

from oracle import naz_oracle as O
from tests.parity import assert_parity, grad_floor

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


def _setup(D, C, hidden, L, act, B, seed, steps=8, solver="rk4", **kw):
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    from torch import nn
    spec = dict(flow_type="cnf", D=D, C=C, hidden=hidden, L=L, activation=act, steps=steps)
    state = {k: v.float().numpy() for k, v in O.random_state(spec, seed=seed, last_layer_scale=1.0).items()}
    acts = {"softplus": nn.Softplus(), "tanh": nn.Tanh()}
    f = NormalizingFlow("cnf", None, D, C, hidden, L, activation=acts[act], steps=steps, solver=solver, **kw)
    fio.load_state(f, state)
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((B, D)) * 0.8).astype(np.float32)
    c = rng.standard_normal((B, C)).astype(np.float32) if C else None
    eps = [rng.standard_normal((B, D)).astype(np.float32) for _ in range(L)]
    w = rng.uniform(0.5, 1.5, B).astype(np.float32)  # per-row loss weights: a generic cotangent
    return spec, state, f, x, c, eps, w


def _oracle_grads(spec, state, x, c, eps, w, dt, steps):
    sp = dict(spec, steps=steps)
    st = {k: torch.as_tensor(v).to(dt).requires_grad_(True) for k, v in state.items()}
    of = O.build_flow(sp, st, dt)
    for l, layer in enumerate(of.layers):
        layer.eps = torch.as_tensor(eps[l]).to(dt)
    xt = torch.as_tensor(x).to(dt).requires_grad_(True)
    ct = None if c is None else torch.as_tensor(c).to(dt).requires_grad_(True)
    lp = of.log_prob(xt, ct)
    loss = (lp * torch.as_tensor(w).to(dt)).sum()
    keys = list(st)
    wrt = [st[k] for k in keys] + [xt] + ([ct] if ct is not None else [])
    gs = torch.autograd.grad(loss, wrt)
    out = dict(zip(keys, gs))
    out["x"] = gs[len(keys)]
    if ct is not None:
        out["ctx"] = gs[len(keys) + 1]
    return lp.detach(), out


def _product_grads(f, x, c, eps, w):
    from naz_amd.flows import io as fio
    for l, t in enumerate(f.transforms):
        t.noise = _cuda(eps[l])
    xt = _cuda(x).requires_grad_(True)
    ct = None if c is None else _cuda(c).requires_grad_(True)
    lp = f.log_prob(xt, condition=ct)
    assert lp.requires_grad, "grad mode with trainable weights must record the CNF solve"
    (lp * _cuda(w)).sum().backward()
    g = {k: p.grad for k, p in fio.named_state_params(f).items()}
    g["x"] = xt.grad
    if ct is not None:
        g["ctx"] = ct.grad
    return lp, g


# the last two: naz's POSYDON CNF (eposydon/train_cnf_mle.py:91, D = 4, H = [128] x 4, the lambda width from the
# data) on the per-layer solve (no fused kernel fits its weights)
CASES = [(4, 2, [32, 32], 2, "softplus"), (4, 2, [32, 32], 1, "tanh"), (5, 3, [48, 32, 16, 16], 1, "softplus"),
         (16, 0, [128, 128, 128], 1, "softplus"), (4, 4, [128] * 4, 1, "softplus"), (4, 6, [128] * 4, 1, "tanh")]


@pytest.mark.parametrize("D,C,hidden,L,act", CASES, ids=lambda v: str(v))
def test_cnf_rk4_gradient_vs_oracle_autograd(D, C, hidden, L, act):
    spec, state, f, x, c, eps, w = _setup(D, C, hidden, L, act, B=256, seed=D + C + L)
    lp, g = _product_grads(f, x, c, eps, w)
    lp64, g64 = _oracle_grads(spec, state, x, c, eps, w, torch.float64, 8)
    lp32, g32 = _oracle_grads(spec, state, x, c, eps, w, torch.float32, 8)
    assert_parity(_np(lp), _np(lp64), _np(lp32), what="cnf graph log_prob")
    assert set(g) == set(g64)
    for k in g64:
        assert g[k] is not None, f"{k}: no gradient"
        ref64, ref32 = _np(g64[k]), _np(g32[k])
        assert_parity(_np(g[k]), ref64, ref32, what=f"cnf d/d{k}", floor=grad_floor(ref64), count_factor=None)


def test_cnf_reductions_side_stream_match():
    """NAZ_CNF_DW_STREAM / NAZ_CNF_PREFETCH: the VJP's weight / bias reductions on a side stream beside
    the next layer's input-adjoint GEMM, and the next RK4 step's forward recompute on another beside
    this step's VJPs (joined before use) give the one-stream gradients, to the reductions' atomic-order
    rounding, at a batch where the kernels overlap."""
    from naz_amd.flows import cnf_adjoint as adj
    res = {}
    prev = adj._DW_STREAM, adj._PREFETCH
    try:
        for side in (False, True):  # (with it: the next RK4 step's recompute on its own stream too)
            adj._DW_STREAM = adj._PREFETCH = side
            spec, state, f, x, c, eps, w = _setup(16, 0, [128, 128, 128], 1, "softplus", B=1 << 15, seed=3)
            res[side] = _product_grads(f, x, c, eps, w)
            torch.cuda.synchronize()
    finally:
        adj._DW_STREAM, adj._PREFETCH = prev
    assert torch.equal(res[False][0], res[True][0])
    for k, a in res[False][1].items():
        b = res[True][1][k]
        rel = float((a - b).norm() / a.norm().clamp_min(1e-30))
        assert rel < 1e-5, f"{k}: side-stream reductions vs one stream {rel:.2e}"


def test_cnf_broadcast_context_gradient():
    """One context row for the whole batch (naz sample/log_prob with condition=[C]): its gradient
    is the sum over rows."""
    D, C, hidden, L, act = 4, 2, [32, 32], 1, "softplus"
    spec, state, f, x, c, eps, w = _setup(D, C, hidden, L, act, B=200, seed=7)
    c1 = c[:1]
    lp, g = _product_grads(f, x, c1, eps, w)
    _, g64 = _oracle_grads(spec, state, x, np.repeat(c1, x.shape[0], 0), eps, w, torch.float64, 8)
    _, g32 = _oracle_grads(spec, state, x, np.repeat(c1, x.shape[0], 0), eps, w, torch.float32, 8)
    r64, r32 = _np(g64["ctx"]).sum(0, keepdims=True), _np(g32["ctx"]).sum(0, keepdims=True)
    assert g["ctx"].shape == (1, C)
    assert_parity(_np(g["ctx"]), r64, r32, what="broadcast ctx grad", floor=grad_floor(r64), count_factor=None)


@pytest.mark.parametrize("D,C,hidden", [(4, 2, [32, 32]), (16, 0, [128, 128, 128]), (4, 4, [128] * 4)])
def test_cnf_dopri5_adjoint_gradient_vs_converged(D, C, hidden):
    spec, state, f, x, c, eps, w = _setup(D, C, hidden, 1, "softplus", B=192, seed=3, solver="dopri5")
    lp, g = _product_grads(f, x, c, eps, w)
    _, g64 = _oracle_grads(spec, state, x, c, eps, w, torch.float64, 64)
    for k in g64:
        ref = _np(g64[k])
        err = np.abs(_np(g[k]) - ref) / grad_floor(ref)
        assert float(err.max()) < 2e-3, (k, float(err.max()))


def test_cnf_training_steps_reduce_nll():
    """A few Adam steps of the naz training loop's NLL (train_flows.py:194-213) on a CNF."""
    D, C, hidden, L, act = 4, 2, [32, 32], 1, "softplus"
    _, _, f, x, c, _, _ = _setup(D, C, hidden, L, act, B=2048, seed=11)
    x = _cuda(x) * 0.5 + 1.0
    c = _cuda(c)
    opt = torch.optim.Adam(f.parameters(), lr=3e-3)
    losses = []
    for _ in range(25):
        opt.zero_grad()
        for t in f.transforms:
            t.noise = None
        loss = -f.log_prob(x, condition=c).mean()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(f.parameters(), 1.0)
        opt.step()
        losses.append(float(loss.detach()))
    assert all(np.isfinite(losses))
    assert np.mean(losses[-5:]) < np.mean(losses[:5]) - 0.05, losses
