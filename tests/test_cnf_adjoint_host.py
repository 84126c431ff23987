"""CPU: the host logic of the CNF backward (naz_amd/flows/cnf_adjoint.py) — the stacked
value/tangent walk, the discrete RK4 adjoint recursion and the continuous adjoint — with every HIP
launch replaced by a float64 torch statement of the kernel's documented semantics
(include/naz_hip.h: naz_linear_act, naz_gemm_dact, naz_gemm_jvp_bwd, naz_gemm, naz_colsum).  Checked
against the oracle's float64 autograd through the same RK4 solve (oracle hutchinson_rhs with
create_graph).  The kernels themselves are covered on the GPU by tests/test_gpu_cnf_grad.py."""
import types

import pytest
import torch
from torch import nn

from oracle import naz_oracle as O


def _d1_ratio(act, h):
    if act == "softplus":
        d1 = -torch.expm1(-h)
        return d1, 1 - d1
    return 1 - h * h, -2 * h


def _fake_ops():
    acts = {"identity": lambda v: v, "softplus": lambda v: torch.where(v > 20, v, torch.log1p(torch.exp(v))),
            "tanh": torch.tanh}

    def _put(out, r):
        if out is None:
            return r
        out.copy_(r)
        return out

    def linear_act(x, W, b, act="identity", context=None, mask=None, out=None):
        inp = x if context is None else torch.cat([context.reshape(-1, context.shape[-1]).expand(x.shape[0], -1), x], 1)
        pre = inp @ W.t() + (0 if b is None else b)
        return _put(out, acts[act](pre))

    def gemm_dact(a, W, y, act, mask=None, out=None):
        return _put(out, (a @ W) * _d1_ratio(act, y)[0])

    def gemm_jvp_bwd(a, W, S, act, out=None):
        G = a @ W
        d1, r = _d1_ratio(act, S[0::2])
        C = torch.empty_like(G)
        C[0::2] = G[0::2] * d1 + G[1::2] * S[1::2] * r
        C[1::2] = G[1::2] * d1
        return _put(out, C)

    def gemm(a, b, out=None, accumulate=False, **kw):
        r = a @ b
        if out is None:
            return r
        if accumulate:
            out += r
        else:
            out.copy_(r)
        return out

    def colsum(a, out=None):
        if out is None:
            return a.sum(0)
        out += a.sum(0)
        return out

    return types.SimpleNamespace(linear_act=linear_act, gemm_dact=gemm_dact, gemm_jvp_bwd=gemm_jvp_bwd, gemm=gemm,
                                 colsum=colsum)


class _Net:
    def __init__(self, Ws, bs, act, D, C):
        self._lins = []
        for W, b in zip(Ws, bs):
            lin = nn.Linear(W.shape[1], W.shape[0]).double()
            lin.weight.data.copy_(W)
            lin.bias.data.copy_(b)
            self._lins.append(lin)
        self.act, self.input_dim, self.context_dim = act, D, C

    def linears(self):
        return self._lins


def _problem(D, C, hidden, act, B, seed):
    spec = dict(flow_type="cnf", D=D, C=C, hidden=hidden, L=1, activation=act)
    st = O.random_state(spec, seed=seed, last_layer_scale=1.0)
    n = len(hidden) + 1
    Ws = [st[f"layers.0.nn.layers.{i}.weight"].double() for i in range(n)]
    bs = [st[f"layers.0.nn.layers.{i}.bias"].double() for i in range(n)]
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, D, generator=g, dtype=torch.float64) * 0.8
    c = torch.randn(B, C, generator=g, dtype=torch.float64) if C else None
    eps = torch.randn(B, D, generator=g, dtype=torch.float64)
    lam = torch.randn(B, D, generator=g, dtype=torch.float64)
    mu = torch.randn(B, generator=g, dtype=torch.float64)
    return Ws, bs, x, c, eps, lam, mu


def _oracle(Ws, bs, act, x, c, eps, lam, mu, t0, t1, steps):
    Wg = [W.clone().requires_grad_(True) for W in Ws]
    bg = [b.clone().requires_grad_(True) for b in bs]
    xg = x.clone().requires_grad_(True)
    cg = None if c is None else c.clone().requires_grad_(True)
    y, a = O.rk4_augmented(O.FCNN(Wg, bg, act), xg, cg, eps, t0, t1, steps)
    loss = (y * lam).sum() + (a * mu).sum()
    wrt = Wg + bg + [xg] + ([cg] if cg is not None else [])
    return torch.autograd.grad(loss, wrt)


@pytest.fixture
def adj(monkeypatch):
    from naz_amd.flows import cnf_adjoint
    monkeypatch.setattr(cnf_adjoint, "ops", _fake_ops())
    return cnf_adjoint


@pytest.mark.parametrize("D,C,hidden,act", [(4, 2, [32, 32], "softplus"), (3, 0, [16, 8, 8], "tanh")])
@pytest.mark.parametrize("t0,t1", [(0.0, 1.0), (1.0, 0.0)])
def test_discrete_adjoint_equals_autograd(adj, D, C, hidden, act, t0, t1):
    Ws, bs, x, c, eps, lam, mu = _problem(D, C, hidden, act, 40, seed=D + C)
    steps = 4
    walk = adj.CnfWalk(_Net(Ws, bs, act, D, C))
    # forward checkpoints x_n (the product takes them from the fused kernel, one launch per step)
    xs, h = [x], (t1 - t0) / steps
    with torch.no_grad():
        for n in range(steps):
            y, _ = O.rk4_augmented(O.FCNN(Ws, bs, act), xs[-1], c, eps, t0 + n * h, t0 + (n + 1) * h, 1)
            xs.append(y)
    gW = [torch.zeros_like(W) for W in Ws]
    gb = [torch.zeros_like(b) for b in bs]
    gc = None if c is None else torch.zeros_like(c)
    l = lam.clone()
    for n in reversed(range(steps)):
        l = adj._rk4_step_adjoint(walk, xs[n], c, eps, h, l, mu, gW, gb, gc)
    ref = _oracle(Ws, bs, act, x, c, eps, lam, mu, t0, t1, steps)
    n = len(Ws)
    got = gW + gb + [l] + ([gc] if c is not None else [])
    for i, (g, r) in enumerate(zip(got, ref)):
        assert torch.allclose(g, r, rtol=1e-9, atol=1e-11), (i, float((g - r).abs().max()))


def test_continuous_adjoint_converges_to_autograd(adj):
    D, C, hidden, act = 4, 2, [32, 32], "softplus"
    Ws, bs, x, c, eps, lam, mu = _problem(D, C, hidden, act, 40, seed=5)
    with torch.no_grad():
        y1, _ = O.rk4_augmented(O.FCNN(Ws, bs, act), x, c, eps, 0.0, 1.0, 64)
    ref = _oracle(Ws, bs, act, x, c, eps, lam, mu, 0.0, 1.0, 64)
    walk = adj.CnfWalk(_Net(Ws, bs, act, D, C))
    gW = [torch.zeros_like(W) for W in Ws]
    gb = [torch.zeros_like(b) for b in bs]
    gc = torch.zeros_like(c)
    l = adj._continuous_adjoint(walk, y1, c, eps, 0.0, 1.0, 16, lam.clone(), mu, gW, gb, gc)
    for g, r in zip(gW + gb + [l, gc], ref):
        scale = max(float(r.abs().max()), 1e-3)
        assert float((g - r).abs().max()) / scale < 1e-5
