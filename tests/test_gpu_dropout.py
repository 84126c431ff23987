"""GPU: MC dropout conditioners (naz transforms.py:29-95) and MCDPNormalizingFlow
(mcdpflow.py:29-56) — SURVEY.md §8f rank 2.  Dropout masks come from a hash of
(seed, row, col) inside naz_dropout; the checks use the mask the kernel applied (recovered by
running it on ones) with a float64 torch restatement of the conditioner chain."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from naz_amd import _lib
    _lib.lib()


def test_dropout_kernel_mask_statistics_and_determinism():
    from naz_amd import ops
    x = torch.randn(4096, 150, device=DEV)
    for p in (0.1, 0.25, 0.5):
        y = ops.dropout(x, p, 1234)
        keep = y != 0
        rate = float(keep.double().mean())
        assert abs(rate - (1 - p)) < 4 * np.sqrt(p * (1 - p) / x.numel()) + 1e-4, (p, rate)
        torch.testing.assert_close(y[keep], x[keep] / (1 - p), rtol=1e-6, atol=0)
        assert torch.equal(ops.dropout(x, p, 1234), y), "same seed must give the same mask"
        assert not torch.equal(ops.dropout(x, p, 1235) != 0, keep), "another seed must change the mask"
        z = x.clone()
        ops.dropout(z, p, 1234, out=z)
        assert torch.equal(z, y), "in place"
        # rows / columns are not correlated: per-column keep rates all near 1 - p
        col = keep.double().mean(0)
        assert float((col - (1 - p)).abs().max()) < 6 * np.sqrt(p * (1 - p) / 4096)
    assert torch.equal(ops.dropout(x, 0.0, 7), x)


def _masks(drop, shapes):
    from naz_amd import ops
    p, seeds = drop
    return [ops.dropout(torch.ones(s, device=DEV), p, sd).double() for s, sd in zip(shapes, seeds)]


@pytest.mark.parametrize("masked", [False, True])
def test_chain_with_dropout_matches_torch_fp64(masked):
    """ChainFn forward and backward with dropout == float64 torch with the kernel's masks."""
    from naz_amd import autograd as ag
    torch.manual_seed(0)
    M, dims = 3000, [6, 64, 48, 10]
    Ws = [(torch.randn(dims[i + 1], dims[i], device=DEV) / dims[i] ** 0.5).requires_grad_(True) for i in range(3)]
    bs = [(torch.randn(dims[i + 1], device=DEV) * 0.1).requires_grad_(True) for i in range(3)]
    x = torch.randn(M, dims[0], device=DEV, requires_grad=True)
    drop = (0.3, [11, 22])
    y = ag.chain(x, Ws, bs, "tanh", drop=drop)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    masks = _masks(drop, [(M, dims[1]), (M, dims[2])])
    W64 = [w.detach().double().requires_grad_(True) for w in Ws]
    b64 = [b.detach().double().requires_grad_(True) for b in bs]
    x64 = x.detach().double().requires_grad_(True)
    h = x64
    for i in range(3):
        h = h @ W64[i].t() + b64[i]
        if i < 2:
            h = torch.tanh(h) * masks[i]
    (h * g.double()).sum().backward()
    torch.testing.assert_close(y.double(), h, rtol=1e-4, atol=1e-5)
    for a, b in zip(Ws + bs + [x], W64 + b64 + [x64]):
        torch.testing.assert_close(a.grad.double(), b.grad, rtol=1e-3, atol=1e-4 * float(b.grad.abs().max()))


@pytest.mark.parametrize("ftype,extra", [("maf", ()), ("nsa", (8,)), ("nsc", (8, 2))])
def test_dropout_flows_train_and_eval(ftype, extra):
    """train mode: dropout active (per-layer kernels, fresh masks per call, gradients flow);
    eval mode: deterministic and equal to the same flow built without dropout."""
    from naz_amd.flows import NormalizingFlow
    D, C = 4, 2
    torch.manual_seed(3)
    f = NormalizingFlow(ftype, None, D, C, [32, 32], 2, *extra, dropout_p=0.2)
    torch.manual_seed(3)
    f0 = NormalizingFlow(ftype, None, D, C, [32, 32], 2, *extra)
    f0.load_state_dict(f.state_dict())
    x = torch.randn(600, D, device=DEV) * 0.8
    c = torch.randn(600, C, device=DEV)
    f.eval()
    f0.eval()
    with torch.no_grad():
        torch.testing.assert_close(f.log_prob(x, condition=c), f0.log_prob(x, condition=c), rtol=0, atol=0)
    f.train()
    with torch.no_grad():
        a, b = f.log_prob(x, condition=c), f.log_prob(x, condition=c)
    assert bool(torch.isfinite(a).all()) and not torch.equal(a, b), "dropout must redraw masks per call"
    lp = f.log_prob(x, condition=c)
    (-lp.mean()).backward()
    assert all(p.grad is not None and bool(torch.isfinite(p.grad).all()) for p in f.parameters() if p.requires_grad)


def test_mcdp_sample_uncertain():
    """MCDPNormalizingFlow.sample_uncertain (mcdpflow.py:39-56): niter stochastic sample sets."""
    from naz_amd.flows.mcdpflow import MCDPNormalizingFlow
    from naz.flows.mcdpflow import MCDPNormalizingFlow as Compat
    assert Compat is MCDPNormalizingFlow
    torch.manual_seed(5)
    f = MCDPNormalizingFlow("maf", None, 2, 2, [48, 48], 3, dropout_p=0.25)
    c = torch.tensor([0.3, -0.7], device=DEV)
    s = f.sample_uncertain(4, [5000], condition=c)
    assert s.shape == (4, 5000, 2) and np.isfinite(s).all()
    assert not np.array_equal(s[0], s[1])
    with pytest.raises(AssertionError):
        MCDPNormalizingFlow("maf", None, 2, 2, [48, 48], 3)
