"""GPU: the degree-scheduled autoregressive inverse (naz_amd.nn.ARInversePlan) — naz's maf / nsa
log_prob (pyro AffineAutoregressive / SplineAutoregressive ``_inverse``, the D-pass loop of
naz/flows/transforms.py:133-198) computing every MADE hidden unit once.

Checked against the float64 oracle (pyro's D full passes) on fresh shapes (context / no
context, several D, ragged hidden widths, one and three hidden layers), and against this
library's own D-full-pass path on the same weights."""
import numpy as np
import pytest
import torch

from oracle import naz_oracle as O
from tests.parity import assert_parity

pytestmark = pytest.mark.gpu

DEV = "cuda"

CASES = [
    dict(flow_type="maf", D=2, C=2, hidden=[150, 150, 150], L=3),
    dict(flow_type="maf", D=5, C=0, hidden=[37], L=2),
    dict(flow_type="maf", D=6, C=3, hidden=[64, 50], L=2),
    dict(flow_type="nsa", D=4, C=2, hidden=[128, 128], L=2, K=8),
    dict(flow_type="nsa", D=3, C=0, hidden=[33, 20], L=2, K=5),
    # SURVEY §8d's config-3 AR variant (bench.py --flow nsa16): D=16 | C=32, K=8, H=[128,128], L=8
    dict(flow_type="nsa", D=16, C=32, hidden=[128, 128], L=8, K=8, n=512),
]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _flow(spec):
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    state = {k: v.float() for k, v in O.random_state(spec, seed=7).items()}
    extra = (spec["K"],) if spec["flow_type"] == "nsa" else ()
    f = NormalizingFlow(spec["flow_type"], None, spec["D"], spec["C"], spec["hidden"], spec["L"], *extra)
    fio.load_state(f, {k: v.numpy() for k, v in state.items()})
    return f.to(DEV), state


def _set_schedule(f, on):
    for net in f.nets:
        net.degree_schedule = on


def _id(spec):
    return f"{spec['flow_type']}-D{spec['D']}C{spec['C']}-{'x'.join(map(str, spec['hidden']))}"


@pytest.mark.parametrize("spec", CASES, ids=_id)
def test_scheduled_inverse_vs_oracle(spec):
    f, state = _flow(spec)
    n = spec.get("n", 2048)
    x = torch.as_tensor(O.gaussian_mixture(n, spec["D"], seed=5))
    c = torch.as_tensor(O.context_normal(n, spec["C"], seed=6)) if spec["C"] else None
    with torch.no_grad():
        _set_schedule(f, True)
        lp = f.log_prob(x.to(DEV), condition=None if c is None else c.to(DEV)).cpu().numpy()
        _set_schedule(f, False)
        lp_full = f.log_prob(x.to(DEV), condition=None if c is None else c.to(DEV)).cpu().numpy()
    cd = None if c is None else c.double()
    lp64 = O.build_flow(spec, state, torch.float64).log_prob(x.double(), cd).numpy()
    lp32 = O.build_flow(spec, state, torch.float32).log_prob(x, c).numpy()
    st = assert_parity(lp, lp64, lp32, what=f"{_id(spec)} scheduled")
    assert_parity(lp_full, lp64, lp32, what=f"{_id(spec)} full passes")
    # the two HIP paths differ only by summation order inside the GEMMs
    np.testing.assert_allclose(lp, lp_full, rtol=1e-5, atol=1e-4)
    print(_id(spec), st)


@pytest.mark.parametrize("spec", CASES[:1] + CASES[3:4], ids=_id)
def test_scheduled_inverse_sample_round_trip(spec):
    """sample (one forward pass per layer) then log_prob through the scheduled inverse: the
    inverse must recover the base draw's density."""
    f, _ = _flow(spec)
    n = 4096
    with torch.no_grad():
        c1 = torch.as_tensor(O.context_normal(1, spec["C"], seed=9)).to(DEV)[0] if spec["C"] else None
        xs = f.sample((n,), condition=c1).reshape(n, spec["D"])
        cond = None if c1 is None else c1.expand(n, -1).contiguous()
        _set_schedule(f, True)
        lp = f.log_prob(xs, condition=cond)
        _set_schedule(f, False)
        lp_full = f.log_prob(xs, condition=cond)
    assert torch.isfinite(lp).all()
    torch.testing.assert_close(lp, lp_full, rtol=1e-5, atol=2e-4)


@pytest.mark.parametrize("spec", [s for s in CASES if s["C"]], ids=_id)
def test_broadcast_context_folding(spec):
    """log_prob(x, condition=<one context vector>): the context-only (degree-0) MADE units are
    evaluated once and folded into biases (ARInversePlan._run_folded); same values as the plain
    schedule and the oracle."""
    from naz_amd.nn import ARInversePlan
    f, state = _flow(spec)
    n = spec.get("n", 2048)
    x = torch.as_tensor(O.gaussian_mixture(n, spec["D"], seed=5))
    c1 = torch.as_tensor(O.context_normal(1, spec["C"], seed=6))[0]
    with torch.no_grad():
        lp = f.log_prob(x.to(DEV), condition=c1.to(DEV)).cpu().numpy()
        ARInversePlan.fold_context = False
        try:
            lp_plain = f.log_prob(x.to(DEV), condition=c1.to(DEV)).cpu().numpy()
        finally:
            ARInversePlan.fold_context = True
    cn = c1.expand(n, -1)
    lp64 = O.build_flow(spec, state, torch.float64).log_prob(x.double(), cn.double()).numpy()
    lp32 = O.build_flow(spec, state, torch.float32).log_prob(x, cn).numpy()
    assert_parity(lp, lp64, lp32, what=f"{_id(spec)} folded")
    np.testing.assert_allclose(lp, lp_plain, rtol=1e-5, atol=1e-4)
