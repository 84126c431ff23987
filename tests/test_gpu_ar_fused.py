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
