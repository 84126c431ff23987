"""GPU: the per-layer CNF solve (flows/cnf_adjoint.py walk_rk4 / walk_dopri5) -- every FFJORD shape
without a fused solve kernel, first of all naz's production POSYDON CNF
(examples/papers/eposydon/train_cnf_mle.py:91, train_cnf_mle_q.py:92:
NormalizingFlow("cnf", None, 4, C, [128, 128, 128, 128], 1), C = the data's lambda width), whose
~200 KB of weights do not fit one CU's LDS.  Checked against the REFERENCE'S OWN RK4 and trace
estimator (tests/golden/cnf_refode_d4c4_h128x4.npz, oracle/gen_refode_fixtures.py), the fp64
oracle (rk4_augmented, dopri5_global: torchdyn's batch-global control), and through the flow API."""
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


def _flow(D, C, hidden, act="softplus", seed=3, **kw):
    from torch import nn

    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    spec = dict(flow_type="cnf", D=D, C=C, hidden=hidden, L=1, activation=act)
    state = {k: v.float() for k, v in O.random_state(spec, seed=seed, last_layer_scale=1.0).items()}
    acts = {"softplus": nn.Softplus(), "tanh": nn.Tanh()}
    f = NormalizingFlow("cnf", None, D, C, hidden, 1, activation=acts[act], **kw)
    fio.load_state(f, {k: v.numpy() for k, v in state.items()})
    return spec, state, f


def test_posydon_cnf_constructs_on_the_per_layer_solve():
    from naz_amd.flows import NormalizingFlow
    for C in (2, 4, 6):
        f = NormalizingFlow("cnf", None, 4, C, [128, 128, 128, 128], 1)
        assert not f.transforms[0]._plan.fused
    f = NormalizingFlow("cnf", None, 4, 2, [32, 32], 1)
    assert f.transforms[0]._plan.fused  # compiled shapes keep the fused kernel


def test_posydon_cnf_vs_reference_odeint():
    """8 RK4 steps t 0 -> 1 (log_prob) and 1 -> 0 (sample) against naz's own odeint + Hutchinson
    estimator run in the build container (ref32 = that run in float32)."""
    from naz_amd import ops
    fx = load_golden("cnf_refode_d4c4_h128x4.npz")
    spec = {k[5:]: fx[k].tolist() for k in fx if k.startswith("spec/")}
    state = {k[6:]: fx[k] for k in fx if k.startswith("state/")}
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    f = NormalizingFlow("cnf", None, spec["D"], spec["C"], spec["hidden"], spec["L"], steps=8)
    fio.load_state(f, state)
    t = f.transforms[0]
    assert not t._plan.fused
    t.noise = _cuda(fx["eps"])
    tt = t.condition(_cuda(fx["ctx"]))
    with torch.no_grad():
        for direction, (t0, t1), v in (("inv", (0.0, 1.0), fx["x"]), ("fwd", (1.0, 0.0), fx["z"])):
            y, a = tt._solve(_cuda(v), t0, t1, None, ops.LD_ROWSUM)
            assert_parity(_np(y), fx[f"{direction}_x64"], fx[f"{direction}_x32"], what=f"posydon {direction} x")
            assert_parity(_np(a), fx[f"{direction}_a64"], fx[f"{direction}_a32"], what=f"posydon {direction} a")


@pytest.mark.parametrize("C,act", [(2, "softplus"), (6, "tanh"), (0, "softplus")])
def test_per_layer_log_prob_and_sample_vs_oracle(C, act):
    """The flow API (log_prob with base + log-det, sample) on the per-layer rk4 solve vs the fp64
    oracle's Flow over the same weights and probes; ragged batch, per-row contexts."""
    D, hidden, B = 4, [128] * 4, 777
    spec, state, f = _flow(D, C, hidden, act, seed=C + 1)
    rng = np.random.default_rng(C)
    x = (rng.standard_normal((B, D)) * 0.8).astype(np.float32)
    c = rng.standard_normal((B, C)).astype(np.float32) if C else None
    eps = rng.standard_normal((B, D)).astype(np.float32)
    f.transforms[0].noise = _cuda(eps)
    with torch.no_grad():
        lp = f.log_prob(_cuda(x), condition=None if c is None else _cuda(c))
    ref = {}
    for dt in (torch.float64, torch.float32):
        of = O.build_flow(dict(spec, steps=8), {k: v.to(dt) for k, v in state.items()}, dt)
        of.layers[0].eps = torch.as_tensor(eps).to(dt)
        ref[dt] = of.log_prob(torch.as_tensor(x).to(dt), None if c is None else torch.as_tensor(c).to(dt)).numpy()
    assert_parity(_np(lp), ref[torch.float64], ref[torch.float32], what=f"per-layer cnf C={C} {act} log_prob")
    # the sampling direction inverts the log_prob direction (to the RK4 truncation at 8 steps)
    t = f.transforms[0]
    tt = t.condition(_cuda(c)) if C else t
    with torch.no_grad():
        z = tt._inverse(_cuda(x))
        xr = tt._call(z)
    assert float((xr - _cuda(x)).abs().max()) < 1e-2


@pytest.mark.parametrize("direction", [(0.0, 1.0), (1.0, 0.0)])
def test_per_layer_dopri5_global_vs_oracle(direction):
    """torchdyn's batch-global dopri5 (naz's solver='dopri5', atol = rtol = 1e-4) on the per-layer
    RHS: the same accepted / rejected step sequence as oracle.dopri5_global in fp64 (same RHS count)
    and the same solution within 2e-4."""
    from naz_amd import ops
    D, C, hidden, B = 4, 4, [128] * 4, 200
    spec, state, f = _flow(D, C, hidden, "softplus", seed=11, solver="dopri5")
    rng = np.random.default_rng(12)
    x = (rng.standard_normal((B, D)) * 0.8).astype(np.float32)
    c = rng.standard_normal((B, C)).astype(np.float32)
    eps = rng.standard_normal((B, D)).astype(np.float32)
    t0, t1 = direction
    net = O.build_flow(spec, {k: v.double() for k, v in state.items()}, torch.float64).layers[0].nn
    y64, a64, nfe64 = O.dopri5_global(net, torch.as_tensor(x).double(), torch.as_tensor(c).double(),
                                      torch.as_tensor(eps).double(), t0, t1, 1e-4, 1e-4)
    t = f.transforms[0]
    t.noise = _cuda(eps)
    tt = t.condition(_cuda(c))
    with torch.no_grad():
        y, a = tt._solve(_cuda(x), t0, t1, None, ops.LD_ROWSUM)
    assert int(tt.last_nfe.item()) == nfe64
    assert np.abs(_np(y) - y64.numpy()).max() <= 2e-4 and np.abs(_np(a) - a64.numpy()).max() <= 2e-4
    with pytest.raises(NotImplementedError, match="group"):
        t.step_control = "group"
        with torch.no_grad():
            tt._solve(_cuda(x), t0, t1, None, ops.LD_ROWSUM)
