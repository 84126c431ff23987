"""CPU: the oracle's CNF arithmetic pinned to the REFERENCE'S OWN ODE code.

tests/golden/cnf_refode_*.npz hold outputs of naz's in-tree pure-torch solver and trace estimator
(src/naz/neural_nets/__deprecated__/neural_odes/odeint.py RK4 :39-52 / integrate :12-19 / Dopri5
:96-112,136-160, cnf.py:22-37 trace_df_dz_hutchinson), run in this container by
oracle/gen_refode_fixtures.py over a fixed FFJORD field.  The oracle's restatements
(rk4_augmented, dopri5_step, hutchinson_rhs) must reproduce them to float64 round-off; the HIP
kernel is checked against the same fixtures in tests/test_gpu_cnf.py.
"""
import numpy as np
import pytest
import torch

from oracle import naz_oracle as O
from tests.conftest import load_golden, spec_state

NAMES = ["cnf_refode_d4c2.npz", "cnf_refode_d16c0.npz", "cnf_refode_d4c4_h128x4.npz"]


def _net_inputs(fx):
    spec, state = spec_state(fx)
    net = O.build_flow(spec, state, torch.float64).layers[0].nn
    x = torch.tensor(fx["x"], dtype=torch.float64)
    c = torch.tensor(fx["ctx"], dtype=torch.float64) if "ctx" in fx else None
    e = torch.tensor(fx["eps"], dtype=torch.float64)
    return net, x, c, e


def _close(a, b, tol=1e-10):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    err = np.abs(a - b).max() / max(1.0, np.abs(b).max())
    assert err < tol, err


@pytest.mark.parametrize("name", NAMES)
def test_oracle_trace_matches_reference_estimator(name):
    fx = load_golden(name)
    net, x, c, e = _net_inputs(fx)
    f, negtr = O.hutchinson_rhs(net, x, c, e)
    _close(f.numpy(), fx["f64"])
    _close(negtr.numpy(), fx["negtr64"])


@pytest.mark.parametrize("name", NAMES)
def test_oracle_rk4_matches_reference_odeint(name):
    fx = load_golden(name)
    net, x, c, e = _net_inputs(fx)
    z = torch.tensor(fx["z"], dtype=torch.float64)
    n = int(fx["steps"])
    xi, ai = O.rk4_augmented(net, x, c, e, 0.0, 1.0, n)  # log_prob direction
    _close(xi.numpy(), fx["inv_x64"])
    _close(ai.numpy(), fx["inv_a64"])
    xf, af = O.rk4_augmented(net, z, c, e, 1.0, 0.0, n)  # sampling direction
    _close(xf.numpy(), fx["fwd_x64"])
    _close(af.numpy(), fx["fwd_a64"])
    xs, as_ = O.rk4_augmented(net, x, c, e, 0.0, 0.125, 1)  # one step
    _close(xs.numpy(), fx["step_x64"])
    _close(as_.numpy(), fx["step_a64"])
    # the float32 reference run is the ref32 the GPU test uses: it must be a float32-level
    # perturbation of the float64 one
    assert np.abs(fx["inv_x32"] - fx["inv_x64"]).max() < 1e-4


@pytest.mark.parametrize("name", NAMES)
def test_oracle_dopri5_step_matches_reference(name):
    fx = load_golden(name)
    net, x, c, e = _net_inputs(fx)
    h = float(fx["dp5_h"])
    a = torch.zeros(x.shape[0], dtype=torch.float64)
    y5, a5, _, en = O.dopri5_step(net, x, a, c, e, h, 1e-4, 1e-4)
    _close((y5 - x).numpy(), fx["dp5_dx64"])
    _close((a5 - a).numpy(), fx["dp5_da64"])
    # the reference returns dt_new = h (0.5 / err_norm)^(1/5): recover its error norm
    en_ref = 0.5 / (float(fx["dp5_dt_new64"]) / h) ** 5
    assert abs(en - en_ref) <= 1e-8 * max(1.0, en_ref), (en, en_ref)
