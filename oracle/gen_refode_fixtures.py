"""TEST INFRASTRUCTURE ONLY — pins the CNF solver and trace arithmetic to the reference's OWN code.

    python -m oracle.gen_refode_fixtures        # in the build container (needs /root/reference)

naz ships a pure-torch ODE toolkit (src/naz/neural_nets/__deprecated__/neural_odes/): fixed-step
``RK4`` (odeint.py:39-52, integrated by ``ODESolver.integrate`` :12-19 through ``odeint`` :200-212),
the ``Dopri5`` tableau and step (odeint.py:96-112,136-160) and Hutchinson's estimator
``trace_df_dz_hutchinson`` (cnf.py:22-37).  Unlike the pyro / torchdyn arithmetic of the flows, these
IMPORT here (torch only), so this script runs them and stores their outputs as fixtures:

  * an 8-step RK4 solve of the FFJORD augmented field d[x, a]/dt = [f(x, ctx), -eps^T (df/dx) eps]
    (torchdyn's CNF sign, continuous_transforms.py:85-89) in both directions (t 0 -> 1 = log_prob,
    1 -> 0 = sample), run by the reference's ``odeint(..., 'rk4')`` in float64 and float32;
  * one RK4 step;
  * the trace term at x: the reference's ``trace_df_dz_hutchinson(f, x, n_samples=1)`` with its probe
    drawn under a fixed seed (the same probe re-drawn every call = one probe per solve, torchdyn's
    FFJORD semantics), and the probe itself;
  * one Dormand-Prince step of the reference's ``Dopri5._step_fn`` (dx and its dt_new, whose
    error norm the oracle's step restates).

The vector field f is the oracle's FCNN (naz ``ConditionalFCNN``: Linear + Softplus, input
cat([x, ctx])) with fixed fp32 weights: a field, not the thing pinned.  Nothing from the reference
travels to the GPU box or is committed: only the .npz arrays (inputs and outputs) under
tests/golden/ do.  ``tests/test_refode_pin.py`` checks the oracle against them (CPU) and
``tests/test_gpu_cnf.py::test_cnf_kernel_vs_reference_odeint`` the HIP solve (GPU).
"""
from __future__ import annotations

import importlib.util
import sys
import types
from pathlib import Path

import numpy as np
import torch

from . import naz_oracle as O

REF = Path("/root/reference/src/naz/neural_nets/__deprecated__/neural_odes")
OUT = Path(__file__).resolve().parent.parent / "tests" / "golden"
SEED_PROBE = 4242


def _load_reference():
    """odeint.py and cnf.py as modules of a private package (their relative imports: .misc,
    .odeint), without importing naz's top-level package (which needs jax / pyro)."""
    pkg = types.ModuleType("_naz_ref_neural_odes")
    pkg.__path__ = [str(REF)]
    sys.modules[pkg.__name__] = pkg
    mods = {}
    for name in ("misc", "odeint", "cnf"):
        spec = importlib.util.spec_from_file_location(f"{pkg.__name__}.{name}", REF / f"{name}.py")
        m = importlib.util.module_from_spec(spec)
        sys.modules[spec.name] = m
        spec.loader.exec_module(m)
        mods[name] = m
    return mods["odeint"], mods["cnf"]


def _field(cnf_mod, net, ctx):
    """The reference's RHS form: func(t, (z, logp)) -> (dz/dt, dlogp/dt), the trace by the
    reference's own estimator with the probe drawn under SEED_PROBE (identical every call)."""
    def func(t, states):
        z = states[0]
        with torch.enable_grad():
            zz = z.detach().requires_grad_(True)
            f = net(zz, ctx)
            torch.manual_seed(SEED_PROBE)
            tr = cnf_mod.trace_df_dz_hutchinson(f, zz, n_samples=1, is_training=False)
        return f.detach(), -tr.detach()
    return func


def _fixture(name, spec, n, seed_w=1234, seed_x=0, seed_c=1):
    odeint_mod, cnf_mod = _load_reference()
    state = O.random_state(spec, seed=seed_w, last_layer_scale=1.0)
    state32 = {k: v.float() for k, v in state.items()}
    D, C = spec["D"], spec["C"]
    x = (torch.as_tensor(O.gaussian_mixture(n, D, seed=seed_x)) * 0.5).float()
    z = torch.randn(n, D, generator=torch.Generator().manual_seed(seed_x + 9)).float()
    c = torch.as_tensor(O.context_normal(n, C, seed=seed_c)).float() if C > 0 else None
    torch.manual_seed(SEED_PROBE)  # the probe the reference's estimator draws ([B, 1, D], then cast)
    eps = torch.randn([n, 1, D])[:, 0, :].float()
    arrays = {"x": x.numpy(), "z": z.numpy(), "eps": eps.numpy(), "steps": np.asarray(8)}
    for dt, key in ((torch.float64, "64"), (torch.float32, "32")):
        f = O.build_flow(spec, state32, dt)
        net = f.layers[0].nn
        cc = None if c is None else c.to(dt)
        func = _field(cnf_mod, net, cc)
        a0 = torch.zeros(n, dtype=dt)
        for direction, (t0, t1) in (("inv", (0.0, 1.0)), ("fwd", (1.0, 0.0))):
            times = torch.linspace(t0, t1, 9, dtype=torch.float64)
            v0 = x if direction == "inv" else z
            v1, a1 = odeint_mod.odeint(func, (v0.to(dt), a0), times, "rk4")
            arrays[f"{direction}_x{key}"], arrays[f"{direction}_a{key}"] = v1.numpy(), a1.numpy()
        # one RK4 step (t 0 -> 1/8)
        s1, sa1 = odeint_mod.odeint(func, (x.to(dt), a0), torch.tensor([0.0, 0.125], dtype=torch.float64), "rk4")
        arrays[f"step_x{key}"], arrays[f"step_a{key}"] = s1.numpy(), sa1.numpy()
        # the trace term and the field at x
        fx, tr = func(None, (x.to(dt), a0))
        arrays[f"f{key}"], arrays[f"negtr{key}"] = fx.numpy(), tr.numpy()
        if key == "64":
            # one Dormand-Prince step of the reference (flattened [x, a] state, atol = rtol = 1e-4)
            shapes = [torch.Size([n, D]), torch.Size([n])]
            solver = odeint_mod.Dopri5(odeint_mod._tuple_func_wrapper(func, shapes), rtol=1e-4, atol=1e-4)
            st0 = odeint_mod._to_flat((x.to(dt), a0))
            h = torch.tensor(0.1, dtype=dt)
            dxf, dt_new = solver._step_fn(torch.tensor(0.0, dtype=dt), st0, h)
            arrays["dp5_h"] = np.asarray(0.1)
            arrays["dp5_dx64"], arrays["dp5_da64"] = dxf[:n * D].reshape(n, D).numpy(), dxf[n * D:].numpy()
            arrays["dp5_dt_new64"] = np.asarray(float(dt_new))
    if c is not None:
        arrays["ctx"] = c.numpy()
    for k, v in state32.items():
        arrays["state/" + k] = v.numpy()
    for k, v in spec.items():
        arrays["spec/" + k] = np.asarray(v)
    np.savez(OUT / name, **arrays)
    print("wrote", OUT / name)


def main():
    if not REF.exists():
        raise SystemExit(f"{REF} not found: the fixtures are generated in the build container only")
    _fixture("cnf_refode_d4c2.npz", dict(flow_type="cnf", D=4, C=2, hidden=[32, 32], L=1, activation="softplus",
                                         steps=8), 192)
    # config 5's block shape (D=16, H=[128]*3, unconditional)
    _fixture("cnf_refode_d16c0.npz", dict(flow_type="cnf", D=16, C=0, hidden=[128, 128, 128], L=1,
                                          activation="softplus", steps=8), 160)
    # naz's POSYDON CNF (examples/papers/eposydon/train_cnf_mle.py:91, train_cnf_mle_q.py:92: 4 parameters,
    # H = [128] x 4, one block; the lambda width comes from the data file: 4 here)
    _fixture("cnf_refode_d4c4_h128x4.npz", dict(flow_type="cnf", D=4, C=4, hidden=[128] * 4, L=1,
                                                activation="softplus", steps=8), 128)


if __name__ == "__main__":
    main()
