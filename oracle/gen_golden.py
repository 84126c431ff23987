"""TEST INFRASTRUCTURE ONLY — writes the committed parity fixtures under tests/golden/.

    python -m oracle.gen_golden

Every fixture stores fp32 inputs/weights and the oracle's float64 outputs computed from
those exact fp32 values (plus, for flows, the oracle's own float32 result = what the
reference's fp32 CPU path produces), so the GPU kernels are compared with the same
numbers on the GPU box without the oracle having to run there.
Parity status: see oracle/__init__.py (pyro semantics restated; no reference-run pin).
"""
from __future__ import annotations

import os
from pathlib import Path

import numpy as np
import torch

from . import jax_maf_np as J
from . import naz_oracle as O

OUT = Path(__file__).resolve().parent.parent / "tests" / "golden"


def _spline_fixture(name, B, Dt, K, layout, seed, scale=2.5, tail_frac=0.15):
    g = torch.Generator().manual_seed(seed)
    raw = (torch.randn(B, Dt * (3 * K - 1), generator=g) * scale).float()
    x = (torch.rand(B, Dt, generator=g) * 6 - 3).float()
    # tails, exact knots-of-the-box and exact zeros
    nt = int(B * tail_frac)
    x[:nt] = (torch.randn(nt, Dt, generator=g) * 5).float()
    x[nt, :] = 3.0
    x[nt + 1, :] = -3.0
    x[nt + 2, :] = 0.0
    x64, raw64 = x.double(), raw.double()
    yf, ldf = O.rqs_from_raw(x64, raw64, Dt, K, layout, inverse=False)
    yi, ldi = O.rqs_from_raw(x64, raw64, Dt, K, layout, inverse=True)
    np.savez(OUT / name, x=x.numpy(), raw=raw.numpy(), y_fwd=yf.numpy(), ld_fwd=ldf.numpy(), y_inv=yi.numpy(),
             ld_inv=ldi.numpy(), K=K, Dt=Dt, layout=layout)


def _flow_fixture(name, spec, n, seed_w=1234, seed_x=0, seed_c=1):
    state = O.random_state(spec, seed=seed_w)
    state32 = {k: (v.float() if v.is_floating_point() else v) for k, v in state.items()}
    f64 = O.build_flow(spec, state32, torch.float64)
    f32 = O.build_flow(spec, state32, torch.float32)
    x = torch.as_tensor(O.gaussian_mixture(n, spec["D"], seed=seed_x))
    c = torch.as_tensor(O.context_normal(n, spec["C"], seed=seed_c)) if spec["C"] > 0 else None
    lp64 = f64.log_prob(x.double(), None if c is None else c.double())
    lp32 = f32.log_prob(x, c)
    z = torch.randn(n, spec["D"], generator=torch.Generator().manual_seed(seed_x + 7)).float()
    ys, lds = f64.forward_with_logdet(z.double(), None if c is None else c.double())
    arrays = {"x": x.numpy(), "lp64": lp64.numpy(), "lp32": lp32.numpy(), "z": z.numpy(), "y_sample": ys.numpy(),
              "ld_sample": lds.numpy()}
    if c is not None:
        arrays["ctx"] = c.numpy()
    for k, v in state32.items():
        arrays["state/" + k] = v.numpy()
    for k, v in spec.items():
        if k != "bounds":
            arrays["spec/" + k] = np.asarray(v)
    np.savez(OUT / name, **arrays)
    return f64, state32, x, c


def _cnf_fixture(name, spec, n, seed_w=1234, seed_x=0, seed_c=1, seed_e=5):
    """a11: FFJORD blocks with the Hutchinson probes fixed and stored (eps_l/{l}: log_prob
    direction, eps_s/{l}: sampling direction)."""
    state = O.random_state(spec, seed=seed_w, last_layer_scale=1.0)
    state32 = {k: v.float() for k, v in state.items()}
    D, C, L = spec["D"], spec["C"], spec["L"]
    x = torch.as_tensor(O.gaussian_mixture(n, D, seed=seed_x)) * 0.5
    c = torch.as_tensor(O.context_normal(n, C, seed=seed_c)) if C > 0 else None
    g = torch.Generator().manual_seed(seed_e)
    eps_l = [torch.randn(n, D, generator=g).float() for _ in range(L)]
    eps_s = [torch.randn(n, D, generator=g).float() for _ in range(L)]
    z = torch.randn(n, D, generator=g).float()
    out = {}
    for dt, key in ((torch.float64, "64"), (torch.float32, "32")):
        f = O.build_flow(spec, state32, dt)
        for layer, e in zip(f.layers, eps_l):
            layer.eps = e
        out["lp" + key] = f.log_prob(x.to(dt), None if c is None else c.to(dt)).numpy()
        for layer, e in zip(f.layers, eps_s):
            layer.eps = e
        ys, lds = f.forward_with_logdet(z.to(dt), None if c is None else c.to(dt))
        out["y_sample" + key], out["ld_sample" + key] = ys.numpy(), lds.numpy()
    arrays = {"x": x.numpy(), "z": z.numpy(), **out}
    for l in range(L):
        arrays[f"eps_l/{l}"], arrays[f"eps_s/{l}"] = eps_l[l].numpy(), eps_s[l].numpy()
    if c is not None:
        arrays["ctx"] = c.numpy()
    for k, v in state32.items():
        arrays["state/" + k] = v.numpy()
    for k, v in spec.items():
        arrays["spec/" + k] = np.asarray(v)
    np.savez(OUT / name, **arrays)


def cnf_fixtures():
    _cnf_fixture("cnf_d4c2.npz", dict(flow_type="cnf", D=4, C=2, hidden=[32, 32], L=2, activation="softplus",
                                      steps=8), 256)
    # config 5's block shape (D=16, H=[128]*3, unconditional), one block
    _cnf_fixture("cnf_d16c0.npz", dict(flow_type="cnf", D=16, C=0, hidden=[128, 128, 128], L=1,
                                       activation="softplus", steps=8), 256)


def main():
    OUT.mkdir(parents=True, exist_ok=True)
    cnf_fixtures()
    _spline_fixture("rqs_dense_k8.npz", 512, 4, 8, O.LAYOUT_DENSE, seed=11)
    _spline_fixture("rqs_arn_k5.npz", 384, 3, 5, O.LAYOUT_ARN, seed=12)
    _spline_fixture("rqs_dense_k16.npz", 256, 6, 16, O.LAYOUT_DENSE, seed=13)
    # the metric configuration's layer shapes (D16 | C32, K8, H[128,128]) at L=2 to keep the file small
    _flow_fixture("nsc_d16c32_l2.npz", dict(flow_type="nsc", D=16, C=32, hidden=[128, 128], L=2, K=8, split=8), 256)
    _flow_fixture("nsc_d8c0_l6.npz", dict(flow_type="nsc", D=8, C=0, hidden=[128, 128], L=6, K=8, split=4), 256)
    _flow_fixture("nsc_d6c2_small.npz", dict(flow_type="nsc", D=6, C=2, hidden=[32, 32], L=3, K=4, split=2), 300)
    _flow_fixture("nsa_d4c2.npz", dict(flow_type="nsa", D=4, C=2, hidden=[32, 32], L=2, K=8), 200)
    spec = dict(flow_type="maf", D=3, C=2, hidden=[16, 16], L=3)
    f64, state32, x, c = _flow_fixture("maf_d3c2.npz", spec, 200)
    # cross-check pin: the reference's in-tree JAX restatement (numpy) of the same affine MAF
    lp_jax = J.log_prob(x.numpy().astype(np.float64), J.layers_from_state(spec, {k: v.numpy() for k, v in
                                                                              state32.items()}), c.numpy())
    with np.load(OUT / "maf_d3c2.npz") as z:
        arrays = {k: z[k] for k in z.files}
    arrays["lp_jaxref"] = lp_jax
    np.savez(OUT / "maf_d3c2.npz", **arrays)
    # config 1: 2-D two-moons unconditional affine MAF, L=8 (the paper scripts use H=[150]*3;
    # H=[64,64] keeps the committed fixture small — same code path)
    spec1 = dict(flow_type="maf", D=2, C=0, hidden=[64, 64], L=8)
    state = O.random_state(spec1, seed=1234, last_layer_scale=1.0)
    state32 = {k: (v.float() if v.is_floating_point() else v) for k, v in state.items()}
    xm = torch.as_tensor(O.two_moons(2048, seed=0))
    f = O.build_flow(spec1, state32, torch.float64)
    arrays = {"x": xm.numpy(), "lp64": f.log_prob(xm.double()).numpy(),
              "lp32": O.build_flow(spec1, state32, torch.float32).log_prob(xm).numpy()}
    for k, v in state32.items():
        arrays["state/" + k] = v.numpy()
    for k, v in spec1.items():
        arrays["spec/" + k] = np.asarray(v)
    np.savez(OUT / "maf_twomoons.npz", **arrays)
    for p in sorted(OUT.glob("*.npz")):
        print(f"{p.name:28s} {os.path.getsize(p) / 1024:8.1f} KiB")


if __name__ == "__main__":
    import sys
    if sys.argv[1:] == ["cnf"]:
        OUT.mkdir(parents=True, exist_ok=True)
        cnf_fixtures()
    else:
        main()
