"""Diagnostic: NLL gradients of the config-3 flow over a batch vs the sum over two ragged halves,
and each against the fp64 oracle, per parameter tensor (norm-wise relative errors)."""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oracle import naz_oracle as O  # noqa: E402
from naz_amd.flows import NormalizingFlow  # noqa: E402
from naz_amd.flows import io as fio  # noqa: E402

spec = dict(flow_type="nsc", D=16, C=32, hidden=[128, 128], L=int(sys.argv[1]) if len(sys.argv) > 1 else 8, K=8, split=8)
state = {k: v.numpy() for k, v in O.random_state(spec, seed=99).items()}
G = 3001
x = O.gaussian_mixture(G, 16, seed=5)
c = O.context_normal(G, 32, seed=6)


def grads(rows_list):
    f = NormalizingFlow("nsc", None, 16, 32, [128, 128], spec["L"], 8, 8)
    fio.load_state(f, state)
    for a, b in rows_list:
        lp = f.log_prob(torch.as_tensor(x[a:b], device="cuda"), condition=torch.as_tensor(c[a:b], device="cuda"))
        (-lp.sum() / G).backward()
    return {k: p.grad.detach().double().cpu().numpy() for k, p in fio.named_state_params(f).items()}


def oracle(a, b):
    st = {k: torch.as_tensor(v).double().requires_grad_(True) for k, v in state.items()}
    of = O.build_flow(spec, st, torch.float64)
    lp = of.log_prob(torch.as_tensor(x[a:b]).double(), torch.as_tensor(c[a:b]).double())
    keys = list(st)
    gs = torch.autograd.grad(-lp.sum() / G, [st[k] for k in keys])
    return {k: g.numpy() for k, g in zip(keys, gs)}


full = grads([(0, G)])
halves = grads([(0, 1501), (1501, G)])
o_full = oracle(0, G)
for k in full:
    r = lambda a, b: np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)
    print(f"{k:55s} full-vs-halves {r(halves[k], full[k]):.2e}  full-vs-oracle {r(full[k], o_full[k]):.2e}  "
          f"halves-vs-oracle {r(halves[k], o_full[k]):.2e}")
