"""Diagnose the fused maf gradient: repeat eager / graph calls, locate differing entries."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from tests.test_bayes_maf import _setup, _flow
from naz_amd.flows import bflow_maf as BM

spec = dict(flow_type="maf", D=2, C=2, hidden=[150, 150, 150], L=3, P=2, B=int(sys.argv[1]) if len(sys.argv) > 1 else 1500,
            ctx="rows")
layers, draws, x, ctx = _setup(spec, seed=11)
flow = _flow(spec, layers, x, ctx, "cuda")
def flat_of(d):
    return BM.ravel([[(torch.tensor(W, dtype=torch.float32, device="cuda"),
                       torch.tensor(b, dtype=torch.float32, device="cuda")) for (W, b) in lay] for lay in d])
H, C, D = 150, 2, 2
names = []
for l in range(3):
    for i, (r, c) in enumerate([(H, C + D), (H, H), (H, H), (2 * D, H)]):
        names += [f"L{l}W{i}"] * (r * c) + [f"L{l}b{i}"] * r
names = np.array(names)
for k, d in enumerate(draws):
    p = flat_of(d)
    res = [flow["lp_and_grad"](p, use_graph=False)[1].cpu().numpy() for _ in range(3)]
    res += [flow["lp_and_grad"](p)[1].cpu().numpy() for _ in range(2)]
    for j in range(1, len(res)):
        diff = np.abs(res[j] - res[0])
        bad = np.nonzero(diff > 1e-4 * np.abs(res[0]).max())[0]
        print(f"draw {k} call {j} ({'eager' if j < 3 else 'graph'}): max rel {diff.max() / np.abs(res[0]).max():.3e}, "
              f"{len(bad)} bad, nonfinite {int((~np.isfinite(res[j])).sum())}/{int((~np.isfinite(res[0])).sum())}",
              sorted(set(names[bad]))[:12])
