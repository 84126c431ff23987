"""diagnostic: non-finite rows of the config-3 headline flow at 2^20 rows (test_full_size_exact_properties)"""
import torch
from oracle import naz_oracle as O
from tests.test_gpu_parity import _config3_flow

DEV = "cuda"
f, spec, state = _config3_flow()
f = f.to(DEV)
B = 1 << 20
g = torch.Generator(device=DEV).manual_seed(0)
x = torch.as_tensor(O.gaussian_mixture(B, 16, seed=0), device=DEV)
c = torch.randn(B, 32, device=DEV, generator=g)
for trial in range(3):
    lp = f.log_prob(x, condition=c)
    bad = torch.nonzero(~torch.isfinite(lp)).reshape(-1)
    print("trial", trial, "non-finite rows", bad.numel(), bad[:10].tolist(), lp[bad[:10]].tolist())
    if bad.numel():
        r = bad[:4]
        print("  rows alone:", f.log_prob(x[r], condition=c[r]).tolist())
        print("  |x| max", float(x[r].abs().max()), "|c| max", float(c[r].abs().max()))
        blk = (bad // 128).unique()
        print("  128-row blocks", blk[:10].tolist())
print("x absmax", float(x.abs().max()), "c absmax", float(c.abs().max()))
