"""Time the batch-row GEMM shapes of the CNF walk (python scripts/rg_res_bench.py).

Measured r02 (one MI355X, 2^18 rows): linear_act softplus 128->128 230 us (37 TF), gemm_dact 185 us,
16->128 136 us, 128->16 38 us, [2^19 x 128]·[128 x 128] 264 us (65 TF).  A weight-resident
persistent variant (weights in LDS for the kernel's lifetime, batch rows straight from HBM as the
transposed MFMA's B operand) measured the same times and was dropped; so did 32-deep k chunks
(NAZ_RG_BK=32, 20-40 % slower) and 256-row workgroups (NAZ_RG_BM=256, within 3 %)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from naz_amd import ops  # noqa: E402

dev = "cuda"
B = 1 << 18
g = torch.Generator(device=dev).manual_seed(0)
res = {}
for (K, N, kind) in [(128, 128, "linear_act softplus"), (128, 128, "gemm_dact"), (16, 128, "linear_act softplus"),
                     (128, 16, "linear_act identity"), (128, 128, "gemm 2B rows")]:
    M = 2 * B if kind.startswith("gemm 2B") else B
    a = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) * 0.1
    b = torch.randn(N, device=dev, generator=g)
    y = torch.rand(M, N, device=dev, generator=g)
    Wt = W.t().contiguous()
    if kind.startswith("linear_act"):
        f = lambda: ops.linear_act(a, W, b, kind.split()[1])
    elif kind == "gemm_dact":
        f = lambda: ops.gemm_dact(a, Wt, y, "softplus")
    else:
        f = lambda: ops.gemm(a, Wt)
    ref = (a.double() @ W.double().t()).float()
    out = f()
    if kind == "linear_act identity" or kind.startswith("gemm 2B"):
        err = float(((out - ref) if kind.startswith("gemm") else (out - ref - b)).abs().max())
    else:
        err = float("nan")
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 20
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    tf = 2 * M * K * N / dt / 1e12
    print(f"{kind:22s} M={M} K={K} N={N}: {dt * 1e6:8.1f} us  {tf:6.1f} TF  maxerr {err:.2e}", flush=True)
