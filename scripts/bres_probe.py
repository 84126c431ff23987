"""Probe the B-resident f16x3 batch-row GEMM (naz_tuning "rowgemm_bres") against the FP32 rowgemm at the
CNF training shapes (2^19 paired rows, 128 -> 128) and the wide maf's (2^16 / 10,752 rows, K up to 512):
time (us, TF) and the error of each against an fp64 torch product (max |err| / max |ref|).
    python scripts/bres_probe.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from naz_amd import ops  # noqa: E402
from scripts.gemm_bench import timeit  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)


def err(out, ref):
    return float((out.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-300))


cases = [(1 << 19, 128, 128, "softplus"), (1 << 18, 128, 128, "softplus"), (1 << 16, 512, 172, "tanh"),
         (1 << 16, 512, 512, "tanh"), (1 << 16, 86, 170, "tanh"), (10752, 512, 512, "tanh"), (1 << 16, 426, 512, "tanh")]
for M, K, N, act in cases:
    X = torch.randn(M, K, device=dev)
    X[::7] *= 1e-3  # rows of very different scale (gradients)
    W = torch.randn(N, K, device=dev) / K ** 0.5
    b = torch.randn(N, device=dev)
    G = torch.randn(M, N, device=dev)
    Hy = torch.tanh(torch.randn(M, K, device=dev)) if act == "tanh" else torch.nn.functional.softplus(torch.randn(M, K, device=dev))
    pre = X.double() @ W.double().t() + b.double()
    ref_lin = torch.tanh(pre) if act == "tanh" else torch.nn.functional.softplus(pre)
    # gemm_dact: (G @ W) * act'(y) with y = Hy; W here [N, K] -> G [M, N] @ W [N, K]
    dref = G.double() @ W.double()
    dref = dref * ((1 - Hy.double() ** 2) if act == "tanh" else (1 - torch.exp(-Hy.double())))
    f = 2.0 * M * N * K
    for mode in ("fp32", "bres", "h3"):
        ops.rowgemm_bres(mode == "bres")
        ops.rowgemm_h3(mode == "h3")
        o1 = ops.linear_act(X, W, b, act)
        o2 = ops.gemm_dact(G, W, Hy, act)
        torch.cuda.synchronize()
        e1, e2 = err(o1, ref_lin), err(o2, dref)
        t1 = timeit(lambda: ops.linear_act(X, W, b, act))
        t2 = timeit(lambda: ops.gemm_dact(G, W, Hy, act))
        print(f"M={M} K={K} N={N} {mode:5s}: linear_act {t1:8.1f} us {f / t1 / 1e6:6.1f} TF err {e1:.1e} | "
              f"gemm_dact {t2:8.1f} us {f / t2 / 1e6:6.1f} TF err {e2:.1e}", flush=True)
ops.rowgemm_bres(False)
ops.rowgemm_h3(False)
