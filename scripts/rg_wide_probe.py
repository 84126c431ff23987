"""Time the wide maf NLL step's GEMM shapes alone (H = 512 degree blocks) at naz's 10,752-row minibatch
and at 2^16 rows: the batch-row GEMM (linear_act, masked dX, chained act') over the rowgemm_fill
setting, and the dW batch reduction (naz_gemm over transposed views) over split-K.
    python scripts/rg_wide_probe.py
torch.mm of the same product (the platform's fp32 GEMM library) is timed beside it for reference."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from naz_amd import ops  # noqa: E402
from scripts.gemm_bench import timeit  # noqa: E402

dev = torch.device("cuda")
for M in (10752, 65536):
    X = torch.randn(M, 512, device=dev)
    G = torch.randn(M, 512, device=dev)
    H = torch.tanh(torch.randn(M, 512, device=dev))
    W = torch.randn(512, 512, device=dev) / 512 ** 0.5
    b = torch.randn(512, device=dev)
    mask = (torch.rand(512, 512, device=dev) > 0.3).float()
    for K, N in ((512, 512), (512, 172), (426, 512), (86, 170)):
        Xk, Wk, bk = X[:, :K], W[:N, :K].contiguous(), b[:N].contiguous()
        t0 = timeit(lambda: torch.mm(Xk, Wk.t()))
        print(f"M={M} K={K} N={N}: torch.mm (library fp32) {t0:7.1f} us {2.0 * M * N * K / t0 / 1e6:6.1f} TF", flush=True)
        for fill in (0, 1, 2, 4, 8):
            ops.rowgemm_fill(fill)
            t = timeit(lambda: ops.linear_act(Xk, Wk, bk, "tanh"))
            t2 = timeit(lambda: ops.gemm_dact(G[:, :N], Wk, H[:, :K], "tanh"))  # (the wide path's weights come masked)
            f = 2.0 * M * N * K
            print(f"M={M} K={K} N={N} fill={fill}: linear_act {t:7.1f} us {f / t / 1e6:6.1f} TF | "
                  f"gemm_dact {t2:7.1f} us {f / t2 / 1e6:6.1f} TF", flush=True)
    ops.rowgemm_fill(2)
    for N1, N2 in ((512, 512), (172, 512), (512, 86)):
        out = torch.empty(N1, N2, device=dev)
        for sk in (1, 4, 8, 16, 21, 32, 64):
            t = timeit(lambda: ops.gemm(G[:, :N1].t(), H[:, :N2], out=out, split_k=sk, accumulate=sk > 1))
            print(f"M={M} dW {N1}x{N2} split_k={sk}: {t:7.1f} us {2.0 * M * N1 * N2 / t / 1e6:6.1f} TF", flush=True)
