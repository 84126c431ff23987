"""Time the batch-row GEMM paths at config-3 training shapes (2^20 rows) and the maf
degree-schedule shapes (ar*) on one GPU.
    NAZ_LIB=... python scripts/gemm_bench.py [--only NAME[,NAME]] [--reps N]"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from naz_amd import ops  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    only = set(args.only.split(",")) if args.only else None
    dev = torch.device("cuda")
    M = 1 << 20
    g = torch.Generator(device=dev).manual_seed(0)
    out = []

    def timeit_(fn):
        return timeit(fn, args.reps)
    # wgrad: dW = G^T X (+ db)
    for n1, n2, name in [(184, 128, "dW2"), (128, 128, "dW1"), (128, 32, "dW0c"), (128, 8, "dW0x")]:
        if only and name not in only:
            continue
        G = torch.randn(M, n1, device=dev, generator=g)
        X = torch.randn(M, n2, device=dev, generator=g)
        C = torch.empty(n1, n2, device=dev)
        rs = torch.empty(n1, device=dev)
        t = timeit_(lambda: ops.gemm(G.t(), X, out=C, rowsum=rs))
        fl = 2 * M * n1 * (n2 + 1)
        out.append(f"{name:6s} wgrad  {t:8.1f} us  {fl / t / 1e6:6.1f} TF  {(G.numel() + X.numel()) * 4 / t / 1e3:6.0f} GB/s")
    # rowgemm forward: act(X W^T + b)
    for k, n, name in [(40, 128, "fwd1"), (128, 128, "fwd2"), (128, 184, "fwd3"), (152, 76, "ar152"), (76, 76, "ar76"), (150, 150, "s150"), (4, 150, "s4"), (152, 152, "s152"),
                       (128, 128, "fwd2id"), (128, 128, "fwd2relu")]:
        if only and name not in only:
            continue
        act = "identity" if name.endswith("id") else ("relu" if name.endswith("relu") else "tanh")
        X = torch.randn(M, k, device=dev, generator=g)
        W = torch.randn(n, k, device=dev, generator=g) / k ** 0.5
        b = torch.randn(n, device=dev, generator=g)
        Y = torch.empty(M, n, device=dev)
        t = timeit_(lambda: ops.linear_act(X, W, b, act, out=Y))
        fl = 2 * M * n * k
        out.append(f"{name:6s} rowgemm {t:8.1f} us  {fl / t / 1e6:6.1f} TF  {(X.numel() + Y.numel()) * 4 / t / 1e3:6.0f} GB/s")
    # dX = G W
    for n_out, k_in, name in [(184, 128, "dX3"), (128, 128, "dX2"), (128, 8, "dX1")]:
        if only and name not in only:
            continue
        G = torch.randn(M, n_out, device=dev, generator=g)
        W = torch.randn(n_out, k_in, device=dev, generator=g)
        t = timeit_(lambda: ops.gemm(G, W))
        fl = 2 * M * n_out * k_in
        out.append(f"{name:6s} rowgemm {t:8.1f} us  {fl / t / 1e6:6.1f} TF  {(G.numel() + M * k_in) * 4 / t / 1e3:6.0f} GB/s")
    # standalone conditional spline (a1/a2): x [M, 8], DenseNN raw [M, 8 * 23], row-sum ld
    for inv, fast, name in [(False, False, "rqsf"), (True, False, "rqsi"), (False, True, "rqsf_fast"),
                            (True, True, "rqsi_fast")]:
        if only and name not in only:
            continue
        X = torch.randn(M, 8, device=dev, generator=g)
        R = torch.randn(M, 8 * 23, device=dev, generator=g)
        ldb = torch.empty(M, device=dev)
        t = timeit_(lambda: ops.rqs(X, R, 8, ops.LAYOUT_DENSE, inv, 3.0, ops.LD_ROWSUM, ldb, fast=fast))
        nbytes = (X.numel() * 2 + R.numel() + M) * 4
        out.append(f"{name:6s} spline  {t:8.1f} us  {nbytes / t / 1e3:6.0f} GB/s (algorithmic bytes)")
    print("\n".join(out))


if __name__ == "__main__":
    main()
