"""Probe: the NLL step's weight-gradient GEMMs (dW = dPre^T X over 2^20 rows) — naz_gemm
(wgrad_flat) vs torch.mm (rocBLAS / hipBLASLt) for reference."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from naz_amd import ops  # noqa: E402

B = 1 << 20
dev = "cuda"
SHAPES = [(192, 128), (128, 128), (128, 40)]
if os.environ.get("WG_SHAPES"):  # e.g. "192x128,128x40"
    SHAPES = [tuple(int(v) for v in t.split("x")) for t in os.environ["WG_SHAPES"].split(",")]
MM = os.environ.get("WG_TORCH", "1") != "0"
for (n1, n2) in SHAPES:
    g = torch.randn(B, n1, device=dev)
    x = torch.randn(B, n2, device=dev)
    out = torch.empty(n1, n2, device=dev)
    rs = torch.empty(n1, device=dev)
    fns = [("naz_gemm", lambda: ops.gemm(g.t(), x, out=out, rowsum=rs))]
    if MM:
        fns.append(("torch.mm", lambda: torch.mm(g.t(), x)))
    for name, fn in fns:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{n1}x{n2} {name}: {ms:.3f} ms  {2 * n1 * n2 * B / ms / 1e9:.1f} TF", flush=True)
    ref = (g.double().t() @ x.double())
    print("  max rel err naz", float(((out.double() - ref).abs().max() / ref.abs().max())))
