"""One wide-maf GEMM shape, repeated, for PMC passes (scripts/pmc.sh CMD=...):
    python scripts/rg_pmc_probe.py {linear|dact|dw} [M] [K] [N]
linear: naz_linear_act [M, K] -> [M, N] (rowgemm_kernel); dact: naz_gemm_dact (the chains' dX product,
row-major weights); dw: the dW batch reduction of a [M, N] gradient and [M, K] activations (naz_gemm
over transposed views, gemm_tn128_kernel)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from naz_amd import ops  # noqa: E402

what = sys.argv[1]
M, K, N = (int(v) for v in (sys.argv[2:5] if len(sys.argv) >= 5 else (65536, 512, 172)))
dev = torch.device("cuda")
X = torch.randn(M, K, device=dev)
W = torch.randn(N, K, device=dev) / K ** 0.5
b = torch.randn(N, device=dev)
G = torch.randn(M, N, device=dev)
H = torch.tanh(torch.randn(M, K, device=dev))
out = torch.empty(N, K, device=dev)
for _ in range(10):
    if what == "linear":
        ops.linear_act(X, W, b, "tanh")
    elif what == "dact":
        ops.gemm_dact(G, W, H, "tanh")
    else:
        ops.gemm(G.t(), H, out=out)
torch.cuda.synchronize()
print("ok", what, M, K, N)
