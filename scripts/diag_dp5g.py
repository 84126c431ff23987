"""diagnostic: batch-global dopri5 controller state after a solve vs the fp64 oracle, per batch size."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from naz_amd import ops  # noqa: E402
from naz_amd._lib import lib, check  # noqa: E402
from oracle import naz_oracle as O  # noqa: E402
from tests.test_gpu_cnf import _oracle_block, _oracle_dopri5_global  # noqa: E402

D, C, hidden, act = 4, 2, [32, 32], "softplus"
for B in (1, 2, 16, 17, 37, 200, 1000):
    rng = np.random.default_rng(B)
    x = (rng.standard_normal((B, D)) * 0.8).astype(np.float32)
    c = rng.standard_normal((B, C)).astype(np.float32)
    eps = rng.standard_normal((B, D)).astype(np.float32)
    yg, ag, nfe64 = _oracle_dopri5_global(D, C, hidden, act, x, c, eps, 0.0, 1.0, 1e-4, 1e-4)
    _, _, flat = _oracle_block(D, C, hidden, act, x, c, eps, 0.0, 1.0, 1, torch.float64)
    d = ops.cnf_desc(D, C, hidden, act, "f32")
    packed = ops.cnf_pack(d, torch.as_tensor(flat, device="cuda"))
    nb = int(lib().naz_cnf_dopri5_global_workspace_bytes(d, B))
    work = torch.zeros(nb // 4, device="cuda")
    xd, ed, cd = (torch.as_tensor(v, device="cuda") for v in (x, eps, c))
    y = torch.empty_like(xd)
    ld = torch.empty(B, device="cuda")
    nfe = torch.zeros(1, device="cuda", dtype=torch.int32)
    check(lib().naz_cnf_integrate_dopri5_global(d, packed.data_ptr(), xd.data_ptr(), 4, cd.data_ptr(), 2, ed.data_ptr(),
                                                4, 0.0, 1.0, 1e-4, 1e-4, 1000, y.data_ptr(), 4, ld.data_ptr(), 1,
                                                nfe.data_ptr(), work.data_ptr(), B, None), "dp5g")
    torch.cuda.synchronize()
    n = B * (D + 1)
    parts = work[4 * n:4 * n + 8].cpu().numpy()
    ctrl = work[4 * n + 2 * 2048:4 * n + 2 * 2048 + 16].cpu()
    f = ctrl[:5].numpy()
    i = ctrl.view(torch.int32)[5:11].numpy()
    print(f"B={B} nfe={int(nfe.item())} oracle={nfe64} t,h,hh,h0,d1={f} cur,last,steps,nfe,done,exh={i} "
          f"parts0={parts[:2]} |y-yg|={np.abs(y.cpu().numpy() - yg).max():.2e}", flush=True)
