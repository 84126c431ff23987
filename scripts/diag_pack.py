"""diagnostic: words where the device AR pack differs from the host pack (maf paper shape)"""
import numpy as np
import torch
from naz_amd import ops
from tests.test_gpu_ar_fused import CASES, _flow

spec = CASES[4]
f, _ = _flow(spec)
plan = f._plan
flat = plan._flat().astype(np.float32)
perm = np.stack([n.permutation.detach().cpu().numpy() for n in plan._nets()]).astype(np.int32)
dev = ops.ar_flow_pack_batched(plan.desc, torch.tensor(flat[None], device="cuda"), perm)[0].cpu().numpy()
host = ops.ar_flow_pack(plan.desc, flat, perm, "cuda").cpu().numpy()
dv, hv = dev.view(np.uint32), host.view(np.uint32)
bad = np.nonzero(dv != hv)[0]
n = dev.size // spec["L"]
print("layer floats", n, "differing words", bad.size)
for w in bad[:40]:
    print(w // n, w % n, hex(dv[w]), hex(hv[w]), dev[w], host[w])
print("first layers with diffs", np.unique(bad // n)[:20])
