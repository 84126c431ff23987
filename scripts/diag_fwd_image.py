"""GPU diagnostic: the forward (sample) image of a maf flow from the host packer vs the device
packer (word for word), and the sampler on each image vs the fp64 oracle's forward.

    python scripts/diag_fwd_image.py [D C H NHID L]
"""
import sys

import numpy as np
import torch

from naz_amd import ops
from oracle import naz_oracle as O


def main():
    D, C, H, NH, L = (int(a) for a in sys.argv[1:6]) if len(sys.argv) > 5 else (2, 2, 150, 3, 3)
    spec = dict(flow_type="maf", D=D, C=C, hidden=[H] * NH, L=L)
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    state = {k: v.float() for k, v in O.random_state(spec, seed=11).items()}
    f = NormalizingFlow("maf", None, D, C, [H] * NH, L)
    fio.load_state(f, {k: v.numpy() for k, v in state.items()})
    f = f.to("cuda")
    plan = f._plan
    flat = plan._flat()
    host = ops.ar_flow_pack_fwd(plan.desc, flat, "cuda")
    dev = ops.ar_flow_pack_fwd_batched(plan.desc, torch.from_numpy(flat).cuda()[None].contiguous())
    hw, dw = host.view(torch.int32), dev[0].view(torch.int32)
    diff = (hw != dw).nonzero().flatten()
    print("image words", hw.numel(), "differing", diff.numel(), diff[:10].tolist())
    n = 700
    g = torch.Generator().manual_seed(5)
    z = torch.randn(n, D, generator=g)
    c = torch.randn(n, C, generator=g) if C else None
    cd = None if c is None else c.cuda()
    for name, img in (("host", host), ("device", dev[0].contiguous())):
        y, ld = ops.ar_flow_sample(plan.desc, img, z.cuda(), cd, with_logdet=True)
        y = y.cpu().numpy()
        print(name, "finite", bool(np.isfinite(y).all()), "nan rows", int((~np.isfinite(y)).any(1).sum()))
    of = O.build_flow(spec, state, torch.float64)
    y64, _ = of.forward_with_logdet(z.double(), None if c is None else c.double())
    y, _ = ops.ar_flow_sample(plan.desc, host, z.cuda(), cd, with_logdet=True)
    err = np.abs(y.cpu().numpy() - y64.numpy()).max()
    print("host image vs fp64 oracle max |dy|", err)


if __name__ == "__main__":
    main()
