"""Pass-0 constants of the fused autoregressive inverse (include/naz_hip.h naz_ar_flow_pack
``pass0``): with ONE context vector, the first degree pass of every layer — the hidden units of
mask index 0 see only the context, and the first dim in order sees only them — is the same for
every row.  It is computed once per weight draw and layer here (naz_linear_act_batched over
draws x layers, operands gathered from the flat rows by index maps built once) and the packer
writes it in place of that pass's weights; the kernel then skips the pass.  Used by the Bayesian
MAF front end (bflow_maf.lp_batched) and by NormalizingFlow.log_prob with one condition vector
(the density-grid case, naz plot.py:126-127)."""
from __future__ import annotations

from typing import List, Optional

import torch
from torch import Tensor

from .. import ops

_SIG_SCALE = 2.8853900817779268  # 2 / ln 2: the kernel's sigmoid-fold scale of pre-activations


class ArPass0:
    """Index maps and the constant computation for one flow structure (descriptor, permutations).

    flat rows: [P, L * per] in naz_ar_flow_pack_host's layout, per layer W0 [H][C + D] | b0 [H] |
    {Wi [H][H] | bi [H]} | Wout [D Q][H] (ARN rows q D + i) | bout [D Q]; ``mask`` the same layout
    (1 on biases).  ``first[l]`` = the first dim in order of layer l (its permutation's entry 0)."""

    def __init__(self, desc, first: List[int], act: str, device):
        self.desc, self.act, self.dev = desc, act, device
        D, C, H, L, nh = desc.D, desc.C, desc.H, desc.L, desc.n_hidden
        Q = 2 if desc.kind == ops.AR_KIND["maf"] else 3 * desc.K - 1
        deg = torch.as_tensor(ops.ar_flow_degrees(desc))
        self.e0 = e0 = int((deg == 0).sum())
        self.nb, self.nob, self.Q = (e0 + 15) // 16, (Q + 15) // 16, Q
        self.C0 = 16 * (nh * self.nb + self.nob)
        if C <= 0 or e0 <= 0 or ops.ar_flow_pass0_floats(desc) != L * self.C0:
            raise ValueError("ArPass0: no context-only first pass for this descriptor")
        per = H * (C + D) + H + (nh - 1) * (H * H + H) + D * Q * H + D * Q
        maps = []
        for i in range(nh):
            o = 0 if i == 0 else H * (C + D) + H + (i - 1) * (H * H + H)
            cols, ncols = (C, C + D) if i == 0 else (e0, H)
            w = torch.stack([l * per + o + torch.arange(e0)[:, None] * ncols + torch.arange(cols)[None, :]
                             for l in range(L)])
            b = torch.stack([l * per + o + H * ncols + torch.arange(e0) for l in range(L)])
            maps.append((w, b))
        o = H * (C + D) + H + (nh - 1) * (H * H + H)
        rows = [torch.arange(Q) * D + first[l] for l in range(L)]
        w = torch.stack([l * per + o + rows[l][:, None] * H + torch.arange(e0)[None, :] for l in range(L)])
        b = torch.stack([l * per + o + D * Q * H + rows[l] for l in range(L)])
        maps.append((w, b))
        self.maps = [(w.to(device), b.to(device)) for (w, b) in maps]

    def __call__(self, flat: Tensor, context: Tensor, mask: Optional[Tensor] = None) -> Tensor:
        """[P, L * C0] constants of P draws' flat rows under one context vector [C]."""
        P, L, e0, nh = flat.shape[0], self.desc.L, self.e0, self.desc.n_hidden
        ctx = context.reshape(-1).to(self.dev, torch.float32).contiguous()
        h, pres, out = None, [], None
        for i, (wm, bm) in enumerate(self.maps):
            W = flat[:, wm] if mask is None else flat[:, wm] * mask[wm]
            W = W.reshape(P * L, *wm.shape[1:])
            b = flat[:, bm].reshape(P * L, -1)
            if i == nh:
                out = ops.linear_act_batched(h, W, b, "identity")
                break
            pres.append(ops.linear_act_batched(h, W, b, "identity", context=ctx if i == 0 else None))
            h = ops.linear_act_batched(h, W, b, self.act, context=ctx if i == 0 else None)
        c0 = torch.zeros((P, L, self.C0), device=self.dev, dtype=torch.float32)
        for i, z in enumerate(pres):
            c0[:, :, 16 * self.nb * i:16 * self.nb * i + e0] = z.reshape(P, L, e0) * _SIG_SCALE
        o = 16 * self.nb * nh
        c0[:, :, o:o + self.Q] = out.reshape(P, L, self.Q)
        return c0.reshape(P, -1)
