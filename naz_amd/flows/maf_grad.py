"""Fused gradient of Σ_rows log p(x | ctx) over a naz affine MAF.

The NUTS / HMC potential of naz's Bayesian MAF is ``flow_lp(unravel(p)).sum()`` and its gradient
(naz/flows/bflow_jax_maf.py:231-235, examples/papers/2506.05657/hmc_maf_exact.py:118-133): one
forward over the whole training set and one backward per leapfrog step.  Here that is

  * the fused inverse kernel with every layer's output saved (naz_ar_flow_log_prob_train);
  * per layer l = 0 .. L-1 one fused backward launch (naz_ar_flow_bwd_layer, csrc/made_ar_bwd.h:
    dense MADE recompute, the affine VJP, the D-order chain of input gradients, the total δ's)
    writing the weight-gradient operands;
  * per layer the batch reductions dW = δᵀ·h (+ bias column sums) on naz_gemm's bf16x6 wgrad
    kernel, into a padded per-layer workspace;
  * ONE gather of the workspace into ``ravel`` order times the masks (pyro MaskedLinear's
    gradient is mask ⊙ (δᵀ h)).

No autograd graph, no per-block gathers: ~10 launches per layer.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
from torch import Tensor

from .. import ops


class MafGrad:
    """(Σ lp, ∇θ) of one flat θ (``ravel`` order = the naz_ar_flow_pack_host flat layout) over
    fixed rows ``x`` [B, D] and ``ctx`` ([B, C], [C] or None).  ``mask`` [L * per]: the MADE
    masks in the flat layout (1 on biases); ``perms`` [L, D]: dim of order p per layer."""

    def __init__(self, desc, perms: np.ndarray, mask: Tensor, x: Tensor, ctx: Optional[Tensor]):
        if not ops.ar_flow_bwd_supported(desc):
            raise RuntimeError("MafGrad: no fused maf backward for this shape")
        self.desc = desc
        dev = x.device
        self.dev = dev
        D, C, H, L = desc.D, desc.C, desc.H, desc.L
        dm = ops.ar_flow_bwd_dims(desc)
        NH, HP, XA, XB, X0W = dm["n_hidden"], dm["HP"], dm["XA"], dm["XB"], dm["X0W"]
        self.dims = dm
        self.x = x.to(torch.float32).contiguous()
        self.ctx = None if ctx is None else ctx.to(dev, torch.float32).contiguous()
        B = self.x.shape[0]
        self.B = B
        self.perms = np.ascontiguousarray(np.asarray(perms), dtype=np.int32)
        self.perm_dev = torch.from_numpy(self.perms).to(dev)
        self.mask = mask.to(dev, torch.float32).contiguous()
        f32 = dict(device=dev, dtype=torch.float32)
        self.states = torch.empty((L, B, D), **f32)
        self.lp = torch.empty((B,), **f32)
        self.g = torch.empty((B, D), **f32)
        self.g_next = torch.empty((B, D), **f32)
        self.x0 = torch.empty((B, X0W), **f32)
        self.ha = [torch.empty((B, XA), **f32) for _ in range(NH)]
        self.hb = [torch.empty((B, XB), **f32) if XB else None for _ in range(NH)]
        self.dp = [torch.empty((B, HP), **f32) for _ in range(NH)]
        self.gout = torch.empty((B, X0W), **f32)
        self.bufs = [self.x0] + [t for i in range(NH) for t in (self.ha[i], self.hb[i])] + self.dp + [self.gout]
        # padded per-layer dW workspace and its gather map into the flat (ravel) order
        shapes = [(HP, X0W)] + [(HP, HP)] * (NH - 1) + [(X0W, HP)]
        nat = [(H, C + D)] + [(H, H)] * (NH - 1) + [(2 * D, H)]
        offs, o = [], 0
        for (r, c) in shapes:
            offs.append((o, o + r * c))
            o += r * c + r
        self.ws_per = o
        self.ws = torch.zeros((L, o), **f32)
        self.views = []
        for l in range(L):
            v = []
            for (r, c), (ow, ob) in zip(shapes, offs):
                v.append((self.ws[l, ow:ow + r * c].view(r, c), self.ws[l, ob:ob + r]))
            self.views.append(v)
        idx = []
        for l in range(L):
            for (r, c), (nr, nc), (ow, ob) in zip(shapes, nat, offs):
                ii = np.arange(nr)[:, None] * c + np.arange(nc)[None, :]
                idx.append(l * o + ow + ii.reshape(-1))
                idx.append(l * o + ob + np.arange(nr))
        self.idx = torch.from_numpy(np.concatenate(idx).astype(np.int64)).to(dev)
        if self.idx.numel() != self.mask.numel():
            raise ValueError("MafGrad: mask does not match the flow's flat parameter count")

    def __call__(self, flat: Tensor) -> Tuple[Tensor, Tensor]:
        d = self.desc
        flat = flat.to(self.dev, torch.float32).reshape(-1).contiguous()
        inv = ops.ar_flow_pack_batched(d, flat[None], self.perms, mask=self.mask)[0]
        fwd = ops.ar_flow_pack_fwd_batched(d, flat[None], mask=self.mask)[0]
        bwd = ops.ar_flow_pack_bwd(d, flat, self.mask)
        ops.ar_flow_log_prob_train(d, inv, self.x, self.ctx, self.states, out=self.lp)
        torch.neg(self.states[0], out=self.g)  # d/dz of the Normal(0, I) base log-density
        g, g_next = self.g, self.g_next
        NH, XA = self.dims["n_hidden"], self.dims["XA"]
        for l in range(d.L):
            ops.ar_flow_bwd_layer(d, fwd, bwd, self.perm_dev, l, self.states[l], self.ctx, g, None, self.bufs,
                                  g_next)
            v = self.views[l]
            W, b = v[0]
            ops.gemm(self.dp[0].t(), self.x0, out=W, rowsum=b, split_k=1)
            for i in range(1, NH):
                W, b = v[i]
                ops.gemm(self.dp[i].t(), self.ha[i - 1], out=W[:, :XA], rowsum=b, split_k=1)
                if self.hb[i - 1] is not None:
                    ops.gemm(self.dp[i].t(), self.hb[i - 1], out=W[:, XA:], split_k=1)
            W, b = v[NH]
            ops.gemm(self.gout.t(), self.ha[NH - 1], out=W[:, :XA], rowsum=b, split_k=1)
            if self.hb[NH - 1] is not None:
                ops.gemm(self.gout.t(), self.hb[NH - 1], out=W[:, XA:], split_k=1)
            g, g_next = g_next, g
        grad = self.ws.view(-1)[self.idx] * self.mask
        return self.lp.sum(), grad
