"""Fused gradient of Σ_rows log p(x | ctx) over a naz affine MAF.

The NUTS / HMC potential of naz's Bayesian MAF is ``flow_lp(unravel(p)).sum()`` and its gradient
(naz/flows/bflow_jax_maf.py:231-235, examples/papers/2506.05657/hmc_maf_exact.py:118-133): one
forward over the whole training set and one backward per leapfrog step.  Here that is

  * the fused inverse kernel with every layer's output saved (naz_ar_flow_log_prob_train);
  * per layer l = 0 .. L-1 one fused backward launch (naz_ar_flow_bwd_layer, csrc/made_ar_bwd.h:
    dense MADE recompute, the affine VJP, the D-order chain of input gradients, the total δ's)
    writing that layer's weight-gradient operands into its own slice of [L, rows, ...] buffers;
  * per weight matrix ONE batched reduction over all layers (naz_wgrad_batched, bf16x6 MFMA):
    dW_l = δ_lᵀ·h_l and the bias column sums into a padded per-layer workspace;
  * ONE gather of the workspace into ``ravel`` order times the masks (pyro MaskedLinear's
    gradient is mask ⊙ (δᵀ h)).

Rows are processed in chunks so the operands stay within ``operand_bytes`` (4 KB per row and layer
at the paper shape).  No autograd graph, no per-block gathers: L + NHID + 5 launches per chunk.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
from torch import Tensor

from .. import ops


class MafGrad:
    """(Σ lp, ∇θ) of one flat θ (``ravel`` order = the naz_ar_flow_pack_host flat layout) over
    fixed rows ``x`` [B, D] and ``ctx`` ([B, C], [1, C] or None).  ``mask`` [L * per]: the MADE
    masks in the flat layout (1 on biases); ``perms`` [L, D]: dim of order p per layer."""

    def __init__(self, desc, perms: np.ndarray, mask: Tensor, x: Tensor, ctx: Optional[Tensor],
                 operand_bytes: int = 8 << 30):
        if not ops.ar_flow_bwd_supported(desc):
            raise RuntimeError("MafGrad: no fused maf backward for this shape")
        self.desc = desc
        dev = x.device
        self.dev = dev
        D, C, H, L = desc.D, desc.C, desc.H, desc.L
        dm = ops.ar_flow_bwd_dims(desc)
        NH, HP, XA, XB, X0W = dm["n_hidden"], dm["HP"], dm["XA"], dm["XB"], dm["X0W"]
        if XB:
            raise RuntimeError("MafGrad: split hidden operands are not supported")
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
        per_row = L * 4 * (2 * X0W + 2 * NH * HP)
        rows = max(dm["rows"], min(B, operand_bytes // per_row) // dm["rows"] * dm["rows"])
        self.chunk = min(B, rows)
        Bc = self.chunk
        self.x0 = torch.empty((L, Bc, X0W), **f32)
        self.h = [torch.empty((L, Bc, HP), **f32) for _ in range(NH)]
        self.dp = [torch.empty((L, Bc, HP), **f32) for _ in range(NH)]
        self.gout = torch.empty((L, Bc, X0W), **f32)
        # padded per-layer dW workspace [L, ws_per] and its gather map into the flat (ravel) order
        shapes = [(HP, X0W)] + [(HP, HP)] * (NH - 1) + [(X0W, HP)]
        nat = [(H, C + D)] + [(H, H)] * (NH - 1) + [(2 * D, H)]
        offs, o = [], 0
        for (r, c) in shapes:
            offs.append((o, o + r * c))
            o += r * c + r
        self.ws_per = o
        self.ws = torch.zeros((L, o), **f32)
        self.views = [(self.ws[:, ow:ow + r * c].view(L, r, c), self.ws[:, ob:ob + r])
                      for (r, c), (ow, ob) in zip(shapes, offs)]
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
        NH = self.dims["n_hidden"]
        # one fill for every layer's dW / db, then the reductions accumulate into it
        self.ws.zero_()
        for r0 in range(0, self.B, self.chunk):
            r1 = min(self.B, r0 + self.chunk)
            n = r1 - r0
            g, g_next = self.g[r0:r1], self.g_next[r0:r1]
            ctx = None if self.ctx is None else (self.ctx if self.ctx.shape[0] == 1 else self.ctx[r0:r1])
            for l in range(d.L):
                bufs = [self.x0[l, :n]] + [t for i in range(NH) for t in (self.h[i][l, :n], None)] + \
                       [self.dp[i][l, :n] for i in range(NH)] + [self.gout[l, :n]]
                ops.ar_flow_bwd_layer(d, fwd, bwd, self.perm_dev, l, self.states[l, r0:r1], ctx, g, None, bufs,
                                      g_next)
                g, g_next = g_next, g
            # dW of every layer: one batched reduction per weight matrix
            W, b = self.views[0]
            ops.wgrad_batched(self.dp[0][:, :n], self.x0[:, :n], W, b)
            for i in range(1, NH):
                W, b = self.views[i]
                ops.wgrad_batched(self.dp[i][:, :n], self.h[i - 1][:, :n], W, b)
            W, b = self.views[NH]
            ops.wgrad_batched(self.gout[:, :n], self.h[NH - 1][:, :n], W, b)
        grad = self.ws.view(-1)[self.idx] * self.mask
        return self.lp.sum(), grad
