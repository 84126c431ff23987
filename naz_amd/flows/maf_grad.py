"""Fused gradient of Σ_rows g_lp · log p(x | ctx) over a naz affine MAF.

The NUTS / HMC potential of naz's Bayesian MAF is ``flow_lp(unravel(p)).sum()`` and its gradient
(naz/flows/bflow_jax_maf.py:231-235, examples/papers/2506.05657/hmc_maf_exact.py:118-133); the maf
NLL step differentiates the same log-density (naz/trainers/train_flows.py:194-213).  Here that is

  * the fused inverse kernel with every layer's output saved (naz_ar_flow_log_prob_train);
  * per layer l = 0 .. L-1 one fused backward launch (naz_ar_flow_bwd_layer, csrc/made_ar_bwd.h:
    dense MADE recompute, the affine VJP, the D-order chain of input gradients, the total δ's)
    writing that layer's weight-gradient operands into its own slice of [L, rows, ...] buffers;
  * per weight matrix ONE batched reduction over all layers (naz_wgrad_batched, bf16x6 MFMA):
    dW_l = δ_lᵀ·h_l and the bias column sums into a padded per-layer workspace;
  * ONE gather of the workspace into the flat (``ravel``) order times the masks (pyro
    MaskedLinear's gradient is mask ⊙ (δᵀ h)).

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
    """The fused maf log-density and its backward for one flow structure: ``desc`` (an affine
    naz_ar_desc at a compiled shape), ``perms`` [L, D] (dim of order p per layer) and ``mask``
    [L * per] (the MADE masks in the naz_ar_flow_pack_host flat layout, 1 on biases).  Weights
    come as flat rows in that layout (= ``ravel`` order of the JAX front end).  ``clip_zero``: the
    log_scale clip differentiates as jnp.clip (zero outside [-5, 3]: the JAX MAF's potential,
    bflow_jax_maf.py:177-192) instead of pyro's clamp_preserve_gradients (naz's torch maf)."""

    def __init__(self, desc, perms: np.ndarray, mask: Tensor, operand_bytes: int = 4 << 30,
                 clip_zero: bool = False, keep_sizes: int = 2):
        if not ops.ar_flow_bwd_supported(desc):
            raise RuntimeError("MafGrad: no fused maf backward for this shape")
        desc = type(desc).from_buffer_copy(desc)
        desc.flags = ops.AR_CLIP_ZERO_GRAD if clip_zero else 0
        self.desc = desc
        self.keep_sizes = max(1, int(keep_sizes))
        dev = mask.device
        self.dev = dev
        D, C, H, L = desc.D, desc.C, desc.H, desc.L
        dm = ops.ar_flow_bwd_dims(desc)
        NH, HP, XB, X0W = dm["n_hidden"], dm["HP"], dm["XB"], dm["X0W"]
        if XB:
            raise RuntimeError("MafGrad: split hidden operands are not supported")
        self.dims = dm
        self.operand_bytes = operand_bytes
        self.perms = np.ascontiguousarray(np.asarray(perms), dtype=np.int32)
        self.perm_dev = torch.from_numpy(self.perms).to(dev)
        self.mask = mask.to(dev, torch.float32).contiguous()
        self._bufs = {}
        # padded per-layer dW workspace [L, ws_per] and its gather map into the flat order
        shapes = [(HP, X0W)] + [(HP, HP)] * (NH - 1) + [(X0W, HP)]
        nat = [(H, C + D)] + [(H, H)] * (NH - 1) + [(2 * D, H)]
        offs, o = [], 0
        for (r, c) in shapes:
            offs.append((o, o + r * c))
            o += r * c + r
        self.ws = torch.zeros((L, o), device=dev, dtype=torch.float32)
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

    def _buffers(self, B: int) -> dict:
        """Per-row-count buffers.  The most recent ``keep_sizes`` row counts stay allocated (a
        captured graph replays the same addresses; a training loop alternates the full batch and
        a ragged last batch); older ones are released, so a run of distinct batch sizes does not
        pin one operand set each."""
        b = self._bufs.pop(B, None)
        if b is not None:
            self._bufs[B] = b  # most recently used last
        else:
            while len(self._bufs) >= self.keep_sizes:
                self._bufs.pop(next(iter(self._bufs)))
            d, dm = self.desc, self.dims
            NH, HP, X0W = dm["n_hidden"], dm["HP"], dm["X0W"]
            f32 = dict(device=self.dev, dtype=torch.float32)
            per_row = d.L * 4 * (2 * X0W + 2 * NH * HP)
            rows = max(dm["rows"], min(B, self.operand_bytes // per_row) // dm["rows"] * dm["rows"])
            Bc = max(1, min(B, rows))
            b = dict(states=torch.empty((d.L, B, d.D), **f32), lp=torch.empty((B,), **f32),
                     g=torch.empty((B, d.D), **f32), g_next=torch.empty((B, d.D), **f32), chunk=Bc,
                     x0=torch.empty((d.L, Bc, X0W), **f32), gout=torch.empty((d.L, Bc, X0W), **f32),
                     h=[torch.empty((d.L, Bc, HP), **f32) for _ in range(NH)],
                     dp=[torch.empty((d.L, Bc, HP), **f32) for _ in range(NH)])
            self._bufs[B] = b
        return b

    def images(self, flat: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
        """(inverse, forward, backward) images of one flat weight row (device packers, masks applied)."""
        d = self.desc
        flat = flat.to(self.dev, torch.float32).reshape(-1).contiguous()
        inv = ops.ar_flow_pack_batched(d, flat[None], self.perms, mask=self.mask)[0]
        fwd = ops.ar_flow_pack_fwd_batched(d, flat[None], mask=self.mask)[0]
        bwd = ops.ar_flow_pack_bwd(d, flat, self.mask)
        return inv, fwd, bwd

    def forward(self, imgs, x: Tensor, ctx: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
        """log p(x | ctx) [B] (this row count's buffer) and the saved layer outputs [L, B, D]."""
        b = self._buffers(x.shape[0])
        ops.ar_flow_log_prob_train(self.desc, imgs[0], x, ctx, b["states"], out=b["lp"])
        return b["lp"], b["states"]

    def backward(self, imgs, states: Tensor, ctx: Optional[Tensor],
                 g_lp: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
        """(dL/dθ in the flat order, dL/dx [B, D]) for L = Σ_rows g_lp · log p (g_lp None: 1)."""
        d = self.desc
        B = states.shape[1]
        b = self._buffers(B)
        NH = self.dims["n_hidden"]
        g_all, gn_all = b["g"], b["g_next"]
        torch.neg(states[0], out=g_all)  # d/dz of the Normal(0, I) base log-density
        if g_lp is not None:
            g_lp = g_lp.to(self.dev, torch.float32).contiguous()
            g_all.mul_(g_lp[:, None])
        self.ws.zero_()  # one fill for every layer's dW / db; the reductions accumulate into it
        Bc = b["chunk"]
        for r0 in range(0, B, Bc):
            r1 = min(B, r0 + Bc)
            n = r1 - r0
            g, g_next = g_all[r0:r1], gn_all[r0:r1]
            c = None if ctx is None else (ctx if ctx.shape[0] == 1 else ctx[r0:r1])
            gl = None if g_lp is None else g_lp[r0:r1]
            for l in range(d.L):
                bufs = [b["x0"][l, :n]] + [t for i in range(NH) for t in (b["h"][i][l, :n], None)] + \
                       [b["dp"][i][l, :n] for i in range(NH)] + [b["gout"][l, :n]]
                ops.ar_flow_bwd_layer(d, imgs[1], imgs[2], self.perm_dev, l, states[l, r0:r1], c, g, gl, bufs,
                                      g_next)
                g, g_next = g_next, g
            # dW of every layer: one batched reduction per weight matrix
            W, bb = self.views[0]
            ops.wgrad_batched(b["dp"][0][:, :n], b["x0"][:, :n], W, bb)
            for i in range(1, NH):
                W, bb = self.views[i]
                ops.wgrad_batched(b["dp"][i][:, :n], b["h"][i - 1][:, :n], W, bb)
            W, bb = self.views[NH]
            ops.wgrad_batched(b["gout"][:, :n], b["h"][NH - 1][:, :n], W, bb)
        g_x = g_all if d.L % 2 == 0 else gn_all  # where dL/dx landed after L swaps
        return self.ws.view(-1)[self.idx] * self.mask, g_x

    def __call__(self, flat: Tensor, x: Tensor, ctx: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
        """(Σ_rows log p(x | ctx), ∇θ) of one flat θ: the NUTS potential and its gradient."""
        imgs = self.images(flat)
        lp, states = self.forward(imgs, x, ctx)
        grad, _ = self.backward(imgs, states, ctx, None)
        return lp.sum(), grad
