"""Differentiable HIP ops for the NLL training step.

naz's ``train`` (naz/trainers/train_flows.py:194-213) differentiates
``-flow.log_prob(x, condition=y).mean()`` through pyro's transforms with torch autograd.
Here every node of that graph is a ``torch.autograd.Function`` whose forward AND backward
are HIP kernels:

  LinearActFn   act(cat[ctx, x] @ (W*mask)^T + b)   bwd: naz_act_bwd, naz_gemm (dX; dW with the
                                                     MADE mask fused and db as an extra ones column)
  RqsFn         RQ spline, either direction          bwd: naz_rqs_bwd (implicit-function rule
                                                     for the inverse)
  AffineARFn    pyro AffineAutoregressive step       bwd: naz_affine_ar_bwd
  BaseLogProbFn Normal(0, 1) log density              bwd: naz_base_log_prob_bwd

Autograd only sequences the kernels; no torch arithmetic runs on the batch except the
[B]-sized log-det sums and index copies (cat / permutation gathers).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
from torch.autograd import Function

from . import ops


def _needs(ctx, i: int) -> bool:
    return bool(ctx.needs_input_grad[i])


class LinearActFn(Function):
    """y = act(cat([context, x]) @ (weight * mask)^T + bias).  ``context`` may be one row
    (broadcast to every row of x), as ``ops.linear_act`` allows."""

    @staticmethod
    def forward(ctx, x, context, weight, bias, mask, act: str):
        y = ops.linear_act(x, weight, bias, act, context=context, mask=mask)
        ctx.act = act
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x, context, weight, mask, y)
        return y

    @staticmethod
    def backward(ctx, g_y):
        x, c, W, mask, y = ctx.saved_tensors
        act = ctx.act
        g_y = g_y.contiguous()
        gpre = g_y if act == "identity" else ops.act_bwd(g_y, y, act)
        M = y.shape[0]
        Cd = 0 if c is None else c.shape[-1]
        g_x = g_c = g_W = g_b = None
        want_b = ctx.has_bias and _needs(ctx, 3)
        if want_b:
            g_b = torch.empty(W.shape[0], device=W.device, dtype=torch.float32)
        gT = gpre.t()  # [N, M] view
        if _needs(ctx, 2):
            g_W = torch.empty_like(W)
            N, Kx = W.shape[0], (0 if x is None else x.shape[-1])
            thin = M >= 1024 and mask is None and bool(N % 4 or Cd % 4 or Kx % 4)
            if thin and (Cd + Kx) <= 256 and N <= 256:
                # the batch-row dW kernel (wgrad_flat) wants both widths in multiples of 4 and
                # one contiguous input: [ctx | x] concatenated, dPre padded with zero columns
                parts = []
                if Cd:
                    parts.append(c.reshape(1, -1).expand(M, Cd) if (c.dim() == 1 or c.shape[0] == 1) and M != 1
                                 else c)
                if Kx:
                    parts.append(x)
                K4, N4 = (Cd + Kx + 3) // 4 * 4, (N + 3) // 4 * 4
                xin = torch.empty((M, K4), device=W.device, dtype=torch.float32)
                xin[:, Cd + Kx:].zero_()  # only the padding columns
                xin[:, :Cd + Kx] = torch.cat(parts, 1) if len(parts) > 1 else parts[0]
                gp = gpre
                if N4 != N:
                    gp = torch.empty((M, N4), device=W.device, dtype=torch.float32)
                    gp[:, N:].zero_()
                    gp[:, :N] = gpre
                gw4 = torch.empty((N4, K4), device=W.device, dtype=torch.float32)
                gb4 = torch.empty(N4, device=W.device, dtype=torch.float32) if want_b else None
                ops.gemm(gp.t(), xin, out=gw4, rowsum=gb4)
                g_W.copy_(gw4[:N, :Cd + Kx])
                if want_b:
                    g_b.copy_(gb4[:N])
            else:
                if Cd:  # db rides on the first dW GEMM as an all-ones column
                    cc = c.reshape(1, -1).expand(M, Cd) if (c.dim() == 1 or c.shape[0] == 1) and M != 1 else c
                    ops.gemm(gT, cc, out=g_W[:, :Cd], mask=None if mask is None else mask[:, :Cd],
                             rowsum=g_b)
                if x is not None:
                    ops.gemm(gT, x, out=g_W[:, Cd:], mask=None if mask is None else mask[:, Cd:],
                             rowsum=None if Cd else g_b)
        elif want_b:
            ops.gemm(gT, gT[:0].t(), out=torch.empty(W.shape[0], 0, device=W.device), rowsum=g_b)
        if x is not None and _needs(ctx, 0):
            g_x = ops.gemm(gpre, W[:, Cd:], mask=None if mask is None else mask[:, Cd:], mask_b=True)
        if Cd and _needs(ctx, 1):
            Wc, mc = W[:, :Cd], (None if mask is None else mask[:, :Cd])
            if c.shape[0] == M and c.dim() == 2:
                g_c = ops.gemm(gpre, Wc, mask=mc, mask_b=True)
            else:  # one broadcast row: sum_m gpre[m] @ W = (sum_m gpre[m]) @ W
                g_c = ops.gemm(ops.colsum(gpre).reshape(1, -1), Wc, mask=mc, mask_b=True).reshape(c.shape)
        return g_x, g_c, g_W, g_b, None, None


def linear_act(x, weight, bias, act="identity", context=None, mask=None):
    return LinearActFn.apply(x, context, weight, bias, mask, act)


_DW_CONCAT = os.environ.get("NAZ_DW_CONCAT", "1") != "0"


def _param_grads(gpre, x, c, W, need_W: bool, need_b: bool):
    """dW (and db riding on it as an all-ones column) of one Linear layer: as LinearActFn."""
    M = gpre.shape[0]
    Cd = 0 if c is None else c.shape[-1]
    g_W = g_b = None
    if need_b:
        g_b = torch.empty(W.shape[0], device=W.device, dtype=torch.float32)
    gT = gpre.t()
    if need_W:
        g_W = torch.empty_like(W)
        Kx = 0 if x is None else x.shape[-1]
        if _DW_CONCAT and Cd and Kx and M >= 1024 and (Cd + Kx) % 4 == 0 and Cd + Kx <= 255 and c.dim() == 2 \
                and c.shape[0] == M:
            # per-row [ctx | x]: one dW GEMM over the concatenated input (one pass over dPre, the
            # flat wgrad kernel on a 16-byte multiple width instead of a narrow x-only GEMM)
            ops.gemm(gT, torch.cat((c, x), 1), out=g_W, rowsum=g_b)
        else:
            if Cd:
                cc = c.reshape(1, -1).expand(M, Cd) if (c.dim() == 1 or c.shape[0] == 1) and M != 1 else c
                ops.gemm(gT, cc, out=g_W[:, :Cd], rowsum=g_b)
            if x is not None:
                ops.gemm(gT, x, out=g_W[:, Cd:], rowsum=None if Cd else g_b)
    elif need_b:
        ops.gemm(gT, gT[:0].t(), out=torch.empty(W.shape[0], 0, device=W.device), rowsum=g_b)
    return g_W, g_b


class ChainFn(Function):
    """A whole Linear/act conditioner chain (pyro DenseNN / MADE forward with masked weights
    already applied) as ONE autograd node.  Backward walks the layers in reverse and forms each
    hidden layer's pre-activation gradient with naz_gemm_dact: dPre_{l-1} = (dPre_l · W_l) ⊙
    act'(h_{l-1}) in the dX GEMM's epilogue, so no separate naz_act_bwd pass reads and writes the
    [B, H] gradient (values identical to the LinearActFn-per-layer walk)."""

    @staticmethod
    def forward(ctx, x, context, act: str, drop, *wb):
        n = len(wb) // 2
        hs, ins = [], []  # post-activation (act') / next layer's input (post-dropout)
        h = x
        for i in range(n):
            a = act if i < n - 1 else "identity"
            h = ops.linear_act(x if i == 0 else ins[-1], wb[2 * i], wb[2 * i + 1], a,
                               context=context if i == 0 else None)
            hs.append(h)
            if i < n - 1:
                ins.append(ops.dropout(h, drop[0], drop[1][i]) if drop is not None else h)
        ctx.act, ctx.n, ctx.drop = act, n, drop
        ctx.has_bias = [wb[2 * i + 1] is not None for i in range(n)]
        extra = ins if drop is not None else []
        ctx.save_for_backward(x, context, *[wb[2 * i] for i in range(n)], *hs[:-1], *extra)
        return hs[-1]

    @staticmethod
    def backward(ctx, g_y):
        n, act, drop = ctx.n, ctx.act, ctx.drop
        saved = ctx.saved_tensors
        x, c = saved[0], saved[1]
        Ws = saved[2:2 + n]
        hs = saved[2 + n:2 + 2 * n - 1]
        ins = saved[2 + 2 * n - 1:] if drop is not None else hs
        grads = [None] * (2 * n)
        gpre = g_y.contiguous()
        g_x = g_c = None
        for i in reversed(range(n)):
            W = Ws[i]
            inp = x if i == 0 else ins[i - 1]
            ci = c if i == 0 else None
            gW, gb = _param_grads(gpre, inp, ci, W, _needs(ctx, 4 + 2 * i), ctx.has_bias[i] and _needs(ctx, 5 + 2 * i))
            grads[2 * i], grads[2 * i + 1] = gW, gb
            Cd = 0 if ci is None else ci.shape[-1]
            if i > 0:
                gpre = ops.gemm_dact(gpre, W, hs[i - 1], act)  # (gpre · W) ⊙ act'(h_{i-1})
                if drop is not None:  # ⊙ the forward's dropout mask / (1 - p)
                    ops.dropout(gpre, drop[0], drop[1][i - 1], out=gpre)
            else:
                if x is not None and _needs(ctx, 0):
                    g_x = ops.gemm(gpre, W[:, Cd:])
                if Cd and _needs(ctx, 1):
                    Wc = W[:, :Cd]
                    if c.shape[0] == gpre.shape[0] and c.dim() == 2:
                        g_c = ops.gemm(gpre, Wc)
                    else:
                        g_c = ops.gemm(ops.colsum(gpre).reshape(1, -1), Wc).reshape(c.shape)
        return (g_x, g_c, None, None, *grads)


def chain(x, weights, biases, act: str, context=None, drop=None):
    """Conditioner forward recorded as one ChainFn node (see there); ``drop`` = (p, seeds)."""
    wb = [t for pair in zip(weights, biases) for t in pair]
    return ChainFn.apply(x, context, act, drop, *wb)


class RqsFn(Function):
    """(y, ld_row) = RQ spline of x over conditioner output ``raw`` (row-sum log-det of THIS
    direction: the forward ldf, or the inverse's -ldf)."""

    @staticmethod
    def forward(ctx, x, raw, count_bins: int, layout: int, inverse: bool, bound: float, broadcast: bool):
        y, ld = ops.rqs(x, raw, count_bins, layout, inverse, bound, ops.LD_ROWSUM, broadcast_raw=broadcast)
        ctx.cfg = (count_bins, layout, inverse, bound, broadcast)
        ctx.save_for_backward(x, raw)
        return y, ld

    @staticmethod
    def backward(ctx, g_y, g_ld):
        x, raw = ctx.saved_tensors
        K, layout, inverse, bound, broadcast = ctx.cfg
        g_x, g_raw = ops.rqs_bwd(x, raw, K, layout, inverse, bound, g_y, g_ld, need_g_in=_needs(ctx, 0),
                                 broadcast_raw=broadcast)
        return g_x, g_raw, None, None, None, None, None


def rqs(x, raw, count_bins, layout=ops.LAYOUT_DENSE, inverse=False, bound=3.0, broadcast=False):
    return RqsFn.apply(x, raw, count_bins, layout, inverse, bound, broadcast)


class AffineARFn(Function):
    """(y, forward ld_row) of pyro's AffineAutoregressive step over MADE output ``raw``."""

    @staticmethod
    def forward(ctx, x, raw, inverse: bool, clip_zero: bool = False):
        y, ld = ops.affine_ar(x, raw, inverse, ops.LD_ROWSUM)
        ctx.inverse, ctx.clip_zero = inverse, clip_zero
        ctx.save_for_backward(x, raw, y)
        return y, ld

    @staticmethod
    def backward(ctx, g_y, g_ld):
        x, raw, y = ctx.saved_tensors
        if g_y is None:
            g_y = torch.zeros_like(y)
        g_x, g_raw = ops.affine_ar_bwd(x, raw, y, ctx.inverse, g_y, g_ld, need_g_x=_needs(ctx, 0),
                                       clip_zero=ctx.clip_zero)
        return g_x, g_raw, None, None


def affine_ar(x, raw, inverse, clip_zero: bool = False):
    """``clip_zero``: jnp.clip's gradient for the log_scale clip (the JAX Bayesian MAF) instead of
    pyro's clamp_preserve_gradients."""
    return AffineARFn.apply(x, raw, inverse, clip_zero)


class BaseLogProbFn(Function):
    """sum_i log N(z_i; 0, 1) per row."""

    @staticmethod
    def forward(ctx, z):
        ctx.save_for_backward(z)
        return ops.base_log_prob(z)

    @staticmethod
    def backward(ctx, g_lp):
        (z,) = ctx.saved_tensors
        return ops.base_log_prob_bwd(z, g_lp.contiguous())


def base_log_prob(z):
    return BaseLogProbFn.apply(z)


def params_require_grad(modules) -> bool:
    """True when autograd must record the walk: grad mode on and some parameter trainable."""
    if not torch.is_grad_enabled():
        return False
    for m in modules:
        if m is None:
            continue
        for p in m.parameters():
            if p.requires_grad:
                return True
    return False


def tensor_requires_grad(*ts: Optional[torch.Tensor]) -> bool:
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts)
