"""Batched-over-parameters affine MAF: the Bayesian front end's log_prob / sampler on MI355X
(SURVEY.md §8f rank 1 and rank 2).

naz's Bayesian flows (``naz/flows/bflow_jax_maf.py``) evaluate ONE trained affine MAF under
many weight draws θ_p — HMC / SVI posterior and prior draws of ``flat_params * (1 + scale *
standard_params)`` (``bflow_jax_maf.py:214-236``) — over the same rows: the density grid of
``plot.py:192-204`` / ``plot_svi.py:184-196``, the training set inside NUTS
(``hmc_maf_exact.py:128-133``), and 10^6 posterior-predictive samples per draw
(``calibrate.py:145-151``).  The reference runs ``flow["lp"](θ_p)`` / ``flow["sampler"](θ_p,
key, n)`` once per draw in a Python loop.  Here all draws of a chunk run together:

* ``lp_batched(params) -> [P, B]``: the degree-scheduled D-pass inverse (``nn.ARInversePlan``)
  with every GEMM one ``naz_linear_act_batched`` launch over (row tiles × column blocks ×
  draws); the schedule depends only on the masks and permutation, so it is built once on
  index-valued weights and each draw set is packed by one gather per block;
* ``sampler_batched(params, key, size) -> ([P, size, D], log_j [P, size])``: one masked MADE
  pass per layer (``naz_linear_act_batched`` with the shared mask) + ``naz_affine_ar``.

``params`` is the reference's pytree (``torch_to_jax``: a list per layer of ``(W, b)`` per
MADE linear) with a leading draw axis on every leaf, i.e. what ``jax.vmap(unravel_fn)`` of
posterior draws gives (``plot.py:140``); ``unravel`` maps the flat ``[P, n]`` draws
(``ravel_pytree`` order) to it.  Scope: ``bounds=None`` and no skip connections (what the
examples use); the bounded branch raises ``NotImplementedError`` (it also carries the
reference's sign bug, ``bflow_jax_maf.py:198-212``).  The sampler takes an integer seed or a
``torch.Generator`` as ``rng_key``: JAX's PRNG stream is not reproduced, only its distribution.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor

from .. import ops
from ..nn import create_mask, degree_schedule
from .ar_pass0 import ArPass0

__all__ = ["torch_to_jax", "make_conditional_autoregressive_nn", "make_masked_affine_autoregressive_transform",
           "make_normalizing_flow", "ravel", "unravel", "MAFSpec"]

Params = List[List[Tuple[Tensor, Tensor]]]


def torch_to_jax(torch_maf):
    """naz ``torch_to_jax`` (bflow_jax_maf.py:26-46) over a naz_amd ``maf`` flow: (params,
    param_shapes, masks, mask_skips, permutations), tensors kept on the flow's device."""
    params, shapes, masks, skips, perms = [], [], [], [], []
    # the layer list (an unconditional flow_dist holds one ComposeTransformModule)
    for t in torch_maf.transforms:
        arn = t.nn
        these = [(l.weight.detach().clone(), l.bias.detach().clone()) for l in arn.layers]
        params.append(these)
        shapes.append([(tuple(w.shape), tuple(b.shape)) for (w, b) in these])
        masks.append([m.detach().to(torch.float32).clone() for m in arn.masks])
        skips.append(arn.mask_skip.detach().to(torch.float32).clone())
        perms.append(arn.permutation.detach().clone())
    return params, shapes, masks, skips, perms


class MAFSpec:
    """What ``make_conditional_autoregressive_nn`` closes over (bflow_jax_maf.py:79-167)."""

    def __init__(self, input_dim: int, context_dim: int, hidden_dims: Sequence[int], activation: str = "tanh"):
        self.input_dim, self.context_dim = int(input_dim), int(context_dim)
        self.hidden_dims = [int(h) for h in hidden_dims]
        self.activation = activation
        self.param_shapes = [((self.hidden_dims[0], self.input_dim + self.context_dim), (self.hidden_dims[0],))]
        for i in range(1, len(self.hidden_dims)):
            self.param_shapes.append(((self.hidden_dims[i], self.hidden_dims[i - 1]), (self.hidden_dims[i],)))
        self.param_shapes.append(((2 * self.input_dim, self.hidden_dims[-1]), (2 * self.input_dim,)))


def make_conditional_autoregressive_nn(input_dim: int, context_dim: int, hidden_dims: Sequence[int],
                                       param_dims: Sequence[int] = (1, 1), permutation=None,
                                       skip_connections: bool = False, activation_fn: str = "tanh",
                                       simple_masking: bool = True):
    """bflow_jax_maf.py:79-167: returns (nn_spec, param_shapes, generate_mask).  Affine MAF
    conditioners only (param_dims [1, 1]), simple masking, no skip connections."""
    if list(param_dims) != [1, 1]:
        raise NotImplementedError("batched MAF: param_dims [1, 1] (affine) only")
    if skip_connections or not simple_masking:
        raise NotImplementedError("batched MAF: skip connections / random masking are not built")
    if activation_fn not in ("tanh", "relu", "sigmoid", "identity"):
        raise ValueError(f"unsupported activation {activation_fn!r}")
    spec = MAFSpec(input_dim, context_dim, hidden_dims, activation_fn)

    def generate_mask(permutation=permutation):
        perm = torch.randperm(input_dim) if permutation is None else torch.as_tensor(permutation)
        masks, mask_skip = create_mask(input_dim, context_dim, spec.hidden_dims, perm, 2)
        return [m.to(torch.float32) for m in masks], mask_skip.to(torch.float32), perm

    return spec, spec.param_shapes, generate_mask


def make_masked_affine_autoregressive_transform(nn_fn: MAFSpec, input_dim: int, context=None):
    """bflow_jax_maf.py:169-194: the (forward, inverse) pair is what ``make_normalizing_flow``
    runs; here it is the spec it runs with."""
    if nn_fn.input_dim != input_dim:
        raise ValueError("input_dim does not match the conditioner")
    return nn_fn


def ravel(params: Params) -> Tensor:
    """``ravel_pytree`` order (layer-major, (W, b) per linear, row-major) of a single-draw
    ([o, i] leaves -> [n]) or batched ([P, o, i] leaves -> [P, n]) pytree."""
    leaves = [t for layer in params for wb in layer for t in wb]
    batched = leaves[0].dim() == 3
    return torch.cat([t.reshape(t.shape[0], -1) if batched else t.reshape(-1) for t in leaves], dim=-1)


def unravel(flat: Tensor, param_shapes) -> Params:
    """Inverse of ``ravel`` (bflow_jax_maf.py:214-216's ``unravel_fn``, vmapped over a leading
    draw axis when ``flat`` is [P, n])."""
    lead = flat.shape[:-1]
    need = sum(int(torch.tensor(ws).prod()) + int(torch.tensor(bs).prod()) for layer in param_shapes
               for (ws, bs) in layer)
    if need != flat.shape[-1]:
        raise ValueError(f"flat params have {flat.shape[-1]} entries, the shapes need {need}")
    out, off = [], 0
    for layer in param_shapes:
        these = []
        for ws, bs in layer:
            nw, nb = int(torch.tensor(ws).prod()), int(torch.tensor(bs).prod())
            w = flat[..., off:off + nw].reshape(*lead, *ws)
            b = flat[..., off + nw:off + nw + nb].reshape(*lead, *bs)
            off += nw + nb
            these.append((w, b))
        out.append(these)
    return out


class _LayerPlan:
    """Degree schedule of one MAF layer as gather maps into its per-draw flat buffer
    ``F[p] = [0, W0.flat, b0, W1.flat, b1, ...]`` (index 0 = a structural zero)."""

    def __init__(self, masks: List[Tensor], perm: Tensor, spec: MAFSpec):
        D, C = spec.input_dim, spec.context_dim
        cpu = dict(device="cpu", dtype=torch.float64)
        wi, bi, off = [], [], 1
        for (ws, bs) in spec.param_shapes:
            nw, nb = ws[0] * ws[1], bs[0]
            wi.append(torch.arange(off, off + nw, **cpu).reshape(ws))
            bi.append(torch.arange(off + nw, off + nw + nb, **cpu))
            off += nw + nb
        self.size = off
        self.masks = [m.to(**cpu) for m in masks]
        widths, hidden, outs = degree_schedule(perm.cpu(), self.masks, wi, bi, D, C, 2)
        self.widths = widths
        self.hidden = [[(li, a, b, n, wb.round().long(), bb.round().long()) for (li, a, b, n, wb, bb) in g]
                       for g in hidden]
        self.outs = [(i, n, wb.round().long(), bb.round().long()) for (i, n, wb, bb) in outs]

    def to(self, dev):
        self.hidden = [[(li, a, b, n, w.to(dev), bb.to(dev)) for (li, a, b, n, w, bb) in g] for g in self.hidden]
        self.outs = [(i, n, w.to(dev), bb.to(dev)) for (i, n, w, bb) in self.outs]
        self.masks_dev = [m.to(dev, torch.float32) for m in self.masks]
        return self


def _feat(o, r, lane):
    """Feature held by accumulator register r of 32-block o in lane ``lane`` (made.hip)."""
    return 32 * o + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)


def made_pack_map(spec: MAFSpec, masks: List[Tensor], nh: int) -> Tensor:
    """Gather map of naz_made_affine_fwd's packed net (layout in csrc/made.hip) into the per-draw
    flat buffer F = [0, W0, b0, W1, b1, ...]: entry = 1-based flat index, 0 for a masked or
    padded slot (so the gather applies the MADE masks)."""
    D, C = spec.input_dim, spec.context_dim
    Wi, Bi, off = [], [], 1
    for (ws, bs), m in zip(spec.param_shapes, masks):
        nw = ws[0] * ws[1]
        Wi.append(torch.arange(off, off + nw).reshape(ws) * (m.cpu() != 0))
        Bi.append(torch.arange(off + nw, off + nw + bs[0]))
        off += nw + bs[0]

    def gw(idx, of, kf):
        ok = (of < idx.shape[0]) & (kf < idx.shape[1])
        return torch.where(ok, idx[of.clamp(max=idx.shape[0] - 1), kf.clamp(max=idx.shape[1] - 1)], 0).reshape(-1)

    def gb(idx, f):
        return torch.where(f < idx.shape[0], idx[f.clamp(max=idx.shape[0] - 1)], 0).reshape(-1)

    def grid(*n):
        return torch.meshgrid(*[torch.arange(k) for k in n], indexing="ij")

    s0 = ((C + D + 1) // 2 + 3) // 4 * 4
    parts = []
    o, t, l, q = grid(nh, s0 // 4, 64, 4)  # A0: W0[32o + l%32][2s + l//32], s = 4t + q
    parts.append(gw(Wi[0], 32 * o + l % 32, 2 * (4 * t + q) + l // 32))
    o, r, l = grid(nh, 16, 64)
    parts.append(gb(Bi[0], _feat(o, r, l)))
    for j in range(1, len(spec.hidden_dims)):
        t, o, l, q = grid(nh * 4, nh, 64, 4)  # t-major: one input 32-block = one contiguous chunk
        s = 4 * t + q
        parts.append(gw(Wi[j], 32 * o + l % 32, _feat(s >> 4, s & 15, l)))
        o, r, l = grid(nh, 16, 64)
        parts.append(gb(Bi[j], _feat(o, r, l)))
    t, l, q = grid(nh * 4, 64, 4)
    s = 4 * t + q
    parts.append(gw(Wi[-1], l % 32, _feat(s >> 4, s & 15, l)))
    r, l = grid(16, 64)
    parts.append(gb(Bi[-1], _feat(0, r, l)))
    return torch.cat(parts)


def _draws(params: Params) -> int:
    return params[0][0][0].shape[0]


def _flat_layer_size(layer) -> int:
    """Floats per draw of one layer's flat parameter row (_flat_layer)."""
    return 1 + sum(w[0].numel() + b[0].numel() for (w, b) in layer)


def _flat_layer(layer, P, dev):
    """F[p] = [0, W0, b0, W1, b1, ...] for one layer of a batched pytree: [P, size]."""
    parts = [torch.zeros((P, 1), device=dev, dtype=torch.float32)]
    for (w, b) in layer:
        parts += [w.reshape(P, -1).to(dev, torch.float32), b.reshape(P, -1).to(dev, torch.float32)]
    return torch.cat(parts, dim=1)


def make_normalizing_flow(transform: MAFSpec, x, masks, mask_skips, perms, bounds=None, context=None,
                          rows_per_chunk: int = 1 << 23, fold_context: bool = True,
                          fuse_pass2: bool = True, batch_layers: bool = True, fused_ar: bool = True,
                          fused_grad: bool = True) -> Dict[str, object]:
    """naz ``make_normalizing_flow`` (bflow_jax_maf.py:196-225) on MI355X.  Returns
    ``{"lp": f(params) -> [B], "sampler": f(params, rng_key, size) -> (y, log_j),
    "lp_batched": f(params_P) -> [P, B], "sampler_batched": f(params_P, rng_key, size)}``.

    ``x`` [B, D] are the evaluation rows; ``context`` None, [C] (broadcast) or [B, C].  The
    single-draw functions are the batched ones at P = 1.  With one context vector,
    ``fold_context`` evaluates the context-only (degree-0) MADE units once per draw and folds
    them into biases (same values up to fp32 reassociation; False = the plain schedule).  ``rows_per_chunk`` bounds the draws
    evaluated together (activation memory ≈ 4·rows·Σwidths bytes)."""
    if bounds is not None:
        raise NotImplementedError("batched MAF: bounds=None only (see module docstring)")
    spec = transform
    D, C = spec.input_dim, spec.context_dim
    x = torch.as_tensor(x)
    dev = x.device
    if dev.type != "cuda":
        raise RuntimeError("naz_amd batched MAF runs on the GPU only; pass x on a cuda device")
    x = x.to(torch.float32).contiguous()
    if x.dim() != 2 or x.shape[1] != D:
        raise ValueError(f"x must be [B, {D}]")
    B = x.shape[0]
    ctx = None
    if C:
        if context is None:
            raise ValueError("conditional flow needs a context")
        ctx = torch.as_tensor(context, device=dev, dtype=torch.float32).contiguous()
        if ctx.shape[-1] != C or (ctx.dim() == 2 and ctx.shape[0] not in (1, B)):
            raise ValueError(f"context must be [{C}] or [B, {C}]")
    plans = [_LayerPlan(m, p, spec).to(dev) for (m, p) in zip(masks, perms)]
    # fused forward (naz_made_affine_fwd): hidden widths <= 160, 2D <= 32, tanh / relu
    nh = (max(spec.hidden_dims) + 31) // 32
    fused_fwd = nh <= 5 and 2 * D <= 32 and spec.activation in ("tanh", "relu")
    if fused_fwd:
        made_maps = [made_pack_map(spec, m, nh).to(dev) for m in masks]
        n_packed = ops.made_packed_floats(len(spec.hidden_dims), nh, C, D)
        assert all(mp.numel() == n_packed for mp in made_maps), "made pack map out of sync with made.hip"
    act = spec.activation
    width_sum = max(sum(pl.widths) for pl in plans)
    # the whole flow's sampling direction in ONE launch for all draws (naz_ar_flow_sample_batched,
    # csrc/made_ar_r16.h, f16x3 MFMA) at the compiled shapes (the paper's D=2 | C=2, H=[150]*3)
    ar_desc = None
    hd = list(spec.hidden_dims)
    if fused_ar and act == "tanh" and len(set(hd)) == 1:
        d_ = ops.ar_flow_desc("maf", D, C, hd[0], len(masks), len(hd))
        if ops.ar_flow_fwd_supported(d_):
            ar_desc = d_
            # per layer: F[:, 1:] * mask-vector = the flat layout naz_ar_flow_pack_fwd reads
            ar_maskvec = [torch.cat([t for m, (ws, bs) in zip(ms, spec.param_shapes)
                                     for t in (m.reshape(-1).to(torch.float32), torch.ones(bs[0]))]).to(dev)
                          for ms in masks]
    # the whole log-density in ONE launch for all draws (naz_ar_flow_log_prob_batched): the
    # inverse kernel's degree passes assume pyro's create_mask for each layer's permutation, one
    # context vector (or none) and rows inside the f16x3 input split's range
    ar_perm = ar_pass0 = ar_grad_perm = None
    if ar_desc is not None and ops.ar_flow_supported(ar_desc) and \
            float(x.abs().max()) < 32768.0 and \
            (C == 0 or float(ctx.abs().max()) < 32768.0):
        pm = [torch.as_tensor(p_).cpu().to(torch.int64) for p_ in perms]
        ok = True
        for ms, p_ in zip(masks, pm):
            ref, _ = create_mask(D, C, hd, p_, 2)
            ok = ok and len(ref) == len(ms) and all(
                torch.equal(r.to(torch.float32), m.detach().cpu().to(torch.float32)) for r, m in zip(ref, ms))
        # the NUTS potential's gradient (lp_and_grad) on the fused maf backward: any context rows
        if ok and ops.ar_flow_bwd_supported(ar_desc):
            ar_grad_perm = torch.stack(pm).numpy()
        if ok and (C == 0 or ctx.dim() == 1):
            ar_perm = torch.stack(pm).numpy()
            # one context vector: the first degree pass (units of mask index 0 see only the
            # context; the first dim's outputs see only them) is a per-draw constant, computed
            # once per draw below and packed in place of that pass's weights
            if C > 0 and fold_context and ops.ar_flow_pass0_floats(ar_desc) > 0 and \
                    int((torch.as_tensor(ops.ar_flow_degrees(ar_desc)) == 0).sum()):
                ar_pass0 = ArPass0(ar_desc, [int(p_[0]) for p_ in pm], act, dev)

    def _chunks(P, rows, max_draws=65535):
        """Draw ranges per launch set: at most ``max_draws`` (the grid-z limit of the batched
        launches) and ``rows_per_chunk`` budget units (~64 floats each) per chunk."""
        per = max(1, min(P, max_draws, rows_per_chunk // max(rows, 1)))
        return [(p0, min(P, p0 + per)) for p0 in range(0, P, per)]

    def _pack(layer, plan, P):
        F = _flat_layer(layer, P, dev)
        hidden = [[(li, a, b, n, F[:, w], F[:, bb]) for (li, a, b, n, w, bb) in g] for g in plan.hidden]
        outs = [(i, n, F[:, w], F[:, bb]) for (i, n, w, bb) in plan.outs]
        return hidden, outs

    def _lp_chunk(params: Params, out: Tensor):
        """out [P, B] <- log p(x | θ_p): reversed layers, D degree-scheduled passes each."""
        P = _draws(params)
        z = x.expand(P, B, D).contiguous()
        lp = out.reshape(P * B)
        lp.zero_()
        hs_all = torch.empty((P, B, width_sum), device=dev, dtype=torch.float32)
        for l in reversed(range(len(plans))):
            plan = plans[l]
            hidden, outs = _pack(params[l], plan, P)
            hs, o = [], 0
            for w in plan.widths:
                hs.append(hs_all[:, :, o:o + w])
                o += w
            xn = torch.zeros_like(z)
            z2, x2 = z.view(P * B, D), xn.view(P * B, D)
            for k in range(1, D + 1):
                for (li, a, b, n, wb, bb) in hidden[k - 1]:
                    dst = hs[li][:, :, a:b]
                    if li == 0:
                        ops.linear_act_batched(xn, wb, bb, act, context=ctx, out=dst)
                    else:
                        ops.linear_act_batched(hs[li - 1][:, :, :n], wb, bb, act, out=dst)
                i, n, wb, bb = outs[k - 1]
                if n:
                    raw = ops.linear_act_batched(hs[-1][:, :, :n], wb, bb, "identity").reshape(P * B, 2)
                else:  # the first dim in order sees only the bias (unconditional layer)
                    raw = bb.reshape(P, 1, 2).expand(P, B, 2).reshape(P * B, 2)
                ops.affine_ar(z2[:, i:i + 1], raw, True, ops.LD_ROWSUM_SUB, lp, out=x2[:, i:i + 1])
            z = xn
        ops.base_log_prob(z.view(P * B, D), out=lp, accumulate=True)

    # ---- one context vector for every row (the density-grid case, plot.py:189-204): every
    # degree-0 hidden unit (masks reach only the context) is a per-draw constant.  Those units
    # are computed once per draw (M = 1 launches) and their products with the later groups'
    # weights fold into those groups' biases; the per-row GEMMs only see the x-dependent groups.
    const_ctx = C > 0 and ctx.dim() == 1

    def _split_maps(plan):
        """Per block: (index maps of the constant columns, of the per-row columns, split e)."""
        if hasattr(plan, "split"):
            return plan.split
        e_out = {}  # layer -> width of its degree-0 group (its constant columns)
        for (li, a, b, n, w, bb) in plan.hidden[0]:
            e_out[li] = b
        split = []
        for g in plan.hidden:
            row = []
            for (li, a, b, n, w, bb) in g:
                e = C if li == 0 else e_out.get(li - 1, 0)
                row.append((e, w[:, :e].contiguous(), w[:, e:].contiguous()))
            split.append(row)
        e_last = e_out.get(len(plan.widths) - 1, 0)
        outs = [(e_last, w[:, :e_last].contiguous(), w[:, e_last:].contiguous()) for (i, n, w, bb) in plan.outs]
        plan.split = (split, outs)
        return plan.split

    def _lp_chunk_const(params: Params, out: Tensor):
        """_lp_chunk with the context's degree-0 units folded into per-draw biases."""
        P = _draws(params)
        z = x.expand(P, B, D).contiguous()
        lp = out.reshape(P * B)
        lp.zero_()
        hs_all = torch.empty((P, B, width_sum), device=dev, dtype=torch.float32)
        c1 = ctx.reshape(1, 1, C).expand(P, 1, C)
        for l in reversed(range(len(plans))):
            plan = plans[l]
            F = _flat_layer(params[l], P, dev)
            split, osplit = _split_maps(plan)
            hs, o = [], 0
            for w in plan.widths:
                hs.append(hs_all[:, :, o:o + w])
                o += w
            # per-draw constants: the degree-0 group of every hidden layer ([P, 1, e])
            hc = {}
            for (li, a, b, n, w, bb) in plan.hidden[0]:
                src = torch.cat((c1, torch.zeros((P, 1, D), device=dev)), 2) if li == 0 else hc[li - 1]
                hc[li] = ops.linear_act_batched(src[:, :, :n].contiguous(), F[:, w], F[:, bb], act)
            xn = torch.zeros_like(z)
            z2, x2 = z.view(P * B, D), xn.view(P * B, D)
            for k in range(1, D + 1):
                if k == 2 and _fused_pass2(plan, split):
                    # D = 2: pass 2 is one context-free MADE chain on x -> one fused launch
                    z = _pass2_fused(plan, split, osplit, F, hc, c1, xn, z, lp.view(P, B))
                    break
                for (li, a, b, n, w, bb), (e, wc, wr) in zip(plan.hidden[k - 1], split[k - 1]):
                    if k == 1:
                        continue  # degree-0 groups: the constants above
                    bias = F[:, bb]
                    if e:  # constant columns -> bias (one row per draw)
                        src = c1.contiguous() if li == 0 else hc[li - 1]
                        bias = ops.linear_act_batched(src, F[:, wc], bias, "identity")[:, 0, :].contiguous()
                    dst = hs[li][:, :, a:b]
                    inp = xn if li == 0 else hs[li - 1][:, :, e:n]
                    ops.linear_act_batched(inp, F[:, wr], bias, act, out=dst)
                i, n, wb, bb = plan.outs[k - 1]
                e, wc, wr = osplit[k - 1]
                bias = F[:, bb]
                if e:
                    bias = ops.linear_act_batched(hc[len(plan.widths) - 1], F[:, wc], bias, "identity")[:, 0, :]
                if n > e:
                    raw = ops.linear_act_batched(hs[-1][:, :, e:n], F[:, wr], bias.contiguous(), "identity")
                    raw = raw.reshape(P * B, 2)
                else:  # only constant inputs: one raw row per draw
                    raw = bias.reshape(P, 1, 2).expand(P, B, 2).reshape(P * B, 2)
                ops.affine_ar(z2[:, i:i + 1], raw, True, ops.LD_ROWSUM_SUB, lp, out=x2[:, i:i + 1])
            else:
                z = xn
        ops.base_log_prob(z.reshape(P * B, D), out=lp, accumulate=True)

    def _fused_pass2(plan, split):
        """D = 2 with every layer's degree-1 group in one block of <= 160 units (tanh / relu)."""
        if D != 2 or act not in ("tanh", "relu") or not fuse_pass2:
            return False
        g1 = plan.hidden[1]
        nl = len(plan.widths)
        return (len(g1) == nl and [blk[0] for blk in g1] == list(range(nl)) and
                all(b - a <= 160 for (li, a, b, n, w, bb) in g1))

    def _p2_map(plan, rows):
        """made.hip pack map of the pass-2 chain (context-free, degree-1 widths ``rows``)."""
        key = tuple(rows)
        if getattr(plan, "p2_key", None) != key:
            sp = MAFSpec(D, 0, rows, act)
            sp.param_shapes[-1] = ((2, rows[-1]), (2,))
            ones = [torch.ones(ws) for (ws, _) in sp.param_shapes]
            plan.p2_nh = (max(rows) + 31) // 32
            plan.p2_map = made_pack_map(sp, ones, plan.p2_nh).to(dev)
            plan.p2_key = key

    def _pass2_fused(plan, split, osplit, F, hc, c1, xn, z, lp2):
        """The order-2 dim of a 2-dim MAF layer: layer 0's degree-1 units from x, each later
        layer's from the previous layer's (context / degree-0 parts folded into per-draw biases),
        its two output rows, the inverse affine step — one naz_made_affine_inv1 launch."""
        P = z.shape[0]
        g1, s1 = plan.hidden[1], split[1]
        rows = [b - a for (li, a, b, n, w, bb) in g1]
        _p2_map(plan, rows)
        parts = [torch.zeros((P, 1), device=dev)]
        for (li, a, b, n, w, bb), (e, wc, wr) in zip(g1, s1):
            bias = F[:, bb]
            if e:
                src = c1.contiguous() if li == 0 else hc[li - 1]
                bias = ops.linear_act_batched(src, F[:, wc], bias, "identity")[:, 0, :]
            parts += [F[:, wr].reshape(P, -1), bias.reshape(P, -1)]
        i, n, wb, bb = plan.outs[1]
        e, wc, wr = osplit[1]
        bias = F[:, bb]
        if e:
            bias = ops.linear_act_batched(hc[len(plan.widths) - 1], F[:, wc], bias, "identity")[:, 0, :]
        parts += [F[:, wr].reshape(P, -1), bias.reshape(P, -1)]
        packed = torch.cat(parts, 1)[:, plan.p2_map].contiguous()
        return ops.made_affine_inv1(packed, len(rows), plan.p2_nh, xn, z, i, act, lp2, ops.LD_ROWSUM_SUB)

    def _same_structure():
        """Every layer's schedule has the same block shapes (only the permutation's dims differ):
        then the per-draw constants and packs of ALL layers run as single launches."""
        def sig(pl):
            split, osplit = _split_maps(pl)
            return (tuple(blk[:4] for blk in pl.hidden[0]), tuple(blk[:4] for blk in pl.hidden[1]),
                    tuple(t[0] for t in split[1]), tuple((o[1], t[0]) for o, t in zip(pl.outs, osplit)))
        s0 = sig(plans[0])
        return all(_fused_pass2(pl, None) and sig(pl) == s0 for pl in plans)

    def _lp_chunk_const2(params: Params, out: Tensor):
        """D = 2, one context vector, identical layer structure: the degree-0 constants, bias
        folds and pass-2 packs of all L layers x P draws in one launch each (Q = L P problems),
        then per layer only the order-1 affine step and the fused pass-2 kernel."""
        P = _draws(params)
        L = len(plans)
        Q = L * P
        z = x.expand(P, B, D).contiguous()
        lp = out.reshape(P * B)
        lp.zero_()
        Fa = torch.stack([_flat_layer(params[l], P, dev) for l in range(L)])  # [L, P, size]

        def gat(get):  # per-layer index maps of one shape -> [Q, *shape] (one gather)
            idx = torch.stack([get(l) for l in range(L)])
            return torch.gather(Fa, 2, idx.reshape(L, 1, -1).expand(L, P, -1)).reshape(Q, *idx.shape[1:])
        pl0 = plans[0]
        nl = len(pl0.widths)
        sp = [_split_maps(pl) for pl in plans]
        c1 = ctx.reshape(1, 1, C).expand(Q, 1, C).contiguous()
        hc = {}
        for j, (li, a, b, n, w, bb) in enumerate(pl0.hidden[0]):
            src = torch.cat((c1, torch.zeros((Q, 1, D), device=dev)), 2) if li == 0 else hc[li - 1]
            hc[li] = ops.linear_act_batched(src[:, :, :n].contiguous(), gat(lambda l: plans[l].hidden[0][j][4]),
                                            gat(lambda l: plans[l].hidden[0][j][5]), act)
        parts = [torch.zeros((Q, 1), device=dev)]
        for j, (li, a, b, n, w, bb) in enumerate(pl0.hidden[1]):
            e = sp[0][0][1][j][0]
            bias = gat(lambda l: plans[l].hidden[1][j][5])
            if e:
                bias = ops.linear_act_batched(c1 if li == 0 else hc[li - 1], gat(lambda l: sp[l][0][1][j][1]), bias,
                                              "identity")[:, 0, :]
            parts += [gat(lambda l: sp[l][0][1][j][2]).reshape(Q, -1), bias.reshape(Q, -1)]
        raws = []
        for k in range(2):
            e = sp[0][1][k][0]
            bias = gat(lambda l: plans[l].outs[k][3])
            if e:
                bias = ops.linear_act_batched(hc[nl - 1], gat(lambda l: sp[l][1][k][1]), bias, "identity")[:, 0, :]
            raws.append(bias)
        parts += [gat(lambda l: sp[l][1][1][2]).reshape(Q, -1), raws[1].reshape(Q, -1)]
        rows = [blk[2] - blk[1] for blk in pl0.hidden[1]]
        _p2_map(pl0, rows)
        packed = torch.cat(parts, 1)[:, pl0.p2_map].contiguous()  # [Q, made_packed_floats]
        for l in reversed(range(L)):
            i1, i2 = plans[l].outs[0][0], plans[l].outs[1][0]
            r1 = raws[0][l * P:(l + 1) * P].reshape(P, 1, 2).expand(P, B, 2).reshape(P * B, 2)
            xn = torch.zeros_like(z)
            ops.affine_ar(z.view(P * B, D)[:, i1:i1 + 1], r1, True, ops.LD_ROWSUM_SUB, lp,
                          out=xn.view(P * B, D)[:, i1:i1 + 1])
            z = ops.made_affine_inv1(packed[l * P:(l + 1) * P], nl, pl0.p2_nh, xn, z, i2, act, lp.view(P, B),
                                     ops.LD_ROWSUM_SUB)
        ops.base_log_prob(z.reshape(P * B, D), out=lp, accumulate=True)

    ar_mask = torch.cat(ar_maskvec) if ar_desc is not None else None  # [L * per], the packers apply it

    def _ar_flat(params: Params, P: int) -> Tensor:
        """[P, L * per] unmasked flat rows in the packers' layout (ravel order): a zero-copy view
        when the pytree is unravel()'s views of one [P, n] row buffer, else one concatenation."""
        ts = [t for layer in params for (w, b) in layer for t in (w, b)]
        base, off, ok = ts[0], 0, True
        S = base.stride(0) if base.dim() else 0
        for t in ts:
            ok = ok and t.dtype == torch.float32 and t.device == base.device and t.dim() >= 1 and \
                t.shape[0] == P and (P == 1 or t.stride(0) == S) and t[0].is_contiguous() and \
                t.data_ptr() - base.data_ptr() == 4 * off
            off += t[0].numel()
        if ok and (P == 1 or S >= off):
            return base.as_strided((P, off), (S if P > 1 else off, 1))
        return torch.cat([t.reshape(P, -1).to(dev, torch.float32) for t in ts], 1)

    def _lp_chunk_ar(params: Params, out: Tensor):
        """Every draw's inverse image packed on the device (naz_ar_flow_pack), then the whole flow
        for all draws in one naz_ar_flow_log_prob_batched launch (csrc/made_ar_r16.h)."""
        P = _draws(params)
        flat = _ar_flat(params, P)
        c0 = ar_pass0(flat, ctx, ar_mask) if ar_pass0 is not None else None
        packed = ops.ar_flow_pack_batched(ar_desc, flat, ar_perm, pass0=c0, mask=ar_mask)
        out.copy_(ops.ar_flow_log_prob_batched(ar_desc, packed, x, ctx, pass0_const=c0 is not None))


    def lp_batched(params: Params) -> Tensor:
        P = _draws(params)
        out = torch.empty((P, B), device=dev, dtype=torch.float32)
        if ar_perm is not None:
            # budget: the flat weights and the packed image per draw (~64-float units), plus its rows
            img = int(ops.lib().naz_ar_flow_packed_bytes(ar_desc)) // 4
            per_draw = (img + len(plans) * _flat_layer_size(params[0])) // 64 + B // 64 + 1
            for p0, p1 in _chunks(P, per_draw):
                _lp_chunk_ar([[(w[p0:p1], b[p0:p1]) for (w, b) in layer] for layer in params], out[p0:p1])
            return out
        run = _lp_chunk_const if (const_ctx and fold_context) else _lp_chunk
        per_draw, max_draws = B * max(1, width_sum // 64), 65535
        if run is _lp_chunk_const and batch_layers and _same_structure():
            run = _lp_chunk_const2
            # its launches run over Q = L * P problems (grid z), and it holds every layer's
            # flat parameters and pass-2 pack per draw: cap P and budget those bytes too
            L = len(plans)
            max_draws = max(1, 65535 // L)
            rows2 = [blk[2] - blk[1] for blk in plans[0].hidden[1]]
            pack = ops.made_packed_floats(len(rows2), (max(rows2) + 31) // 32, 0, D)
            per_draw += (L * (pack + _flat_layer_size(params[0]))) // 64 + 1
        for p0, p1 in _chunks(P, per_draw, max_draws):
            run([[(w[p0:p1], b[p0:p1]) for (w, b) in layer] for layer in params], out[p0:p1])
        return out

    def _sample_chunk(params: Params, z: Tensor, y_out: Tensor, lj_out: Tensor):
        """JAX forward_fn composed in flow order (bflow_jax_maf.py:172-178, 218-222):
        log_j = base(z) + Σ clip(ls) (the reference's returned quantity, sign as there)."""
        P, S = z.shape[0], z.shape[1]
        lj = lj_out.reshape(P * S)
        ops.base_log_prob(z.reshape(P * S, D), out=lj)
        if ar_desc is not None and (ctx_s is None or float(ctx_s.abs().max()) < 32768.0):
            packed = ops.ar_flow_pack_fwd_batched(ar_desc, _ar_flat(params, P), mask=ar_mask)
            y, ld = ops.ar_flow_sample_batched(ar_desc, packed, z, ctx_s)
            y_out.copy_(y)
            lj_out.add_(ld)
            return
        cur = z
        if fused_fwd:
            for l in range(len(plans)):
                nxt = y_out if l == len(plans) - 1 else torch.empty_like(cur)
                packed = _flat_layer(params[l], P, dev)[:, made_maps[l]]
                ops.made_affine_fwd(packed, len(spec.hidden_dims), nh, cur, ctx_s, act, lj_out, ops.LD_ROWSUM_ADD,
                                    out=nxt)
                cur = nxt
            return
        for l, plan in enumerate(plans):
            h = None
            layer = params[l]
            nlin = len(layer)
            for j, (w, b) in enumerate(layer):
                m = plan.masks_dev[j]
                a = "identity" if j == nlin - 1 else act
                w, b = w.to(torch.float32), b.to(torch.float32)
                if j == 0:
                    h = ops.linear_act_batched(cur, w, b, a, context=ctx_s, mask=m)
                else:
                    h = ops.linear_act_batched(h, w, b, a, mask=m)
            nxt = y_out if l == len(plans) - 1 else torch.empty_like(cur)
            ops.affine_ar(cur.reshape(P * S, D), h.reshape(P * S, 2 * D), False, ops.LD_ROWSUM_ADD, lj,
                          out=nxt.view(P * S, D))
            cur = nxt

    def sampler_batched(params: Params, rng_key: Union[int, torch.Generator, None] = None, size: int = 1,
                        z: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
        nonlocal ctx_s
        P = _draws(params)
        S = int(size)
        if z is None:
            g = rng_key if isinstance(rng_key, torch.Generator) else \
                torch.Generator(device=dev).manual_seed(int(rng_key or 0))
            z = torch.randn((P, S, D), device=dev, dtype=torch.float32, generator=g)
        else:
            z = z.to(dev, torch.float32).reshape(P, S, D).contiguous()
        if C:
            if ctx.dim() != 1 and ctx.shape[0] != 1:
                raise ValueError("sampler: the reference conditions on one context vector")
            ctx_s = ctx.reshape(-1)
        y = torch.empty((P, S, D), device=dev, dtype=torch.float32)
        lj = torch.empty((P, S), device=dev, dtype=torch.float32)
        for p0, p1 in _chunks(P, S * max(1, sum(spec.hidden_dims) // 64)):
            _sample_chunk([[(w[p0:p1], b[p0:p1]) for (w, b) in layer] for layer in params], z[p0:p1], y[p0:p1],
                          lj[p0:p1])
        return y, lj

    ctx_s = None

    grad_flow = {}

    def _grad_model():
        from torch import nn as tnn
        from .flow import NormalizingFlow
        f = grad_flow.get("f")
        if f is None:
            acts = {"tanh": tnn.Tanh(), "relu": tnn.ReLU(), "sigmoid": tnn.Sigmoid(), "identity": tnn.Identity()}
            f = NormalizingFlow("maf", None, D, C, spec.hidden_dims, len(plans), activation=acts[act]).to(dev)
            for t, perm in zip(f.transforms, perms):
                t.nn.set_permutation(torch.as_tensor(perm))
                t.nn.clip_zero_grad = True  # the potential differentiates jnp.clip (bflow_jax_maf.py:177-192)
            grad_flow["f"] = f
        return f

    def _grad_step(flat: Tensor):
        """flat θ -> (Σ lp, ∇θ): MafGrad, or the weights copied into a naz_amd maf and the NLL
        training walk forward + backward."""
        mg = _fused_grad()
        if mg is not None:
            return mg(flat, x, None if ctx is None else (ctx.reshape(1, -1) if ctx.dim() == 1 else ctx))
        f = _grad_model()
        params = unravel(flat, [spec.param_shapes] * len(plans))
        with torch.no_grad():
            for t, layer in zip(f.transforms, params):
                for lin, (w, b) in zip(t.nn.layers, layer):
                    lin.weight.copy_(w)
                    lin.bias.copy_(b)
        with torch.enable_grad():
            total = f.log_prob(x, condition=ctx).sum()
            total.backward()
        g = [[(lin.weight.grad, lin.bias.grad) for lin in t.nn.layers] for t in f.transforms]
        return total.detach(), ravel(g)

    def _capture(flat0: Tensor):
        """The whole gradient step as one HIP graph (the walk is ~1,000 small launches eager)."""
        fused = _fused_grad() is not None
        f = None if fused else _grad_model()
        static = flat0.detach().clone()
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):  # warm the caches (schedules, packs) outside the capture
                if f is not None:
                    f.zero_grad(set_to_none=True)
                _grad_step(static)
        torch.cuda.current_stream(dev).wait_stream(side)
        if f is not None:
            f.zero_grad(set_to_none=True)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = _grad_step(static)
        grad_flow["graph"] = (graph, static, out)

    def _fused_grad():
        """MafGrad over these rows (maf_grad.py: the fused inverse with saved states, one fused
        backward launch per layer, bf16x6 batch reductions), or None where it does not apply."""
        if ar_grad_perm is None or not fused_grad:
            return None
        mg = grad_flow.get("mafgrad")
        if mg is None:
            from .maf_grad import MafGrad
            # jnp.clip's gradient for the log_scale clip, as jax.grad of the reference's potential
            mg = grad_flow["mafgrad"] = MafGrad(ar_desc, ar_grad_perm, torch.cat(ar_maskvec), clip_zero=True)
        return mg

    def lp_and_grad(params, use_graph: bool = True) -> Tuple[Tensor, Tensor]:
        """(Σ_rows log p(x | θ), ∇θ of it in ``ravel`` order): the NUTS / HMC potential of
        ``bayesian_normalizing_flow`` (bflow_jax_maf.py:233-235: ``flow_lp(unravel(p)).sum()``
        and its gradient).  One draw (pytree or flat [n]).  At the fused backward's shapes (the
        paper maf, pyro masks, rows inside the f16 split's range): MafGrad.  Otherwise the NLL
        training walk (HIP forward + backward kernels, nn autograd) on a naz_amd maf with these
        weights.  Either is replayed as one captured HIP graph after the first call
        (``use_graph=False``: eager launches)."""
        flat = params if torch.is_tensor(params) else ravel(params)
        flat = flat.to(dev, torch.float32).reshape(-1)
        if use_graph and "graph" not in grad_flow and not grad_flow.get("no_graph"):
            try:
                _capture(flat)
            except RuntimeError:  # capture unsupported here: eager launches (same kernels)
                grad_flow["no_graph"] = True
                torch.cuda.synchronize(dev)
        if use_graph and "graph" in grad_flow:
            graph, static, (total, grad) = grad_flow["graph"]
            static.copy_(flat)
            graph.replay()
            return total.clone(), grad.clone()
        if _fused_grad() is None:
            _grad_model().zero_grad(set_to_none=True)
        return _grad_step(flat)

    def _one(params):
        return [[(w.unsqueeze(0), b.unsqueeze(0)) for (w, b) in layer] for layer in params]

    def lp(params: Params) -> Tensor:
        return lp_batched(_one(params))[0]

    def sampler(params: Params, rng_key=None, size: int = 1):
        y, lj = sampler_batched(_one(params), rng_key, size)
        return y[0], lj[0]

    def lp_flops_per_row() -> int:
        """GEMM FLOPs per (draw, row) of lp_batched: on the fused AR kernel the FLOPs it executes
        (ops.ar_executed_flop_per_row: block rounding and padding included); otherwise the degree
        schedule's (every MADE unit once), or with the context folded the per-row part."""
        if ar_perm is not None:
            return ops.ar_executed_flop_per_row(ar_desc, pass0_const=ar_pass0 is not None)["inverse"]
        tot = 0
        for plan in plans:
            if const_ctx and fold_context and ar_perm is None:
                split, osplit = _split_maps(plan)
                for g in range(1, D):
                    for (li, a, b, n, w, bb), (e, wc, wr) in zip(plan.hidden[g], split[g]):
                        tot += 2 * (b - a) * (n - e)
                tot += sum(2 * 2 * max(n - e, 0) for (i, n, w, bb), (e, wc, wr) in zip(plan.outs, osplit))
            else:
                tot += sum(2 * (b - a) * n for g in plan.hidden for (li, a, b, n, w, bb) in g)
                tot += sum(2 * 2 * n for (i, n, w, bb) in plan.outs)
        return tot

    return {"lp": lp, "sampler": sampler, "lp_batched": lp_batched, "sampler_batched": sampler_batched,
            "lp_and_grad": lp_and_grad, "grad_state": grad_flow, "lp_flops_per_row": lp_flops_per_row,
            "grad_fused": ar_grad_perm is not None and fused_grad,
            "plans": plans, "fused_fwd": fused_fwd, "lp_fused_ar": ar_perm is not None}
