"""Flow transforms and factories with naz's API (naz/flows/transforms.py), HIP-executed.

Factories keep naz's signatures and return ``(flow, transforms, nets)``:
  masked_affine_autoregressive  ("maf", naz/flows/transforms.py:133-160)
  neural_spline_autoregressive  ("nsa", naz/flows/transforms.py:165-198)
  neural_spline_coupling        ("nsc", naz/flows/transforms.py:201-236 — naz's intent;
                                 the reference body is broken)

Transform classes follow the pyro protocol the reference relies on: ``condition(ctx)``
on conditional modules, ``__call__``/``_call``, ``inv``/``_inverse``,
``log_abs_det_jacobian(x, y) -> [B]`` with a size-1 cache, ``.nn`` conditioners with
``layers.{i}.weight|bias``.  Each transform also offers ``_inverse_acc(y, lp)`` /
``_call_acc(x, ld)`` — the same map with the row log-det accumulated in-kernel — which
``TransformedDistribution.log_prob``/``sample`` use so no torch arithmetic runs.
"""
from __future__ import annotations

from typing import List, Optional

import torch
from torch import nn
from torch.distributions import Transform, constraints
import torch.nn.functional as F

from .. import autograd as ag
from .. import ops
from ..nn import (AutoRegressiveNN, ConditionalAutoRegressiveNN, ConditionalDenseNN, DenseNN, cache_epoch)
from ..utils import device, set_device

# per-Transform spline-coupling calls on the fused one-layer kernel (naz_coupling_layer_{fwd,inv});
# NAZ_LAYER_FUSED=0 keeps the per-kernel chain (naz_linear_act + naz_rqs)
_LAYER_FUSED = __import__("os").environ.get("NAZ_LAYER_FUSED", "1") != "0"

__all__ = ["TransformModule", "ConditionalTransformModule", "ComposeTransformModule",
           "ConditionalComposeTransformModule", "Spline", "SplineCoupling", "ConditionalSplineCoupling",
           "SplineAutoregressive", "ConditionalSplineAutoregressive", "AffineAutoregressive",
           "ConditionalAffineAutoregressive", "Permute", "bounding_transform", "inverse_bounding_transform",
           "masked_affine_autoregressive", "neural_spline_autoregressive", "neural_spline_coupling"]


# ----------------------------------------------------------------------------- protocol
class TransformModule(Transform, nn.Module):
    """[pyro] distributions/torch_transform.py::TransformModule."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)

    def __hash__(self):
        return super(nn.Module, self).__hash__()


class ConditionalTransformModule(nn.Module):
    """[pyro] distributions/conditional.py::ConditionalTransformModule."""

    def condition(self, context):
        raise NotImplementedError


class ComposeTransformModule(TransformModule):
    """[pyro] ComposeTransformModule: an nn.ModuleList of transforms applied in order."""

    bijective = True

    def __init__(self, parts: List[Transform]):
        super().__init__(cache_size=0)
        self.parts = nn.ModuleList([p for p in parts if isinstance(p, nn.Module)])
        self._all = list(parts)

    @property
    def domain(self):
        return constraints.real_vector

    @property
    def codomain(self):
        return constraints.real_vector

    def __iter__(self):
        return iter(self._all)

    def __len__(self):
        return len(self._all)

    def _call(self, x):
        for p in self._all:
            x = p(x)
        return x

    def _inverse(self, y):
        for p in reversed(self._all):
            y = p.inv(y)
        return y

    def log_abs_det_jacobian(self, x, y):
        raise NotImplementedError("use TransformedDistribution.log_prob (per-layer caches are consumed there)")

    def _inverse_acc(self, y, lp):
        for p in reversed(self._all):
            y = p._inverse_acc(y, lp)
        return y

    def _call_acc(self, x, ld):
        for p in self._all:
            x = p._call_acc(x, ld)
        return x

    def _inv_ld(self, y):
        total = None
        for p in reversed(self._all):
            y, ld = p._inv_ld(y)
            if ld is not None:
                total = ld if total is None else total + ld
        return y, total


class ConditionalComposeTransformModule(ConditionalTransformModule):
    """[pyro] ConditionalComposeTransformModule (naz/flows/transforms.py:157,196,234):
    iterable over its layers; ``parts`` registers the module layers' parameters."""

    def __init__(self, transforms, cache_size=0):
        super().__init__()
        self.parts = nn.ModuleList([t for t in transforms if isinstance(t, nn.Module)])
        self._all = list(transforms)

    def __iter__(self):
        return iter(self._all)

    def __len__(self):
        return len(self._all)

    def condition(self, context):
        return [t.condition(context) if isinstance(t, ConditionalTransformModule) else t for t in self._all]


# ----------------------------------------------------------------------------- bounding
def bounding_transform(x, low, high):
    """naz/flows/transforms.py:20-23 — HIP kernel naz_bounding_fwd."""
    return ops.bounding_fwd(x, low, high)


def inverse_bounding_transform(y, low, high):
    """naz/flows/transforms.py:25-27 — HIP kernel naz_bounding_inv."""
    return ops.bounding_inv(y, low, high)


# ----------------------------------------------------------------------------- splines
def _degree_plan(arn, v, ld_mode):
    """The MADE net's degree-scheduled inverse (nn.ARInversePlan) when it applies: 2-D batch,
    a row-sum log-det (each pass adds its own dim's term)."""
    if ld_mode == ops.LD_PERDIM or v.dim() != 2:
        return None
    return arn.inverse_plan()


def _pass_ld_mode(ld_mode, k):
    """Row-sum mode of pass k's single-dim term: an overwriting mode overwrites on pass 1 only."""
    return ops.LD_ROWSUM if (ld_mode == ops.LD_ROWSUM and k == 1) else (
        ops.LD_ROWSUM_ADD if ld_mode == ops.LD_ROWSUM else ld_mode)


def _zeros_rows(x):
    return torch.zeros(x.shape[:-1], device=x.device, dtype=torch.float32)


class _LDCache:
    """pyro-style size-1 cache of the per-row forward log|det J|."""

    def _set_ld(self, ld):
        self._cache_log_detJ = ld

    def log_abs_det_jacobian(self, x, y):
        x_old, y_old = self._cached_x_y
        if getattr(self, "_cache_log_detJ", None) is None or x is not x_old or y is not y_old:
            self(x)
        return self._cache_log_detJ


class Spline(TransformModule):
    """[pyro] distributions/transforms/spline.py::Spline (order="quadratic") — elementwise,
    unconditional; used as SplineCoupling's lower spline.  Parameters are unnormalised."""

    domain = constraints.real
    codomain = constraints.real
    bijective = True

    def __init__(self, input_dim: int, count_bins: int = 8, bound: float = 3.0, order: str = "quadratic"):
        super().__init__(cache_size=1)
        if order != "quadratic":
            raise NotImplementedError("naz_amd: only order='quadratic' (naz's default) is implemented")
        self.input_dim, self.count_bins, self.bound, self.order = input_dim, count_bins, bound, order
        self.unnormalized_widths = nn.Parameter(torch.randn(input_dim, count_bins))
        self.unnormalized_heights = nn.Parameter(torch.randn(input_dim, count_bins))
        self.unnormalized_derivatives = nn.Parameter(torch.randn(input_dim, count_bins - 1))
        self._cache_log_detJ = None

    def flat_raw(self):
        """[w(S*K) | h(S*K) | d(S*(K-1))] — one broadcast conditioner row (DENSE layout)."""
        return torch.cat([self.unnormalized_widths.reshape(-1), self.unnormalized_heights.reshape(-1),
                          self.unnormalized_derivatives.reshape(-1)])

    def spline_apply(self, x, inverse, ld_mode, ld_out, out=None):
        return ops.rqs(x, self.flat_raw(), self.count_bins, ops.LAYOUT_DENSE, inverse, self.bound, ld_mode, ld_out,
                       out=out, broadcast_raw=True, fast=True)

    def _call(self, x):
        y, ld = self.spline_apply(x, False, ops.LD_PERDIM, None)
        self._cache_log_detJ = ld
        return y

    def _inverse(self, y):
        x, ld = self.spline_apply(y, True, ops.LD_PERDIM, None)
        self._cache_log_detJ = None  # per-dim forward ld needs a negation; recomputed on demand
        return x

    def log_abs_det_jacobian(self, x, y):
        _, ld = self.spline_apply(x, False, ops.LD_PERDIM, None)
        return ld


def _fused_coupling_layer(m, v, inverse, context, ld_buf, ld_mode):
    """One spline-coupling layer as ONE naz_coupling_layer_{fwd,inv} launch for the
    per-Transform protocol (pyro's t(x) / t.inv(y)): the conditioner, the lower and upper splines and
    the log-det fused, on the module's own one-layer 16-row f16x3 image (re-packed when a parameter
    changes).  None where it does not apply (autograd recording, dropout active, a shape without a
    16-row instantiation, per-dim log-dets): the per-kernel chain runs."""
    if (v.dim() != 2 or ld_mode not in (ops.LD_ROWSUM, ops.LD_ROWSUM_ADD, ops.LD_ROWSUM_SUB) or v.requires_grad
            or (torch.is_grad_enabled() and any(p.requires_grad for p in m.parameters()))):
        return None
    net = m.nn
    if not isinstance(net, ConditionalDenseNN) or net.dropout_active() or len(net.hidden_dims) != 2 or \
            net.hidden_dims[0] != net.hidden_dims[1]:
        return None
    C = net.context_dim
    if C and (context is None or context.dim() > 2 or (context.dim() == 2 and context.shape[0] not in (1, v.shape[0]))):
        return None
    plan = m.__dict__.get("_layer_plan")
    if plan is None:
        from .flow import _FusedCoupling
        plan = _FusedCoupling([m], m.input_dim, C, m.split_dim, m.count_bins, net.hidden_dims[0], net.act,
                              m.lower_spline is not None, m.bound, mfma="f16x3r16")
        if not ops.coupling_supported(plan.desc):
            plan = False
        m.__dict__["_layer_plan"] = plan
    if plan is False:
        return None
    packed = plan.packed()
    if plan.mode != "f16x3r16":
        return None
    # the ABI reports the layer's FORWARD log-det; the per-kernel chain's inverse modes act on the
    # inverse's (its negation): swap += and -= for the inverse direction
    mode = ld_mode
    if inverse and ld_mode != ops.LD_ROWSUM:
        mode = ops.LD_ROWSUM_SUB if ld_mode == ops.LD_ROWSUM_ADD else ops.LD_ROWSUM_ADD
    if inverse and ld_mode == ops.LD_ROWSUM:
        return None
    ctx = None if not C else (context.reshape(1, -1) if context.dim() == 1 else context)
    return ops.coupling_layer(plan.desc, packed, 0, v, ctx, inverse, ld_buf, mode)


class _ConditionedSplineCoupling(_LDCache, Transform):
    """[pyro] SplineCoupling with the hypernet bound to a context (naz/flows/transforms.py:126-129)."""

    domain = constraints.real_vector
    codomain = constraints.real_vector
    bijective = True

    def __init__(self, module: "ConditionalSplineCoupling", context: Optional[torch.Tensor]):
        super().__init__(cache_size=1)
        self.module, self.context = module, context
        self._cache_log_detJ = None

    @property
    def nn(self):
        return self.module.nn

    def _map(self, v, inverse: bool, ld_buf, ld_mode):
        m = self.module
        if _LAYER_FUSED:
            y = _fused_coupling_layer(m, v, inverse, self.context, ld_buf, ld_mode)
            if y is not None:
                return y
        s = m.split_dim
        out = torch.empty_like(v)
        v1, v2 = v[:, :s], v[:, s:]
        if inverse:
            if m.lower_spline is not None:
                m.lower_spline.spline_apply(v1, True, ld_mode, ld_buf, out=out[:, :s])
            else:
                out[:, :s].copy_(v1)
            x1 = out[:, :s]
        else:
            x1 = v1
        raw = m.nn.raw(x1, self.context)
        ops.rqs(v2, raw, m.count_bins, ops.LAYOUT_DENSE, inverse, m.bound, ld_mode, ld_buf, out=out[:, s:], fast=True)
        if not inverse:
            if m.lower_spline is not None:
                m.lower_spline.spline_apply(v1, False, ld_mode, ld_buf, out=out[:, :s])
            else:
                out[:, :s].copy_(v1)
        return out

    def _call(self, x):
        ld = _zeros_rows(x)
        y = self._map(x, False, ld, ops.LD_ROWSUM_ADD)
        self._set_ld(ld)
        return y

    def _inverse(self, y):
        ld = _zeros_rows(y)
        x = self._map(y, True, ld, ops.LD_ROWSUM_SUB)  # forward ld = -(inverse ld)
        self._set_ld(ld)
        return x

    def _inverse_acc(self, y, lp):
        """x = T^-1(y) and lp -= log|det J_T(x)| in-kernel."""
        return self._map(y, True, lp, ops.LD_ROWSUM_ADD)

    def _call_acc(self, x, ld):
        return self._map(x, False, ld, ops.LD_ROWSUM_ADD)

    def _inv_ld(self, y):
        """Differentiable x = T^-1(y) and the FORWARD row log-det (training walk, a10)."""
        m = self.module
        s = m.split_dim
        y1, y2 = y[:, :s], y[:, s:]
        ld_inv = None
        if m.lower_spline is not None:
            x1, ld_inv = ag.rqs(y1, m.lower_spline.flat_raw(), m.count_bins, ops.LAYOUT_DENSE, True, m.bound,
                                broadcast=True)
        else:
            x1 = y1
        raw = m.nn.raw(x1, self.context)
        x2, ld2 = ag.rqs(y2, raw, m.count_bins, ops.LAYOUT_DENSE, True, m.bound)
        ld_inv = ld2 if ld_inv is None else ld_inv + ld2
        return torch.cat([x1, x2], dim=1), -ld_inv


class ConditionalSplineCoupling(ConditionalTransformModule):
    """naz ``ConditionalSplineCoupling`` (naz/flows/transforms.py:113-129), made runnable:
    pyro SplineCoupling(input_dim, split_dim, partial(nn, context), count_bins, bound, order)
    with a PERSISTENT lower spline (naz rebuilt it with fresh random parameters on every
    ``condition`` call — see DESIGN.md).  ``identity=True`` drops the lower spline."""

    def __init__(self, input_dim: int, split_dim: int, dense_nn: nn.Module, count_bins: int = 8,
                 bound: float = 3.0, order: str = "quadratic", identity: bool = False):
        super().__init__()
        if order != "quadratic":
            raise NotImplementedError("naz_amd: only order='quadratic' (naz's default) is implemented")
        self.input_dim, self.split_dim, self.count_bins, self.bound, self.order = (
            input_dim, split_dim, count_bins, bound, order)
        self.nn = dense_nn
        self.lower_spline = None if identity else Spline(split_dim, count_bins, bound, order)

    def condition(self, context):
        return _ConditionedSplineCoupling(self, context)


class SplineCoupling(_ConditionedSplineCoupling, nn.Module):
    """[pyro] SplineCoupling, unconditional (hypernet = DenseNN on x1)."""

    def __init__(self, input_dim: int, split_dim: int, hypernet: nn.Module, count_bins: int = 8,
                 bound: float = 3.0, order: str = "quadratic", identity: bool = False):
        inner = ConditionalSplineCoupling(input_dim, split_dim, hypernet, count_bins, bound, order, identity)
        Transform.__init__(self, cache_size=1)
        self.inner = inner
        self.context = None
        self._cache_log_detJ = None

    @property
    def module(self):
        return self.inner

    @property
    def nn(self):
        return self.inner.nn

    @property
    def lower_spline(self):
        return self.inner.lower_spline

    def __hash__(self):
        return nn.Module.__hash__(self)


class _ConditionedSplineAutoregressive(_LDCache, Transform):
    """[pyro] ConditionedSplineAutoregressive: ``_call`` is one MADE pass, ``_inverse`` the
    D-pass loop (naz ``nsa``, naz/flows/transforms.py:165-198)."""

    domain = constraints.real_vector
    codomain = constraints.real_vector
    bijective = True

    def __init__(self, arn, context, count_bins, bound):
        super().__init__(cache_size=1)
        self.arn, self.context, self.count_bins, self.bound = arn, context, count_bins, bound
        self._cache_log_detJ = None

    @property
    def nn(self):
        return self.arn

    def _map(self, v, inverse, ld_buf, ld_mode):
        if not inverse:
            y = _fused_made_forward(self.arn, v, self.context, ld_buf, ld_mode)
            if y is not None:
                return y
            raw = self.arn.raw(v, self.context)
            y, _ = ops.rqs(v, raw, self.count_bins, ops.LAYOUT_ARN, False, self.bound, ld_mode, ld_buf, fast=True)
            return y
        plan = _degree_plan(self.arn, v, ld_mode)
        if plan is not None:
            def step(k, i, raw, x):
                ops.rqs(v[:, i:i + 1], raw, self.count_bins, ops.LAYOUT_ARN, True, self.bound,
                        _pass_ld_mode(ld_mode, k), ld_buf, out=x[:, i:i + 1], fast=True)
            return plan.run(v, self.context, step)
        x = torch.zeros_like(v)
        D = v.shape[-1]
        scratch = _zeros_rows(v)
        for k in range(D):
            raw = self.arn.raw(x, self.context)
            last = k == D - 1
            x, _ = ops.rqs(v, raw, self.count_bins, ops.LAYOUT_ARN, True, self.bound,
                           ld_mode if last else ops.LD_ROWSUM, ld_buf if last else scratch, fast=True)
        return x

    def _call(self, x):
        ld = _zeros_rows(x)
        y = self._map(x, False, ld, ops.LD_ROWSUM_ADD)
        self._set_ld(ld)
        return y

    def _inverse(self, y):
        ld = _zeros_rows(y)
        x = self._map(y, True, ld, ops.LD_ROWSUM_SUB)
        self._set_ld(ld)
        return x

    def _inverse_acc(self, y, lp):
        return self._map(y, True, lp, ops.LD_ROWSUM_ADD)

    def _call_acc(self, x, ld):
        return self._map(x, False, ld, ops.LD_ROWSUM_ADD)

    def _inv_ld(self, y):
        """Differentiable inverse.  Degree-scheduled (every MADE unit once, ARInversePlan.run_grad:
        per pass the order-k dim's spline on its 3K-1 ARN rows, single-dim naz_rqs_inv + its VJP)
        unless the conditioner's degree_schedule is off; then pyro's D full passes, autograd running
        back through every pass as pyro's does."""
        plan = self.arn.inverse_plan() if y.dim() == 2 else None
        if plan is not None:
            x, ld = plan.run_grad(y, self.context, lambda k, i, raw: ag.rqs(
                y[:, i:i + 1], raw, self.count_bins, ops.LAYOUT_ARN, True, self.bound))
            return x, -ld  # the steps' log-dets are the inverse's; the walk wants the forward's
        x = torch.zeros_like(y)
        ld = None
        for _ in range(y.shape[-1]):
            raw = self.arn.raw(x, self.context)
            x, ld = ag.rqs(y, raw, self.count_bins, ops.LAYOUT_ARN, True, self.bound)
        return x, -ld


class ConditionalSplineAutoregressive(ConditionalTransformModule):
    """[pyro] ConditionalSplineAutoregressive (naz/flows/transforms.py:190)."""

    def __init__(self, input_dim, autoregressive_nn, count_bins=8, bound=3.0, order="quadratic"):
        super().__init__()
        if order != "quadratic":
            raise NotImplementedError("naz_amd: only order='quadratic' (naz's default) is implemented")
        self.input_dim, self.count_bins, self.bound, self.order = input_dim, count_bins, bound, order
        self.nn = autoregressive_nn

    def condition(self, context):
        return _ConditionedSplineAutoregressive(self.nn, context, self.count_bins, self.bound)


class SplineAutoregressive(_ConditionedSplineAutoregressive, nn.Module):
    """[pyro] SplineAutoregressive (unconditional)."""

    def __init__(self, input_dim, autoregressive_nn, count_bins=8, bound=3.0, order="quadratic"):
        if order != "quadratic":
            raise NotImplementedError("naz_amd: only order='quadratic' (naz's default) is implemented")
        Transform.__init__(self, cache_size=1)
        self.input_dim, self.order = input_dim, order
        self.arn_module = autoregressive_nn
        self.context, self.count_bins, self.bound = None, count_bins, bound
        self._cache_log_detJ = None

    @property
    def arn(self):
        return self.arn_module

    @property
    def nn(self):
        return self.arn_module

    def __hash__(self):
        return nn.Module.__hash__(self)


def _fused_made_forward(arn, v, context, ld_buf, ld_mode):
    """AffineAutoregressive._call as ONE naz_made_affine_fwd launch (the whole masked MADE
    conditioner + affine step, csrc/made.hip) when nothing is recorded for autograd and the
    shape fits the kernel (hidden widths <= 160, 2D <= 32, tanh / relu, row-sum log-det);
    None otherwise (the per-GEMM path runs)."""
    from .bflow_maf import MAFSpec, made_pack_map
    layers = list(arn.layers)
    if (v.dim() != 2 or arn.dropout_active() or arn.output_multiplier != 2 or 2 * arn.input_dim > 32
            or arn.act not in ("tanh", "relu")
            or max(arn.hidden_dims) > 160 or ld_mode == ops.LD_PERDIM or v.requires_grad
            or (torch.is_grad_enabled() and any(p.requires_grad for p in arn.parameters()))):
        return None
    C = arn.context_dim
    if C and (context is None or context.dim() > 2 or (context.dim() == 2 and context.shape[0] not in (1, v.shape[0]))):
        return None
    nh = (max(arn.hidden_dims) + 31) // 32
    key = tuple((l.weight.data_ptr(), l.weight._version, l.bias.data_ptr(), l.bias._version, l.mask._version)
                for l in layers) + (cache_epoch(),)
    cache = arn.__dict__.get("_made_fwd")
    if cache is None or cache[0] != key:
        spec = MAFSpec(arn.input_dim, C, arn.hidden_dims, arn.act)
        mp = made_pack_map(spec, [l.mask for l in layers], nh).to(v.device)
        flat = torch.cat([torch.zeros(1, device=v.device)] +
                         [t.detach().reshape(-1).float() for l in layers for t in (l.weight, l.bias)])
        cache = (key, flat[mp].reshape(1, -1).contiguous())
        arn.__dict__["_made_fwd"] = cache
    x = v.contiguous().unsqueeze(0)
    ctx = None if not C else context.reshape(-1, C)
    y = ops.made_affine_fwd(cache[1], len(arn.hidden_dims), nh, x, ctx, arn.act, ld_buf.view(1, -1), ld_mode)
    return y[0]


class _ConditionedAffineAutoregressive(_LDCache, Transform):
    """[pyro] AffineAutoregressive(stable=False), clip (-5, 3) (naz ``maf``,
    naz/flows/transforms.py:133-160; JAX restatement bflow_jax_maf.py:169-194)."""

    domain = constraints.real_vector
    codomain = constraints.real_vector
    bijective = True
    log_scale_min_clip, log_scale_max_clip = -5.0, 3.0

    def __init__(self, arn, context):
        super().__init__(cache_size=1)
        self.arn, self.context = arn, context
        self._cache_log_detJ = None

    @property
    def nn(self):
        return self.arn

    def _map(self, v, inverse, ld_buf, ld_mode):
        if not inverse:
            raw = self.arn.raw(v, self.context)
            y, _ = ops.affine_ar(v, raw, False, ld_mode, ld_buf)
            return y
        plan = _degree_plan(self.arn, v, ld_mode)
        if plan is not None:
            def step(k, i, raw, x):  # naz_affine_ar reports the FORWARD log-det in both directions
                ops.affine_ar(v[:, i:i + 1], raw, True, _pass_ld_mode(ld_mode, k), ld_buf, out=x[:, i:i + 1])
            if ld_mode != ops.LD_PERDIM:  # D = 2, one context vector: pass 2 fused
                y = plan.run_affine2(v, self.context, step, ld_buf, _pass_ld_mode(ld_mode, 2))
                if y is not None:
                    return y
            return plan.run(v, self.context, step)
        # pyro loops over the permutation updating one dim per pass; updating every dim per
        # pass gives identical values (masked weights are exact zeros for non-predecessors)
        x = torch.zeros_like(v)
        D = v.shape[-1]
        scratch = _zeros_rows(v)
        for k in range(D):
            raw = self.arn.raw(x, self.context)
            last = k == D - 1
            x, _ = ops.affine_ar(v, raw, True, ld_mode if last else ops.LD_ROWSUM, ld_buf if last else scratch)
        return x

    def _call(self, x):
        ld = _zeros_rows(x)
        y = self._map(x, False, ld, ops.LD_ROWSUM_ADD)
        self._set_ld(ld)
        return y

    def _inverse(self, y):
        ld = _zeros_rows(y)
        x = self._map(y, True, ld, ops.LD_ROWSUM_ADD)  # affine kernel already reports forward ld
        self._set_ld(ld)
        return x

    def _inverse_acc(self, y, lp):
        return self._map(y, True, lp, ops.LD_ROWSUM_SUB)

    def _call_acc(self, x, ld):
        return self._map(x, False, ld, ops.LD_ROWSUM_ADD)

    def _inv_ld(self, y):
        """Differentiable inverse; the affine kernel reports the forward log-det.  Degree-
        scheduled (every MADE unit once, ARInversePlan.run_grad) unless the conditioner's
        degree_schedule is off, then pyro's D full passes."""
        plan = self.arn.inverse_plan() if y.dim() == 2 else None
        cz = bool(getattr(self.arn, "clip_zero_grad", False))  # the JAX MAF's jnp.clip gradient
        if plan is not None:
            return plan.run_grad(y, self.context, lambda k, i, raw: ag.affine_ar(y[:, i:i + 1], raw, True, cz))
        x = torch.zeros_like(y)
        ld = None
        for _ in range(y.shape[-1]):
            raw = self.arn.raw(x, self.context)
            x, ld = ag.affine_ar(y, raw, True, cz)
        return x, ld


class ConditionalAffineAutoregressive(ConditionalTransformModule):
    """[pyro] ConditionalAffineAutoregressive (naz/flows/transforms.py:159)."""

    def __init__(self, autoregressive_nn, **kwargs):
        super().__init__()
        self.nn = autoregressive_nn

    def condition(self, context):
        return _ConditionedAffineAutoregressive(self.nn, context)


class AffineAutoregressive(_ConditionedAffineAutoregressive, nn.Module):
    """[pyro] AffineAutoregressive (unconditional)."""

    def __init__(self, autoregressive_nn, **kwargs):
        Transform.__init__(self, cache_size=1)
        self.arn_module = autoregressive_nn
        self.context = None
        self._cache_log_detJ = None

    @property
    def arn(self):
        return self.arn_module

    @property
    def nn(self):
        return self.arn_module

    def __hash__(self):
        return nn.Module.__hash__(self)


class Permute(Transform):
    """[pyro] T.Permute (naz random_perm=True).  The gather is a pure index copy."""

    domain = constraints.real_vector
    codomain = constraints.real_vector
    bijective = True

    def __init__(self, permutation):
        super().__init__(cache_size=1)
        self.permutation = permutation
        inv = torch.empty_like(permutation)
        inv[permutation] = torch.arange(permutation.numel(), device=permutation.device)
        self.inv_permutation = inv

    def _call(self, x):
        return x[..., self.permutation.to(x.device)]

    def _inverse(self, y):
        return y[..., self.inv_permutation.to(y.device)]

    def log_abs_det_jacobian(self, x, y):
        return _zeros_rows(x)

    def _inverse_acc(self, y, lp):
        return self._inverse(y)

    def _call_acc(self, x, ld):
        return self._call(x)

    def _inv_ld(self, y):
        return self._inverse(y), None


# ----------------------------------------------------------------------------- factories
def _hidden(hidden_dim):
    return list(hidden_dim) if isinstance(hidden_dim, (list, tuple)) else [hidden_dim]


def _unsupported(use_batchnorm, dropout_p):
    """use_batchnorm is rejected; returns the conditioners' dropout probability (naz's
    *Dropout conditioners when dropout_p is not None, transforms.py:141-147,178-184,224-227)."""
    if use_batchnorm:
        raise NotImplementedError("naz_amd: use_batchnorm is outside the log_prob hot path (SURVEY.md §8)")
    if dropout_p is not None and not 0.0 <= float(dropout_p) < 1.0:
        raise ValueError("dropout_p must be in [0, 1)")
    return 0.0 if dropout_p is None else float(dropout_p)


def masked_affine_autoregressive(theta_dim, condition_dim, hidden_dim, num_layers, activation=nn.Tanh(),
                                 use_batchnorm=False, random_mask=True, random_perm=False, dropout_p=None):
    """naz/flows/transforms.py:133-160."""
    p = _unsupported(use_batchnorm, dropout_p)
    transforms, nets = [], []
    for _ in range(num_layers):
        perm = None if random_mask else torch.arange(theta_dim)
        arn = (ConditionalAutoRegressiveNN(theta_dim, condition_dim, _hidden(hidden_dim), nonlinearity=activation,
                                           permutation=perm, dropout_p=p) if condition_dim > 0 else
               AutoRegressiveNN(theta_dim, _hidden(hidden_dim), nonlinearity=activation, permutation=perm,
                                dropout_p=p))
        nets.append(arn)
        t = ConditionalAffineAutoregressive(arn) if condition_dim > 0 else AffineAutoregressive(arn)
        transforms.append(t)
        if random_perm:
            transforms.append(Permute(torch.randperm(theta_dim)))
    flow = (ConditionalComposeTransformModule(transforms) if condition_dim > 0 else ComposeTransformModule(transforms))
    return flow, transforms, nets


def neural_spline_autoregressive(theta_dim, condition_dim, hidden_dim, num_layers, count_bins, order="quadratic",
                                 activation=nn.Tanh(), use_batchnorm=False, random_mask=True, random_perm=False,
                                 dropout_p=None):
    """naz/flows/transforms.py:165-198."""
    p = _unsupported(use_batchnorm, dropout_p)
    if order != "quadratic":
        raise NotImplementedError("naz_amd: only order='quadratic' (naz's default) is implemented")
    paramdim = [count_bins, count_bins, count_bins - 1]
    transforms, nets = [], []
    for _ in range(num_layers):
        perm = None if random_mask else torch.arange(theta_dim)
        arn = (ConditionalAutoRegressiveNN(theta_dim, condition_dim, _hidden(hidden_dim), param_dims=paramdim,
                                           nonlinearity=activation, permutation=perm, dropout_p=p)
               if condition_dim > 0 else
               AutoRegressiveNN(theta_dim, _hidden(hidden_dim), param_dims=paramdim, nonlinearity=activation,
                                permutation=perm, dropout_p=p))
        nets.append(arn)
        t = (ConditionalSplineAutoregressive(theta_dim, arn, count_bins=count_bins, order=order)
             if condition_dim > 0 else SplineAutoregressive(theta_dim, arn, count_bins=count_bins, order=order))
        transforms.append(t)
        if random_perm:
            transforms.append(Permute(torch.randperm(theta_dim)))
    flow = (ConditionalComposeTransformModule(transforms) if condition_dim > 0 else ComposeTransformModule(transforms))
    return flow, transforms, nets


def neural_spline_coupling(theta_dim, condition_dim, hidden_dim, num_layers, count_bins, split_dim,
                           order="quadratic", activation=nn.Tanh(), use_batchnorm=False, random_perm=False,
                           dropout_p=None, identity=False):
    """naz/flows/transforms.py:201-236 (intent): DenseNN hypernet input cat([ctx, x1]),
    param_dims [(D-s)K, (D-s)K, (D-s)(K-1)], SplineCoupling per layer.  dropout_p: the
    ConditionalDenseNNDropout intent (the reference's _forward indexes an undefined
    ``self.dropout_layers[i]``, transforms.py:82): dropout after every hidden activation."""
    p = _unsupported(use_batchnorm, dropout_p)
    if order != "quadratic":
        raise NotImplementedError("naz_amd: only order='quadratic' (naz's default) is implemented")
    Dt = theta_dim - split_dim
    param_dims = [Dt * count_bins, Dt * count_bins, Dt * (count_bins - 1)]
    transforms, nets = [], []
    for _ in range(num_layers):
        net = (ConditionalDenseNN(split_dim, condition_dim, _hidden(hidden_dim), param_dims=param_dims,
                                  nonlinearity=activation, dropout_p=p) if condition_dim > 0 else
               DenseNN(split_dim, _hidden(hidden_dim), param_dims=param_dims, nonlinearity=activation, dropout_p=p))
        nets.append(net)
        t = (ConditionalSplineCoupling(theta_dim, split_dim, net, count_bins=count_bins, order=order,
                                       identity=identity) if condition_dim > 0 else
             SplineCoupling(theta_dim, split_dim, net, count_bins=count_bins, order=order, identity=identity))
        transforms.append(t)
        if random_perm:
            transforms.append(Permute(torch.randperm(theta_dim)))
    flow = (ConditionalComposeTransformModule(transforms) if condition_dim > 0 else ComposeTransformModule(transforms))
    return flow, transforms, nets
