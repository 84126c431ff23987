"""TEST INFRASTRUCTURE ONLY — pure-torch CPU restatement of naz's flow hot path.

naz (``/root/reference/src/naz``) delegates every hot-path number to pyro-ppl
(unpinned in ``pip_requirements.txt:2``; 1.9.x at the 2025-08-08 snapshot) and
to torch's ``TransformedDistribution``.  This module restates those semantics
with plain torch tensor ops so the oracle runs on the CPU in float32 (the
reference's dtype, ``utils.py:7``) or float64.  It deliberately keeps the
reference's *eager, layer-by-layer* structure (cumsum → pad → searchsorted →
gather …) rather than anything fused, so that it is also an honest stand-in for
the reference's CPU path in ``bench.py``'s ``cpu_baseline`` leg.

Citations: ``naz:`` = ``/root/reference/src/naz/<file>:<line>`` (naz call site);
``[pyro]`` = the upstream pyro-ppl module the call site reaches (not vendored).

Nothing here imports the product package ``naz_amd``.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor

# Constants of [pyro] distributions/transforms/spline.py::_monotonic_rational_spline
MIN_BIN_WIDTH = 1e-3
MIN_BIN_HEIGHT = 1e-3
MIN_DERIVATIVE = 1e-3
SEARCH_EPS = 1e-6
DEFAULT_BOUND = 3.0
# [pyro] AffineAutoregressive defaults (naz: flows/transforms.py:159 constructs it with defaults)
LOG_SCALE_MIN_CLIP = -5.0
LOG_SCALE_MAX_CLIP = 3.0

ACTIVATIONS = {
    "tanh": torch.tanh,             # naz default: flows/transforms.py:133,165,201 (activation = nn.Tanh())
    "relu": torch.relu,             # pyro's own default nonlinearity
    "softplus": F.softplus,         # CNF vector field (naz: flows/continuous_transforms.py:47)
    "sigmoid": torch.sigmoid,
    "identity": lambda t: t,
}


# ---------------------------------------------------------------------------
# a1: the monotonic rational-quadratic spline
# ---------------------------------------------------------------------------
def _searchsorted(sorted_sequence: Tensor, values: Tensor) -> Tensor:
    """[pyro] spline.py::_searchsorted — count of knots <= value, minus one."""
    return torch.sum(values[..., None] >= sorted_sequence, dim=-1) - 1


def _select_bins(x: Tensor, idx: Tensor) -> Tensor:
    """[pyro] spline.py::_select_bins — gather with the index clamped to the bins."""
    idx = idx.clamp(min=0, max=x.size(-1) - 1)
    if idx.dim() > x.dim():
        x = x.reshape((1,) * (idx.dim() - x.dim()) + x.shape)
    x = x.expand(idx.shape[:-1] + (x.size(-1),))
    return x.gather(-1, idx).squeeze(-1)


def _calculate_knots(lengths: Tensor, lower: float, upper: float) -> Tuple[Tensor, Tensor]:
    """[pyro] spline.py::_calculate_knots — cumsum, left-pad 0, map [0,1]→[lower,upper],
    pin the end knots, and recompute the bin lengths from the knots."""
    knots = torch.cumsum(lengths, dim=-1)
    knots = F.pad(knots, pad=(1, 0), mode="constant", value=0.0)
    knots = (upper - lower) * knots + lower
    knots[..., 0] = lower
    knots[..., -1] = upper
    lengths = knots[..., 1:] - knots[..., :-1]
    return lengths, knots


def monotonic_rqs(inputs: Tensor, widths: Tensor, heights: Tensor, derivatives: Tensor,
                  inverse: bool = False, bound: float = DEFAULT_BOUND,
                  min_bin_width: float = MIN_BIN_WIDTH, min_bin_height: float = MIN_BIN_HEIGHT,
                  min_derivative: float = MIN_DERIVATIVE, eps: float = SEARCH_EPS) -> Tuple[Tensor, Tensor]:
    """[pyro] spline.py::_monotonic_rational_spline, ``lambdas=None`` (order="quadratic",
    the naz default: flows/transforms.py:165,201).

    inputs [..., Dt]; widths/heights [..., Dt, K] (already softmaxed); derivatives
    [..., Dt, K-1] (already softplus'ed).  Returns (outputs, logabsdet) both
    [..., Dt]; for ``inverse=True`` logabsdet is the log-det of the inverse map.
    Identity with zero log-det outside [-bound, bound].
    """
    num_bins = widths.shape[-1]
    left, right = -bound, bound
    bottom, top = -bound, bound
    inside = (inputs >= left) & (inputs <= right)
    outside = ~inside

    widths = min_bin_width + (1.0 - min_bin_width * num_bins) * widths
    heights = min_bin_height + (1.0 - min_bin_height * num_bins) * heights
    derivatives = min_derivative + derivatives

    widths, cumwidths = _calculate_knots(widths, left, right)
    heights, cumheights = _calculate_knots(heights, bottom, top)
    # edge slopes pinned to 1 - min_derivative, padded AFTER adding min_derivative
    derivatives = F.pad(derivatives, pad=(1, 1), mode="constant", value=1.0 - min_derivative)

    bin_idx = _searchsorted(cumheights + eps if inverse else cumwidths + eps, inputs).unsqueeze(-1)

    input_widths = _select_bins(widths, bin_idx)
    input_cumwidths = _select_bins(cumwidths, bin_idx)
    input_cumheights = _select_bins(cumheights, bin_idx)
    input_delta = _select_bins(heights / widths, bin_idx)
    input_derivatives = _select_bins(derivatives, bin_idx)
    input_derivatives_plus_one = _select_bins(derivatives[..., 1:], bin_idx)
    input_heights = _select_bins(heights, bin_idx)

    if inverse:
        a = (inputs - input_cumheights) * (input_derivatives + input_derivatives_plus_one - 2 * input_delta) \
            + input_heights * (input_delta - input_derivatives)
        b = input_heights * input_derivatives \
            - (inputs - input_cumheights) * (input_derivatives + input_derivatives_plus_one - 2 * input_delta)
        c = -input_delta * (inputs - input_cumheights)
        discriminant = b.pow(2) - 4 * a * c
        discriminant = discriminant.masked_fill(outside, 0)
        root = (2 * c) / (-b - torch.sqrt(discriminant))
        outputs = root * input_widths + input_cumwidths
        theta_one_minus_theta = root * (1 - root)
        denominator = input_delta + (input_derivatives + input_derivatives_plus_one - 2 * input_delta) \
            * theta_one_minus_theta
        derivative_numerator = input_delta.pow(2) * (
            input_derivatives_plus_one * root.pow(2) + 2 * input_delta * theta_one_minus_theta
            + input_derivatives * (1 - root).pow(2))
        logabsdet = -(torch.log(derivative_numerator) - 2 * torch.log(denominator))
    else:
        theta = (inputs - input_cumwidths) / input_widths
        theta_one_minus_theta = theta * (1 - theta)
        numerator = input_heights * (input_delta * theta.pow(2) + input_derivatives * theta_one_minus_theta)
        denominator = input_delta + (input_derivatives + input_derivatives_plus_one - 2 * input_delta) \
            * theta_one_minus_theta
        outputs = input_cumheights + numerator / denominator
        derivative_numerator = input_delta.pow(2) * (
            input_derivatives_plus_one * theta.pow(2) + 2 * input_delta * theta_one_minus_theta
            + input_derivatives * (1 - theta).pow(2))
        logabsdet = torch.log(derivative_numerator) - 2 * torch.log(denominator)

    outputs = torch.where(outside, inputs, outputs)
    logabsdet = torch.where(outside, torch.zeros_like(logabsdet), logabsdet)
    return outputs, logabsdet


# ---------------------------------------------------------------------------
# a2: conditioner output -> (w, h, d)
# ---------------------------------------------------------------------------
LAYOUT_DENSE = 0   # DenseNN hypernet: raw column i*K+k | Dt*K + i*K+k | 2*Dt*K + i*(K-1)+k
LAYOUT_ARN = 1     # AutoRegressiveNN: raw column p*Dt + i  (p in [0, 3K-1))


def split_raw_params(raw: Tensor, Dt: int, K: int, layout: int) -> Tuple[Tensor, Tensor, Tensor]:
    """Split a conditioner's flat output ``raw [..., Dt*(3K-1)]`` into the unnormalised
    (w [..,Dt,K], h [..,Dt,K], d [..,Dt,K-1]) exactly as [pyro] ConditionalSpline._params
    sees them: DenseNN output is reshaped, ARN output ``[.., 3K-1, Dt]`` is transposed."""
    if layout == LAYOUT_DENSE:
        w = raw[..., : Dt * K].reshape(raw.shape[:-1] + (Dt, K))
        h = raw[..., Dt * K: 2 * Dt * K].reshape(raw.shape[:-1] + (Dt, K))
        d = raw[..., 2 * Dt * K:].reshape(raw.shape[:-1] + (Dt, K - 1))
    else:
        r = raw.reshape(raw.shape[:-1] + (3 * K - 1, Dt))
        w = r[..., :K, :].transpose(-1, -2)
        h = r[..., K: 2 * K, :].transpose(-1, -2)
        d = r[..., 2 * K:, :].transpose(-1, -2)
    return w, h, d


def normalize_spline_params(w: Tensor, h: Tensor, d: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    """[pyro] ConditionalSpline._params / Spline._params: softmax, softmax, softplus."""
    return F.softmax(w, dim=-1), F.softmax(h, dim=-1), F.softplus(d)


def rqs_from_raw(x: Tensor, raw: Tensor, Dt: int, K: int, layout: int, inverse: bool,
                 bound: float = DEFAULT_BOUND) -> Tuple[Tensor, Tensor]:
    """a1+a2 composed: the standalone spline primitive the HIP ``naz_rqs_{fwd,inv}`` replaces.
    Returns (y, ld) with ld the log-det of the map actually applied."""
    w, h, d = normalize_spline_params(*split_raw_params(raw, Dt, K, layout))
    return monotonic_rqs(x, w, h, d, inverse=inverse, bound=bound)


# ---------------------------------------------------------------------------
# a6/a7: conditioner networks
# ---------------------------------------------------------------------------
def sample_mask_indices(input_dim: int, hidden_dim: int) -> Tensor:
    """[pyro] auto_reg_nn.py::sample_mask_indices(simple=True): round half-to-even of a
    float32 linspace (JAX restatement: naz: flows/bflow_jax_maf.py:48-50)."""
    indices = torch.linspace(1, input_dim, steps=hidden_dim, dtype=torch.float32)
    return torch.round(indices)


def create_mask(input_dim: int, context_dim: int, hidden_dims: Sequence[int], permutation: Tensor,
                output_dim_multiplier: int) -> Tuple[List[Tensor], Tensor]:
    """[pyro] auto_reg_nn.py::create_mask (JAX restatement: naz: flows/bflow_jax_maf.py:52-72).
    Context inputs get index 0; variable ``permutation[k]`` gets index k+1."""
    var_index = torch.empty(permutation.shape, dtype=torch.float32)
    var_index[permutation] = torch.arange(input_dim, dtype=torch.float32)
    input_indices = torch.cat((torch.zeros(context_dim), 1 + var_index))
    if context_dim > 0:
        hidden_indices = [sample_mask_indices(input_dim, h) - 1 for h in hidden_dims]
    else:
        hidden_indices = [sample_mask_indices(input_dim - 1, h) for h in hidden_dims]
    output_indices = (var_index + 1).repeat(output_dim_multiplier)
    mask_skip = (output_indices.unsqueeze(-1) > input_indices.unsqueeze(0)).float()
    masks = [(hidden_indices[0].unsqueeze(-1) >= input_indices.unsqueeze(0)).float()]
    for i in range(1, len(hidden_dims)):
        masks.append((hidden_indices[i].unsqueeze(-1) >= hidden_indices[i - 1].unsqueeze(0)).float())
    masks.append((output_indices.unsqueeze(-1) > hidden_indices[-1].unsqueeze(0)).float())
    return masks, mask_skip


class MLP:
    """[pyro] nn/dense_nn.py::ConditionalDenseNN._forward and nn/auto_reg_nn.py::
    ConditionalAutoRegressiveNN._forward (MaskedLinear = F.linear(x, mask*W, b)).
    Input is ``cat([context, x])`` — context FIRST (naz: transforms.py:142,180,223)."""

    def __init__(self, weights: List[Tensor], biases: List[Tensor], activation: str = "tanh",
                 masks: Optional[List[Tensor]] = None):
        self.weights = weights
        self.biases = biases
        self.masks = masks
        self.f = ACTIVATIONS[activation]

    def __call__(self, x: Tensor, context: Optional[Tensor] = None) -> Tensor:
        if context is not None:
            context = context.expand(x.shape[:-1] + (context.shape[-1],))
            h = torch.cat([context, x], dim=-1)
        else:
            h = x
        n = len(self.weights)
        for i in range(n):
            W = self.weights[i] if self.masks is None else self.masks[i].to(self.weights[i].dtype) * self.weights[i]
            h = F.linear(h, W, self.biases[i])
            if i < n - 1:
                h = self.f(h)
        return h


# ---------------------------------------------------------------------------
# Transforms (Pyro protocol, restated): every transform exposes
#   inverse(y, ctx) -> (x, ld_per_dim_of_forward_map)   and   forward(x, ctx) -> (y, ld)
# ---------------------------------------------------------------------------
class SplineCoupling:
    """a3: [pyro] distributions/transforms/spline_coupling.py::SplineCoupling with a
    (Conditional)DenseNN hypernet — naz's *intended* ``nsc`` (naz: transforms.py:113-129,
    201-236, broken as written).  The lower (unconditional, elementwise) spline is a
    persistent parameter set here (naz rebuilds it per ``condition()`` call, transforms.py:126-129).
    ``identity=True`` passes x1 through unchanged (pyro's ``identity`` flag)."""

    def __init__(self, D: int, split: int, K: int, nn: MLP, lower: Optional[Tuple[Tensor, Tensor, Tensor]],
                 bound: float = DEFAULT_BOUND):
        self.D, self.s, self.K, self.nn, self.lower, self.bound = D, split, K, nn, lower, bound

    def _upper_params(self, x1: Tensor, ctx: Optional[Tensor]):
        raw = self.nn(x1, ctx)
        return normalize_spline_params(*split_raw_params(raw, self.D - self.s, self.K, LAYOUT_DENSE))

    def _lower_params(self):
        uw, uh, ud = self.lower
        return normalize_spline_params(uw, uh, ud)

    def forward(self, x: Tensor, ctx: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
        x1, x2 = x[..., : self.s], x[..., self.s:]
        if self.lower is not None:
            y1, ldk = monotonic_rqs(x1, *self._lower_params(), inverse=False, bound=self.bound)
        else:
            y1 = x1
        y2, ld = monotonic_rqs(x2, *self._upper_params(x1, ctx), inverse=False, bound=self.bound)
        if self.lower is not None:
            ld = torch.cat([ld, ldk], dim=-1)
        return torch.cat([y1, y2], dim=-1), ld

    def inverse(self, y: Tensor, ctx: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
        y1, y2 = y[..., : self.s], y[..., self.s:]
        if self.lower is not None:
            x1, ldk = monotonic_rqs(y1, *self._lower_params(), inverse=True, bound=self.bound)
            ldk = -ldk
        else:
            x1 = y1
        x2, ld = monotonic_rqs(y2, *self._upper_params(x1, ctx), inverse=True, bound=self.bound)
        ld = -ld
        if self.lower is not None:
            ld = torch.cat([ld, ldk], dim=-1)
        return torch.cat([x1, x2], dim=-1), ld


class SplineAutoregressive:
    """a4: [pyro] spline_autoregressive.py::(Conditioned)SplineAutoregressive with a MADE
    conditioner (naz ``nsa``: transforms.py:165-198).  ``inverse`` is the D-pass loop."""

    def __init__(self, D: int, K: int, arn: MLP, bound: float = DEFAULT_BOUND):
        self.D, self.K, self.nn, self.bound = D, K, arn, bound

    def _params(self, x: Tensor, ctx: Optional[Tensor]):
        raw = self.nn(x, ctx)
        return normalize_spline_params(*split_raw_params(raw, self.D, self.K, LAYOUT_ARN))

    def forward(self, x, ctx=None):
        return monotonic_rqs(x, *self._params(x, ctx), inverse=False, bound=self.bound)

    def inverse(self, y, ctx=None):
        x = torch.zeros_like(y)
        ld = None
        for _ in range(self.D):
            x, ld = monotonic_rqs(y, *self._params(x, ctx), inverse=True, bound=self.bound)
        return x, -ld


def _clamp(t: Tensor, lo: float, hi: float) -> Tensor:
    """[pyro] distributions/transforms/utils.py::clamp_preserve_gradients, which
    AffineAutoregressive applies to log_scale: clamped value, identity gradient."""
    return t + (t.clamp(min=lo, max=hi) - t).detach()


def _clip(t: Tensor, lo: float, hi: float) -> Tensor:
    """jnp.clip as the reference's JAX MAF applies it to log_scale (bflow_jax_maf.py:177,188,192):
    clamped value, ZERO gradient outside [lo, hi] (torch.clamp's gradient)."""
    return t.clamp(min=lo, max=hi)


class AffineAutoregressive:
    """a5: [pyro] affine_autoregressive.py::AffineAutoregressive(stable=False) with clip
    (-5, 3) (naz ``maf``: transforms.py:133-160; JAX restatement bflow_jax_maf.py:169-194).
    ``clip_grad``: "preserve" = pyro's clamp_preserve_gradients (naz's torch flows), "zero" =
    jnp.clip's gradient (the JAX Bayesian MAF whose potential NUTS differentiates)."""

    def __init__(self, D: int, arn: MLP, permutation: Tensor, clip_grad: str = "preserve"):
        self.D, self.nn, self.permutation = D, arn, permutation
        if clip_grad not in ("preserve", "zero"):
            raise ValueError(f"clip_grad must be 'preserve' or 'zero', not {clip_grad!r}")
        self._cl = _clamp if clip_grad == "preserve" else _clip

    def _mean_logscale(self, x, ctx):
        out = self.nn(x, ctx).reshape(x.shape[:-1] + (2, self.D))
        return out[..., 0, :], out[..., 1, :]

    def forward(self, x, ctx=None):
        mean, log_scale = self._mean_logscale(x, ctx)
        log_scale = self._cl(log_scale, LOG_SCALE_MIN_CLIP, LOG_SCALE_MAX_CLIP)
        return torch.exp(log_scale) * x + mean, log_scale

    def inverse(self, y, ctx=None):
        xs = [torch.zeros(y.shape[:-1], dtype=y.dtype)] * self.D
        log_scale = None
        for idx in self.permutation.tolist():
            mean, log_scale = self._mean_logscale(torch.stack(xs, dim=-1), ctx)
            inverse_scale = torch.exp(-self._cl(log_scale[..., idx], LOG_SCALE_MIN_CLIP, LOG_SCALE_MAX_CLIP))
            xs[idx] = (y[..., idx] - mean[..., idx]) * inverse_scale
        return torch.stack(xs, dim=-1), self._cl(log_scale, LOG_SCALE_MIN_CLIP, LOG_SCALE_MAX_CLIP)


class Permute:
    """[pyro] T.Permute (naz: random_perm=True, transforms.py:155,194,232)."""

    def __init__(self, perm: Tensor):
        self.perm = perm
        self.inv_perm = torch.empty_like(perm)
        self.inv_perm[perm] = torch.arange(perm.numel())

    def forward(self, x, ctx=None):
        return x[..., self.perm], torch.zeros_like(x)

    def inverse(self, y, ctx=None):
        return y[..., self.inv_perm], torch.zeros_like(y)


# ---------------------------------------------------------------------------
# a11: continuous normalizing flow (FFJORD with Hutchinson's trace), pinned RK4 solver
# ---------------------------------------------------------------------------
class FCNN:
    """naz: flows/continuous_transforms.py:38-60 ``ConditionalFCNN``: Linear/act chain (Softplus
    default, no dropout when dropout_p is None), input ``cat([x, context])`` — x FIRST
    (``_conditioned_forward``, :54-56), output D."""

    def __init__(self, weights: List[Tensor], biases: List[Tensor], activation: str = "softplus"):
        self.weights, self.biases = weights, biases
        self.f = ACTIVATIONS[activation]

    def __call__(self, x: Tensor, context: Optional[Tensor] = None) -> Tensor:
        h = x if context is None else torch.cat([x, context.expand(x.shape[:-1] + (context.shape[-1],))], -1)
        n = len(self.weights)
        for i in range(n):
            h = F.linear(h, self.weights[i], self.biases[i])
            if i < n - 1:
                h = self.f(h)
        return h


def hutchinson_rhs(net: FCNN, x: Tensor, ctx: Optional[Tensor], eps: Tensor) -> Tuple[Tensor, Tensor]:
    """torchdyn ``CNF.forward`` with naz's ``hutch_trace`` (continuous_transforms.py:78,85-89):
    d[a, x]/dt = [-eps^T (df/dx) eps, f(x)], the VJP eps^T J taken by reverse-mode autograd
    exactly as the reference does; eps is fixed for one solve.

    Under grad mode with a trainable input or weight (the CNF training step), the VJP is taken
    with ``create_graph=True`` and nothing is detached, as torchdyn's hutch_trace must for the
    trace to carry a gradient: autograd through this RHS is the gradient oracle of the adjoint."""
    if torch.is_grad_enabled() and (x.requires_grad or any(w.requires_grad for w in net.weights + net.biases)
                                    or (ctx is not None and ctx.requires_grad)):
        x_in = x if x.requires_grad else x.detach().requires_grad_(True)
        f = net(x_in, ctx)
        vjp = torch.autograd.grad(f, x_in, eps, create_graph=True)[0]
        return f, -torch.einsum("bi,bi->b", vjp, eps)
    with torch.enable_grad():
        x_in = x.detach().requires_grad_(True)
        f = net(x_in, ctx)
        vjp = torch.autograd.grad(f, x_in, eps)[0]
    tr = torch.einsum("bi,bi->b", vjp, eps)
    return f.detach(), -tr.detach()


def rk4_augmented(net: FCNN, x: Tensor, ctx: Optional[Tensor], eps: Tensor, t0: float, t1: float,
                  steps: int) -> Tuple[Tensor, Tensor]:
    """Fixed-step classical RK4 on the augmented state [a, x], a(t0) = 0, in the form of naz's
    in-tree solver (neural_nets/__deprecated__/neural_odes/odeint.py:12-19 integrate,
    :46-52 RK4._step_fn): k_i = dt f(.), x += (k1 + 2 k2 + 2 k3 + k4) / 6.  SURVEY.md §8d pins
    config 5 to this solver with 8 steps (NFE 32); torchdyn's adaptive dopri5 is §8f rank 3."""
    times = torch.linspace(t0, t1, steps + 1, dtype=torch.float64)
    a = torch.zeros(x.shape[:-1], dtype=x.dtype)
    for i in range(steps):
        dt = float(times[i + 1] - times[i])
        f1, g1 = hutchinson_rhs(net, x, ctx, eps)
        k1x, k1a = dt * f1, dt * g1
        f2, g2 = hutchinson_rhs(net, x + 0.5 * k1x, ctx, eps)
        k2x, k2a = dt * f2, dt * g2
        f3, g3 = hutchinson_rhs(net, x + 0.5 * k2x, ctx, eps)
        k3x, k3a = dt * f3, dt * g3
        f4, g4 = hutchinson_rhs(net, x + k3x, ctx, eps)
        k4x, k4a = dt * f4, dt * g4
        x = x + (k1x + 2.0 * k2x + 2.0 * k3x + k4x) / 6.0
        a = a + (k1a + 2.0 * k2a + 2.0 * k3a + k4a) / 6.0
    return x, a


# Dormand-Prince 5(4) tableau: naz's in-tree Dopri5 (neural_nets/__deprecated__/neural_odes/
# odeint.py:136-160; c_x rows = a_ij, last row = b, c_err = b - b*)
DOPRI5_A = [[1 / 5], [3 / 40, 9 / 40], [44 / 45, -56 / 15, 32 / 9],
            [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
            [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656]]
DOPRI5_B = [35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84]
DOPRI5_E = [35 / 384 - 5179 / 57600, 0.0, 500 / 1113 - 7571 / 16695, 125 / 192 - 393 / 640,
            -2187 / 6784 + 92097 / 339200, 11 / 84 - 187 / 2100, -1 / 40]


def _rms(u: Tensor, ua: Tensor) -> float:
    """RMS over the augmented state's elements ([x] and [a] together)."""
    return float(torch.sqrt((torch.sum(u ** 2) + torch.sum(ua ** 2)) / (u.numel() + ua.numel())))


def dopri5_step(net: FCNN, y: Tensor, a: Tensor, ctx: Optional[Tensor], eps: Tensor, hh: float,
                atol: float, rtol: float, k0: Optional[Tuple[Tensor, Tensor]] = None):
    """One Dormand-Prince 5(4) step of the augmented field, naz's in-tree ``Dopri5._step_fn``
    (neural_nets/__deprecated__/neural_odes/odeint.py:96-112 with the tableau :136-160): stages
    k_i = f(y + hh sum_j a_ij k_j), the 5th-order update y5 = y + hh sum b_i k_i, the FSAL stage
    f(y5), the embedded error hh sum e_i k_i and its RMS norm over err / (atol + rtol max(|y|, |y5|)).
    Returns (y5, a5, k6 = f(y5) pair, error norm).  Pinned to the reference's own step by
    tests/golden/cnf_refode_*.npz (oracle/gen_refode_fixtures.py)."""
    f0, f0a = hutchinson_rhs(net, y, ctx, eps) if k0 is None else k0
    ks, kas = [f0], [f0a]
    for row in DOPRI5_A:
        ki, kia = hutchinson_rhs(net, y + hh * sum(c * k for c, k in zip(row, ks)), ctx, eps)
        ks.append(ki)
        kas.append(kia)
    y5 = y + hh * sum(c * k for c, k in zip(DOPRI5_B, ks))
    a5 = a + hh * sum(c * k for c, k in zip(DOPRI5_B, kas))
    k6, k6a = hutchinson_rhs(net, y5, ctx, eps)
    ks.append(k6)
    kas.append(k6a)
    err = hh * sum(c * k for c, k in zip(DOPRI5_E, ks))
    erra = hh * sum(c * k for c, k in zip(DOPRI5_E, kas))
    en = _rms(err / (atol + rtol * torch.maximum(y.abs(), y5.abs())),
              erra / (atol + rtol * torch.maximum(a.abs(), a5.abs())))
    return y5, a5, (k6, k6a), en


def dopri5_augmented(net: FCNN, x: Tensor, ctx: Optional[Tensor], eps: Tensor, t0: float, t1: float,
                     atol: float = 1e-4, rtol: float = 1e-4, group: int = 16, max_steps: int = 1000):
    """Adaptive Dormand-Prince 5(4) on the augmented state [x, a] (naz
    FFJORDTransform solver='dopri5', atol = rtol = 1e-4, continuous_transforms.py:73-81).

    torchdyn (absent, unpinned) is restated by the standard embedded-RK controller it shares
    with torchdiffeq: RMS error norm of err / (atol + rtol max(|y0|, |y1|)) over the state,
    accept when <= 1, h *= clamp(0.9 norm^(-1/5), 0.2 (1 on accept), 10); Hairer's initial-step
    heuristic (order 5); FSAL.  The last step is clipped to end exactly at t1 (no dense-output
    interpolation).  One step size per GROUP of consecutive rows — the kernel's 16-row wave —
    instead of torchdyn's single step size for the whole batch (a finer control; the same
    tolerance).  Returns x(t1), a(t1) and the number of RHS evaluations per group."""
    B = x.shape[0]
    xs, as_, nfes = [], [], []
    for g0 in range(0, B, group):
        sl = slice(g0, min(B, g0 + group))
        cg = None if ctx is None else (ctx[sl] if ctx.dim() == 2 and ctx.shape[0] == B else ctx)
        y = x[sl].clone()
        a = torch.zeros(y.shape[0], dtype=y.dtype)
        e = eps[sl]

        def f(v):
            return hutchinson_rhs(net, v, cg, e)
        rms = _rms
        direction = 1.0 if t1 > t0 else -1.0
        k0, k0a = f(y)
        sc, sca = atol + rtol * y.abs(), atol + rtol * a.abs()
        d0, d1 = rms(y / sc, a / sca), rms(k0 / sc, k0a / sca)
        h0 = 1e-6 if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
        f1, f1a = f(y + direction * h0 * k0)
        d2 = rms((f1 - k0) / sc, (f1a - k0a) / sca) / h0
        h1 = max(1e-6, h0 * 1e-3) if max(d1, d2) <= 1e-15 else (0.01 / max(d1, d2)) ** (1.0 / 6.0)
        h = min(100 * h0, h1)
        nfe, t, steps = 2, t0, 0
        while steps < max_steps and t != t1:
            rem = abs(t1 - t)
            last = h >= rem
            hh = direction * (rem if last else h)
            y5, a5, (k6, k6a), en = dopri5_step(net, y, a, cg, e, hh, atol, rtol, k0=(k0, k0a))
            nfe += 6
            if en <= 1.0:
                y, a, k0, k0a = y5, a5, k6, k6a
                t = t1 if last else t + hh
            factor = 10.0 if en == 0 else min(10.0, max(0.9 / en ** 0.2, 1.0 if en <= 1.0 else 0.2))
            h = abs(hh) * factor
            steps += 1
        xs.append(y)
        as_.append(a)
        nfes.append(nfe)
    return torch.cat(xs), torch.cat(as_), nfes


def dopri5_global(net: FCNN, x: Tensor, ctx: Optional[Tensor], eps: Tensor, t0: float, t1: float,
                  atol: float = 1e-4, rtol: float = 1e-4, max_steps: int = 1000):
    """torchdyn's controller as naz configures it (FFJORDTransform solver='dopri5', atol = rtol =
    1e-4, continuous_transforms.py:73-81; torchdyn.numerics odeint with an adaptive solver): ONE
    step size for the whole batch.  The error ratio is torchdyn's ``hairer_norm`` — the RMS over
    every element of the augmented state tensor [B, D + 1] — of err / (atol + rtol max(|y0|, |y1|)),
    with the same accept rule, step factor (0.9 r^(-1/5) clamped to [0.2 (1 on accept), 10]) and
    Hairer initial step as ``dopri5_augmented``, which this is with one group spanning the batch.
    torchdyn is absent here (parity unpinned); the last step is clipped to t1 as the kernel does
    (torchdyn instead interpolates its dense output at t1 — the same solution within tolerance).
    Returns x(t1), a(t1) and the batch's number of RHS evaluations."""
    y, a, nfe = dopri5_augmented(net, x, ctx, eps, t0, t1, atol, rtol, group=x.shape[0], max_steps=max_steps)
    return y, a, nfe[0]


class FFJORD:
    """a11: naz ``FFJORDTransform`` (continuous_transforms.py:70-106).  ``inverse`` = its
    ``_inverse`` (integrate t 0 -> 1, the log_prob direction), ``forward`` = ``_call``
    (t 1 -> 0, sampling).  Both return the cached log-det a(t_end) = int -eps^T J eps dt as a
    [B, 1] 'per-dim' ld so Flow.log_prob's ``lp -= ld.sum(-1)`` applies it as torch's
    TransformedDistribution does with ``log_abs_det_jacobian``.  ``eps`` [B, D] must be set
    before each call (torchdyn draws it per solve)."""

    def __init__(self, D: int, net: FCNN, steps: int = 8):
        self.D, self.nn, self.steps = D, net, steps
        self.eps: Optional[Tensor] = None

    def inverse(self, y, ctx=None):
        x, a = rk4_augmented(self.nn, y, ctx, self.eps.to(y.dtype), 0.0, 1.0, self.steps)
        return x, a[..., None]

    def forward(self, z, ctx=None):
        x, a = rk4_augmented(self.nn, z, ctx, self.eps.to(z.dtype), 1.0, 0.0, self.steps)
        return x, a[..., None]


# ---------------------------------------------------------------------------
# a8/a9: flow composition, bounding, density and sampling
# ---------------------------------------------------------------------------
def bounding_transform(x: Tensor, low: Tensor, high: Tensor) -> Tuple[Tensor, Tensor]:
    """naz: flows/transforms.py:20-23 (verbatim semantics)."""
    y = (x - low.expand(x.shape)) / ((high - low).expand(x.shape))
    log_jac = -torch.sum(torch.log(y) + torch.log1p(-y), dim=-1) - torch.sum(torch.log(high - low))
    return torch.logit(y), log_jac


def inverse_bounding_transform(y: Tensor, low: Tensor, high: Tensor) -> Tensor:
    """naz: flows/transforms.py:25-27."""
    x = torch.sigmoid(y)
    return x * ((high - low).expand(y.shape)) + low.expand(y.shape)


def base_log_prob(z: Tensor) -> Tensor:
    """Independent(Normal(0,1), 1).log_prob (naz: flow.py:37; torch Normal.log_prob)."""
    return (-(z ** 2) / 2 - math.log(math.sqrt(2 * math.pi))).sum(-1)


class Flow:
    """naz: flows/flow.py:26-129 restated over torch TransformedDistribution semantics:
    ``log_prob`` walks the layers in reverse (lp -= ld.sum(-1)), then adds the base."""

    def __init__(self, layers: list, D: int, bounds: Optional[Dict[str, Tensor]] = None):
        self.layers, self.D, self.bounds = layers, D, bounds

    def log_prob(self, x: Tensor, ctx: Optional[Tensor] = None) -> Tensor:
        if self.bounds is None:
            y, log_jac = x, 0.0
        else:
            y, log_jac = bounding_transform(x, self.bounds["low"], self.bounds["high"])
        lp = 0.0
        for layer in reversed(self.layers):
            y, ld = layer.inverse(y, ctx)
            lp = lp - ld.sum(-1)
        return lp + base_log_prob(y) + log_jac

    def sample_from_base(self, z: Tensor, ctx: Optional[Tensor] = None) -> Tensor:
        y = z
        for layer in self.layers:
            y, _ = layer.forward(y, ctx)
        if self.bounds is not None:
            y = inverse_bounding_transform(y, self.bounds["low"], self.bounds["high"])
        return y

    def forward_with_logdet(self, z: Tensor, ctx: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
        y, tot = z, torch.zeros(z.shape[:-1], dtype=z.dtype)
        for layer in self.layers:
            y, ld = layer.forward(y, ctx)
            tot = tot + ld.sum(-1)
        return y, tot


# ---------------------------------------------------------------------------
# Building an oracle flow from a spec + a canonical state dict
# ---------------------------------------------------------------------------
def _hidden_list(hidden) -> List[int]:
    return list(hidden) if isinstance(hidden, (list, tuple)) else [int(hidden)]


def build_flow(spec: dict, state: Dict[str, Tensor], dtype=torch.float64) -> Flow:
    """Build an oracle flow from ``spec`` (flow_type, D, C, hidden, L, K, split, activation,
    bounds, clip_grad for maf) and a canonical state dict (numpy or torch values):

      layers.{l}.nn.layers.{i}.weight/bias                      conditioner
      layers.{l}.nn.permutation                                 ARN variable order (maf/nsa)
      layers.{l}.lower_spline.unnormalized_{widths,heights,derivatives}   coupling lower spline
      layers.{l}.perm                                           optional Permute after layer l
    """
    t = {k: torch.as_tensor(v) for k, v in state.items()}
    ft, D, C = spec["flow_type"], spec["D"], spec["C"]
    hidden = _hidden_list(spec["hidden"])
    K = spec.get("K", 8)
    act = spec.get("activation", "tanh")
    bound = spec.get("bound", DEFAULT_BOUND)
    layers = []
    for l in range(spec["L"]):
        p = f"layers.{l}."
        n_lin = len(hidden) + 1
        Ws = [t[p + f"nn.layers.{i}.weight"].to(dtype) for i in range(n_lin)]
        bs = [t[p + f"nn.layers.{i}.bias"].to(dtype) for i in range(n_lin)]
        if ft == "nsc":
            s = spec["split"]
            lower = None
            if (p + "lower_spline.unnormalized_widths") in t:
                lower = tuple(t[p + "lower_spline.unnormalized_" + n].to(dtype)
                              for n in ("widths", "heights", "derivatives"))
            layers.append(SplineCoupling(D, s, K, MLP(Ws, bs, act), lower, bound))
        elif ft == "cnf":
            layers.append(FFJORD(D, FCNN(Ws, bs, spec.get("activation", "softplus")), spec.get("steps", 8)))
        elif ft in ("nsa", "maf"):
            perm = t[p + "nn.permutation"].long()
            mult = (3 * K - 1) if ft == "nsa" else 2
            masks, _ = create_mask(D, C, hidden, perm, mult)
            arn = MLP(Ws, bs, act, masks=[m.to(dtype) for m in masks])
            if ft == "nsa":
                layers.append(SplineAutoregressive(D, K, arn, bound))
            else:
                layers.append(AffineAutoregressive(D, arn, perm, spec.get("clip_grad", "preserve")))
        else:
            raise ValueError(f"oracle: unsupported flow_type {ft!r}")
        if (p + "perm") in t:
            layers.append(Permute(t[p + "perm"].long()))
    bounds = None
    if spec.get("bounds") is not None:
        bounds = {k: torch.as_tensor(v).to(dtype) for k, v in spec["bounds"].items()}
    return Flow(layers, D, bounds)


def random_state(spec: dict, seed: int = 1234, last_layer_scale: float = 3.0) -> Dict[str, Tensor]:
    """Deterministic synthetic weights with nn.Linear's default init (kaiming-uniform,
    bound 1/sqrt(fan_in) for weight and bias), last conditioner layer ×``last_layer_scale``
    so the bins are non-uniform (BASELINE.md §Synthetic inputs).  Lower-spline params ~ randn
    ([pyro] Spline init); ARN permutations ~ randperm ([pyro] ConditionalAutoRegressiveNN)."""
    g = torch.Generator().manual_seed(seed)
    ft, D, C = spec["flow_type"], spec["D"], spec["C"]
    hidden = _hidden_list(spec["hidden"])
    K = spec.get("K", 8)
    out = {}
    for l in range(spec["L"]):
        p = f"layers.{l}."
        if ft == "nsc":
            s = spec["split"]
            dims = [s + C] + hidden + [(D - s) * (3 * K - 1)]
        elif ft == "nsa":
            dims = [D + C] + hidden + [D * (3 * K - 1)]
        elif ft == "cnf":
            dims = [D + C] + hidden + [D]  # ConditionalFCNN, continuous_transforms.py:41-50
        else:
            dims = [D + C] + hidden + [2 * D]
        n_lin = len(dims) - 1
        for i in range(n_lin):
            fan_in = dims[i]
            bnd = 1.0 / math.sqrt(fan_in)
            W = (torch.rand(dims[i + 1], dims[i], generator=g) * 2 - 1) * bnd
            b = (torch.rand(dims[i + 1], generator=g) * 2 - 1) * bnd
            if i == n_lin - 1:
                W, b = W * last_layer_scale, b * last_layer_scale
            out[p + f"nn.layers.{i}.weight"] = W
            out[p + f"nn.layers.{i}.bias"] = b
        if ft == "nsc" and spec.get("lower", True):
            s = spec["split"]
            out[p + "lower_spline.unnormalized_widths"] = torch.randn(s, K, generator=g)
            out[p + "lower_spline.unnormalized_heights"] = torch.randn(s, K, generator=g)
            out[p + "lower_spline.unnormalized_derivatives"] = torch.randn(s, K - 1, generator=g)
        if ft in ("nsa", "maf"):
            out[p + "nn.permutation"] = torch.randperm(D, generator=g)
    return out


def gaussian_mixture(n: int, D: int, seed: int = 0, n_comp: int = 8):
    """BASELINE.md §Synthetic inputs: 8-component mixture, means ~ N(0, 2^2 I),
    per-dim sigma ~ U(0.3, 1.0), equal weights, numpy default_rng(seed)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    means = rng.normal(0.0, 2.0, size=(n_comp, D))
    sig = rng.uniform(0.3, 1.0, size=(n_comp, D))
    comp = rng.integers(0, n_comp, size=n)
    x = means[comp] + sig[comp] * rng.standard_normal(size=(n, D))
    return x.astype(np.float32)


def context_normal(n: int, C: int, seed: int = 1):
    import numpy as np
    return np.random.default_rng(seed).standard_normal(size=(n, C)).astype(np.float32)


def two_moons(n: int, noise: float = 0.1, seed: int = 0):
    """Config 1 data: outer (cos t, sin t), inner (1-cos t, 0.5-sin t)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    n_out = n // 2
    t_out = rng.uniform(0, math.pi, n_out)
    t_in = rng.uniform(0, math.pi, n - n_out)
    outer = np.stack([np.cos(t_out), np.sin(t_out)], 1)
    inner = np.stack([1 - np.cos(t_in), 0.5 - np.sin(t_in)], 1)
    x = np.concatenate([outer, inner], 0) + noise * rng.standard_normal((n, 2))
    return x.astype(np.float32)
