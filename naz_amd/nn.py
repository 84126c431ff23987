"""Conditioner networks with pyro's module surface, executed by the HIP kernels.

Mirrors the pyro-ppl 1.9 classes naz instantiates (naz/flows/transforms.py:142,180,223):
``ConditionalDenseNN``/``DenseNN`` and ``ConditionalAutoRegressiveNN``/``AutoRegressiveNN``
with ``layers.{i}.weight|bias`` parameter names, ``masks``, ``mask_skip``, ``permutation``
and the pyro output shapes (so ``torch_to_jax`` in naz/flows/bflow_jax_maf.py:26-46 and
``get_params``/``set_params`` in naz/trainers/train_flows.py:20-71 work unchanged).
Every forward runs ``naz_linear_act`` (fused concat + mask + bias + activation).
"""
from __future__ import annotations

import os

from typing import List, Optional, Sequence

import torch
from torch import nn

from . import autograd as ag
from . import ops


def activation_name(f: nn.Module) -> str:
    """Map a torch activation module to the kernel's activation code."""
    if isinstance(f, nn.Tanh):
        return "tanh"
    if isinstance(f, nn.ReLU):
        return "relu"
    if isinstance(f, nn.Sigmoid):
        return "sigmoid"
    if isinstance(f, nn.Softplus) and f.beta == 1 and f.threshold == 20:
        return "softplus"
    if isinstance(f, nn.Identity):
        return "identity"
    raise NotImplementedError(f"naz_amd: activation {f!r} has no HIP kernel (tanh, relu, sigmoid, softplus)")


# ----------------------------------------------------------------------------- MADE masks
def sample_mask_indices(input_dim: int, hidden_dim: int) -> torch.Tensor:
    """[pyro] auto_reg_nn.sample_mask_indices(simple=True): round-half-to-even of a float32 linspace."""
    return torch.round(torch.linspace(1, input_dim, steps=hidden_dim, dtype=torch.float32))


def create_mask(input_dim: int, context_dim: int, hidden_dims: Sequence[int], permutation: torch.Tensor,
                output_dim_multiplier: int):
    """[pyro] auto_reg_nn.create_mask: context inputs get index 0, variable perm[k] gets k+1."""
    permutation = permutation.cpu()
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


# Weight-derived caches (masked weights, degree schedules, packed kernel images) are keyed on
# (data_ptr, _version) of the tensors they come from plus this epoch.  An in-place write through
# ``param.data`` does not bump ``_version``: call ``invalidate_caches()`` after one (io.load_state
# and trainers.set_params do), or update weights with in-place ops under torch.no_grad().
_CACHE_EPOCH = [0]


def invalidate_caches() -> None:
    """Drop every weight-derived cache (see _CACHE_EPOCH)."""
    _CACHE_EPOCH[0] += 1


def cache_epoch() -> int:
    return _CACHE_EPOCH[0]


class MaskedLinear(nn.Linear):
    """[pyro] nn.auto_reg_nn.MaskedLinear: F.linear(x, mask * W, b); mask is a buffer."""

    def __init__(self, in_features: int, out_features: int, mask: torch.Tensor, bias: bool = True):
        super().__init__(in_features, out_features, bias)
        self.register_buffer("mask", mask.data.clone())

    def forward(self, x):  # pragma: no cover - kept for API completeness; the nets call the fused kernel
        return ops.linear_act(x, self.weight, self.bias, "identity", mask=self.mask)

    def masked_weight(self) -> torch.Tensor:
        """W ⊙ mask, the weight MaskedLinear applies.  Formed once (a [out, in] tensor) instead of
        per element inside every GEMM tile; under autograd it is a differentiable torch product,
        so dW = mask ⊙ dWm exactly as pyro's F.linear(x, mask * W, b).  Cached across the D
        passes of an autoregressive inverse while the weight is unchanged (version counter)."""
        if torch.is_grad_enabled() and self.weight.requires_grad:
            return self.weight * self.mask
        key = (self.weight.data_ptr(), self.weight._version, self.mask.data_ptr(), self.mask._version, cache_epoch())
        if getattr(self, "_wm_key", None) != key:
            self._wm = (self.weight * self.mask).detach()
            self._wm_key = key
        return self._wm


def _slices(param_dims: Sequence[int]):
    ends = torch.cumsum(torch.tensor(param_dims), dim=0)
    starts = torch.cat((torch.zeros(1).type_as(ends), ends[:-1]))
    return [slice(int(s), int(e)) for s, e in zip(starts, ends)]


# conditioner chains under autograd run as one ChainFn node (act' fused into the dX GEMMs);
# NAZ_CHAIN_NODE=0 selects the LinearActFn-per-layer walk (A/B, tests)
_CHAIN_NODE = os.environ.get("NAZ_CHAIN_NODE", "1") != "0"
# run_grad's block gathers: every masked / padding entry gets its own zero slot, so a gather's
# indices are unique and its backward is a plain scatter (NAZ_GATHER_SORT=1: torch's indexing
# backward, which sorts the indices to accumulate the duplicates of a shared zero slot)
_GATHER_UNIQUE = os.environ.get("NAZ_GATHER_SORT", "0") != "1"


class _GatherBlocks(torch.autograd.Function):
    """(F[idx_0], F[idx_1], ...) for index sets without duplicates (within and across sets):
    backward scatters every block's gradient into ONE zero buffer (no per-block full-size
    gradients for autograd to sum, no accumulation)."""

    @staticmethod
    def forward(ctx, F, *idxs):
        ctx.save_for_backward(*idxs)
        ctx.n = F.numel()
        return tuple(F[i] for i in idxs)

    @staticmethod
    def backward(ctx, *grads):
        idxs = ctx.saved_tensors
        g0 = next(g for g in grads if g is not None)
        gF = g0.new_zeros(ctx.n)
        for i, g in zip(idxs, grads):
            if g is not None:
                gF[i] = g
        return (gF,) + (None,) * len(idxs)


def _run_chain(layers, f_name: str, x: torch.Tensor, context: Optional[torch.Tensor], masked: bool,
               drop=None) -> torch.Tensor:
    """The conditioner pass; recorded for autograd (HIP backward kernels) when grad mode is on
    and a weight, the input or the context requires grad.  ``drop`` = (p, seeds): MC dropout
    after every hidden activation (naz_dropout, one seed per hidden layer)."""
    n = len(layers)
    grad = ag.params_require_grad(layers) or ag.tensor_requires_grad(x, context)
    if grad and n >= 2 and x is not None and (_CHAIN_NODE or drop is not None):
        # one autograd node, act' fused into dX (and the dropout mask re-applied to it)
        ws = [layer.masked_weight() if masked else layer.weight for layer in layers]
        return ag.chain(x, ws, [layer.bias for layer in layers], f_name, context=context, drop=drop)
    if grad and drop is not None:
        raise NotImplementedError("naz_amd: dropout under autograd needs a conditioner with hidden layers and an input")
    lin = ag.linear_act if grad else ops.linear_act
    h = None
    for i, layer in enumerate(layers):
        act = f_name if i < n - 1 else "identity"
        w = layer.masked_weight() if masked else layer.weight
        if i == 0:
            h = lin(x, w, layer.bias, act, context=context)
        else:
            h = lin(h, w, layer.bias, act)
        if drop is not None and i < n - 1:
            h = ops.dropout(h, drop[0], drop[1][i], out=h)
    return h


class _DropoutMixin:
    """naz's MC-dropout conditioners (ConditionalAutoRegressiveNNDropout /
    ConditionalDenseNNDropout, naz/flows/transforms.py:29-95): nn.Dropout(dropout_p) after every
    hidden activation, active in train mode only (torch semantics).  Each conditioner pass draws
    fresh masks: one 64-bit seed per hidden layer from torch's CPU generator (so
    torch.manual_seed makes a run reproducible); the kernel hashes (seed, row, column)."""

    dropout_p = 0.0

    def dropout_active(self) -> bool:
        return bool(self.dropout_p) and self.training

    def _drop_args(self):
        if not self.dropout_active():
            return None
        n_hidden = len(self.layers) - 1
        seeds = torch.randint(0, 2 ** 62, (max(n_hidden, 1),), dtype=torch.int64).tolist()
        return float(self.dropout_p), seeds


class ConditionalDenseNN(_DropoutMixin, nn.Module):
    """[pyro] nn/dense_nn.py::ConditionalDenseNN — input cat([context, x])."""

    def __init__(self, input_dim: int, context_dim: int, hidden_dims: Sequence[int],
                 param_dims: Sequence[int] = (1, 1), nonlinearity: nn.Module = nn.ReLU(), dropout_p: float = 0.0):
        super().__init__()
        self.dropout_p = float(dropout_p or 0.0)
        self.input_dim, self.context_dim = input_dim, context_dim
        self.hidden_dims = list(hidden_dims)
        self.param_dims = list(param_dims)
        self.count_params = len(self.param_dims)
        self.output_multiplier = sum(self.param_dims)
        self.param_slices = _slices(self.param_dims)
        dims = [input_dim + context_dim] + self.hidden_dims + [self.output_multiplier]
        self.layers = nn.ModuleList([nn.Linear(dims[i], dims[i + 1]) for i in range(len(dims) - 1)])
        self.f = nonlinearity
        self.act = activation_name(nonlinearity)

    def raw(self, x: torch.Tensor, context: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Flat conditioner output [B, sum(param_dims)] (what the spline kernels consume)."""
        return _run_chain(self.layers, self.act, x, context, masked=False, drop=self._drop_args())

    def _shape(self, h, lead):
        if self.output_multiplier == 1:
            return h
        h = h.reshape(list(lead) + [self.output_multiplier])
        if self.count_params == 1:
            return h
        return tuple(h[..., s] for s in self.param_slices)

    def forward(self, x, context=None):
        return self._shape(self.raw(x, context), x.shape[:-1])


class DenseNN(ConditionalDenseNN):
    """[pyro] nn/dense_nn.py::DenseNN."""

    def __init__(self, input_dim, hidden_dims, param_dims=(1, 1), nonlinearity=nn.ReLU(), dropout_p=0.0):
        super().__init__(input_dim, 0, hidden_dims, param_dims, nonlinearity, dropout_p)

    def forward(self, x):
        return self._shape(self.raw(x, None), x.shape[:-1])


class ConditionalAutoRegressiveNN(_DropoutMixin, nn.Module):
    """[pyro] nn/auto_reg_nn.py::ConditionalAutoRegressiveNN (MADE, Germain et al. 2015)."""

    def __init__(self, input_dim: int, context_dim: int, hidden_dims: Sequence[int],
                 param_dims: Sequence[int] = (1, 1), permutation: Optional[torch.Tensor] = None,
                 skip_connections: bool = False, nonlinearity: nn.Module = nn.ReLU(), dropout_p: float = 0.0):
        super().__init__()
        self.dropout_p = float(dropout_p or 0.0)
        if skip_connections:
            raise NotImplementedError("naz_amd: MADE skip connections are not on naz's path (transforms.py:142,180)")
        self.input_dim, self.context_dim = input_dim, context_dim
        self.hidden_dims = list(hidden_dims)
        self.param_dims = list(param_dims)
        self.count_params = len(self.param_dims)
        self.output_multiplier = sum(self.param_dims)
        self.all_ones = all(p == 1 for p in self.param_dims)
        self.param_slices = _slices(self.param_dims)
        for h in self.hidden_dims:
            if h < input_dim:
                raise ValueError("Hidden dimension must not be less than input dimension.")
        if permutation is None:
            P = torch.randperm(input_dim, device="cpu")
        else:
            P = permutation.type(dtype=torch.int64).cpu()
        self.register_buffer("permutation", P)
        self.masks, self.mask_skip = create_mask(input_dim, context_dim, self.hidden_dims, P,
                                                 self.output_multiplier)
        dims = [input_dim + context_dim] + self.hidden_dims + [input_dim * self.output_multiplier]
        self.layers = nn.ModuleList([MaskedLinear(dims[i], dims[i + 1], self.masks[i])
                                     for i in range(len(dims) - 1)])
        self.skip_layer = None
        self.f = nonlinearity
        self.act = activation_name(nonlinearity)

    # inverse passes run degree-scheduled (ARInversePlan); False = pyro's D full passes
    degree_schedule = True

    def inverse_plan(self) -> Optional["ARInversePlan"]:
        """The cached degree-scheduled inverse (None when disabled, or while MC dropout is active:
        pyro's D-pass inverse then draws fresh dropout masks on every pass, which the schedule's
        compute-each-unit-once cannot reproduce)."""
        if not self.degree_schedule or self.dropout_active():
            return None
        plan = self.__dict__.get("_inverse_plan")
        if plan is None:
            plan = ARInversePlan(self)
            self.__dict__["_inverse_plan"] = plan
        return plan

    def get_permutation(self):
        return self.permutation

    def set_permutation(self, permutation: torch.Tensor) -> None:
        """Replace the variable order and rebuild every MADE mask (e.g. when importing weights)."""
        P = torch.as_tensor(permutation).to(torch.int64).cpu()
        self.masks, self.mask_skip = create_mask(self.input_dim, self.context_dim, self.hidden_dims, P,
                                                 self.output_multiplier)
        dev = self.layers[0].weight.device
        self.permutation = P.to(self.permutation.device)
        for layer, m in zip(self.layers, self.masks):
            layer.mask = m.to(dev)

    def raw(self, x: torch.Tensor, context: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Flat MADE output [B, mult*D], column p*D + i (pyro's reshape to [mult, D])."""
        return _run_chain(self.layers, self.act, x, context, masked=True, drop=self._drop_args())

    def _shape(self, h, lead):
        if self.output_multiplier == 1:
            return h
        h = h.reshape(list(lead) + [self.output_multiplier, self.input_dim])
        if self.count_params == 1:
            return h
        if self.all_ones:
            return torch.unbind(h, dim=-2)
        return tuple(h[..., s, :] for s in self.param_slices)

    def forward(self, x, context=None):
        return self._shape(self.raw(x, context), x.shape[:-1])


def degree_schedule(perm: torch.Tensor, masks, weights, biases, D: int, C: int, mult: int):
    """The degree schedule of ``ARInversePlan`` (see there) from float64 CPU tensors: per layer
    mask, weight, bias (pyro's MaskedLinear order).  Returns (widths, hidden, outs):
    hidden[g] = [(layer, a, b, n, w_block [b-a, n], bias_block [b-a])] run in pass g + 1,
    outs[k-1] = (dim i, n, w_rows [mult, max(n, 1)], bias_rows [mult]) of pass k.  Every block
    entry is one masked weight (or 0), so the schedule is linear in the weights: run on
    index-valued weights it yields the gather map of a per-draw pack (flows/bflow_maf.py)."""
    if len(weights) < 2:
        raise ValueError("MADE conditioner without hidden layers")
    order = torch.empty(D, dtype=torch.float64)
    order[perm] = torch.arange(1, D + 1, dtype=torch.float64)  # var perm[j] has order j + 1
    prev_deg = torch.cat((torch.zeros(C, dtype=torch.float64), order))
    prev_cols = None  # previous layer: padded column of each unit (None = natural [ctx | x])
    prev_ends = None  # previous layer: padded column end of degree groups <= m
    hidden = [[] for _ in range(D)]  # hidden[m] = blocks of degree m (run in pass m + 1)
    widths = []
    for li in range(len(weights) - 1):
        m = masks[li]
        deg = (m * prev_deg[None, :]).amax(dim=1)  # max order reached (0: context/bias only)
        w = weights[li] * m
        bias = biases[li]
        cols = torch.empty(w.shape[0], dtype=torch.int64)
        ends, off = [], 0
        for g in range(D):
            units = torch.nonzero(deg == g).flatten()
            a = off
            cols[units] = torch.arange(a, a + units.numel())
            off = a + (units.numel() + 3) // 4 * 4
            ends.append(off)
            if units.numel() == 0:
                continue
            if prev_cols is None:
                n = C + D
                wb = torch.zeros(off - a, n, dtype=torch.float64)
                wb[:units.numel()] = w[units]
            else:
                n = prev_ends[g]
                wb = torch.zeros(off - a, prev_ends[-1], dtype=torch.float64)
                wb[:units.numel(), prev_cols] = w[units]  # inputs scattered to padded columns
                wb = wb[:, :n]
            bb = torch.zeros(off - a, dtype=torch.float64)
            bb[:units.numel()] = bias[units]
            hidden[g].append((li, a, off, n, wb, bb))
        if deg.max() >= D:
            raise RuntimeError("MADE masks: a hidden unit sees a variable of order D")
        widths.append(off)
        prev_deg, prev_cols, prev_ends = deg, cols, ends
    # output rows of each dim (flat column p*D + i), from last-layer groups < order(i)
    m = masks[-1]
    w = weights[-1] * m
    bias = biases[-1]
    outs = []
    for k in range(1, D + 1):
        i = int(perm[k - 1])
        rows = torch.tensor([p * D + i for p in range(mult)])
        if ((m[rows] * prev_deg[None, :]).amax() if m.shape[1] else 0) >= k:
            raise RuntimeError("MADE masks are not autoregressive in the permutation's order")
        n = prev_ends[k - 1]
        full = torch.zeros(mult, prev_ends[-1], dtype=torch.float64)
        full[:, prev_cols] = w[rows]
        outs.append((i, n, full[:, :max(n, 1)], bias[rows]))
    return widths, hidden, outs


class _InverseBlock:
    """One GEMM of the degree-scheduled inverse: columns [a, b) of a layer's (padded, degree-sorted)
    activation from input columns [0, n) of the previous one (layer 0: the full [ctx | x])."""

    __slots__ = ("a", "b", "n", "w", "bias")

    def __init__(self, a, b, n, w, bias):
        self.a, self.b, self.n, self.w, self.bias = a, b, n, w, bias


class ARInversePlan:
    """Degree-scheduled D-pass inverse of a MADE conditioner (pyro's AffineAutoregressive /
    SplineAutoregressive ``_inverse``, naz/flows/transforms.py:133-198).

    pyro runs the WHOLE network D times; pass k makes the dim of order k final.  A hidden unit's
    value depends only on the inputs its masks reach, so a unit whose inputs all have order ≤ m
    ("degree" m, read off the actual masks) has its final value from pass m + 1 on and never
    changes afterwards.  Here every unit is computed exactly once, in pass (degree + 1):
      * each layer's units are sorted by degree into groups, each group padded to a multiple of
        4 columns (dummy units: zero weights and bias, zero weight in the next layer) so every
        group is a 16-byte-aligned column slice of the activation buffer;
      * pass k runs, per layer, the GEMM block [group k−1] × [prev-layer groups ≤ k−1] (masked
        weights; the block is the non-zero part of that product), then only the output rows of
        the dim of order k from last-layer groups ≤ k−1, then the elementwise map on that dim.
    Same values as pyro's loop (the skipped products are exact zeros of the masks); the
    conditioner work drops from D full networks to about one (triangular) network."""

    def __init__(self, arn: "ConditionalAutoRegressiveNN"):
        self.arn = arn
        self._key = None

    def _cache_key(self):
        return tuple((l.weight.data_ptr(), l.weight._version, l.bias.data_ptr(), l.bias._version,
                      l.mask.data_ptr(), l.mask._version) for l in self.arn.layers) + (cache_epoch(),)

    def _build(self):
        arn = self.arn
        layers = list(arn.layers)
        dev = layers[0].weight.device
        cpu = dict(device="cpu", dtype=torch.float64)
        widths, hidden, outs = degree_schedule(
            arn.permutation.cpu(), [l.mask.detach().to(**cpu) for l in layers],
            [l.weight.detach().to(**cpu) for l in layers], [l.bias.detach().to(**cpu) for l in layers],
            arn.input_dim, arn.context_dim, arn.output_multiplier)
        f32 = dict(device=dev, dtype=torch.float32)
        self.widths = widths
        self.hidden = [[(li, _InverseBlock(a, b, n, wb.to(**f32).contiguous(), bb.to(**f32)))
                        for (li, a, b, n, wb, bb) in hidden[g]] for g in range(arn.input_dim)]
        self.outs = [(i, n, wb.to(**f32).contiguous(), bb.to(**f32).contiguous()) for (i, n, wb, bb) in outs]

    def plan(self):
        key = self._cache_key()
        if key != self._key:
            self._build()
            self._key = key
        return self

    def run(self, v: torch.Tensor, context: Optional[torch.Tensor], step) -> torch.Tensor:
        """x with pass k's dim of order k set by step(k, dim, raw_k [B, mult], x) (raw_k is the
        conditioner output of that dim only, pyro's column order p)."""
        self.plan()
        B, D = v.shape
        if context is not None and self.fold_context and (
                context.dim() == 1 or context.shape[0] == 1 or context.stride(0) == 0):
            return self._run_folded(v, context.reshape(-1, context.shape[-1])[0], step)
        x = torch.zeros_like(v)
        hs = [torch.empty((B, w), device=v.device, dtype=torch.float32) for w in self.widths]
        act = self.arn.act
        for k in range(1, D + 1):
            for li, blk in self.hidden[k - 1]:
                dst = hs[li][:, blk.a:blk.b]
                if li == 0:
                    ops.linear_act(x, blk.w, blk.bias, act, context=context, out=dst)
                else:
                    ops.linear_act(hs[li - 1][:, :blk.n], blk.w, blk.bias, act, out=dst)
            i, n, wb, bb = self.outs[k - 1]
            if n:
                raw = ops.linear_act(hs[-1][:, :n], wb, bb, "identity")
            else:
                raw = bb.reshape(1, -1).expand(B, -1)
            step(k, i, raw, x)
        return x


    # one context vector for all rows: evaluate the context-only (degree-0) units once and fold
    # them into the later groups' biases (flows/bflow_maf.py does the same per weight draw)
    fold_context = True

    def _splits(self):
        """Per block (e, W[:, :e], W[:, e:]): e = the input columns that are constant under a
        broadcast context (layer 0: the context; later layers: the previous degree-0 group)."""
        key = self._key
        if getattr(self, "_split_key", None) == key:
            return self._split
        C = self.arn.context_dim
        e_out = {li: blk.b for li, blk in self.hidden[0]}
        split = [[(e, blk.w[:, :e].contiguous(), blk.w[:, e:].contiguous())
                  for li, blk in g for e in [C if li == 0 else e_out.get(li - 1, 0)]] for g in self.hidden]
        e_last = e_out.get(len(self.widths) - 1, 0)
        outs = [(e_last, wb[:, :e_last].contiguous(), wb[:, e_last:].contiguous()) for (_, _, wb, _) in self.outs]
        self._split, self._split_key = (split, outs), key
        return self._split

    def _run_folded(self, v: torch.Tensor, c: torch.Tensor, step) -> torch.Tensor:
        B, D = v.shape
        C = c.shape[0]
        act = self.arn.act
        split, osplit = self._splits()
        hc = {}  # layer -> [1, e] constant activations of its degree-0 group
        for li, blk in self.hidden[0]:
            src = torch.cat((c, torch.zeros(D, device=v.device))).reshape(1, -1) if li == 0 else hc[li - 1]
            hc[li] = ops.linear_act(src[:, :blk.n].contiguous(), blk.w, blk.bias, act)
        x = torch.zeros_like(v)
        hs = [torch.empty((B, w), device=v.device, dtype=torch.float32) for w in self.widths]
        c1 = c.reshape(1, C)
        for k in range(1, D + 1):
            if k > 1:
                for (li, blk), (e, wc, wr) in zip(self.hidden[k - 1], split[k - 1]):
                    bias = blk.bias
                    if e:
                        src = c1 if li == 0 else hc[li - 1]
                        bias = ops.linear_act(src, wc, bias, "identity").reshape(-1)
                    inp = x if li == 0 else hs[li - 1][:, e:blk.n]
                    ops.linear_act(inp, wr, bias, act, out=hs[li][:, blk.a:blk.b])
            i, n, wb, bb = self.outs[k - 1]
            e, wc, wr = osplit[k - 1]
            bias = bb if not e else ops.linear_act(hc[len(self.widths) - 1], wc, bb, "identity").reshape(-1)
            if n > e:
                raw = ops.linear_act(hs[-1][:, e:n], wr, bias, "identity")
            else:
                raw = bias.reshape(1, -1).expand(B, -1)
            step(k, i, raw, x)
        return x


    def index_maps(self):
        """The schedule as gather maps into F = [0, W0, b0, W1, b1, ...] (flat, unmasked): the
        schedule is linear in the weights, so running it on index-valued weights (1-based, masks
        applied) gives, per block, the flat index of every entry (0 = masked / padding)."""
        arn = self.arn
        layers = list(arn.layers)
        key = tuple((l.mask.data_ptr(), l.mask._version) for l in layers) + (
            arn.permutation.data_ptr(), arn.permutation._version, cache_epoch())  # no device sync (graph capture)
        if getattr(self, "_imap_key", None) == key:
            return self._imap
        cpu = dict(device="cpu", dtype=torch.float64)
        wi, bi, off = [], [], 1
        for l in layers:
            nw = l.weight.numel()
            wi.append(torch.arange(off, off + nw, **cpu).reshape(l.weight.shape))
            bi.append(torch.arange(off + nw, off + nw + l.bias.numel(), **cpu))
            off += nw + l.bias.numel()
        widths, hidden, outs = degree_schedule(arn.permutation.cpu(), [l.mask.detach().to(**cpu) for l in layers],
                                               wi, bi, arn.input_dim, arn.context_dim, arn.output_multiplier)
        dev = layers[0].weight.device
        nxt = [off]  # next zero slot past F's parameters

        def ix(t):
            t = t.round().long()
            if _GATHER_UNIQUE:  # each masked / padding entry its own zero slot
                z = t == 0
                k = int(z.sum())
                t[z] = torch.arange(nxt[0], nxt[0] + k)
                nxt[0] += k
            return t
        hidden = [[(li, a, b, n, ix(w), ix(bb)) for (li, a, b, n, w, bb) in g] for g in hidden]
        outs = [(i, n, ix(w), ix(bb)) for (i, n, w, bb) in outs]
        if _GATHER_UNIQUE:
            allix = torch.cat([t.reshape(-1) for g in hidden for blk in g for t in blk[4:]] +
                              [t.reshape(-1) for o in outs for t in o[2:]])
            assert allix.unique().numel() == allix.numel(), "degree schedule gathers a parameter twice"
        to = lambda t: t.to(dev)  # noqa: E731
        hidden = [[(li, a, b, n, to(w), to(bb)) for (li, a, b, n, w, bb) in g] for g in hidden]
        outs = [(i, n, to(w), to(bb)) for (i, n, w, bb) in outs]
        self._imap, self._imap_key, self._nzero = (widths, hidden, outs), key, nxt[0] - off
        return self._imap

    def run_grad(self, v: torch.Tensor, context: Optional[torch.Tensor], step):
        """Differentiable degree-scheduled inverse (training walk, a10): the blocks are gathered
        from the live parameters (torch indexing, so autograd scatters their gradients back) and
        run through LinearActFn; step(k, dim, raw_k) -> (x_dim [B, 1], forward ld [B]).  Same
        values as pyro's D-pass loop with every hidden unit computed once."""
        B, D = v.shape
        widths, hidden, outs = self.index_maps()
        layers = list(self.arn.layers)
        F = torch.cat([v.new_zeros(1)] + [t.reshape(-1) for l in layers for t in (l.weight, l.bias)] +
                      [v.new_zeros(self._nzero)])
        if _GATHER_UNIQUE:  # every block of the layer in one gather node
            order = [t for g in hidden for blk in g for t in blk[4:]] + [t for o in outs for t in o[2:]]
            got = dict(zip((id(t) for t in order), _GatherBlocks.apply(F, *order)))

            def G(idx):
                return got[id(idx)]
        else:
            def G(idx):
                return F[idx]
        act = self.arn.act
        cols = [v.new_zeros(B, 1) for _ in range(D)]
        done = [[] for _ in widths]  # per hidden layer: its group outputs in degree order
        ld = None
        for k in range(1, D + 1):
            x = torch.cat(cols, 1)
            for (li, a, b, n, wi, bi) in hidden[k - 1]:
                if li == 0:
                    h = ag.linear_act(x, G(wi), G(bi), act, context=context)
                else:
                    h = ag.linear_act(torch.cat(done[li - 1], 1)[:, :n], G(wi), G(bi), act)
                done[li].append(h)
            i, n, wi, bi = outs[k - 1]
            if n:
                raw = ag.linear_act(torch.cat(done[-1], 1)[:, :n], G(wi), G(bi), "identity")
            else:
                raw = G(bi).reshape(1, -1).expand(B, -1)
            xi, ldi = step(k, i, raw)
            cols[i] = xi
            ld = ldi if ld is None else ld + ldi
        return torch.cat(cols, 1), ld

    def run_affine2(self, v: torch.Tensor, context: Optional[torch.Tensor], step, ld_buf: torch.Tensor,
                    ld_mode2: int) -> Optional[torch.Tensor]:
        """Affine MAF inverse for D = 2 with one context vector: pass 1 as in ``run`` (folded),
        pass 2 = the context-free chain of degree-1 units + the inverse affine step of the order-2
        dim in ONE naz_made_affine_inv1 launch (csrc/made.hip).  None when not applicable."""
        self.plan()
        B, D = v.shape
        arn = self.arn
        if (D != 2 or context is None or not self.fold_context or arn.output_multiplier != 2
                or arn.act not in ("tanh", "relu") or ld_buf is None or not ld_buf.is_contiguous()
                or not (context.dim() == 1 or context.shape[0] == 1 or context.stride(0) == 0)):
            return None
        g1 = self.hidden[1]
        nl = len(self.widths)
        if [li for li, _ in g1] != list(range(nl)) or any(blk.b - blk.a > 160 for _, blk in g1):
            return None
        from .flows.bflow_maf import MAFSpec, made_pack_map
        c = context.reshape(-1, context.shape[-1])[0]
        C = c.shape[0]
        split, osplit = self._splits()
        act = arn.act
        hc = {}
        for li, blk in self.hidden[0]:
            src = torch.cat((c, torch.zeros(D, device=v.device))).reshape(1, -1) if li == 0 else hc[li - 1]
            hc[li] = ops.linear_act(src[:, :blk.n].contiguous(), blk.w, blk.bias, act)
        x = torch.zeros_like(v)
        i, n, wb, bb = self.outs[0]
        e, wc, wr = osplit[0]
        raw = bb if not e else ops.linear_act(hc[nl - 1], wc, bb, "identity").reshape(-1)
        step(1, i, raw.reshape(1, -1).expand(B, -1), x)  # order-1 dim: constant conditioner output
        rows = [blk.b - blk.a for _, blk in g1]
        if getattr(self, "_p2_key", None) != (self._key, tuple(rows)):
            sp = MAFSpec(D, 0, rows, act)
            sp.param_shapes[-1] = ((2, rows[-1]), (2,))
            self._p2_nh = (max(rows) + 31) // 32
            self._p2_map = made_pack_map(sp, [torch.ones(ws) for (ws, _) in sp.param_shapes], self._p2_nh).to(v.device)
            self._p2_key = (self._key, tuple(rows))
        c1 = c.reshape(1, C)
        parts = [torch.zeros(1, device=v.device)]
        for (li, blk), (e, wc, wr) in zip(g1, split[1]):
            bias = blk.bias if not e else ops.linear_act(c1 if li == 0 else hc[li - 1], wc, blk.bias,
                                                         "identity").reshape(-1)
            parts += [wr.reshape(-1), bias.reshape(-1)]
        i2, n2, wb2, bb2 = self.outs[1]
        e, wc, wr = osplit[1]
        bias = bb2 if not e else ops.linear_act(hc[nl - 1], wc, bb2, "identity").reshape(-1)
        parts += [wr.reshape(-1), bias.reshape(-1)]
        packed = torch.cat(parts)[self._p2_map].reshape(1, -1).contiguous()
        y = ops.made_affine_inv1(packed, nl, self._p2_nh, x.unsqueeze(0), v.contiguous().unsqueeze(0), i2, act,
                                 ld_buf.view(1, -1), ld_mode2)
        return y[0]


class AutoRegressiveNN(ConditionalAutoRegressiveNN):
    """[pyro] nn/auto_reg_nn.py::AutoRegressiveNN."""

    def __init__(self, input_dim, hidden_dims, param_dims=(1, 1), permutation=None, skip_connections=False,
                 nonlinearity=nn.ReLU(), dropout_p=0.0):
        super().__init__(input_dim, 0, hidden_dims, param_dims, permutation, skip_connections, nonlinearity,
                         dropout_p)

    def forward(self, x):
        return self._shape(self.raw(x, None), x.shape[:-1])
