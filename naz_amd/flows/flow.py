"""``NormalizingFlow`` — naz's flow facade (naz/flows/flow.py:21-129), MI355X-native.

Same constructor (``NormalizingFlow(flow_type, bounds, D, C, hidden, L, [K, [split]],
embedding_net=None, **kw)``), same methods (``log_prob``, ``bounded_log_prob``,
``average_log_prob``, ``sample``) and attributes (``flow``, ``transforms``, ``nets``,
``flow_dist``, ``base_dist``, ``bounds``, ``conditional``, ``embedding_net``).

For flow_type "nsc" with a compiled shape, log_prob / sample run as ONE fused HIP
launch over all layers (``_FusedCoupling``); everything else runs the per-layer HIP
kernels through the Transform objects.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import numpy as np
import torch
from torch import nn
from torch.distributions import Normal

from .. import ops
from ..nn import activation_name, cache_epoch
from ..utils import device
from .continuous_transforms import continuous_free_form
from .distributions import ConditionalTransformedDistribution, TransformedDistribution
from .transforms import (ConditionalSplineCoupling, Permute, SplineCoupling, masked_affine_autoregressive,
                         neural_spline_autoregressive, neural_spline_coupling)


flow_makers = {"maf": masked_affine_autoregressive, "nsa": neural_spline_autoregressive,
               "nsc": neural_spline_coupling, "cnf": continuous_free_form}


class _FusedCoupling:
    """All L spline-coupling layers as one HIP launch (naz_coupling_log_prob / _sample).

    Parameters are gathered into the C ABI's flat per-layer order and re-laid into the
    kernel's MFMA panel order by ``naz_coupling_pack`` — only when a parameter changed
    (tracked by tensor version counters), so inference pays it once."""

    # fp16 pieces of the PACKED GEMM2/3 weights must stay finite with margin: |W'| < 2^15.  The
    # packer's sigmoid fold scales W1 by -2*(2 log2 e) and W2 by -2 (coupling.hip, kSigScale).
    F16_WEIGHT_LIMIT = 32768.0
    F16_PACK_SCALE = {1: 2.0 * 2.88539008177792681, 2: 2.0}

    def __init__(self, layers: List[nn.Module], D: int, C: int, S: int, K: int, H: int, act: str, lower: bool,
                 bound: float, mfma: str = "auto"):
        self.layers = layers
        self.shape = (D, C, S, K, H, act, lower, bound)
        self.mfma = mfma
        self.mode = "f16x3" if mfma == "auto" else mfma
        self.desc = ops.coupling_desc(D, C, S, K, len(layers), H, act, lower, bound, self.mode)
        self._sig = None
        self._packed = None

    def set_mfma(self, mfma: str) -> None:
        """"auto" (default: the 16-row-wave f16x3 kernel when the packed GEMM2/3 weights fit
        fp16's range and the shape allows it, else the 32-row f16x3 kernel, else bf16x6),
        "f16x3r16", "f16x3", "bf16x6" or "f32" (exact FP32 MFMA kernel); invalidates the
        packed weights."""
        self.mfma = mfma
        self._sig, self._packed = None, None

    def _resolve_mode(self) -> str:
        if self.mfma != "auto":
            return self.mfma
        big = max(float(t.nn.layers[i].weight.detach().abs().max()) * self.F16_PACK_SCALE[i]
                  for t in self.layers for i in (1, 2))
        if big >= self.F16_WEIGHT_LIMIT:
            return "bf16x6"
        D, C, S, K, H, act, lower, bound = self.shape
        r16 = ops.coupling_desc(D, C, S, K, len(self.layers), H, act, lower, bound, "f16x3r16")
        return "f16x3r16" if ops.coupling_supported(r16) else "f16x3"

    def usable(self) -> bool:
        """False while a conditioner's MC dropout is active (train mode, dropout_p > 0): the
        fused kernel has no dropout, so the per-layer kernels run."""
        return not any(t.nn.dropout_active() for t in self.layers)

    def params(self) -> List[torch.Tensor]:
        out = []
        for t in self.layers:
            net = t.nn
            for lin in net.layers:
                out += [lin.weight, lin.bias]
            low = t.lower_spline
            if low is not None:
                out += [low.unnormalized_widths, low.unnormalized_heights, low.unnormalized_derivatives]
        return out

    def packed(self) -> torch.Tensor:
        ps = self.params()
        sig = tuple((p.data_ptr(), p._version) for p in ps) + (cache_epoch(),)
        if sig != self._sig or self._packed is None:
            D, C, S, K, H, act, lower, bound = self.shape
            if self._packed is None or not _capturing(ps[0].device):
                # (a capture keeps the mode its eager warm-up step resolved: reading the weights back
                # is a host sync; the graph's packer kernel re-packs every replay in that mode)
                self.mode = self._resolve_mode()
            self.desc = ops.coupling_desc(D, C, S, K, len(self.layers), H, act, lower, bound, self.mode)
            flat = torch.cat([p.detach().reshape(-1) for p in ps])
            # a fresh image per repack: a training forward's backward (_CouplingTrainFn) still
            # holds the previous one, which must not change under it
            self._packed = ops.coupling_pack(self.desc, flat, None)
            self._flat, self._packed_bwd = flat, None
            self._sig = sig
        return self._packed

    # ---- the fused NLL training step (a10; coupling_train.h)
    F16_DATA_LIMIT = 32768.0

    def train_ready(self, x, context) -> bool:
        """The fused training path applies: the 16-row f16x3 image, data and context inside
        fp16's range (the kernels' GEMM1 split; one small device reduction + host read), and no
        gradient wanted for x or the context (train's data).  NAZ_TRAIN_FUSED=0 disables it."""
        if _TRAIN_FUSED == "0" or x.dim() != 2 or x.requires_grad or (context is not None and context.requires_grad):
            return False
        self.packed()
        if self.mode != "f16x3r16":
            return False
        if _RANGE_CHECKED.get():  # a HIP-graph capture whose caller checks the range before every replay
            return True
        return ops.absmax(x, context) < self.F16_DATA_LIMIT

    def packed_bwd(self) -> torch.Tensor:
        packed = self.packed()
        if getattr(self, "_packed_bwd", None) is None:
            self._packed_bwd = ops.coupling_pack_bwd(self.desc, self._flat)
        return packed, self._packed_bwd, self._flat

    def train_log_prob(self, x, context=None, bounds=None):
        """log p(x | ctx) recorded as ONE autograd node whose backward is the fused per-layer
        HIP backward (naz_coupling_bwd_layer) + weight-gradient GEMMs (naz_gemm)."""
        return _CouplingTrainFn.apply(x, context, bounds, self, *self.params())


    def log_prob(self, x, context=None, bounds=None, out=None):
        low = high = None
        if bounds is not None:
            low, high = bounds["low"].to(x.device, torch.float32), bounds["high"].to(x.device, torch.float32)
        packed = self.packed()  # may re-resolve the mode: read self.desc only after it
        return ops.coupling_log_prob(self.desc, packed, x, context, low, high, out=out)

    def sample(self, z, context=None, bounds=None, with_logdet=False):
        low = high = None
        if bounds is not None:
            low, high = bounds["low"].to(z.device, torch.float32), bounds["high"].to(z.device, torch.float32)
        packed = self.packed()
        return ops.coupling_sample(self.desc, packed, z, context, low, high, with_logdet=with_logdet)


class _FusedAR:
    """All L nsa / maf layers' log_prob as ONE HIP launch (naz_ar_flow_log_prob,
    csrc/made_ar_r16.h): every layer's D-pass MADE inverse (pyro ConditionedSplineAutoregressive /
    ConditionedAffineAutoregressive._inverse, naz transforms.py:133-198) with each hidden unit
    computed once, in registers, on the f16x3 MFMA path.  sample() is one naz_ar_flow_sample launch
    (the forward direction: one MADE pass per layer, then every dim's map); the autograd walk keeps
    the per-layer kernels.  The kernel is compiled for pyro's hidden mask indices; the masks are
    checked against them once per parameter change."""

    can_sample = True  # sample(): naz_ar_flow_sample (the forward direction, one launch)
    inverse = True  # log_prob fused too (False for a forward-only instance: per-layer log_prob)
    F16_DATA_LIMIT = 32768.0  # the kernel's f16x3 input split (|x|, |ctx| < 2^15)

    def __init__(self, layers: List[nn.Module], kind: str, D: int, C: int, H: int, n_hidden: int, K: int, act: str,
                 bound: float):
        self.layers = layers
        self.kind = kind
        self.shape = (D, C, H, n_hidden, K)
        self.P = 2 if kind == "maf" else 3 * K - 1
        self.desc = ops.ar_flow_desc(kind, D, C, H, len(layers), n_hidden, K, act, bound)
        self.act = act
        self._sig = None
        self._packed = None
        self._fsig, self._fpacked = None, None
        self._masks = None
        self._p0sig, self._p0, self._p0fn = None, None, (None, None)

    def _nets(self):
        return [t.nn for t in self.layers]

    def masks_ok(self) -> bool:
        """The ARN masks are pyro's create_mask for the kernel's compiled hidden indices
        (re-checked whenever a mask or permutation tensor changes: load_state rewrites them)."""
        sig = tuple((t.data_ptr(), t._version) for n in self._nets()
                    for t in [n.permutation] + [l.mask for l in n.layers])
        if self._masks is None or self._masks[0] != sig:
            D, C, H, NH, K = self.shape
            deg = ops.ar_flow_degrees(self.desc).astype(np.int64)
            ok = True
            for arn in self._nets():
                m = [l.mask.detach().cpu().numpy() != 0 for l in arn.layers]
                perm = arn.permutation.detach().cpu().numpy().astype(np.int64)
                order = np.empty(D, dtype=np.int64)
                order[perm] = np.arange(D)
                in_idx = np.concatenate([np.zeros(C, dtype=np.int64), order + 1])
                out_idx = np.tile(order + 1, self.P)
                ok = ok and len(m) == NH + 1 and m[0].shape == (H, C + D) and m[-1].shape == (D * self.P, H)
                ok = ok and bool((m[0] == (deg[:, None] >= in_idx[None, :])).all())
                for i in range(1, NH):
                    ok = ok and m[i].shape == (H, H) and bool((m[i] == (deg[:, None] >= deg[None, :])).all())
                ok = ok and bool((m[-1] == (out_idx[:, None] > deg[None, :])).all())
            self._masks = (sig, ok)
        return self._masks[1]

    def usable(self) -> bool:
        return self.masks_ok() and not any(n.dropout_active() for n in self._nets())

    def log_prob_ready(self, x, context) -> bool:
        if not self.inverse or x.dim() != 2:
            return False
        if _RANGE_CHECKED.get():  # a HIP-graph capture whose caller checks the range before every replay
            return True
        return ops.absmax(x, context) < self.F16_DATA_LIMIT

    def train_ready(self, x, context) -> bool:
        """The maf NLL step on the fused backward (made_ar_bwd.h, flows/maf_grad.py): an affine flow
        at a compiled shape, rows inside the f16 split's range, no gradient wanted for x or the
        context (train's data).  NAZ_TRAIN_FUSED=0 keeps the autograd walk."""
        if self.kind != "maf" or _TRAIN_FUSED == "0" or x.dim() != 2 or x.requires_grad or \
                (context is not None and context.requires_grad) or not self._train_kernels():
            return False
        return self.log_prob_ready(x, context)

    def _train_kernels(self) -> bool:
        """The fused backward kernel (made_ar_bwd.h) at its compiled shapes; elsewhere a fused inverse
        (naz_ar_flow_log_prob_train) + the GEMM-composed backward (flows/maf_grad_wide.py).
        NAZ_TRAIN_WIDE=0 keeps the autograd walk at the latter's shapes."""
        if ops.ar_flow_bwd_supported(self.desc):
            return True
        return _TRAIN_WIDE != "0" and self.inverse and ops.ar_flow_supported(self.desc) == 1

    def maf_grad(self):
        """MafGrad for the current permutations and masks (rebuilt when one of them changes)."""
        nets = self._nets()
        ts = [t for n in nets for l in n.layers for t in (l.mask,)] + [n.permutation for n in nets]
        cz = any(bool(getattr(n, "clip_zero_grad", False)) for n in nets)  # jnp.clip's gradient (bflow)
        sig = tuple((t.data_ptr(), t._version) for t in ts) + (cache_epoch(), cz)
        if getattr(self, "_mg", None) is None or self._mg[0] != sig:
            from .maf_grad import MafGrad
            from .maf_grad_wide import WideMafGrad
            mask = torch.cat([t for n in nets for l in n.layers
                              for t in (l.mask.detach().reshape(-1).float(), torch.ones_like(l.bias.detach()))])
            perm = np.stack([n.permutation.detach().cpu().numpy() for n in nets]).astype(np.int32)
            cls = MafGrad if ops.ar_flow_bwd_supported(self.desc) else WideMafGrad
            self._mg = (sig, cls(self.desc, perm, mask.contiguous(), clip_zero=cz))
        return self._mg[1]

    def train_params(self) -> List[torch.Tensor]:
        return [p for n in self._nets() for l in n.layers for p in (l.weight, l.bias)]

    def train_log_prob(self, x, context=None, bounds=None):
        """log p(x | ctx) recorded as ONE autograd node whose backward is the fused maf backward."""
        lj = None
        if bounds is not None:  # naz bounding_transform: a constant of the parameters here
            with torch.no_grad():
                x, lj = ops.bounding_fwd(x.detach(), bounds["low"], bounds["high"])
        lp = _MafTrainFn.apply(x, context, self, *self.train_params())
        return lp if lj is None else lp + lj

    def packed(self) -> torch.Tensor:
        ps = [p for n in self._nets() for l in n.layers for p in (l.weight, l.bias, l.mask)]
        sig = tuple((p.data_ptr(), p._version) for p in ps) + (cache_epoch(),)
        if sig != self._sig or self._packed is None:
            flats, perms = [], []
            for n in self._nets():
                for l in n.layers:
                    flats += [(l.weight.detach() * l.mask).float().cpu().numpy().ravel(),
                              l.bias.detach().float().cpu().numpy()]
                perms.append(n.permutation.detach().cpu().numpy())
            dev = self._nets()[0].layers[0].weight.device
            self._packed = ops.ar_flow_pack(self.desc, np.concatenate(flats), np.stack(perms), dev)
            self._sig = sig
        return self._packed

    def _flat(self):
        flats = []
        for n in self._nets():
            for l in n.layers:
                flats += [(l.weight.detach() * l.mask).float().cpu().numpy().ravel(),
                          l.bias.detach().float().cpu().numpy()]
        return np.concatenate(flats)

    def packed_fwd(self) -> torch.Tensor:
        """The forward (sample) image, re-packed when a weight, bias or mask changes."""
        ps = [p for n in self._nets() for l in n.layers for p in (l.weight, l.bias, l.mask)]
        sig = tuple((p.data_ptr(), p._version) for p in ps) + (cache_epoch(),)
        if sig != self._fsig or self._fpacked is None:
            dev = self._nets()[0].layers[0].weight.device
            self._fpacked = ops.ar_flow_pack_fwd(self.desc, self._flat(), dev)
            self._fsig = sig
        return self._fpacked

    def sample_ready(self, z, context) -> bool:
        """The kernel splits the context into f16 pieces (|ctx| < 2^15); z is rescaled per row."""
        if z.dim() != 2:
            return False
        if context is not None and context.numel():
            return ops.absmax(context) < self.F16_DATA_LIMIT
        return True

    def sample(self, z, context=None, bounds=None, with_logdet=False):
        low = high = None
        if bounds is not None:
            low, high = bounds["low"].contiguous(), bounds["high"].contiguous()
        return ops.ar_flow_sample(self.desc, self.packed_fwd(), z, context, low, high, with_logdet=with_logdet)

    def _pass0_operands(self):
        """(unmasked flat rows [1, L per], mask vector, permutations, ArPass0) on the device, for
        the one-context-vector path; re-read when a parameter, mask or permutation changes."""
        nets = self._nets()
        ts = [t for n in nets for l in n.layers for t in (l.weight, l.bias, l.mask)] + [n.permutation for n in nets]
        sig = tuple((t.data_ptr(), t._version) for t in ts) + (cache_epoch(),)
        if sig != self._p0sig:
            flats, masks = [], []
            for n in nets:
                for l in n.layers:
                    flats += [l.weight.detach().reshape(-1), l.bias.detach().reshape(-1)]
                    masks += [l.mask.detach().reshape(-1), torch.ones_like(l.bias.detach()).reshape(-1)]
            perm = np.stack([n.permutation.detach().cpu().numpy() for n in nets]).astype(np.int32)
            flat = torch.cat(flats).to(torch.float32)[None].contiguous()
            key = perm.tobytes()
            if self._p0fn[0] != key:
                from .ar_pass0 import ArPass0
                self._p0fn = (key, ArPass0(self.desc, [int(p[0]) for p in perm], self.act, flat.device))
            self._p0 = (flat, torch.cat(masks).to(torch.float32).contiguous(), perm, self._p0fn[1])
            self._p0sig = sig
        return self._p0

    def _pass0_form(self) -> bool:
        """The instance has the pass-0-constants image (the wide H = 512 inverse does not)."""
        if getattr(self, "_p0form", None) is None:
            self._p0form = ops.ar_flow_pass0_floats(self.desc) > 0
        return self._p0form

    def log_prob(self, x, context=None, bounds=None, out=None):
        low = high = None
        if bounds is not None:
            low, high = bounds["low"].to(x.device, torch.float32), bounds["high"].to(x.device, torch.float32)
        if (_AR_PASS0 and bounds is None and self.shape[1] > 0 and context is not None and x.dim() == 2 and
                x.shape[0] >= 4096 and (context.dim() == 1 or context.shape[0] == 1) and self._pass0_form()):
            # one condition vector (the density grid): the context-only first degree pass once,
            # packed as constants in place of its weights (naz_ar_flow_pack pass0)
            flat, mask, perm, p0 = self._pass0_operands()
            img = ops.ar_flow_pack_batched(self.desc, flat, perm, pass0=p0(flat, context, mask), mask=mask)
            lp = ops.ar_flow_log_prob_batched(self.desc, img, x, context.reshape(-1), pass0_const=True)[0]
            if out is None:
                return lp
            out.copy_(lp)
            return out
        return ops.ar_flow_log_prob(self.desc, self.packed(), x, context, low, high, out=out)

    def executed_flop_per_row(self) -> int:
        """FP32-equivalent FLOPs the inverse kernel executes per row (ops.ar_executed_flop_per_row)."""
        return ops.ar_executed_flop_per_row(self.desc)["inverse"]


_TRAIN_FUSED = __import__("os").environ.get("NAZ_TRAIN_FUSED", "1")
# set by trainers.GraphedNllStep around the capture of a step (a context variable: only the capturing
# thread's calls skip the check): the fused paths' f16-range check reads the data back to the host
# (no sync is allowed in a capture), so the graph's owner checks each replay's rows itself before
# replaying (and runs an out-of-range minibatch eagerly)
_RANGE_CHECKED = __import__("contextvars").ContextVar("naz_range_checked", default=False)


def _capturing(dev) -> bool:
    return dev.type == "cuda" and torch.cuda.is_current_stream_capturing()
_TRAIN_WIDE = __import__("os").environ.get("NAZ_TRAIN_WIDE", "1")  # the GEMM-composed maf backward
_AR_FUSED = __import__("os").environ.get("NAZ_AR_FUSED", "1")
_AR_PASS0 = __import__("os").environ.get("NAZ_AR_PASS0", "1") != "0"  # one-context-vector first-pass folding


class _MafTrainFn(torch.autograd.Function):
    """NormalizingFlow.log_prob of a maf flow under autograd at the fused backward's shapes (naz
    train's loss, train_flows.py:195, 208): forward = the fused inverse kernel with every layer's
    output saved; backward = one fused backward launch per layer + batched dW (flows/maf_grad.py)."""

    @staticmethod
    def forward(ctx, x, context, plan, *params):
        mg = plan.maf_grad()
        flat = torch.cat([p.detach().reshape(-1) for p in params])
        imgs = mg.images(flat)
        c = None if context is None else (context.detach().reshape(1, -1) if context.dim() == 1 else context.detach())
        lp, states = mg.forward(imgs, x.detach().float().contiguous(), c)
        ctx.mg, ctx.imgs, ctx.c = mg, imgs, c
        ctx.shapes = [p.shape for p in params]
        ctx.save_for_backward(states.clone())  # the buffer is reused by the next forward of this size
        return lp.clone()

    @staticmethod
    def backward(ctx, g_lp):
        (states,) = ctx.saved_tensors
        grad, _ = ctx.mg.backward(ctx.imgs, states, ctx.c, g_lp.contiguous().float())
        outs, o = [], 0
        for shp in ctx.shapes:
            n = int(np.prod(shp))
            outs.append(grad[o:o + n].view(shp))
            o += n
        return (None, None, None, *outs)


# layer l's dW reductions on a side stream while layer l + 1's backward kernel runs (NAZ_TRAIN_DW_STREAM=1).
# Off by default since r06: the r05 gain (164-165 -> 157-159 ms per 2^23-row step) was measured on runs
# whose loss went NaN; on the fixed step, same box, interleaved (profiles/r06_g7_*): 158.5 / 159.1 / 158.9
# ms with it vs 157.4 / 158.2 / 158.5 without.  The two kernels share the CUs (the backward kernel holds
# every register slot), so the overlap buys nothing, and one stream needs half the operand memory.
_DW_STREAM = os.environ.get("NAZ_TRAIN_DW_STREAM", "0") == "1"
# operand sets the backward kernels rotate through (a set is rewritten once its dW reductions are done)
_DW_SETS = max(2, int(os.environ.get("NAZ_TRAIN_DW_SETS", "2")))
_SIDE: Dict[int, "torch.cuda.Stream"] = {}


def _side_stream(dev: torch.device) -> "torch.cuda.Stream":
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i not in _SIDE:
        _SIDE[i] = torch.cuda.Stream(dev)
    return _SIDE[i]


def _nullcontext():
    import contextlib
    return contextlib.nullcontext()


class _CouplingTrainFn(torch.autograd.Function):
    """NormalizingFlow.log_prob of an nsc flow under autograd (naz train's loss, train_flows.py:
    195, 208).  forward: naz_coupling_log_prob_train (all layers, one launch, layer inputs
    saved); backward: for l = 0 .. L-1 one naz_coupling_bwd_layer launch (recomputes the layer's
    conditioner, spline VJPs, exact-fp32 MFMA dX chain, lower-spline gradients) and three
    batch-reduction GEMMs for dW / db."""

    @staticmethod
    def forward(ctx, x, context, bounds, plan, *params):
        packed, pbwd, flat = plan.packed_bwd()
        d = plan.desc
        B = x.shape[0]
        low = high = None
        if bounds is not None:
            low = bounds["low"].to(x.device, torch.float32).contiguous()
            high = bounds["high"].to(x.device, torch.float32).contiguous()
        states = torch.empty((d.L + 1, B, d.D), device=x.device, dtype=torch.float32)
        lp = ops.coupling_log_prob_train(d, packed, x.detach(), None if context is None else context.detach(),
                                         low, high, states)
        ctx.plan, ctx.packed, ctx.pbwd, ctx.flat = plan, packed, pbwd, flat
        ctx.desc, ctx.shape = d, plan.shape  # the forward's; a later repack replaces plan.desc
        ctx.save_for_backward(states, context)
        ctx.n_params = len(params)
        return lp

    @staticmethod
    def backward(ctx, g_lp):
        states, context = ctx.saved_tensors
        plan = ctx.plan
        d = ctx.desc
        D, C, S, K, H, act, lower, bound = ctx.shape
        L, B = d.L, states.shape[1]
        dev = states.device
        g_lp = g_lp.contiguous().float()
        g = (-states[0]) * g_lp[:, None]  # d/dz of the Normal(0, I) base log-density
        g = g.contiguous()
        g_next = torch.empty_like(g)
        rows = plan.__dict__.get("_dp3_rows")
        if rows is None or rows.device != dev:
            rows = ops.coupling_dp3_columns(d).to(dev)
            plan._dp3_rows = rows
            valid = rows >= 0
            perm = torch.empty((int(valid.sum()),), dtype=torch.int64, device=dev)
            perm[rows[valid]] = torch.nonzero(valid).flatten()  # DenseNN output row -> its dp3 column
            plan._dp3_perm = perm
        perm = plan._dp3_perm
        NC = rows.numel()
        f32 = dict(device=dev, dtype=torch.float32)

        def operand_set():
            return {"h1": torch.empty((B, H), **f32), "h2": torch.empty((B, H), **f32),
                    "dp1": torch.empty((B, H), **f32), "dp2": torch.empty((B, H), **f32),
                    "dp3": torch.empty((B, NC), **f32), "x0": torch.empty((B, C + S), **f32)}

        # every layer's dW / db in ONE zeroed buffer (one fill on the main stream before the loop): the
        # reductions accumulate into it, so the side stream launches only the three dW kernels per
        # layer — r06 trace (profiles/r06_g3_*): the per-call zero fills queued behind the concurrent
        # backward kernel and took ~2 ms per layer on the side stream, its critical path
        sizes = [H * (C + S), H, H * H, H, NC * H, NC]
        offs = np.concatenate([[0], np.cumsum(sizes)]).tolist()
        gall = torch.zeros((L, offs[-1]), **f32)
        # layer l's dW reductions on a side stream, overlapping layer l + 1's backward kernel
        # (_DW_SETS operand sets; fork / join by events, capture-safe; NAZ_TRAIN_DW_STREAM=0: one stream)
        overlap = _DW_STREAM and dev.type == "cuda" and not _capturing(dev)  # (a captured step: one stream)
        sets = [operand_set() for _ in range(_DW_SETS if overlap else 1)]
        main = torch.cuda.current_stream(dev) if overlap else None
        side = _side_stream(dev) if overlap else None
        if overlap:
            gall.record_stream(side)
            for bufs in sets:
                for t in bufs.values():
                    t.record_stream(side)
        done = [None] * len(sets)  # the side stream's event after the dW of the last layer that used set i
        n_low = S * (3 * K - 1) if lower else 0
        g_low = torch.zeros((L, max(n_low, 1)), **f32)
        per = 9 if lower else 6
        grads = [None] * ctx.n_params
        for l in range(L):
            si = l % len(sets)
            bufs = sets[si]
            if overlap and done[si] is not None:
                main.wait_event(done[si])  # this set's previous dW reads are over
            ops.coupling_bwd_layer(d, ctx.packed, ctx.pbwd, ctx.flat, l, states[l + 1], context, g, g_lp, bufs, g_next,
                                   g_low[l] if lower else None)
            gw = [gall[l, offs[i]:offs[i + 1]] for i in range(6)]
            if overlap:
                ev = torch.cuda.Event()
                ev.record(main)
                side.wait_event(ev)
            with torch.cuda.stream(side) if overlap else _nullcontext():
                ops.gemm(bufs["dp1"].t(), bufs["x0"], out=gw[0].view(H, C + S), rowsum=gw[1], accumulate=True)
                ops.gemm(bufs["dp2"].t(), bufs["h1"], out=gw[2].view(H, H), rowsum=gw[3], accumulate=True)
                ops.gemm(bufs["dp3"].t(), bufs["h2"], out=gw[4].view(NC, H), rowsum=gw[5], accumulate=True)
            if overlap:
                done[si] = torch.cuda.Event()
                done[si].record(side)
            g, g_next = g_next, g
        if overlap:
            for e in done:
                if e is not None:
                    main.wait_event(e)  # the gradients are read on the main stream
        # dp3 columns (lane-slot order, padding included) -> DenseNN output rows, all layers at once
        w2 = gall[:, offs[4]:offs[5]].view(L, NC, H).index_select(1, perm)
        b2 = gall[:, offs[5]:offs[6]].index_select(1, perm)
        for l in range(L):
            out = [gall[l, offs[0]:offs[1]].view(H, C + S), gall[l, offs[1]:offs[2]],
                   gall[l, offs[2]:offs[3]].view(H, H), gall[l, offs[3]:offs[4]], w2[l], b2[l]]
            if lower:
                gl = g_low[l]
                out += [gl[:S * K].view(S, K), gl[S * K:2 * S * K].view(S, K), gl[2 * S * K:].view(S, K - 1)]
            grads[l * per:(l + 1) * per] = out
        return (None, None, None, None, *grads)


def _maker_args(flow_type, flow_args, flow_kwargs):
    """The maker's arguments by name, however the caller passed them (positionally as naz's
    examples do, or by keyword); None when they do not bind."""
    import inspect
    try:
        b = inspect.signature(flow_makers[flow_type]).bind(*flow_args, **flow_kwargs)
    except TypeError:
        return None
    b.apply_defaults()
    return b.arguments


def _fused_plan(flow_type, flow_args, flow_kwargs, transforms):
    if any(isinstance(t, Permute) for t in transforms):
        return None
    a = _maker_args(flow_type, flow_args, flow_kwargs)
    if a is None or "theta_dim" not in a:
        return None
    if flow_type in ("nsa", "maf") and _AR_FUSED != "0":
        D, C, hidden, L = a["theta_dim"], a["condition_dim"], a["hidden_dim"], a["num_layers"]
        K = a["count_bins"] if flow_type == "nsa" else 8
        hidden = list(hidden) if isinstance(hidden, (list, tuple)) else [hidden]
        act = activation_name(a["activation"])
        if any(h != hidden[0] for h in hidden):
            return None
        try:
            bound = transforms[0].bound if flow_type == "nsa" else 3.0
            plan = _FusedAR(list(transforms), flow_type, D, C, hidden[0], len(hidden), K, act, bound)
            if not ops.ar_flow_fwd_supported(plan.desc) or not plan.masks_ok():
                return None
            plan.inverse = ops.ar_flow_supported(plan.desc)  # False: fused sampling only (wide MAFs)
            return plan
        except Exception:
            return None
    if flow_type != "nsc":
        return None
    D, C, hidden, L = a["theta_dim"], a["condition_dim"], a["hidden_dim"], a["num_layers"]
    K, S = a["count_bins"], a["split_dim"]
    hidden = list(hidden) if isinstance(hidden, (list, tuple)) else [hidden]
    if len(hidden) != 2 or hidden[0] != hidden[1]:
        return None
    act = activation_name(a["activation"])
    layers = list(transforms)
    inner = [t.module if isinstance(t, SplineCoupling) else t for t in layers]
    lower = all(t.lower_spline is not None for t in inner)
    if not lower and any(t.lower_spline is not None for t in inner):
        return None
    try:
        plan = _FusedCoupling(inner, D, C, S, K, hidden[0], act, lower, inner[0].bound)
        return plan if ops.coupling_supported(plan.desc) else None
    except Exception:
        return None


class NormalizingFlow(nn.Module):
    """naz/flows/flow.py:24-129."""

    def __init__(self, flow_type, bounds, *flow_maker_args, embedding_net=None, **flow_maker_kwargs):
        super().__init__()
        assert flow_type in list(flow_makers.keys())
        flow_maker = flow_makers[flow_type]
        self.flow_type = flow_type
        self.conditional = True if flow_maker_args[1] > 0 else False
        if embedding_net is not None:
            assert self.conditional
            self.embedding_net = embedding_net
        else:
            self.embedding_net = nn.Identity()
        self.bounds = bounds
        D = flow_maker_args[0]
        self.register_buffer("_base_loc", torch.zeros(D))
        self.register_buffer("_base_scale", torch.ones(D))
        self.flow, self.transforms, self.nets = flow_maker(*flow_maker_args, **flow_maker_kwargs)
        self._plan = _fused_plan(flow_type, flow_maker_args, flow_maker_kwargs, self.transforms)
        self.to(device)
        self._make_dist()

    # -- distribution objects are rebuilt after device moves (the base Normal holds tensors)
    def _make_dist(self):
        self.base_dist = Normal(self._base_loc, self._base_scale)
        if self.conditional:
            self.flow_dist = ConditionalTransformedDistribution(self.base_dist, self.flow, fused=self._plan)
        else:
            self.flow_dist = TransformedDistribution(self.base_dist, self.flow, fused=self._plan)

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        if "_base_loc" in self._buffers and hasattr(self, "flow"):
            self._make_dist()
        return out

    def set_fused(self, enabled: bool) -> None:
        """Switch between the single fused launch and the per-layer kernels (testing aid)."""
        if not enabled:
            if self._plan is not None:
                self._plan_saved, self._plan = self._plan, None
        elif self._plan is None:
            if getattr(self, "_plan_saved", None) is None:
                raise RuntimeError("no fused instantiation for this flow")
            self._plan = self._plan_saved
        self._make_dist()

    @property
    def fused(self) -> bool:
        """True when log_prob (and, for nsc, sample) run as one fused launch."""
        return self._plan is not None

    def _bounds_dev(self, ref):
        if self.bounds is None:
            return None
        return {k: torch.as_tensor(v, dtype=torch.float32, device=ref.device) for k, v in self.bounds.items()}

    def _pdf(self, condition):
        if self.conditional:
            assert condition is not None
            return self.flow_dist.condition(self.embedding_net(condition))
        return self.flow_dist

    def log_prob(self, x, *args, condition=None, **kwargs):
        """log p(theta | lambda) for x [B, D] (naz/flows/flow.py:45-79)."""
        pdf = self._pdf(condition)
        return pdf.log_prob(x, bounds=self._bounds_dev(x))

    def bounded_log_prob(self, x, *args, condition=None, **kwargs):
        """naz/flows/flow.py:81-87: -inf outside the bounding box."""
        if self.bounds is None:
            return self.log_prob(x, *args, condition=condition, **kwargs)
        b = self._bounds_dev(x)
        lp = torch.full(x.shape[:1], float("-inf"), device=x.device, dtype=torch.float32)
        valid = torch.prod((x > b["low"].expand(x.shape)) * (x < b["high"].expand(x.shape)), dim=1).to(torch.bool)
        if bool(valid.any()):
            lp[valid] = self.log_prob(x[valid, :], *args, condition=condition, **kwargs)
        return lp

    def average_log_prob(self, x, *args, condition=None, **kwargs):
        """naz/flows/flow.py:90-91."""
        return torch.mean(self.bounded_log_prob(x, *args, condition=condition, **kwargs))

    def sample(self, *args, condition=None, **kwargs):
        """theta ~ p(theta | lambda) (naz/flows/flow.py:94-129); ``args[0]`` is the sample shape."""
        pdf = self._pdf(condition)
        shape = args[0] if args else kwargs.get("sample_shape", ())
        ref = self._base_loc
        return pdf.sample(shape, bounds=self._bounds_dev(ref))
