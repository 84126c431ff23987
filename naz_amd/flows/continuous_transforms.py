"""naz's continuous normalizing flow (naz/flows/continuous_transforms.py), MI355X-native.

``continuous_free_form(input_dim, condition_dim, hidden_dims, num_blocks, activation=nn.Softplus(),
...)`` keeps naz's signature and returns ``(flow, transforms, nets)``.  Each block is an FFJORD
transform over a ``ConditionalFCNN`` vector field (naz :38-60 — same ``.nn`` Sequential, so
parameter names ``nn.{i}.weight|bias`` match), integrated by ONE ``naz_cnf_integrate``
launch: the whole fixed-step RK4 solve, the Hutchinson trace and the log-det accumulation in
registers, the MLP resident in LDS (csrc/cnf.hip).

Solver: naz constructs torchdyn ``NeuralODE(solver='dopri5', atol=rtol=1e-4, sensitivity=
'adjoint')`` (:73-81).  SURVEY.md §8d pins config 5 to fixed-step classical RK4 with 8 steps
(NFE 32) — the default here (``solver='rk4', steps=8``); ``solver='dopri5'`` runs the adaptive
Dormand-Prince solve (``step_control="global"``, the default: torchdyn's one step size for the
batch, naz_cnf_integrate_dopri5_global — one launch per attempted step, the host polling the
controller every 4 attempts, so the call blocks the host and cannot be captured into a HIP graph;
``"group"``: naz_cnf_integrate_dopri5, one launch per solve, one step size per 16 rows, capturable).  Under autograd
the solve is one ``CnfSolveFn`` node (flows/cnf_adjoint.py, §8f rank 3): rk4 backpropagates by the
discrete adjoint of the pinned solve from per-step checkpoints, dopri5 by the continuous adjoint
(``adjoint_steps`` RK4 steps back from t1), every RHS and VJP on HIP kernels.  The Hutchinson probe eps ~ N(0, I)
is drawn per solve on the device, as torchdyn does; assign ``transform.noise`` to fix it.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn
from torch.distributions import Transform, constraints

from .. import ops
from ..nn import activation_name, cache_epoch
from .transforms import ComposeTransformModule, ConditionalComposeTransformModule, ConditionalTransformModule, \
    TransformModule

__all__ = ["ConditionalFCNN", "FCNN", "FFJORDTransform", "ConditionalFFJORDTransform", "continuous_free_form"]


class ConditionalFCNN(nn.Module):
    """naz/flows/continuous_transforms.py:38-60: Linear/act (/Dropout) chain, input cat([x, ctx])."""

    def __init__(self, input_dim, context_dim, hidden_dims, act=nn.Softplus(), dropout_p=0.0):
        super().__init__()
        hidden_dims = list(hidden_dims)
        if dropout_p:
            raise NotImplementedError("naz_amd CNF: dropout in the vector field is SURVEY.md §8f rank 2")
        layers = [nn.Linear(input_dim + context_dim, hidden_dims[0]), act]
        if dropout_p is not None:
            layers.append(nn.Dropout(p=dropout_p))
        for i, hidden_dim in enumerate(hidden_dims[1:]):
            layers.append(nn.Linear(hidden_dims[i], hidden_dim))
            layers.append(act)
            if dropout_p is not None:
                layers.append(nn.Dropout(p=dropout_p))
        layers.append(nn.Linear(hidden_dims[-1], input_dim))
        self.nn = nn.Sequential(*layers)
        self.input_dim, self.context_dim, self.hidden_dims = input_dim, context_dim, hidden_dims
        self.act = activation_name(act)

    def linears(self):
        return [m for m in self.nn if isinstance(m, nn.Linear)]

    def forward(self, x):
        raise NotImplementedError("naz_amd: the vector field runs inside naz_cnf_integrate")


class FCNN(ConditionalFCNN):
    """naz :62-67 (whose ``super().__init__(self, ...)`` call is broken in the reference; this is
    the evident intent: an unconditional ConditionalFCNN)."""

    def __init__(self, input_dim, hidden_dims, act=nn.Softplus(), dropout_p=0.0):
        super().__init__(input_dim, 0, hidden_dims, act=act, dropout_p=dropout_p)


class _CnfPlan:
    """The block's packed LDS image, re-packed when a parameter changes (version counters).

    ``mfma``: "auto" (default: "f16x3" when the shape allows it and every hidden/output weight
    fits fp16's range with margin, |W| < 2^15; else "f32"), "f16x3" or "f32"."""

    F16_WEIGHT_LIMIT = 32768.0

    def __init__(self, net: ConditionalFCNN, mfma: str = "auto"):
        self.net = net
        self.mfma = mfma
        self.mode = None
        # fused: the whole solve in one launch (csrc/cnf.hip, the vector field resident in one CU's
        # LDS); otherwise (e.g. naz's POSYDON CNF, D = 4, H = [128] x 4: ~200 KB of weights) the
        # per-layer solve over the walk's RHS (flows/cnf_adjoint.py walk_rk4 / walk_dopri5)
        try:
            self.desc = ops.cnf_desc(net.input_dim, net.context_dim, net.hidden_dims, net.act)
            self.fused = bool(ops.cnf_supported(self.desc))
        except ValueError:  # more hidden layers than the fused kernels take
            self.desc, self.fused = None, False
        self._sig, self._packed = None, None
        self._wsig, self._walk = None, None

    def set_mfma(self, mfma: str) -> None:
        self.mfma = mfma
        self._sig, self._packed = None, None

    def _resolve_mode(self) -> str:
        if self.mfma != "auto":
            return self.mfma
        x3 = ops.cnf_desc(self.net.input_dim, self.net.context_dim, self.net.hidden_dims, self.net.act, "f16x3")
        if not ops.cnf_supported(x3):
            return "f32"
        lins = self.net.linears()
        big = max(float(lin.weight.detach().abs().max()) for lin in lins[1:])
        return "f16x3" if big < self.F16_WEIGHT_LIMIT else "f32"

    def walk(self):
        """The per-layer RHS over the current parameters (rebuilt when one changes)."""
        from .cnf_adjoint import CnfWalk
        ps = [t for lin in self.net.linears() for t in (lin.weight, lin.bias)]
        sig = tuple((p.data_ptr(), p._version) for p in ps) + (cache_epoch(),)
        if sig != self._wsig or self._walk is None:
            self._walk, self._wsig = CnfWalk(self.net), sig
        return self._walk

    def packed(self):
        if not self.fused:
            raise RuntimeError("naz_amd CNF: no fused solve kernel at this shape (the per-layer solve runs instead)")
        ps = [t for lin in self.net.linears() for t in (lin.weight, lin.bias)]
        sig = tuple((p.data_ptr(), p._version) for p in ps) + (cache_epoch(),)
        if sig != self._sig or self._packed is None:
            self.mode = self._resolve_mode()
            n = self.net
            self.desc = ops.cnf_desc(n.input_dim, n.context_dim, n.hidden_dims, n.act, self.mode)
            flat = torch.cat([p.detach().reshape(-1) for p in ps])
            self._packed = ops.cnf_pack(self.desc, flat, self._packed)
            self._sig = sig
        return self._packed


class _FFJORDCore:
    """Shared solve logic of the conditional and unconditional transforms."""

    def _needs_graph(self, v) -> bool:
        return torch.is_grad_enabled() and (v.requires_grad or any(p.requires_grad for p in self._net.parameters())
                                            or (self._context is not None and self._context.requires_grad))

    def _noise(self, v):
        return self.noise if self.noise is not None else torch.randn(v.shape, device=v.device, dtype=torch.float32)

    def _dopri5(self, desc, packed, v, noise, t0, t1, ld_buf, ld_mode):
        """§8f rank 3: adaptive Dormand-Prince.  ``step_control="global"`` (default): torchdyn's
        one step size for the whole batch (naz_cnf_integrate_dopri5_global); ``"group"``: one per
        16-row group (naz_cnf_integrate_dopri5, one launch, no host sync)."""
        glob = self.step_control == "global"
        nfe = self._nfe_buffer(v, glob)
        fn = ops.cnf_integrate_dopri5_global if glob else ops.cnf_integrate_dopri5
        y, ld = fn(desc, packed, v, noise, t0, t1, self.atol, self.rtol, self.max_steps, context=self._context,
                   ld_out=ld_buf, ld_mode=ld_mode, nfe=nfe)
        # a solve that hit max_steps before t1 writes a negative count (cnf.hip): its state and
        # log-det are from partway through the interval, so fail loudly (strict, the default)
        if self.strict and nfe.numel() and bool((nfe < 0).any()):
            bad = int((nfe < 0).sum())
            what = "the batch" if glob else f"{bad} of {nfe.numel()} 16-row groups"
            raise RuntimeError(f"naz_amd CNF dopri5: {what} reached max_steps="
                               f"{self.max_steps} before t1 (step size collapsed or non-finite state); "
                               "raise max_steps, loosen atol/rtol, or set strict=False to accept partial solves")
        return y, ld

    def _solve_walk(self, v, noise, t0, t1, ld_buf, ld_mode):
        """The per-layer solve (no fused kernel at this shape): rk4 or dopri5 with torchdyn's
        batch-global control over the walk's RHS (flows/cnf_adjoint.py)."""
        from .cnf_adjoint import walk_dopri5, walk_rk4
        walk = self._plan.walk()
        v = v.detach().contiguous()
        if self.solver == "dopri5":
            if self.step_control != "global":
                raise NotImplementedError("naz_amd CNF: step_control='group' needs the fused solve kernel; this "
                                          "shape runs the per-layer solve with torchdyn's batch-global control")
            y, ld, nfe = walk_dopri5(walk, v, self._context, noise, t0, t1, self.atol, self.rtol, self.max_steps)
            self.last_nfe = torch.tensor([nfe], device=v.device, dtype=torch.int32)
            if self.strict and nfe < 0:
                raise RuntimeError(f"naz_amd CNF dopri5: the batch reached max_steps={self.max_steps} before t1 "
                                   "(step size collapsed or non-finite state); raise max_steps, loosen atol/rtol, "
                                   "or set strict=False to accept partial solves")
        else:
            y, ld = walk_rk4(walk, v, self._context, noise, t0, t1, self.steps)
        if ld_buf is None:
            return y, ld
        if ld_mode == ops.LD_ROWSUM_ADD:
            ld_buf.add_(ld)
        elif ld_mode == ops.LD_ROWSUM_SUB:
            ld_buf.sub_(ld)
        else:
            ld_buf.copy_(ld)
        return y, ld_buf

    def _solve(self, v, t0, t1, ld_buf, ld_mode):
        if ld_buf is None and self._needs_graph(v):
            # (the in-place accumulating forms, _inverse_acc / _call_acc, serve the no-grad walk and
            # sample; their outputs are not differentiable)
            from .cnf_adjoint import CnfSolveFn
            ps = [t for lin in self._net.linears() for t in (lin.weight, lin.bias)]
            return CnfSolveFn.apply(v, self._context, self._noise(v), self, float(t0), float(t1), *ps)
        noise = self._noise(v)
        if not self._plan.fused:
            return self._solve_walk(v, noise, t0, t1, ld_buf, ld_mode)
        packed = self._plan.packed()  # may re-resolve the mode: read desc only after it
        if self.solver == "dopri5":
            return self._dopri5(self._plan.desc, packed, v, noise, t0, t1, ld_buf, ld_mode)
        return ops.cnf_integrate(self._plan.desc, packed, v, noise, t0, t1, self.steps,
                                 context=self._context, ld_out=ld_buf, ld_mode=ld_mode)

    def _nfe_buffer(self, v, glob=False):
        """RHS evaluations of the last dopri5 solve (``last_nfe``): one count for the batch
        (global step control) or one per 16-row group."""
        n = 1 if glob else (v.shape[0] + 15) // 16
        self.last_nfe = torch.empty(n, device=v.device, dtype=torch.int32)
        return self.last_nfe

    def _inverse(self, x):  # naz :91-95: integrate t 0 -> 1, cache int -tr J
        y, ld = self._solve(x, 0.0, 1.0, None, ops.LD_ROWSUM)
        self._cached_logdet = ld
        return y

    def _call(self, z):  # naz :97-102: integrate t 1 -> 0
        y, ld = self._solve(z, 1.0, 0.0, None, ops.LD_ROWSUM)
        self._cached_logdet = ld
        return y

    def log_abs_det_jacobian(self, x, y):
        return self._cached_logdet

    def _inverse_acc(self, y, lp):
        x, _ = self._solve(y, 0.0, 1.0, lp, ops.LD_ROWSUM_SUB)
        return x

    def _call_acc(self, x, ld):
        y, _ = self._solve(x, 1.0, 0.0, ld, ops.LD_ROWSUM_ADD)
        return y

    def _inv_ld(self, y):
        """The autograd walk's step (flows/distributions.py): x and the forward log-det, both
        differentiable through the solve (flows/cnf_adjoint.py)."""
        return self._solve(y, 0.0, 1.0, None, ops.LD_ROWSUM)


def _check_solver(solver, steps, step_control="global"):
    if step_control not in ("global", "group"):
        raise ValueError("step_control must be 'global' (torchdyn's batch step size) or 'group' (per 16 rows)")
    if solver not in ("rk4", "dopri5"):
        raise NotImplementedError(f"naz_amd CNF: solver {solver!r}: fixed-step 'rk4' (SURVEY.md §8d config 5) and "
                                  "adaptive 'dopri5' are built")
    if int(steps) < 1:
        raise ValueError("steps must be >= 1")


class FFJORDTransform(_FFJORDCore, TransformModule):
    """naz :70-106 FFJORDTransform(net, input_dim, solver, sensitivity, atol, rtol)."""

    domain = constraints.real_vector
    codomain = constraints.real_vector
    bijective = True

    def __init__(self, net, input_dim, solver="rk4", sensitivity="adjoint", atol=1e-4, rtol=1e-4, steps=8,
                 max_steps=1000, strict=True, adjoint_steps=16, step_control="global"):
        super().__init__()
        _check_solver(solver, steps, step_control)
        self.step_control = step_control
        self.net, self.input_dim, self.steps = net, input_dim, int(steps)
        self.solver, self.sensitivity, self.atol, self.rtol = solver, sensitivity, atol, rtol
        self.max_steps = int(max_steps)
        self.strict = bool(strict)
        self.adjoint_steps = int(adjoint_steps)
        self.last_nfe = None
        self._plan = _CnfPlan(net)
        self._cached_logdet = None
        self._context = None
        self.noise: Optional[torch.Tensor] = None

    @property
    def _net(self):
        return self.net

    def __hash__(self):
        return nn.Module.__hash__(self)


class _ConditionedFFJORD(_FFJORDCore, Transform):
    domain = constraints.real_vector
    codomain = constraints.real_vector
    bijective = True

    def __init__(self, module: "ConditionalFFJORDTransform", context):
        super().__init__(cache_size=0)
        self.module, self._context = module, context
        self._cached_logdet = None

    @property
    def _net(self):
        return self.module.net

    @property
    def _plan(self):
        return self.module._plan

    @property
    def steps(self):
        return self.module.steps

    @property
    def noise(self):
        return self.module.noise

    def __getattr__(self, name):  # solver settings live on the module
        if name in ("solver", "atol", "rtol", "max_steps", "strict", "adjoint_steps", "step_control"):
            return getattr(self.module, name)
        raise AttributeError(name)


class ConditionalFFJORDTransform(ConditionalTransformModule):
    """naz :109-121.  ``condition(ctx)`` returns a conditioned transform instead of naz's
    monkey-patch of the vector field's ``forward``."""

    def __init__(self, net, input_dim, context_dim, solver="rk4", sensitivity="adjoint", atol=1e-4, rtol=1e-4,
                 steps=8, max_steps=1000, strict=True, adjoint_steps=16, step_control="global"):
        super().__init__()
        _check_solver(solver, steps, step_control)
        self.step_control = step_control
        self.net, self.input_dim, self.context_dim, self.steps = net, input_dim, context_dim, int(steps)
        self.solver, self.sensitivity, self.atol, self.rtol = solver, sensitivity, atol, rtol
        self.max_steps = int(max_steps)
        self.strict = bool(strict)
        self.adjoint_steps = int(adjoint_steps)
        self._plan = _CnfPlan(net)
        self.noise: Optional[torch.Tensor] = None

    def condition(self, context):
        return _ConditionedFFJORD(self, context)


def continuous_free_form(input_dim, condition_dim, hidden_dims, num_blocks, activation=nn.Softplus(),
                         use_batchnorm=False, dropout_p=None, **kwargs):
    """naz/flows/continuous_transforms.py:124-139."""
    if use_batchnorm:
        raise NotImplementedError("naz_amd: use_batchnorm is outside the log_prob hot path (SURVEY.md §8)")
    hidden_dims = list(hidden_dims) if isinstance(hidden_dims, (list, tuple)) else [hidden_dims]
    nets, transforms = [], []
    for _ in range(num_blocks):
        if condition_dim == 0:
            net = FCNN(input_dim, hidden_dims, act=activation, dropout_p=dropout_p)
            transform = FFJORDTransform(net, input_dim, **kwargs)
        else:
            net = ConditionalFCNN(input_dim, condition_dim, hidden_dims, act=activation, dropout_p=dropout_p)
            transform = ConditionalFFJORDTransform(net, input_dim, condition_dim, **kwargs)
        nets.append(net)
        transforms.append(transform)
    flow = (ComposeTransformModule(transforms) if condition_dim <= 0 else
            ConditionalComposeTransformModule(transforms))
    return flow, transforms, nets
