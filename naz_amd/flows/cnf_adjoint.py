"""Gradients through a FFJORD block solve: the CNF training step.

naz trains its continuous flows with torchdyn ``NeuralODE(..., sensitivity='adjoint')``
(naz/flows/continuous_transforms.py:73-82) through ``train`` / ``train_lightning``
(naz/trainers/train_flows.py:194-213, :244-278): the loss is -log_prob, whose CNF part is the
augmented solve d[x, a]/dt = [f(x, ctx), -eps^T (df/dx) eps] (hutch_trace, :85-89).

``CnfSolveFn`` is that solve as one autograd node.

* Forward: the fused solve kernels (csrc/cnf.hip).  For ``solver='rk4'`` one ``naz_cnf_integrate``
  launch per step, so the step-start states x_n are kept as checkpoints (B x D floats each);
  for ``'dopri5'`` the adaptive kernel, keeping only x(t1).
* Backward, rk4 (``sensitivity`` 'adjoint' or 'autograd'): the discrete adjoint of the pinned RK4
  solve, i.e. exactly the gradient of what the forward computed.  Per step, last to first: the
  four stages are recomputed from the checkpoint, then the step's adjoint recursion runs in
  reverse (g_k4 = h/6 lam, g_k3 = h/3 lam + h g_z4, g_k2 = h/3 lam + h/2 g_z3,
  g_k1 = h/6 lam + h/2 g_z2; lam <- lam + sum g_z; the log-det's adjoint mu = dL/da is constant
  because the RHS does not read a).  Memory is one step's activations, as with an adjoint solve.
* Backward, dopri5: torchdyn's continuous adjoint — the system [x, lam, theta_bar] integrated from
  t1 back to t0 (dx/dt = f, dlam/dt = -(lam^T df/dx + mu d(-tr)/dx), dtheta_bar/dt = -(lam^T df/dtheta +
  mu d(-tr)/dtheta)) with ``adjoint_steps`` fixed RK4 steps (x reconstructed backwards in time, as
  torchdyn does).  Its gradient approximates the continuous one, not the forward's step sequence.

Every RHS evaluation and VJP is HIP (``CnfWalk``): per hidden layer the value GEMM with its
bias + activation epilogue (``naz_linear_act``) and the tangent GEMM with the act' epilogue
(``naz_gemm_dact``), kept as (value, tangent) row pairs (2B rows); the VJP is the input-adjoint
GEMM with the activation's VJP in its epilogue (``naz_gemm_jvp_bwd``: value rows need act''
because the tangent reads pre through act'; both derivatives come from h), ``naz_gemm`` for the
2B-row dW reductions and ``naz_colsum`` for the bias gradients.  Torch only forms the [B, D]-sized
RK4 combinations.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
from torch.autograd import Function

from .. import ops


def _pairs(B: int, N: int, like: torch.Tensor) -> torch.Tensor:
    """[B, 2 Np] storage of (value, tangent) row pairs, Np = N padded to 16 bytes, returned as its
    [2B, N] view: row 2i = value of batch row i, row 2i + 1 = its tangent."""
    npad = (N + 3) // 4 * 4
    t = torch.empty((2 * B, npad), device=like.device, dtype=like.dtype)
    return t[:, :N] if npad != N else t


# The weight / bias gradient reductions of a VJP only read its adjoints and saved activations, so they
# run on a side stream beside the next layer's input-adjoint GEMM (NAZ_CNF_DW_STREAM, default on); the
# caller joins with _join_reductions before reading the gradients.
_DW_STREAM = os.environ.get("NAZ_CNF_DW_STREAM", "1") == "1"
_SIDE = {}


def _reductions(dev):
    """fn(fn, *tensors_read): run fn on the device's reduction stream after everything the current
    stream has queued (the tensors it reads are kept from the allocator until it is done), or inline."""
    if not (_DW_STREAM and dev.type == "cuda"):
        return lambda fn, *ts: fn()
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i not in _SIDE:
        _SIDE[i] = torch.cuda.Stream(dev)
    side, main = _SIDE[i], torch.cuda.current_stream(dev)

    def run(fn, *ts):
        ev = torch.cuda.Event()
        ev.record(main)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            fn()
        for t in ts:
            t.record_stream(side)
    return run


_PREFETCH = os.environ.get("NAZ_CNF_PREFETCH", "1") == "1"


def _prefetch_stream(dev):
    if not (_PREFETCH and dev.type == "cuda"):
        return None
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if (i, 1) not in _SIDE:
        _SIDE[(i, 1)] = torch.cuda.Stream(dev)
    return _SIDE[(i, 1)]


def _join_reductions(dev) -> None:
    i = dev.index if dev.index is not None else (torch.cuda.current_device() if dev.type == "cuda" else None)
    if dev.type == "cuda" and i in _SIDE:
        torch.cuda.current_stream(dev).wait_stream(_SIDE[i])


class CnfWalk:
    """The FFJORD vector field (ConditionalFCNN, naz continuous_transforms.py:38-60, input
    cat([x, ctx]), x first) with its Hutchinson JVP, evaluated layer by layer on HIP kernels.

    Hidden layer i keeps S_i as (value, tangent) row pairs [2B, H] (row 2r = h_i, 2r + 1 = dh_i of
    batch row r): h_i = act(W_i h + b_i) by naz_linear_act (activation epilogue) written to the
    even rows, dh_i = act'(pre) ⊙ (W_i dh) by naz_gemm_dact (act' from h_i in the epilogue) to the
    odd rows.  The VJP needs nothing else: act' and act''/act' are functions of h_i, applied in the
    input-adjoint GEMM's epilogue (naz_gemm_jvp_bwd)."""

    def __init__(self, net):
        lins = net.linears()
        self.W = [lin.weight.detach() for lin in lins]
        self.b = [lin.bias.detach() for lin in lins]
        self.act = net.act
        self.D, self.C = D, C = net.input_dim, net.context_dim
        W0 = self.W[0]
        # naz_linear_act concatenates [ctx | x]; the CNF input is [x | ctx]: reorder W0's columns
        self.W0_cx = torch.cat([W0[:, D:], W0[:, :D]], 1).contiguous() if C else W0.contiguous()
        self.WT = [W0[:, :D].t().contiguous()] + [W.t().contiguous() for W in self.W[1:]]  # tangent GEMMs

    def rhs(self, z: torch.Tensor, ctx: Optional[torch.Tensor], eps: torch.Tensor):
        """(f(z), -eps^T J eps, saved activations) for z [B, D]."""
        B, n = z.shape[0], len(self.W)
        saved = [z]
        h, dh = None, eps
        for i in range(n - 1):
            S = _pairs(B, self.W[i].shape[0], z)
            hv, tv = S[0::2], S[1::2]  # [B, H] views at row stride 2 Np
            if i == 0:
                ops.linear_act(z, self.W0_cx, self.b[0], self.act, context=ctx if self.C else None, out=hv)
            else:
                ops.linear_act(h, self.W[i], self.b[i], self.act, out=hv)
            ops.gemm_dact(dh, self.WT[i], hv, self.act, out=tv)
            h, dh = hv, tv
            saved.append(S)
        k = ops.linear_act(h, self.W[-1], self.b[-1])
        jv = ops.gemm(dh, self.WT[-1])
        t = -(eps * jv).sum(1)
        return k, t, saved

    def vjp(self, saved: List[torch.Tensor], ctx: Optional[torch.Tensor], eps: torch.Tensor, g_k: torch.Tensor,
            g_t: torch.Tensor, gW: List[torch.Tensor], gb: List[torch.Tensor], g_ctx: Optional[torch.Tensor]):
        """Adjoints (g_k, g_t) of (f, -tr) at the point ``rhs`` saved -> returns g_z [B, D];
        accumulates the weight / bias gradients into gW / gb and the context's into g_ctx."""
        B, D, C, n = g_k.shape[0], self.D, self.C, len(self.W)
        z = saved[0]
        G = _pairs(B, D, g_k)  # output adjoints in row pairs: (g_f, g_(J eps)) = (g_k, -g_t eps)
        G[0::2] = g_k
        G[1::2] = -g_t[:, None] * eps
        red = _reductions(g_k.device)
        red(lambda G=G: (ops.gemm(G.t(), saved[-1], out=gW[-1], accumulate=True), ops.colsum(g_k, out=gb[-1])),
            G, g_k, saved[-1])
        W_next = self.W[-1]
        for i in reversed(range(n - 1)):
            GP = ops.gemm_jvp_bwd(G, W_next, saved[i + 1], self.act)  # pre-activation adjoints, pairs
            if i > 0:
                red(lambda GP=GP, i=i: (ops.colsum(GP[0::2], out=gb[i]),
                                        ops.gemm(GP.t(), saved[i], out=gW[i], accumulate=True)), GP, saved[i])
                G, W_next = GP, self.W[i]
                continue
            ops.colsum(GP[0::2], out=gb[i])
            S0 = torch.zeros((2 * B, D + C), device=z.device, dtype=z.dtype)  # pairs ([z, ctx], [eps, 0])
            S0[0::2, :D] = z
            S0[1::2, :D] = eps
            if C:
                S0[0::2, D:] = ctx.reshape(-1, C).expand(B, C) if ctx.numel() == C else ctx
            ops.gemm(GP.t(), S0, out=gW[0], accumulate=True)
            GPv = GP[0::2]  # the tangent rows' input is eps (no gradient)
            g_z = ops.gemm(GPv, self.W[0][:, :D])
            if C and g_ctx is not None:
                Wc = self.W[0][:, D:]
                if g_ctx.shape[0] == B and g_ctx.dim() == 2:
                    ops.gemm(GPv, Wc, out=g_ctx, accumulate=True)
                else:
                    ops.gemm(ops.colsum(GPv).reshape(1, -1), Wc, out=g_ctx.view(1, C), accumulate=True)
        return g_z


# ----------------------------------------------------------------------------- the per-layer solve
# The fused solve kernels (csrc/cnf.hip) hold the whole vector field in one CU's LDS; naz's POSYDON
# CNF (examples/papers/eposydon/train_cnf_mle.py:91, train_cnf_mle_q.py:92: D = 4, H = [128] x 4) does
# not fit (~200 KB of weights).  Every other shape integrates through the walk's RHS instead: per
# RHS one batch-row GEMM launch per layer for the values and one for the Hutchinson tangents (the
# same kernels as the backward), torch only for the [B, D] stage combinations.

def walk_rk4(walk: CnfWalk, x: torch.Tensor, ctx, eps: torch.Tensor, t0: float, t1: float, steps: int,
             checkpoints: Optional[list] = None):
    """Classical RK4 on the augmented state [x, a] (naz odeint.py:46-52, the config-5 pin) with the
    walk's RHS: returns (x(t1), a(t1) = int -eps^T J eps dt).  ``checkpoints`` receives each step's
    start state (the discrete adjoint's, as the fused forward keeps them)."""
    x = x.contiguous()
    a = torch.zeros(x.shape[0], device=x.device, dtype=torch.float32)
    h = (t1 - t0) / steps
    for _ in range(steps):
        if checkpoints is not None:
            checkpoints.append(x)
        f1, g1, _ = walk.rhs(x, ctx, eps)
        f2, g2, _ = walk.rhs(x + (0.5 * h) * f1, ctx, eps)
        f3, g3, _ = walk.rhs(x + (0.5 * h) * f2, ctx, eps)
        f4, g4, _ = walk.rhs(x + h * f3, ctx, eps)
        x = x + (h / 6.0) * (f1 + 2.0 * f2 + 2.0 * f3 + f4)
        a = a + (h / 6.0) * (g1 + 2.0 * g2 + 2.0 * g3 + g4)
    return x, a


# Dormand-Prince 5(4): naz's in-tree tableau (neural_nets/__deprecated__/neural_odes/odeint.py:136-160;
# rows a_ij, 5th-order weights b, error weights b - b*)
_DP5_A = [[1 / 5], [3 / 40, 9 / 40], [44 / 45, -56 / 15, 32 / 9], [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
          [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656]]
_DP5_B = [35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84]
_DP5_E = [35 / 384 - 5179 / 57600, 0.0, 500 / 1113 - 7571 / 16695, 125 / 192 - 393 / 640, -2187 / 6784 + 92097 / 339200,
          11 / 84 - 187 / 2100, -1 / 40]


def walk_dopri5(walk: CnfWalk, x: torch.Tensor, ctx, eps: torch.Tensor, t0: float, t1: float, atol: float,
                rtol: float, max_steps: int):
    """Adaptive Dormand-Prince 5(4) with torchdyn's batch-global control (naz FFJORDTransform
    solver='dopri5', continuous_transforms.py:73-81), the controller of
    naz_cnf_integrate_dopri5_global on the walk's RHS: ONE step size for the batch, error ratio =
    RMS over every element of [B, D + 1] of err / (atol + rtol max(|y0|, |y1|)), accept at <= 1,
    h *= clamp(0.9 r^(-1/5), 0.2 (1 on accept), 10), Hairer's initial step, FSAL, the last step
    clipped to t1.  The controller reads one scalar per attempt back to the host (torchdyn's is
    host-driven too).  Returns (x(t1), a(t1), nfe) with nfe < 0 when max_steps ran out."""
    y = x.contiguous()
    B = y.shape[0]
    a = torch.zeros(B, device=y.device, dtype=torch.float32)
    n_el = float(B * (y.shape[1] + 1))
    direction = 1.0 if t1 > t0 else -1.0

    def f(v):
        k, g, _ = walk.rhs(v, ctx, eps)
        return k, g

    def rms(u, ua):
        return float(torch.sqrt(((u.double() ** 2).sum() + (ua.double() ** 2).sum()) / n_el))

    k0, k0a = f(y)
    sc, sca = atol + rtol * y.abs(), atol + rtol * a.abs()
    d0, d1 = rms(y / sc, a / sca), rms(k0 / sc, k0a / sca)
    h0 = 1e-6 if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
    f1, f1a = f(y + (direction * h0) * k0)
    d2 = rms((f1 - k0) / sc, (f1a - k0a) / sca) / h0
    h1 = max(1e-6, h0 * 1e-3) if max(d1, d2) <= 1e-15 else (0.01 / max(d1, d2)) ** (1.0 / 6.0)
    h = min(100 * h0, h1)
    nfe, t, steps = 2, t0, 0
    while steps < max_steps and t != t1:
        rem = abs(t1 - t)
        last = h >= rem
        hh = direction * (rem if last else h)
        ks, kas = [k0], [k0a]
        for row in _DP5_A:
            ki, kia = f(y + hh * sum(c * k for c, k in zip(row, ks)))
            ks.append(ki)
            kas.append(kia)
        y5 = y + hh * sum(c * k for c, k in zip(_DP5_B, ks) if c != 0.0)
        a5 = a + hh * sum(c * k for c, k in zip(_DP5_B, kas) if c != 0.0)
        k6, k6a = f(y5)
        ks.append(k6)
        kas.append(k6a)
        err = hh * sum(c * k for c, k in zip(_DP5_E, ks) if c != 0.0)
        erra = hh * sum(c * k for c, k in zip(_DP5_E, kas) if c != 0.0)
        en = rms(err / (atol + rtol * torch.maximum(y.abs(), y5.abs())),
                 erra / (atol + rtol * torch.maximum(a.abs(), a5.abs())))
        nfe += 6
        if en <= 1.0:
            y, a, k0, k0a = y5, a5, k6, k6a
            t = t1 if last else t + hh
        factor = 10.0 if en == 0 else min(10.0, max(0.9 / en ** 0.2, 1.0 if en <= 1.0 else 0.2))
        h = abs(hh) * factor
        steps += 1
    return y, a, (nfe if t == t1 else -nfe)


def _rk4_stages(walk, x, ctx, eps, h):
    """The four RK4 stages' saved activations of one step from checkpoint x (naz odeint.py:46-52)."""
    k1, _, s1 = walk.rhs(x, ctx, eps)
    k2, _, s2 = walk.rhs(x + 0.5 * h * k1, ctx, eps)
    k3, _, s3 = walk.rhs(x + 0.5 * h * k2, ctx, eps)
    _, _, s4 = walk.rhs(x + h * k3, ctx, eps)
    return s1, s2, s3, s4


def _rk4_step_adjoint(walk, x, ctx, eps, h, lam, mu, gW, gb, g_ctx, stages=None):
    """Discrete adjoint of one classical RK4 step from checkpoint x (naz odeint.py:46-52); ``stages``:
    the step's recomputed stages when the caller already has them."""
    s1, s2, s3, s4 = _rk4_stages(walk, x, ctx, eps, h) if stages is None else stages
    del stages
    w1, w2 = h / 6.0, h / 3.0
    gz4 = walk.vjp(s4, ctx, eps, w1 * lam, w1 * mu, gW, gb, g_ctx)
    del s4
    gz3 = walk.vjp(s3, ctx, eps, w2 * lam + h * gz4, w2 * mu, gW, gb, g_ctx)
    del s3
    gz2 = walk.vjp(s2, ctx, eps, w2 * lam + 0.5 * h * gz3, w2 * mu, gW, gb, g_ctx)
    del s2
    gz1 = walk.vjp(s1, ctx, eps, w1 * lam + 0.5 * h * gz2, w1 * mu, gW, gb, g_ctx)
    return lam + gz1 + gz2 + gz3 + gz4


def _continuous_adjoint(walk, y1, ctx, eps, t0, t1, steps, lam, mu, gW, gb, g_ctx):
    """torchdyn-style adjoint: RK4 on [x, lam, theta_bar] from t1 back to t0."""
    h = (t0 - t1) / steps
    x = y1

    def stage(xs, ls, c):
        # derivative of [x, lam, theta_bar]: (f, -g_z, -g_theta); the parameter / context part is
        # accumulated directly with its RK4 weight c (the VJP is linear in its adjoint inputs)
        k, _, sv = walk.rhs(xs, ctx, eps)
        gz = walk.vjp(sv, ctx, eps, -c * ls, -c * mu, gW, gb, g_ctx)
        return k, gz / c

    for _ in range(steps):
        k1, d1 = stage(x, lam, h / 6.0)
        k2, d2 = stage(x + 0.5 * h * k1, lam + 0.5 * h * d1, h / 3.0)
        k3, d3 = stage(x + 0.5 * h * k2, lam + 0.5 * h * d2, h / 3.0)
        k4, d4 = stage(x + h * k3, lam + h * d3, h / 6.0)
        x = x + h / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)
        lam = lam + h / 6.0 * (d1 + 2 * d2 + 2 * d3 + d4)
    return lam


class CnfSolveFn(Function):
    """(y, ld) = FFJORD block solve of v from t0 to t1 (ld = int -eps^T J eps dt), differentiable
    in v, the context and the vector field's parameters (see the module docstring)."""

    @staticmethod
    def forward(ctx, v, context, eps, core, t0: float, t1: float, *params):
        plan = core._plan
        v = v.detach().contiguous()
        if not plan.fused:  # the per-layer solve (no fused kernel at this shape)
            if core.solver == "dopri5":
                y, ld = core._solve_walk(v, eps, t0, t1, None, ops.LD_ROWSUM)
                ctx.checkpoints = None
                ctx.save_for_backward(y, eps, context)
            else:
                xs: list = []
                y, ld = walk_rk4(plan.walk(), v, context, eps, t0, t1, core.steps, checkpoints=xs)
                ctx.checkpoints = len(xs)
                ctx.save_for_backward(eps, context, *xs)
            ctx.core, ctx.t0, ctx.t1 = core, t0, t1
            return y, ld
        packed = plan.packed()
        desc = plan.desc
        if core.solver == "dopri5":
            y, ld = core._dopri5(desc, packed, v, eps, t0, t1, None, ops.LD_ROWSUM)
            ctx.checkpoints = None
            ctx.save_for_backward(y, eps, context)
        else:
            steps = core.steps
            ld = torch.zeros(v.shape[0], device=v.device, dtype=torch.float32)
            xs = [v]
            dt = (t1 - t0) / steps
            for n in range(steps):
                y, _ = ops.cnf_integrate(desc, packed, xs[-1], eps, t0 + n * dt, t0 + (n + 1) * dt, 1,
                                         context=context, ld_out=ld, ld_mode=ops.LD_ROWSUM_ADD)
                xs.append(y)
            ctx.checkpoints = len(xs) - 1
            ctx.save_for_backward(eps, context, *xs[:-1])
        ctx.core, ctx.t0, ctx.t1 = core, t0, t1
        return y, ld

    @staticmethod
    def backward(ctx, g_y, g_ld):
        core, t0, t1 = ctx.core, ctx.t0, ctx.t1
        saved = ctx.saved_tensors
        walk = CnfWalk(core._net)
        if ctx.checkpoints is None:
            y1, eps, context = saved
            B = y1.shape[0]
        else:
            eps, context = saved[0], saved[1]
            xs = saved[2:]
            B = xs[0].shape[0]
        dev = eps.device
        lam = torch.zeros((B, walk.D), device=dev) if g_y is None else g_y.contiguous().clone()
        mu = torch.zeros(B, device=dev) if g_ld is None else g_ld.contiguous()
        gW = [torch.zeros_like(W) for W in walk.W]
        gb = [torch.zeros_like(b) for b in walk.b]
        need_c = context is not None and ctx.needs_input_grad[1]
        g_ctx = torch.zeros(context.shape, device=dev) if need_c else None
        if g_ctx is not None and g_ctx.dim() == 1:
            g_ctx = g_ctx.reshape(1, -1)
        if B:
            if ctx.checkpoints is None:
                lam = _continuous_adjoint(walk, y1, context, eps, t0, t1, core.adjoint_steps, lam, mu, gW, gb, g_ctx)
            else:
                h = (t1 - t0) / ctx.checkpoints
                # the next (earlier) step's forward recompute on its own stream while this step's
                # VJPs run: the recompute reads only its checkpoint (NAZ_CNF_PREFETCH, default on)
                rec = _prefetch_stream(dev)
                main = torch.cuda.current_stream(dev) if rec is not None else None
                nxt = None
                for n in reversed(range(ctx.checkpoints)):
                    stages, nxt = nxt, None
                    if rec is not None and n > 0:
                        ev = torch.cuda.Event()
                        ev.record(main)
                        rec.wait_event(ev)
                        with torch.cuda.stream(rec):
                            nxt = _rk4_stages(walk, xs[n - 1], context, eps, h)
                        done = torch.cuda.Event()
                        done.record(rec)
                    lam = _rk4_step_adjoint(walk, xs[n], context, eps, h, lam, mu, gW, gb, g_ctx, stages=stages)
                    if nxt is not None:
                        main.wait_event(done)
                        for sv in nxt:  # made on the prefetch stream, read on this one
                            for t in sv:
                                t.record_stream(main)
        _join_reductions(dev)
        if g_ctx is not None:
            g_ctx = g_ctx.reshape(context.shape)
        grads = [t for pair in zip(gW, gb) for t in pair]
        return (lam if ctx.needs_input_grad[0] else None, g_ctx, None, None, None, None, *grads)
