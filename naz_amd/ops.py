"""Torch-facing wrappers of the HIP kernels (the only compute path of naz_amd).

Tensors must be fp32 on a HIP device (``torch.device("cuda")`` on PyTorch-ROCm);
outputs are allocated here, kernels are launched on the current stream of the
input's device.  Row strides are passed through, so contiguous-last-dim views work
without copies.
"""
from __future__ import annotations

import ctypes as C
import weakref
from typing import List, Optional, Tuple

import numpy as np
import torch

from ._lib import (ACT, FLOW_AR, FLOW_COUPLING, LAYOUT_ARN, LAYOUT_DENSE, RQS_FAST, LD_PERDIM, LD_ROWSUM, LD_ROWSUM_ADD,
                   LD_ROWSUM_SUB, ArDesc, CnfDesc, CouplingDesc, FlowDesc, check, lib)

Tensor = torch.Tensor

__all__ = ["rqs", "rqs_bwd", "spline_elementwise", "linear_act", "linear_act_batched", "made_packed_floats", "made_affine_fwd", "made_affine_inv1", "gemm_dact", "affine_ar", "affine_ar_bwd", "base_log_prob",
           "base_log_prob_bwd", "gemm", "colsum", "act_bwd", "bounding_fwd", "bounding_inv",
           "coupling_desc", "coupling_supported", "coupling_param_count", "coupling_pack", "coupling_log_prob",
           "coupling_sample", "cnf_desc", "cnf_supported", "cnf_param_count", "cnf_pack", "cnf_integrate", "cnf_integrate_dopri5", "cnf_integrate_dopri5_global", "gemm_jvp_bwd", "flow_desc", "flow_log_prob", "flow_sample",
           "LAYOUT_ARN", "LAYOUT_DENSE", "LD_PERDIM", "LD_ROWSUM", "LD_ROWSUM_ADD",
           "LD_ROWSUM_SUB"]


def _dev(*ts: Optional[Tensor]) -> torch.device:
    dev = None
    for t in ts:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError(f"naz_amd kernels run on the GPU only; got a tensor on {t.device} "
                               "(no CPU fallback exists)")
        if t.dtype != torch.float32:
            raise TypeError(f"naz_amd kernels compute in float32; got {t.dtype}")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError("naz_amd: tensors on different devices")
    return dev


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _rows(t: Tensor) -> Tuple[Tensor, int]:
    """2-D view with unit last-dim stride; returns (tensor, row stride)."""
    if t.dim() != 2:
        raise ValueError(f"expected a 2-D tensor, got shape {tuple(t.shape)}")
    if t.stride(1) != 1:
        t = t.contiguous()
    return t, t.stride(0)


def _p(t: Optional[Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


_WS: dict = {}
_WS_PER_DEVICE = 4  # streams whose workspace is kept per device (least recently used dropped first)


def workspace(dev: torch.device, nbytes: int) -> Tuple[Optional[int], int]:
    """Caller-owned device workspace of the autoregressive log_prob entries (include/naz_hip.h
    naz_ar_flow_workspace_bytes: the wide MAF inverse's per-wave hidden layers; no entry allocates):
    one buffer per (device, stream), grown on demand and kept, so a captured HIP graph replays one
    fixed address.  Returns (pointer, bytes) for the call.

    The key is the device INDEX ('cuda' and 'cuda:0' are one device) and the stream; at most
    _WS_PER_DEVICE streams keep a buffer per device.  Dropping the least recently used one is safe:
    the caching allocator reuses a freed block only for allocations on the stream it was allocated
    on (here: the stream it served), so later work is ordered after the dropped buffer's last use."""
    if nbytes <= 0:
        return None, 0
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (idx, _stream(dev))
    buf = _WS.pop(key, None)  # re-inserted below: dict order = recency
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(nbytes, dtype=torch.uint8, device=torch.device("cuda", idx))
    _WS[key] = buf
    mine = [k for k in _WS if k[0] == idx]
    for k in mine[:max(0, len(mine) - _WS_PER_DEVICE)]:
        del _WS[k]
    return buf.data_ptr(), buf.numel()


def absmax(*ts: Optional[Tensor]) -> float:
    """max |t| over the given tensors (None / empty skipped) as a host float: the fused kernels'
    f16-split range check.  One reduction pass per tensor (an inf-norm) with no |t| temporary —
    r06 PMC: x.abs().amax() wrote and re-read a full |x| copy, 100 of the 348 MB per nsa16 call."""
    m = None
    for t in ts:
        if t is None or t.numel() == 0:
            continue
        v = torch.linalg.vector_norm(t.detach(), float("inf"))
        m = v if m is None else torch.maximum(m, v)
    return 0.0 if m is None else float(m)


def rowgemm_split(value: Optional[bool] = None) -> bool:
    """The batch-row GEMM's panel split (naz_tuning "rowgemm_split": outputs wider than 128 columns
    as balanced panels of at most 128; no result changes).  ``value`` sets it; returns the setting
    before."""
    r = int(lib().naz_tuning(b"rowgemm_split", -1 if value is None else int(bool(value))))
    if r < 0:
        check(r, "rowgemm_split")
    return bool(r)


def rowgemm_h3(value: Optional[bool] = None) -> bool:
    """The batch-row GEMM's f16x3 form (naz_tuning "rowgemm_h3": A rows split at a per-row
    power-of-two scale, B at 2^6, three products on the f16 matrix pipe; fp32-grade, other rounding).
    The caller keeps |B| < 2^9 while it is on.  ``value`` sets it; returns the setting before."""
    r = int(lib().naz_tuning(b"rowgemm_h3", -1 if value is None else int(bool(value))))
    if r < 0:
        check(r, "rowgemm_h3")
    return bool(r)


def rowgemm_bres(value: Optional[bool] = None) -> bool:
    """The batch-row GEMM's B-resident f16x3 form (naz_tuning "rowgemm_bres": a persistent workgroup
    keeps its column panel of B split into f16 pieces in LDS, A rows split at per-row power-of-two
    scales; fp32-grade, other rounding).  ``value`` sets it; returns the setting before."""
    r = int(lib().naz_tuning(b"rowgemm_bres", -1 if value is None else int(bool(value))))
    if r < 0:
        check(r, "rowgemm_bres")
    return bool(r)


def rowgemm_fill(value: Optional[int] = None) -> int:
    """The batch-row GEMM's small-batch grid fill (naz_tuning "rowgemm_fill": column panels narrowed
    until the grid holds ``value`` workgroups per CU, 0 = off; no result changes).  Returns the
    setting before."""
    r = int(lib().naz_tuning(b"rowgemm_fill", -1 if value is None else int(value)))
    if r < 0:
        check(r, "rowgemm_fill")
    return r


def _release_image(ptr: int) -> None:
    lib().naz_image_release(ptr)  # (an image packed over it since has replaced the record: no-op)


def track_image(img: Tensor) -> Tensor:
    """Forget the library's registry record of a packed image when its tensor is freed: the caching
    allocator hands the memory to the next tensor, which must not pass for an image."""
    if not getattr(img, "_naz_tracked", False):
        weakref.finalize(img, _release_image, img.data_ptr()).atexit = False
        img._naz_tracked = True
    return img


def rowgemm_x6(value: Optional[bool] = None) -> bool:
    """The batch-row GEMM's arithmetic (naz_tuning "rowgemm_x6"): exact FP32 MFMA (False) or the
    exact bf16x6 split on the bf16 matrix pipe (True; fp32-grade, 2.67x the FP32 MFMA rate).
    ``value`` sets it; returns the setting before."""
    r = int(lib().naz_tuning(b"rowgemm_x6", -1 if value is None else int(bool(value))))
    if r < 0:
        check(r, "rowgemm_x6")
    return bool(r)


def attach_image(img: Tensor, what: str) -> Tensor:
    """Register a host-packed image copied to the device (naz_image_attach reads its header once)."""
    check(lib().naz_image_attach(_p(img), img.numel() * img.element_size(), _stream(img.device)), what)
    return track_image(img)


# ----------------------------------------------------------------------------- a1 + a2
def rqs(x: Tensor, raw: Tensor, count_bins: int, layout: int = LAYOUT_DENSE, inverse: bool = False,
        bound: float = 3.0, ld_mode: int = LD_PERDIM, ld_out: Optional[Tensor] = None,
        out: Optional[Tensor] = None, broadcast_raw: bool = False, fast: bool = False) -> Tuple[Tensor, Tensor]:
    """Conditional RQ spline over a conditioner output (naz_rqs_fwd / naz_rqs_inv).

    ``out`` may be a strided 2-D view (unit last stride) to write into; ``broadcast_raw``
    passes a single parameter row (row stride 0) shared by every batch row, which is how
    the unconditional lower spline of a coupling layer runs.  ``fast`` selects the
    select-first hardware-math evaluator (NAZ_RQS_FAST; fp32-grade, HBM-bound) instead of
    the libm-grade one that ``rqs_bwd``'s VJP matches (the autograd walk keeps the latter)."""
    dev = _dev(x, raw, ld_out, out)
    x, ldx = _rows(x)
    B, Dt = x.shape
    P = Dt * (3 * count_bins - 1)
    if broadcast_raw:
        raw = raw.reshape(1, -1).contiguous()
        ldr = 0
        if raw.shape[1] != P:
            raise ValueError(f"broadcast raw must have {P} entries, got {raw.shape[1]}")
    else:
        raw, ldr = _rows(raw)
        if raw.shape != (B, P):
            raise ValueError(f"raw must be [B, Dt*(3K-1)] = {(B, P)}, got {tuple(raw.shape)}")
    if out is None:
        out = torch.empty_like(x)
    elif out.shape != (B, Dt) or out.stride(1) != 1:
        raise ValueError("out must be a [B, Dt] view with unit last stride")
    if ld_out is None:
        ld_out = torch.empty((B, Dt) if ld_mode == LD_PERDIM else (B,), device=dev, dtype=torch.float32)
    fn = lib().naz_rqs_inv if inverse else lib().naz_rqs_fwd
    check(fn(_p(x), ldx, _p(raw), ldr, _p(out), out.stride(0), _p(ld_out), ld_mode, B, Dt, count_bins,
             layout | (RQS_FAST if fast else 0), float(bound), _stream(dev)), "rqs")
    return out, ld_out


def spline_elementwise(x: Tensor, uw: Tensor, uh: Tensor, ud: Tensor, inverse: bool = False,
                       bound: float = 3.0) -> Tuple[Tensor, Tensor]:
    """Unconditional elementwise spline ([pyro] Spline); returns (y, per-dim ld)."""
    dev = _dev(x, uw, uh, ud)
    x, ldx = _rows(x)
    B, Dt = x.shape
    K = uw.shape[-1]
    uw, uh, ud = uw.contiguous(), uh.contiguous(), ud.contiguous()
    y = torch.empty_like(x)
    ld = torch.empty((B, Dt), device=dev, dtype=torch.float32)
    check(lib().naz_spline_elementwise(int(inverse), _p(x), ldx, _p(uw), _p(uh), _p(ud), _p(y), y.stride(0), _p(ld),
                                       B, Dt, K, float(bound), _stream(dev)), "spline_elementwise")
    return y, ld


# ----------------------------------------------------------------------------- a6 / a7
def linear_act(x: Optional[Tensor], weight: Tensor, bias: Optional[Tensor], act: str = "identity",
               context: Optional[Tensor] = None, mask: Optional[Tensor] = None,
               out: Optional[Tensor] = None) -> Tensor:
    """act(cat([context, x]) @ (weight * mask)^T + bias) with the concat fused."""
    dev = _dev(x, weight, bias, context, mask)
    C = 0 if context is None else context.shape[-1]
    Kx = 0 if x is None else x.shape[-1]
    M = x.shape[0] if x is not None else context.shape[0]
    ldc = 0
    if context is not None:
        if context.dim() == 1 or context.shape[0] == 1 and M != 1:
            context = context.reshape(1, -1).contiguous()
            ldc = 0  # broadcast one context row
        else:
            context, ldc = _rows(context)
            if context.shape[0] != M:
                raise ValueError("context rows must match x rows (or be a single row)")
    ldx = 0
    if x is not None:
        x, ldx = _rows(x)
    N = weight.shape[0]
    if weight.shape[1] != C + Kx:
        raise ValueError(f"weight must be [N, {C + Kx}], got {tuple(weight.shape)}")
    weight = weight.contiguous()
    if mask is not None:
        mask = mask.to(torch.float32).contiguous()
    if out is None:
        # rows padded to 16 bytes: the batch-row kernels then use 16-byte loads/stores on this
        # activation here and in the next layer (the [M, N] view is what callers see)
        npad = (N + 3) // 4 * 4
        out = torch.empty((M, npad), device=dev, dtype=torch.float32)[:, :N] if npad != N else \
            torch.empty((M, N), device=dev, dtype=torch.float32)
    check(lib().naz_linear_act(_p(context), ldc, C, _p(x), ldx, Kx, _p(weight), _p(mask), _p(bias), _p(out),
                               out.stride(0), M, N, ACT[act], _stream(dev)), "linear_act")
    return out


def linear_act_batched(x: Optional[Tensor], weight: Tensor, bias: Optional[Tensor], act: str = "identity",
                       context: Optional[Tensor] = None, mask: Optional[Tensor] = None,
                       out: Optional[Tensor] = None) -> Tensor:
    """Per-draw conditioner layer (naz_linear_act_batched):
    out[z] = act(cat([context[z], x[z]]) @ (weight[z] * mask)^T + bias[z]) for z < P.

    x / out: [P, M, *] with unit column stride (any row stride, draw stride); weight [P, N, C+Kx]
    and bias [P, N] contiguous; context [C] / [M, C] (shared by every draw) or [P, M, C]."""
    dev = _dev(x, weight, bias, context, mask)
    P, N = weight.shape[0], weight.shape[1]
    C = 0 if context is None else context.shape[-1]
    Kx = 0 if x is None else x.shape[-1]
    M = x.shape[1] if x is not None else (context.shape[-2] if context.dim() >= 2 else 1)

    def _pm(t, what):  # (draw stride, row stride) of a [P, M, k] operand with unit column stride
        if t.stride(-1) != 1 or t.shape[:2] != (P, M):
            raise ValueError(f"{what} must be [P={P}, M={M}, *] with unit column stride, got "
                             f"{tuple(t.shape)} / {t.stride()}")
        return t.stride(0), t.stride(1)

    sctx = ldc = 0
    if context is not None:
        if context.dim() == 3:
            sctx, ldc = _pm(context, "context")
        else:
            context = context.reshape(-1, C).contiguous()
            if context.shape[0] not in (1, M):
                raise ValueError("context rows must match x rows (or be a single row)")
            ldc = 0 if context.shape[0] == 1 else C
    sx = ldx = 0
    if x is not None:
        sx, ldx = _pm(x, "x")
    if weight.shape != (P, N, C + Kx):
        raise ValueError(f"weight must be [P, N, {C + Kx}], got {tuple(weight.shape)}")
    weight = weight.contiguous()
    if bias is not None:
        if bias.shape != (P, N):
            raise ValueError(f"bias must be [P, N] = {(P, N)}, got {tuple(bias.shape)}")
        bias = bias.contiguous()
    if mask is not None:
        mask = mask.to(torch.float32).contiguous()
    if out is None:
        npad = (N + 3) // 4 * 4
        out = torch.empty((P, M, npad), device=dev, dtype=torch.float32)[:, :, :N]
    sy, ldy = _pm(out, "out")
    check(lib().naz_linear_act_batched(_p(context), ldc, sctx, C, _p(x), ldx, sx, Kx, _p(weight), N * (C + Kx),
                                       _p(mask), _p(bias), N, _p(out), ldy, sy, M, N, P, ACT[act], _stream(dev)),
          "linear_act_batched")
    return out


def made_packed_floats(nhid: int, nh: int, C: int, D: int) -> int:
    return int(lib().naz_made_packed_floats(nhid, nh, C, D))


def made_affine_fwd(packed: Tensor, nhid: int, nh: int, x: Tensor, context: Optional[Tensor], act: str,
                    ld: Tensor, ld_mode: int = LD_ROWSUM_ADD, out: Optional[Tensor] = None) -> Tensor:
    """Fused MADE conditioner + affine forward step for P draws (naz_made_affine_fwd):
    packed [P, n] (``flows.bflow_maf`` packer), x [P, S, D], ld [P, S]; context [C] or [S, C]."""
    dev = _dev(packed, x, context, ld, out)
    P, S, D = x.shape
    C = 0 if context is None else context.shape[-1]
    n = made_packed_floats(nhid, nh, C, D)
    if packed.shape != (P, n) or not packed.is_contiguous():
        raise ValueError(f"packed must be contiguous [P={P}, {n}], got {tuple(packed.shape)}")
    if x.stride(-1) != 1 or ld.shape != (P, S) or ld.stride(-1) != 1:
        raise ValueError("x needs unit column stride and ld must be [P, S]")
    ldc = sctx = 0
    if context is not None:
        context = context.reshape(-1, C).contiguous()
        if context.shape[0] not in (1, S):
            raise ValueError("context must be [C] or [S, C]")
        ldc = 0 if context.shape[0] == 1 else C
    if out is None:
        out = torch.empty_like(x)
    check(lib().naz_made_affine_fwd(_p(packed), n, nhid, nh, C, D, _p(context), ldc, sctx, _p(x), x.stride(1),
                                    x.stride(0), _p(out), out.stride(1), out.stride(0), _p(ld), ld.stride(0), ld_mode,
                                    S, P, ACT[act], _stream(dev)), "made_affine_fwd")
    return out


def made_affine_inv1(packed: Tensor, nhid: int, nh: int, x: Tensor, v: Tensor, dim: int, act: str, ld: Tensor,
                     ld_mode: int = LD_ROWSUM_SUB, out: Optional[Tensor] = None) -> Tensor:
    """Context-free MADE chain + inverse affine step of one dim (naz_made_affine_inv1):
    x, v [P, S, D] (unit column stride), ld [P, S], packed [P, naz_made_packed_floats(nhid, nh, 0, D)]."""
    dev = _dev(packed, x, v, ld, out)
    P, S, D = x.shape
    n = made_packed_floats(nhid, nh, 0, D)
    if packed.shape != (P, n) or not packed.is_contiguous():
        raise ValueError(f"packed must be contiguous [P={P}, {n}], got {tuple(packed.shape)}")
    if v.shape != x.shape or x.stride(-1) != 1 or v.stride(-1) != 1 or ld.shape != (P, S) or ld.stride(-1) != 1:
        raise ValueError("x, v must be [P, S, D] with unit column stride and ld [P, S]")
    if out is None:
        out = torch.empty_like(x)
    check(lib().naz_made_affine_inv1(_p(packed), n, nhid, nh, D, _p(x), x.stride(1), x.stride(0), _p(v), v.stride(1),
                                     v.stride(0), int(dim), _p(out), out.stride(1), out.stride(0), _p(ld), ld.stride(0),
                                     ld_mode, S, P, ACT[act], _stream(dev)), "made_affine_inv1")
    return out


# ----------------------------------------------------------------------------- a5
def affine_ar(x: Tensor, raw: Tensor, inverse: bool, ld_mode: int = LD_PERDIM,
              ld_out: Optional[Tensor] = None, out: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    dev = _dev(x, raw, ld_out, out)
    x, ldx = _rows(x)
    raw, ldr = _rows(raw)
    B, D = x.shape
    if raw.shape != (B, 2 * D):
        raise ValueError(f"raw must be [B, 2D] = {(B, 2 * D)}, got {tuple(raw.shape)}")
    if out is None:
        out = torch.empty_like(x)
    if ld_out is None:
        ld_out = torch.empty((B, D) if ld_mode == LD_PERDIM else (B,), device=dev, dtype=torch.float32)
    check(lib().naz_affine_ar(int(inverse), _p(x), ldx, _p(raw), ldr, _p(out), out.stride(0), _p(ld_out), ld_mode,
                              B, D, _stream(dev)), "affine_ar")
    return out, ld_out


# ----------------------------------------------------------------------------- a8
def base_log_prob(z: Tensor, out: Optional[Tensor] = None, accumulate: bool = False) -> Tensor:
    dev = _dev(z, out)
    z, ldz = _rows(z)
    B, D = z.shape
    if out is None:
        out = torch.empty((B,), device=dev, dtype=torch.float32)
        accumulate = False
    check(lib().naz_base_log_prob(_p(z), ldz, _p(out), B, D, int(accumulate), _stream(dev)), "base_log_prob")
    return out


def bounding_fwd(x: Tensor, low: Tensor, high: Tensor) -> Tuple[Tensor, Tensor]:
    dev = _dev(x, low, high)
    x, ldx = _rows(x)
    B, D = x.shape
    y = torch.empty_like(x)
    lj = torch.empty((B,), device=dev, dtype=torch.float32)
    check(lib().naz_bounding_fwd(_p(x), ldx, _p(low.contiguous()), _p(high.contiguous()), _p(y), y.stride(0), _p(lj),
                                 B, D, _stream(dev)), "bounding_fwd")
    return y, lj


def bounding_inv(y: Tensor, low: Tensor, high: Tensor) -> Tensor:
    dev = _dev(y, low, high)
    y, ldy = _rows(y)
    B, D = y.shape
    x = torch.empty_like(y)
    check(lib().naz_bounding_inv(_p(y), ldy, _p(low.contiguous()), _p(high.contiguous()), _p(x), x.stride(0), B, D,
                                 _stream(dev)), "bounding_inv")
    return x


# ----------------------------------------------------------------------------- a10 backward
def rqs_bwd(x: Tensor, raw: Tensor, count_bins: int, layout: int, inverse: bool, bound: float,
            g_out: Optional[Tensor], g_ld: Optional[Tensor], need_g_in: bool = True,
            broadcast_raw: bool = False) -> Tuple[Optional[Tensor], Tensor]:
    """VJP of ``rqs`` (naz_rqs_bwd).  ``g_ld``: [B] (gradient of the row-sum ld) or [B, Dt]
    (per-dim ld) or None.  Returns (g_x or None, g_raw shaped like ``raw``)."""
    dev = _dev(x, raw, g_out, g_ld)
    x, ldx = _rows(x)
    B, Dt = x.shape
    P = Dt * (3 * count_bins - 1)
    if broadcast_raw:
        raw_c = raw.reshape(1, -1).contiguous()
        ldr = 0
        g_raw = torch.zeros(P, device=dev, dtype=torch.float32)
        ldgr = 0
    else:
        raw_c, ldr = _rows(raw)
        g_raw = torch.empty((B, P), device=dev, dtype=torch.float32)
        ldgr = P
    ldgo = 0
    if g_out is not None:
        g_out, ldgo = _rows(g_out)
    mode = 0
    if g_ld is not None:
        g_ld = g_ld.contiguous()
        mode = 1 if g_ld.dim() == 1 else 2
    g_in = torch.empty((B, Dt), device=dev, dtype=torch.float32) if need_g_in else None
    check(lib().naz_rqs_bwd(int(inverse), _p(x), ldx, _p(raw_c), ldr, _p(g_out), ldgo, _p(g_ld), mode, _p(g_in), Dt,
                            _p(g_raw), ldgr, B, Dt, count_bins, layout, float(bound), _stream(dev)), "rqs_bwd")
    return g_in, (g_raw.reshape(raw.shape) if broadcast_raw else g_raw)


def affine_ar_bwd(x: Tensor, raw: Tensor, y: Tensor, inverse: bool, g_y: Tensor, g_ld: Optional[Tensor],
                  need_g_x: bool = True, clip_zero: bool = False) -> Tuple[Optional[Tensor], Tensor]:
    """VJP of ``affine_ar`` with a row-sum ld (naz_affine_ar_bwd).  ``clip_zero``: the log_scale
    clip differentiates as jnp.clip (0 outside [-5, 3], bflow_jax_maf.py:177-192) instead of pyro's
    clamp_preserve_gradients."""
    dev = _dev(x, raw, y, g_y, g_ld)
    x, ldx = _rows(x)
    raw, ldr = _rows(raw)
    y, ldy = _rows(y)
    g_y, ldgy = _rows(g_y)
    B, D = x.shape
    g_ld = None if g_ld is None else g_ld.contiguous()
    g_x = torch.empty((B, D), device=dev, dtype=torch.float32) if need_g_x else None
    g_raw = torch.empty((B, 2 * D), device=dev, dtype=torch.float32)
    check(lib().naz_affine_ar_bwd(int(bool(inverse)) | (2 if clip_zero else 0), _p(x), ldx, _p(raw), ldr, _p(y), ldy, _p(g_y), ldgy, _p(g_ld),
                                  _p(g_x), D, _p(g_raw), 2 * D, B, D, _stream(dev)), "affine_ar_bwd")
    return g_x, g_raw


def maf_dim_vjp(raw: Tensor, s: Tensor, g: Tensor, g_lp: Optional[Tensor], dim: int, g_next: Tensor, tot: Tensor,
                chain: Optional[Tensor] = None, clip_zero: bool = False) -> None:
    """One dim of the maf inverse layer's VJP (naz_maf_dim_vjp): raw [B, 2D] the MADE output, s [B, D]
    the layer output, g [B, D] = dL/ds; writes g_next[:, dim], tot[:, dim], tot[:, D + dim] and,
    when given, chain [B, 2D] (zero but for those two columns)."""
    dev = _dev(raw, s, g, g_lp, g_next, tot, chain)
    B, D = s.shape
    ts = [raw, s, g, g_next, tot] + ([] if chain is None else [chain])
    if any(t.stride(-1) != 1 or t.shape[0] != B for t in ts) or raw.shape[1] != 2 * D or tot.shape[1] != 2 * D or \
            g.shape[1] != D or g_next.shape[1] != D or (chain is not None and chain.shape[1] != 2 * D):
        raise ValueError("maf_dim_vjp: raw/tot/chain [B, 2D], s/g/g_next [B, D] with unit column stride")
    if g_lp is not None and (g_lp.shape != (B,) or not g_lp.is_contiguous()):
        raise ValueError("maf_dim_vjp: g_lp must be a contiguous [B] tensor")
    check(lib().naz_maf_dim_vjp(AFFINE_CLIP_ZERO_GRAD if clip_zero else 0, _p(raw), raw.stride(0), _p(s), s.stride(0),
                                _p(g), g.stride(0), _p(g_lp), _p(g_next), g_next.stride(0), _p(tot), tot.stride(0),
                                _p(chain), 0 if chain is None else chain.stride(0), B, D, int(dim), _stream(dev)),
          "maf_dim_vjp")


def base_log_prob_bwd(z: Tensor, g_lp: Tensor) -> Tensor:
    dev = _dev(z, g_lp)
    z, ldz = _rows(z)
    B, D = z.shape
    g_z = torch.empty((B, D), device=dev, dtype=torch.float32)
    check(lib().naz_base_log_prob_bwd(_p(z), ldz, _p(g_lp.contiguous()), _p(g_z), D, B, D, _stream(dev)),
          "base_log_prob_bwd")
    return g_z


def _split_k(M: int, N: int, K: int) -> int:
    # about 2048 64 x 64 tiles over the grid, each split at least 192 batch rows deep (at naz's
    # 10,752-row minibatch a 512-row floor held the wide maf's dW at 21 splits: 58 vs 70 TF at 32,
    # profiles/r05_g8_rg_probe.txt)
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    want = max(1, 2048 // tiles)
    return int(max(1, min(want, K // 192)))


def gemm(a: Tensor, b: Tensor, out: Optional[Tensor] = None, mask: Optional[Tensor] = None, mask_b: bool = False,
         accumulate: bool = False, split_k: Optional[int] = None, rowsum: Optional[Tensor] = None) -> Tensor:
    """out (+)= a @ b for arbitrary-strided 2-D views (transposes / stride-0 broadcasts are
    free); ``mask`` multiplies the output (mask_b False) or ``b`` (mask_b True).  Exact fp32
    MFMA (naz_gemm); long reductions are split over the grid with atomic accumulation.
    ``rowsum`` [M] (contiguous) also receives a.sum(1) through the same MFMA reduction
    (accumulated like ``out``)."""
    dev = _dev(a, b, out, mask, rowsum)
    M, K = a.shape
    K2, N = b.shape
    if K2 != K:
        raise ValueError(f"gemm: inner dims differ ({K} vs {K2})")
    if out is None:
        out = torch.empty((M, N), device=dev, dtype=torch.float32)
        accumulate = False
    if out.shape != (M, N):
        raise ValueError(f"gemm: out must be {(M, N)}")
    if mask is not None and mask.shape != ((K, N) if mask_b else (M, N)):
        raise ValueError("gemm: mask shape mismatch")
    if rowsum is not None and (rowsum.shape != (M,) or not rowsum.is_contiguous()):
        raise ValueError("gemm: rowsum must be a contiguous [M] tensor")
    sk = _split_k(M, N + (rowsum is not None), K) if split_k is None else int(split_k)
    if sk > 1 and not accumulate:
        out.zero_()
        if rowsum is not None:
            rowsum.zero_()
    smm, smn = (0, 0) if mask is None else mask.stride()
    check(lib().naz_gemm(M, N, K, _p(a), a.stride(0), a.stride(1), _p(b), b.stride(0), b.stride(1), _p(out),
                         out.stride(0), out.stride(1), _p(mask), smm, smn, int(mask_b), int(accumulate), sk,
                         _p(rowsum), _stream(dev)), "gemm")
    return out


def wgrad_batched(g: Tensor, x: Tensor, c: Tensor, rowsum: Optional[Tensor] = None) -> Tensor:
    """c[b] += g[b]ᵀ @ x[b] and rowsum[b] += g[b].sum(0) for every b in ONE launch (naz_wgrad_batched,
    bf16x6 MFMA): g [nb, M, N1], x [nb, M, N2] with contiguous rows; c [nb, N1, N2] with unit column
    stride (a strided view of a workspace is fine); rowsum [nb, N1] with unit stride."""
    dev = _dev(g, x, c, rowsum)
    nb, M, N1 = g.shape
    if x.shape[:2] != (nb, M) or c.shape != (nb, N1, x.shape[2]):
        raise ValueError("wgrad_batched: shapes must be g [nb, M, N1], x [nb, M, N2], c [nb, N1, N2]")
    for t in (g, x):
        if t.stride(2) != 1 or t.stride(1) != t.shape[2]:
            raise ValueError("wgrad_batched: g and x need contiguous rows")
    if c.stride(2) != 1 or (rowsum is not None and (rowsum.shape != (nb, N1) or rowsum.stride(1) != 1)):
        raise ValueError("wgrad_batched: c / rowsum need a unit column stride")
    check(lib().naz_wgrad_batched(M, N1, x.shape[2], nb, _p(g), g.stride(1), g.stride(0), _p(x), x.stride(1),
                                  x.stride(0), _p(c), c.stride(1), c.stride(0), _p(rowsum),
                                  0 if rowsum is None else rowsum.stride(0), _stream(dev)), "wgrad_batched")
    return c


def gemm_dact(a: Tensor, weight: Tensor, y: Tensor, act: str, mask: Optional[Tensor] = None,
              out: Optional[Tensor] = None) -> Tensor:
    """(a @ (weight * mask)) * act'(y) in one batch-row GEMM (naz_gemm_dact): the input
    gradient of a Linear layer chained with the derivative of the activation that produced its
    input (``y`` = that activation's output)."""
    dev = _dev(a, weight, y, mask, out)
    a, lda = _rows(a)
    M, K = a.shape
    if weight.shape[0] != K or weight.stride(1) != 1:
        raise ValueError("gemm_dact: weight must be [K, N] with unit column stride")
    N = weight.shape[1]
    y, lddy = _rows(y)
    if y.shape != (M, N):
        raise ValueError(f"gemm_dact: y must be {(M, N)}")
    if mask is not None and (mask.shape != weight.shape or mask.stride(1) != 1):
        raise ValueError("gemm_dact: mask must match weight")
    if out is None:
        npad = (N + 3) // 4 * 4
        out = torch.empty((M, npad), device=dev, dtype=torch.float32)[:, :N]
    check(lib().naz_gemm_dact(_p(a), lda, K, _p(weight), weight.stride(0), _p(mask),
                              0 if mask is None else mask.stride(0), _p(out), out.stride(0), _p(y), lddy, ACT[act], M, N,
                              _stream(dev)), "gemm_dact")
    return out


def colsum(a: Tensor, out: Optional[Tensor] = None) -> Tensor:
    """out (+)= a.sum(0) (naz_colsum; ``out`` is zeroed when allocated here)."""
    dev = _dev(a, out)
    a, lda = _rows(a)
    M, N = a.shape
    if out is None:
        out = torch.zeros(N, device=dev, dtype=torch.float32)
    check(lib().naz_colsum(_p(a), lda, M, N, _p(out), _stream(dev)), "colsum")
    return out


def act_bwd(g_y: Tensor, y: Tensor, act: str) -> Tensor:
    """dL/d(pre-activation) from dL/dy and the post-activation y (naz_act_bwd)."""
    dev = _dev(g_y, y)
    g_y, ldg = _rows(g_y)
    y, ldy = _rows(y)
    M, N = y.shape
    gp = torch.empty((M, N), device=dev, dtype=torch.float32)
    check(lib().naz_act_bwd(_p(g_y), ldg, _p(y), ldy, _p(gp), N, M, N, ACT[act], _stream(dev)), "act_bwd")
    return gp


def gemm_jvp_bwd(a: Tensor, weight: Tensor, S: Tensor, act: str, out: Optional[Tensor] = None) -> Tensor:
    """Input adjoints of a CNF vector-field layer under the Hutchinson JVP (naz_gemm_jvp_bwd): rows in
    (value, tangent) pairs 2i, 2i + 1.  a [2B, K] = the next layer's pre-activation adjoints,
    weight [K, N] (unit column stride), S [2B, N] = this layer's (h, dh) pairs -> the adjoints of
    this layer's pre-activations (a @ weight through the activation's VJP), [2B, N]."""
    dev = _dev(a, weight, S, out)
    a, lda = _rows(a)
    S, lds = _rows(S)
    M, K = a.shape
    if weight.shape[0] != K or weight.stride(1) != 1:
        raise ValueError("gemm_jvp_bwd: weight must be [K, N] with unit column stride")
    N = weight.shape[1]
    if M % 2 or S.shape != (M, N):
        raise ValueError(f"gemm_jvp_bwd: S must be [{M}, {N}] with M even (value/tangent row pairs)")
    if out is None:
        npad = (N + 3) // 4 * 4
        out = torch.empty((M, npad), device=dev, dtype=torch.float32)[:, :N]
    check(lib().naz_gemm_jvp_bwd(_p(a), lda, K, _p(weight), weight.stride(0), _p(out), out.stride(0), _p(S), lds,
                                 ACT[act], M, N, _stream(dev)), "gemm_jvp_bwd")
    return out


def dropout(x: Tensor, p: float, seed: int, out: Optional[Tensor] = None) -> Tensor:
    """MC dropout of a conditioner activation (naz_dropout): x / (1 - p) where the hash of
    (seed, row, col) keeps it, else 0.  The same (p, seed) on a same-shape gradient applies
    the forward's mask (the backward).  ``out`` may be ``x`` (in place)."""
    dev = _dev(x, out)
    x, ldx = _rows(x)
    M, N = x.shape
    if out is None:
        out = torch.empty((M, N), device=dev, dtype=torch.float32)
    o, ldo = _rows(out)
    if o.data_ptr() != out.data_ptr():
        raise ValueError("dropout: out must be a row-strided 2-D tensor")
    check(lib().naz_dropout(_p(x), ldx, _p(o), ldo, M, N, float(p), int(seed) & (2 ** 64 - 1), _stream(dev)),
          "dropout")
    return out


# ----------------------------------------------------------------------------- a3 + a8 + a9 fused
def coupling_desc(D: int, C: int, S: int, K: int, L: int, H: int, act: str = "tanh", has_lower: bool = True,
                  bound: float = 3.0, mfma: str = "bf16x6") -> CouplingDesc:
    """``mfma``: "bf16x6" (FP32 GEMMs as six exact-split bf16 products), "f16x3" (three
    exact-split fp16 products; needs packed |W1|,|W2| < 2^15; GEMM1 bf16x6 for workgroups
    outside fp16 range), "f16x3r16" (the same arithmetic on 16-row waves; S and D-S multiples
    of 4; GEMM1 exact fp32 for workgroups outside fp16 range) or "f32" (exact
    v_mfma_f32_32x32x2_f32)."""
    d = CouplingDesc()
    d.D, d.C, d.S, d.K, d.L, d.H = D, C, S, K, L, H
    d.act, d.has_lower, d.bound = ACT.get(act, -1), int(has_lower), float(bound)
    d.mfma_mode = {"bf16x6": 0, "f32": 1, "f16x3": 2, "f16x3r16": 3}[mfma]
    return d


def coupling_supported(d: CouplingDesc) -> bool:
    return bool(lib().naz_coupling_supported(d))


def coupling_param_count(d: CouplingDesc) -> int:
    return int(lib().naz_coupling_param_count(d))


def coupling_pack(d: CouplingDesc, flat: Tensor, packed: Optional[Tensor] = None) -> Tensor:
    dev = _dev(flat)
    n = coupling_param_count(d)
    if flat.numel() != n or not flat.is_contiguous():
        raise ValueError(f"flat params must be a contiguous [{n}] fp32 tensor")
    nbytes = int(lib().naz_coupling_packed_bytes(d))
    if nbytes <= 0:
        raise RuntimeError("naz_amd coupling_pack: unsupported descriptor")
    if packed is None or packed.numel() * 4 != nbytes:
        packed = torch.empty(nbytes // 4, device=dev, dtype=torch.float32)
    check(lib().naz_coupling_pack(d, _p(flat), _p(packed), _stream(dev)), "coupling_pack")
    return track_image(packed)


def _ctx_arg(context: Optional[Tensor], B: int):
    if context is None:
        return None, 0
    if context.dim() == 1 or (context.shape[0] == 1 and B != 1):
        return context.reshape(1, -1).contiguous(), 0
    context, ldc = _rows(context)
    if context.shape[0] != B:
        raise ValueError("condition rows must match x rows (or be a single row)")
    return context, ldc


def coupling_log_prob(d: CouplingDesc, packed: Tensor, x: Tensor, context: Optional[Tensor] = None,
                      low: Optional[Tensor] = None, high: Optional[Tensor] = None,
                      out: Optional[Tensor] = None) -> Tensor:
    dev = _dev(packed, x, context, low, high, out)
    x, ldx = _rows(x)
    B = x.shape[0]
    context, ldc = _ctx_arg(context, B)
    if out is None:
        out = torch.empty((B,), device=dev, dtype=torch.float32)
    check(lib().naz_coupling_log_prob(d, _p(packed), _p(x), ldx, _p(context), ldc, _p(low), _p(high), _p(out), B,
                                      _stream(dev)), "coupling_log_prob")
    return out


def coupling_layer(d: CouplingDesc, packed: Tensor, layer: int, x: Tensor, context: Optional[Tensor], inverse: bool,
                   ld_out: Tensor, ld_mode: int = LD_ROWSUM, out: Optional[Tensor] = None) -> Tensor:
    """ONE coupling layer of a packed flow (naz_coupling_layer_{fwd,inv}): y = T_layer(x) or its
    inverse; ld_out [B] gets the layer's FORWARD log|det J| by ld_mode (=, +=, -=)."""
    dev = _dev(packed, x, context, ld_out, out)
    x, ldx = _rows(x)
    B = x.shape[0]
    context, ldc = _ctx_arg(context, B)
    if ld_out.shape != (B,) or not ld_out.is_contiguous() or ld_out.dtype != torch.float32:
        raise ValueError(f"coupling_layer: ld_out must be a contiguous float32 [{B}] tensor")
    if out is None:
        out = torch.empty((B, d.D), device=dev, dtype=torch.float32)
    if out.dim() != 2 or out.shape != (B, d.D) or out.stride(1) != 1:
        raise ValueError(f"coupling_layer: out must be [{B}, {d.D}] with unit column stride")
    fn = lib().naz_coupling_layer_inv if inverse else lib().naz_coupling_layer_fwd
    check(fn(d, _p(packed), int(layer), _p(x), ldx, _p(context), ldc, _p(out), out.stride(0), _p(ld_out), int(ld_mode),
             B, _stream(dev)), "coupling_layer")
    return out


# ----------------------------------------------------------------------------- §8b naz_{spline,affine}_ar_inv
AR_KIND = {"nsa": 0, "maf": 1}  # NAZ_AR_SPLINE, NAZ_AR_AFFINE
AR_CLIP_ZERO_GRAD = 1  # naz_ar_desc.flags: NAZ_AR_CLIP_ZERO_GRAD
AFFINE_CLIP_ZERO_GRAD = 2  # naz_affine_ar_bwd / naz_maf_dim_vjp mode bit: NAZ_AFFINE_CLIP_ZERO_GRAD


def ar_flow_desc(kind: str, D: int, C: int, H: int, L: int, n_hidden: int = 2, K: int = 8, act: str = "tanh",
                 bound: float = 3.0) -> ArDesc:
    """naz_ar_desc of an L-layer nsa / maf flow with n_hidden tanh hidden layers of width H."""
    d = ArDesc()
    d.D, d.C, d.H, d.K, d.L = D, C, H, K, L
    d.act, d.bound = ACT.get(act, -1), float(bound)
    d.n_hidden, d.kind = n_hidden, AR_KIND.get(kind, -1)
    return d


def ar_flow_supported(d: ArDesc) -> bool:
    """Both directions (log_prob and sample) run fused for this shape."""
    return int(lib().naz_ar_flow_supported(d)) == 1


def ar_flow_fwd_supported(d: ArDesc) -> bool:
    """The sampling direction runs fused (naz_ar_flow_sample*): every fused shape, including a
    forward-only one (naz_ar_flow_supported == 2; none today)."""
    return int(lib().naz_ar_flow_supported(d)) in (1, 2)


def ar_flow_degrees(d: ArDesc) -> np.ndarray:
    """The hidden-unit mask indices the fused kernel is compiled for (pyro create_mask's)."""
    out = np.zeros(d.H, dtype=np.int32)
    check(lib().naz_ar_flow_degrees(d, out.ctypes.data), "ar_flow_degrees")
    return out


def ar_executed_flop_per_row(d: ArDesc, pass0_const: bool = False) -> dict:
    """FP32-equivalent FLOPs per row the fused autoregressive kernels EXECUTE (a split f16x3 /
    bf16x6 product counted once; the 16-unit block recomputation and zero padding included), for
    roofline accounting against the pipe each runs on:

      inverse  made_ar_r16_kernel (log_prob): per pass p, hidden layer 1's blocks holding units of
               degree p over [ctx | x], the further hidden layers' over the units of degree <= p,
               and the output blocks of dim p (made_ar_r16.h; f16x3); the wide H = 512 instances
               (made_ar_inv_wide_kernel) recompute ALL of hidden layer 1's degree <= p blocks;
      bwd      made_ar_bwd_kernel, all layers (maf only): one dense MADE pass plus D chains
               (W_out^T g on the VALU in fp32, the W_i^T chain and the input unit on f16x3);
      dw       the batched weight-gradient reductions over the padded operands (bf16x6).
    pass0_const: the images carry the first degree pass as per-draw constants (no MFMAs in pass 0).
    """
    D, C, H, NH, L = d.D, d.C, d.H, d.n_hidden, d.L
    P = 2 if d.kind == AR_KIND["maf"] else 3 * d.K - 1
    HP = (H + 31) // 32 * 32
    HB, KSH, KI, NOB = HP // 16, HP // 32, (C + 31) // 32 + 1, (P + 15) // 16
    blk = 16 * 32 * 2  # one 16-unit block over one 32-deep k-step, per row
    deg = ar_flow_degrees(d)
    E = [int((deg <= p).sum()) for p in range(D)]
    wide = HP > 256  # made_ar_wide.h: hidden layer 1 recomputed in full (blocks of degree <= p) every pass
    inv = 0
    for p in range(1 if pass0_const else 0, D):  # pass-0 constants: the first pass runs no MFMAs
        e0 = E[p - 1] if p else 0
        nb = ((E[p] - 1) >> 4) - (e0 >> 4) + 1 if E[p] > e0 else 0
        nb1 = (((E[p] - 1) >> 4) + 1 if E[p] > 0 else 0) if wide else nb
        kt = (E[p] + 31) // 32
        inv += (nb1 * KI + nb * (NH - 1) * kt + NOB * kt) * blk
    out = {"inverse": inv * L}
    if d.kind == AR_KIND["maf"] and int(lib().naz_ar_flow_bwd_packed_bytes(d)) > 0:
        X0W = ar_flow_bwd_dims(d)["X0W"]
        dense = (HB * KI + (NH - 1) * HB * KSH + (D + 3) // 4 * KSH) * blk
        chains = D * (2 * 2 * D * HP + (NH - 1) * HB * KSH * blk) + (D - 1) * KSH * blk
        out["bwd"] = (dense + chains) * L
        out["bwd_valu"] = D * 2 * 2 * D * HP * L  # the W_out^T g part, in "bwd"
        out["dw"] = 2 * (HP * X0W + (NH - 1) * HP * HP + X0W * HP) * L
    return out


def ar_flow_pack(d: ArDesc, flat: np.ndarray, perm: np.ndarray, device) -> Tensor:
    """Host-side pack (naz_ar_flow_pack_host) of the masked per-layer weights, then one copy to
    the device.  flat: fp32 per layer W0m|b0|{Wim|bi}|Woutm|bout; perm: int32 [L, D]."""
    flat = np.ascontiguousarray(flat, dtype=np.float32)
    perm = np.ascontiguousarray(perm, dtype=np.int32)
    nbytes = int(lib().naz_ar_flow_packed_bytes(d))
    if nbytes <= 0:
        raise RuntimeError("naz_amd ar_flow_pack: unsupported descriptor")
    host = np.empty(nbytes // 4, dtype=np.float32)
    check(lib().naz_ar_flow_pack_host(d, flat.ctypes.data, perm.ctypes.data, host.ctypes.data), "ar_flow_pack")
    return attach_image(torch.from_numpy(host).to(device), "ar_flow_pack")


def ar_flow_pack_fwd(d: ArDesc, flat: np.ndarray, device) -> Tensor:
    """Host-side pack of the forward (sample) image (naz_ar_flow_pack_fwd_host) from the same flat
    masked weights as ``ar_flow_pack``; one copy to the device."""
    flat = np.ascontiguousarray(flat, dtype=np.float32)
    nbytes = int(lib().naz_ar_flow_fwd_packed_bytes(d))
    if nbytes <= 0:
        raise RuntimeError("naz_amd ar_flow_pack_fwd: unsupported descriptor")
    host = np.empty(nbytes // 4, dtype=np.float32)
    check(lib().naz_ar_flow_pack_fwd_host(d, flat.ctypes.data, host.ctypes.data), "ar_flow_pack_fwd")
    return attach_image(torch.from_numpy(host).to(device), "ar_flow_pack_fwd")


def ar_flow_sample(d: ArDesc, packed_fwd: Tensor, z: Tensor, context: Optional[Tensor] = None,
                   low: Optional[Tensor] = None, high: Optional[Tensor] = None,
                   with_logdet: bool = False) -> Tuple[Tensor, Optional[Tensor]]:
    """y = T_L ∘ … ∘ T_1(z) of an nsa / maf flow in one launch (naz_ar_flow_sample)."""
    dev = _dev(packed_fwd, z, context, low, high)
    z, ldz = _rows(z)
    B = z.shape[0]
    context, ldc = _ctx_arg(context, B)
    y = torch.empty_like(z)
    ld = torch.empty((B,), device=dev, dtype=torch.float32) if with_logdet else None
    check(lib().naz_ar_flow_sample(d, _p(packed_fwd), _p(z), ldz, _p(context), ldc, _p(low), _p(high), _p(y),
                                   y.stride(0), _p(ld), B, _stream(dev)), "ar_flow_sample")
    return y, ld


def _flat_rows(flat: Tensor):
    """(flat, draw stride) of a [P, n] operand with unit column stride (rows may be strided)."""
    if flat.dim() != 2:
        raise ValueError("flat must be [P, L * per]")
    if flat.stride(1) != 1 or (flat.shape[0] > 1 and flat.stride(0) < flat.shape[1]):
        flat = flat.contiguous()
    return flat, (flat.stride(0) if flat.shape[0] > 1 else flat.shape[1])


def ar_flow_pack_fwd_batched(d: ArDesc, flat: Tensor, mask: Optional[Tensor] = None) -> Tensor:
    """Forward images of P weight draws packed on the device (naz_ar_flow_pack_fwd): flat [P, L * per]
    (the naz_ar_flow_pack_host flat layout; masks applied, or given as ``mask`` [L * per]) ->
    [P, image floats]."""
    dev = _dev(flat, mask)
    flat, sflat = _flat_rows(flat)
    P = flat.shape[0]
    n = int(lib().naz_ar_flow_fwd_packed_bytes(d)) // 4
    if n <= 0:
        raise RuntimeError("naz_amd ar_flow_pack_fwd: unsupported descriptor")
    out = torch.empty((P, n), device=dev, dtype=torch.float32)
    if mask is not None and (mask.numel() != flat.shape[1] or not mask.is_contiguous()):
        raise ValueError("ar_flow_pack_fwd_batched: mask must be a contiguous [L * per] tensor")
    check(lib().naz_ar_flow_pack_fwd(d, _p(flat), sflat, _p(out), n, P, _p(mask), _stream(dev)), "ar_flow_pack_fwd")
    return track_image(out)


def ar_flow_sample_batched(d: ArDesc, packed: Tensor, z: Tensor, context: Optional[Tensor] = None,
                           with_logdet: bool = True) -> Tuple[Tensor, Optional[Tensor]]:
    """Draw p of ``packed`` [P, image] maps z[p] ([P, S, D]) -> y[p]; one context vector for all draws
    (naz_ar_flow_sample_batched).  Returns (y [P, S, D], Σ forward log-dets [P, S])."""
    dev = _dev(packed, z, context)
    z = z.contiguous()
    P, S, D = z.shape
    if packed.shape[0] != P or not packed.is_contiguous():
        raise ValueError("ar_flow_sample_batched: packed must be a contiguous [P, image] tensor")
    ctx = None if context is None else context.reshape(1, -1).contiguous()
    y = torch.empty_like(z)
    ld = torch.empty((P, S), device=dev, dtype=torch.float32) if with_logdet else None
    check(lib().naz_ar_flow_sample_batched(d, _p(packed), packed.stride(0), _p(z), D, S * D, _p(ctx), 0, _p(y), D,
                                           S * D, _p(ld), S, S, P, _stream(dev)), "ar_flow_sample_batched")
    return y, ld


_AR_PERMS: dict = {}


def ar_flow_pass0_floats(d: ArDesc) -> int:
    """Floats per draw of naz_ar_flow_pack's pass-0 constants (all L layers)."""
    return int(lib().naz_ar_flow_pass0_floats(d))


def ar_flow_pack_batched(d: ArDesc, flat: Tensor, perm, pass0: Optional[Tensor] = None,
                         mask: Optional[Tensor] = None) -> Tensor:
    """Inverse (log_prob) images of P weight draws packed on the device (naz_ar_flow_pack): flat
    [P, L * per] (the naz_ar_flow_pack_host flat layout, masks applied), perm [L, D] shared by the
    draws (checked here: the kernel indexes its registers by it) -> [P, image floats].  pass0
    [P, ar_flow_pass0_floats]: the first degree pass's per-draw constants (one context vector;
    include/naz_hip.h) written in place of that pass's weights."""
    dev = _dev(flat, mask)
    flat, sflat = _flat_rows(flat)
    P = flat.shape[0]
    if mask is not None and (mask.numel() != flat.shape[1] or not mask.is_contiguous()):
        raise ValueError("ar_flow_pack_batched: mask must be a contiguous [L * per] tensor")
    pm = np.ascontiguousarray(np.asarray(perm), dtype=np.int32)
    key = (pm.shape, pm.tobytes(), str(dev))
    pmd = _AR_PERMS.get(key)
    if pmd is None:  # checked and copied once per permutation set and device
        if pm.shape != (d.L, d.D) or any(sorted(r) != list(range(d.D)) for r in pm.tolist()):
            raise ValueError(f"ar_flow_pack_batched: perm must hold {d.L} permutations of 0..{d.D - 1}")
        pmd = _AR_PERMS[key] = torch.from_numpy(pm).to(dev)
    n = int(lib().naz_ar_flow_packed_bytes(d)) // 4
    if n <= 0:
        raise RuntimeError("naz_amd ar_flow_pack: unsupported descriptor")
    sp0 = 0
    if pass0 is not None:
        pass0 = pass0.contiguous()
        sp0 = ar_flow_pass0_floats(d)
        if pass0.shape != (P, sp0):
            raise ValueError(f"ar_flow_pack_batched: pass0 must be [{P}, {sp0}]")
    out = torch.empty((P, n), device=dev, dtype=torch.float32)
    check(lib().naz_ar_flow_pack(d, _p(flat), sflat, _p(pmd), _p(out), n, P, _p(pass0), sp0, _p(mask),
                                 _stream(dev)), "ar_flow_pack")
    return track_image(out)


def ar_flow_log_prob_batched(d: ArDesc, packed: Tensor, x: Tensor, context: Optional[Tensor] = None,
                             pass0_const: bool = False) -> Tensor:
    """out[p] = log p(x | ctx) under draw p of ``packed`` [P, image] (naz_ar_flow_log_prob_batched);
    x [B, D] (the same rows for every draw) or [P, B, D]; one context vector [C] for all rows.
    pass0_const: the images carry pass-0 constants (ar_flow_pack_batched(pass0=...))."""
    dev = _dev(packed, x, context)
    P = packed.shape[0]
    if not packed.is_contiguous():
        raise ValueError("ar_flow_log_prob_batched: packed must be a contiguous [P, image] tensor")
    x = x.contiguous()
    if x.dim() == 2:
        B, sx = x.shape[0], 0
    elif x.dim() == 3 and x.shape[0] == P:
        B, sx = x.shape[1], x.shape[1] * x.shape[2]
    else:
        raise ValueError("ar_flow_log_prob_batched: x must be [B, D] or [P, B, D]")
    ctx = None if context is None else context.reshape(1, -1).contiguous()
    out = torch.empty((P, B), device=dev, dtype=torch.float32)
    ws, wsb = workspace(dev, int(lib().naz_ar_flow_workspace_bytes(d, B, P)))
    check(lib().naz_ar_flow_log_prob_batched(d, _p(packed), packed.stride(0), _p(x), x.shape[-1], sx, _p(ctx), 0,
                                             _p(out), B, B, P, int(pass0_const), ws, wsb, _stream(dev)),
          "ar_flow_log_prob_batched")
    return out


def ar_flow_log_prob(d: ArDesc, packed: Tensor, x: Tensor, context: Optional[Tensor] = None,
                     low: Optional[Tensor] = None, high: Optional[Tensor] = None,
                     out: Optional[Tensor] = None) -> Tensor:
    dev = _dev(packed, x, context, low, high, out)
    x, ldx = _rows(x)
    B = x.shape[0]
    context, ldc = _ctx_arg(context, B)
    if out is None:
        out = torch.empty((B,), device=dev, dtype=torch.float32)
    ws, wsb = workspace(dev, int(lib().naz_ar_flow_workspace_bytes(d, B, 1)))
    check(lib().naz_ar_flow_log_prob(d, _p(packed), _p(x), ldx, _p(context), ldc, _p(low), _p(high), _p(out), B,
                                     ws, wsb, _stream(dev)), "ar_flow_log_prob")
    return out


# ----------------------------------------------------------------------------- fused maf backward (§8f rank 1)
def ar_flow_bwd_supported(d: ArDesc) -> bool:
    """The fused maf backward (made_ar_bwd.h) is compiled for this shape."""
    return int(lib().naz_ar_flow_bwd_packed_bytes(d)) > 0


def ar_flow_bwd_dims(d: ArDesc) -> dict:
    """Operand widths of naz_ar_flow_bwd_layer (include/naz_hip.h)."""
    out = np.zeros(6, dtype=np.int32)
    check(lib().naz_ar_flow_bwd_dims(d, out.ctypes.data), "ar_flow_bwd_dims")
    return dict(zip(("n_hidden", "HP", "XA", "XB", "X0W", "rows"), (int(v) for v in out)))


def ar_flow_pack_bwd(d: ArDesc, flat: Tensor, mask: Optional[Tensor] = None) -> Tensor:
    """Per-layer backward images (naz_ar_flow_pack_bwd) of one flow's flat [L * per] parameters."""
    dev = _dev(flat, mask)
    flat = flat.reshape(-1).contiguous()
    n = int(lib().naz_ar_flow_bwd_packed_bytes(d)) // 4
    if n <= 0:
        raise RuntimeError("naz_amd ar_flow_pack_bwd: unsupported descriptor")
    if mask is not None and (mask.numel() != flat.numel() or not mask.is_contiguous()):
        raise ValueError("ar_flow_pack_bwd: mask must be a contiguous tensor shaped like flat")
    out = torch.empty(n, device=dev, dtype=torch.float32)
    check(lib().naz_ar_flow_pack_bwd(d, _p(flat), _p(mask), _p(out), _stream(dev)), "ar_flow_pack_bwd")
    return track_image(out)


def ar_flow_log_prob_train(d: ArDesc, packed: Tensor, x: Tensor, context: Optional[Tensor], states: Tensor,
                           out: Optional[Tensor] = None) -> Tensor:
    """log p(x | ctx) (naz_ar_flow_log_prob on the inverse image) also writing states [L, B, D]:
    layer l's output s_l, for naz_ar_flow_bwd_layer."""
    dev = _dev(packed, x, context, states, out)
    x, ldx = _rows(x)
    B = x.shape[0]
    context, ldc = _ctx_arg(context, B)
    if states.shape != (d.L, B, d.D) or not states.is_contiguous():
        raise ValueError(f"ar_flow_log_prob_train: states must be contiguous {(d.L, B, d.D)}")
    if out is None:
        out = torch.empty((B,), device=dev, dtype=torch.float32)
    ws, wsb = workspace(dev, int(lib().naz_ar_flow_workspace_bytes(d, B, 1)))
    check(lib().naz_ar_flow_log_prob_train(d, _p(packed), _p(x), ldx, _p(context), ldc, _p(out), _p(states), B,
                                           ws, wsb, _stream(dev)), "ar_flow_log_prob_train")
    return out


def ar_flow_bwd_layer(d: ArDesc, packed_fwd: Tensor, packed_bwd: Tensor, perm: Tensor, layer: int, state: Tensor,
                      context: Optional[Tensor], g_in: Tensor, g_lp: Optional[Tensor], bufs: List[Tensor],
                      g_out: Tensor) -> None:
    """Layer ``layer``'s fused maf backward (naz_ar_flow_bwd_layer): g_in = dL/ds_l -> g_out =
    dL/ds_{l+1} and the weight-gradient operands ``bufs`` (include/naz_hip.h order)."""
    dev = _dev(packed_fwd, packed_bwd, state, context, g_in, g_lp, g_out)
    if perm.dtype != torch.int32 or perm.device != dev or perm.shape != (d.L, d.D):
        raise ValueError(f"ar_flow_bwd_layer: perm must be an int32 [{d.L}, {d.D}] tensor on {dev}")
    B = state.shape[0]
    context, ldc = _ctx_arg(context, B)
    for t in (state, g_in, g_out, perm) + tuple(b for b in bufs if b is not None) + ((g_lp,) if g_lp is not None else ()):
        if not t.is_contiguous():
            raise ValueError("ar_flow_bwd_layer: buffers must be contiguous")
    if not (0 <= int(layer) < d.L):
        raise ValueError(f"ar_flow_bwd_layer: layer {layer} outside [0, {d.L})")
    for name, t in (("state", state), ("g_in", g_in), ("g_out", g_out)):
        if t.dim() != 2 or t.shape[0] != B or t.shape[1] != d.D or t.dtype != torch.float32:
            raise ValueError(f"ar_flow_bwd_layer: {name} must be float32 [{B}, {d.D}], got {tuple(t.shape)}")
    if g_lp is not None and (g_lp.numel() != B or g_lp.dtype != torch.float32):
        raise ValueError(f"ar_flow_bwd_layer: g_lp must be float32 [{B}]")
    # bufs (include/naz_hip.h): x0, then per hidden layer (h_i, h_i split tail), then dp_i, then gout
    dm = ar_flow_bwd_dims(d)
    NH, HP, X0W, XA, XB = dm["n_hidden"], dm["HP"], dm["X0W"], dm["XA"], dm["XB"]
    if len(bufs) != 2 + 3 * NH:
        raise ValueError(f"ar_flow_bwd_layer: {2 + 3 * NH} operand buffers expected, got {len(bufs)}")
    widths = [X0W] + [w for _ in range(NH) for w in (XA, XB)] + [HP] * NH + [X0W]
    for k, (t, w) in enumerate(zip(bufs, widths)):
        if t is None:
            if w != 0 and not (1 <= k <= 2 * NH and k % 2 == 0 and XB == 0):
                raise ValueError(f"ar_flow_bwd_layer: operand buffer {k} is required")
            continue
        if t.dim() != 2 or t.shape[0] < B or t.shape[1] != w or t.dtype != torch.float32 or t.device != dev:
            raise ValueError(f"ar_flow_bwd_layer: operand buffer {k} must be float32 [>= {B}, {w}] on {dev}, "
                             f"got {tuple(t.shape)}")
    ptrs = (C.c_void_p * len(bufs))(*[_p(b) for b in bufs])
    check(lib().naz_ar_flow_bwd_layer(d, _p(packed_fwd), _p(packed_bwd), _p(perm), int(layer), _p(state),
                                      _p(context), ldc, _p(g_in), _p(g_lp), ptrs, _p(g_out), B, _stream(dev)),
          "ar_flow_bwd_layer")


# ----------------------------------------------------------------------------- a10: fused NLL step
# ----------------------------------------------------------------------------- §8b whole-flow entries
def flow_desc(part) -> FlowDesc:
    """naz_flow_desc wrapping a coupling (nsc) or autoregressive (nsa / maf) descriptor."""
    d = FlowDesc()
    if isinstance(part, CouplingDesc):
        d.kind, d.coupling = FLOW_COUPLING, part
    elif isinstance(part, ArDesc):
        d.kind, d.ar = FLOW_AR, part
    else:
        raise TypeError("flow_desc: a CouplingDesc or an ArDesc")
    return d


def flow_log_prob(d: FlowDesc, packed: Tensor, x: Tensor, context: Optional[Tensor] = None,
                  low: Optional[Tensor] = None, high: Optional[Tensor] = None,
                  out: Optional[Tensor] = None) -> Tensor:
    """NormalizingFlow.log_prob of a fused-kind flow through the generic entry (naz_flow_log_prob)."""
    dev = _dev(packed, x, context, low, high, out)
    x, ldx = _rows(x)
    B = x.shape[0]
    context, ldc = _ctx_arg(context, B)
    if out is None:
        out = torch.empty((B,), device=dev, dtype=torch.float32)
    ws, wsb = workspace(dev, int(lib().naz_workspace_bytes(d, B)))
    check(lib().naz_flow_log_prob(d, _p(packed), _p(x), ldx, _p(context), ldc, _p(low), _p(high), _p(out), B,
                                  ws, wsb, _stream(dev)), "flow_log_prob")
    return out


def flow_sample(d: FlowDesc, packed: Tensor, z: Tensor, context: Optional[Tensor] = None,
                low: Optional[Tensor] = None, high: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """(y, sum log|det|) through the generic entry (naz_flow_sample; coupling flows)."""
    dev = _dev(packed, z, context, low, high)
    z, ldz = _rows(z)
    B = z.shape[0]
    context, ldc = _ctx_arg(context, B)
    y = torch.empty_like(z)
    ld = torch.empty((B,), device=dev, dtype=torch.float32)
    check(lib().naz_flow_sample(d, _p(packed), _p(z), ldz, _p(context), ldc, _p(low), _p(high), _p(y), y.stride(0),
                                _p(ld), B, _stream(dev)), "flow_sample")
    return y, ld


def coupling_pack_bwd(d: CouplingDesc, flat: Tensor, out: Optional[Tensor] = None) -> Tensor:
    """Per-layer fp32 backward images (naz_coupling_pack_bwd) of the flat natural parameters."""
    n = int(lib().naz_coupling_bwd_packed_bytes(d))
    if n < 0:
        raise RuntimeError(f"coupling_pack_bwd: {lib().naz_last_error().decode()}")
    dev = _dev(flat, out)
    if out is None or out.numel() * 4 != n:
        out = torch.empty(n // 4, device=dev, dtype=torch.float32)
    check(lib().naz_coupling_pack_bwd(d, _p(flat.contiguous()), _p(out), _stream(dev)), "coupling_pack_bwd")
    return track_image(out)


def coupling_log_prob_train(d: CouplingDesc, packed: Tensor, x: Tensor, context: Optional[Tensor],
                            low: Optional[Tensor], high: Optional[Tensor], states: Tensor,
                            out: Optional[Tensor] = None) -> Tensor:
    """log p with the reference walk's libm-grade math; states [L+1, B, D] receives every
    layer's input (states[0] = z) for the backward (naz_coupling_log_prob_train)."""
    dev = _dev(packed, x, context, low, high, out, states)
    x, ldx = _rows(x)
    B = x.shape[0]
    context, ldc = _ctx_arg(context, B)
    if states.shape != (d.L + 1, B, d.D) or not states.is_contiguous():
        raise ValueError(f"coupling_log_prob_train: states must be contiguous {(d.L + 1, B, d.D)}")
    if out is None:
        out = torch.empty((B,), device=dev, dtype=torch.float32)
    check(lib().naz_coupling_log_prob_train(d, _p(packed), _p(x), ldx, _p(context), ldc, _p(low), _p(high), _p(out),
                                            _p(states), B, _stream(dev)), "coupling_log_prob_train")
    return out


def coupling_dp3_columns(d: CouplingDesc) -> Tensor:
    """DenseNN output row of every dp3 column of naz_coupling_bwd_layer (-1 = padding)."""
    n = int(lib().naz_coupling_dp3_columns(d, None))
    if n < 0:
        raise RuntimeError(f"coupling_dp3_columns: {lib().naz_last_error().decode()}")
    rows = (C.c_int * n)()
    lib().naz_coupling_dp3_columns(d, rows)
    return torch.tensor(list(rows), dtype=torch.int64)


def coupling_bwd_layer(d: CouplingDesc, packed: Tensor, packed_bwd: Tensor, flat: Tensor, layer: int, state: Tensor,
                       context: Optional[Tensor], g_in: Tensor, g_lp: Tensor, bufs: dict, g_out: Tensor,
                       g_low: Optional[Tensor]) -> None:
    """One layer of the fused NLL backward (naz_coupling_bwd_layer); ``bufs`` holds the
    contiguous h1, h2, dp1, dp2 [B, H], dp3 [B, ncol], x0 [B, C+S] outputs."""
    dev = _dev(packed, packed_bwd, flat, state, context, g_in, g_lp, g_out, g_low)
    B = state.shape[0]
    context, ldc = _ctx_arg(context, B)
    for t in (state, g_in, g_lp, g_out) + tuple(bufs[k] for k in ("h1", "h2", "dp1", "dp2", "dp3", "x0")):
        if not t.is_contiguous():
            raise ValueError("coupling_bwd_layer: buffers must be contiguous")
    check(lib().naz_coupling_bwd_layer(d, _p(packed), _p(packed_bwd), _p(flat), int(layer), _p(state), _p(context), ldc,
                                       _p(g_in), _p(g_lp), _p(bufs["h1"]), _p(bufs["h2"]), _p(bufs["dp1"]),
                                       _p(bufs["dp2"]), _p(bufs["dp3"]), _p(bufs["x0"]), _p(g_out), _p(g_low), B,
                                       _stream(dev)), "coupling_bwd_layer")


def coupling_sample(d: CouplingDesc, packed: Tensor, z: Tensor, context: Optional[Tensor] = None,
                    low: Optional[Tensor] = None, high: Optional[Tensor] = None,
                    with_logdet: bool = False) -> Tuple[Tensor, Optional[Tensor]]:
    dev = _dev(packed, z, context, low, high)
    z, ldz = _rows(z)
    B = z.shape[0]
    context, ldc = _ctx_arg(context, B)
    y = torch.empty_like(z)
    ld = torch.empty((B,), device=dev, dtype=torch.float32) if with_logdet else None
    check(lib().naz_coupling_sample(d, _p(packed), _p(z), ldz, _p(context), ldc, _p(low), _p(high), _p(y),
                                    y.stride(0), _p(ld), B, _stream(dev)), "coupling_sample")
    return y, ld


# ----------------------------------------------------------------------------- a11 CNF
def cnf_desc(D: int, C: int, hidden, act: str = "softplus", mfma: str = "f32") -> CnfDesc:
    """``mfma``: "f32" (exact FP32 MFMA throughout) or "f16x3" (layer 0 exact FP32; hidden and
    output layers as three exact-split fp16 products; hidden widths multiples of 32, packed
    |W| < 2^15 — the caller checks)."""
    hidden = list(hidden)
    if not 1 <= len(hidden) <= 4:
        raise ValueError("naz_amd CNF: 1 to 4 hidden layers")
    d = CnfDesc()
    d.D, d.C, d.n_hidden = D, C, len(hidden)
    for j, h in enumerate(hidden):
        d.H[j] = int(h)
    d.act = ACT.get(act, -1)
    d.mfma_mode = {"f32": 0, "f16x3": 1}[mfma]
    return d


def cnf_supported(d: CnfDesc) -> bool:
    return bool(lib().naz_cnf_supported(d))


def cnf_param_count(d: CnfDesc) -> int:
    return int(lib().naz_cnf_param_count(d))


def cnf_pack(d: CnfDesc, flat: Tensor, packed: Optional[Tensor] = None) -> Tensor:
    dev = _dev(flat)
    n = cnf_param_count(d)
    if flat.numel() != n or not flat.is_contiguous():
        raise ValueError(f"flat CNF params must be a contiguous [{n}] fp32 tensor")
    nbytes = int(lib().naz_cnf_packed_bytes(d))
    if nbytes <= 0:
        raise RuntimeError(f"naz_amd cnf_pack: {lib().naz_last_error().decode()}")
    if packed is None or packed.numel() * 4 != nbytes:
        packed = torch.empty(nbytes // 4, device=dev, dtype=torch.float32)
    check(lib().naz_cnf_pack(d, _p(flat), _p(packed), _stream(dev)), "cnf_pack")
    return track_image(packed)


def cnf_integrate(d: CnfDesc, packed: Tensor, x: Tensor, eps: Tensor, t0: float, t1: float, steps: int,
                  context: Optional[Tensor] = None, ld_out: Optional[Tensor] = None, ld_mode: int = LD_ROWSUM,
                  out: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """One FFJORD block solve (naz_cnf_integrate): (y, ld) with ld = int_{t0}^{t1} -eps^T J eps dt."""
    dev = _dev(packed, x, eps, context, ld_out, out)
    x, ldx = _rows(x)
    eps, lde = _rows(eps)
    B = x.shape[0]
    if eps.shape != x.shape:
        raise ValueError("eps must match x")
    context, ldc = _ctx_arg(context, B)
    if out is None:
        out = torch.empty_like(x)
    if ld_out is None:
        ld_out = torch.empty((B,), device=dev, dtype=torch.float32)
        if ld_mode in (LD_ROWSUM_ADD, LD_ROWSUM_SUB):
            ld_out.zero_()
    check(lib().naz_cnf_integrate(d, _p(packed), _p(x), ldx, _p(context), ldc, _p(eps), lde, float(t0), float(t1),
                                  int(steps), _p(out), out.stride(0), _p(ld_out), ld_mode, B, _stream(dev)),
          "cnf_integrate")
    return out, ld_out


def cnf_integrate_dopri5(d: CnfDesc, packed: Tensor, x: Tensor, eps: Tensor, t0: float, t1: float,
                         atol: float = 1e-4, rtol: float = 1e-4, max_steps: int = 1000,
                         context: Optional[Tensor] = None, ld_out: Optional[Tensor] = None, ld_mode: int = LD_ROWSUM,
                         out: Optional[Tensor] = None, nfe: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """Adaptive dopri5 FFJORD block solve (naz_cnf_integrate_dopri5); ``nfe`` (int32
    [ceil(B/16)], optional) receives the RHS evaluations of every 16-row group."""
    dev = _dev(packed, x, eps, context, ld_out, out)
    x, ldx = _rows(x)
    eps, lde = _rows(eps)
    B = x.shape[0]
    if eps.shape != x.shape:
        raise ValueError("eps must match x")
    context, ldc = _ctx_arg(context, B)
    if out is None:
        out = torch.empty_like(x)
    if ld_out is None:
        ld_out = torch.empty((B,), device=dev, dtype=torch.float32)
        if ld_mode in (LD_ROWSUM_ADD, LD_ROWSUM_SUB):
            ld_out.zero_()
    if nfe is not None and (nfe.dtype != torch.int32 or nfe.numel() < (B + 15) // 16 or nfe.device != dev):
        raise ValueError("nfe must be a device int32 tensor with ceil(B/16) entries")
    check(lib().naz_cnf_integrate_dopri5(d, _p(packed), _p(x), ldx, _p(context), ldc, _p(eps), lde, float(t0),
                                         float(t1), float(atol), float(rtol), int(max_steps), _p(out), out.stride(0),
                                         _p(ld_out), ld_mode, _p(nfe), B, _stream(dev)), "cnf_integrate_dopri5")
    return out, ld_out


def cnf_integrate_dopri5_global(d: CnfDesc, packed: Tensor, x: Tensor, eps: Tensor, t0: float, t1: float,
                                atol: float = 1e-4, rtol: float = 1e-4, max_steps: int = 1000,
                                context: Optional[Tensor] = None, ld_out: Optional[Tensor] = None,
                                ld_mode: int = LD_ROWSUM, out: Optional[Tensor] = None,
                                nfe: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """dopri5 FFJORD block solve with torchdyn's batch-global step control
    (naz_cnf_integrate_dopri5_global: one step size for the batch, the reference's semantics).
    ``nfe`` (int32 [1], optional) receives the batch's RHS evaluations (negative: max_steps ran
    out).  Synchronises the current stream (the controller is polled)."""
    dev = _dev(packed, x, eps, context, ld_out, out)
    x, ldx = _rows(x)
    eps, lde = _rows(eps)
    B = x.shape[0]
    if eps.shape != x.shape:
        raise ValueError("eps must match x")
    context, ldc = _ctx_arg(context, B)
    if out is None:
        out = torch.empty_like(x)
    if ld_out is None:
        ld_out = torch.empty((B,), device=dev, dtype=torch.float32)
        if ld_mode in (LD_ROWSUM_ADD, LD_ROWSUM_SUB):
            ld_out.zero_()
    if nfe is not None and (nfe.dtype != torch.int32 or nfe.numel() < 1 or nfe.device != dev):
        raise ValueError("nfe must be a device int32 tensor with one entry")
    nbytes = int(lib().naz_cnf_dopri5_global_workspace_bytes(d, B))
    if nbytes < 0:
        check(-1, "cnf_dopri5_global_workspace_bytes")
    work = torch.empty((max(nbytes, 4) + 3) // 4, device=dev, dtype=torch.float32)
    check(lib().naz_cnf_integrate_dopri5_global(d, _p(packed), _p(x), ldx, _p(context), ldc, _p(eps), lde, float(t0),
                                                float(t1), float(atol), float(rtol), int(max_steps), _p(out),
                                                out.stride(0), _p(ld_out), ld_mode, _p(nfe), _p(work), B,
                                                _stream(dev)), "cnf_integrate_dopri5_global")
    return out, ld_out
