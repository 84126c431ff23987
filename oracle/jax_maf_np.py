"""TEST INFRASTRUCTURE ONLY — numpy restatement of the reference's in-tree JAX affine MAF.

``/root/reference/src/naz/flows/bflow_jax_maf.py`` is naz's own second statement of
the conditional affine MAF log-density (MADE masks, masked linear, tanh, clip(-5,3),
D-pass inverse, standard-normal base).  JAX is not installed here, so it is re-stated
in numpy (float64) from the text; it is independent of ``naz_oracle`` and is used to
cross-check the affine path (SURVEY.md §8c known-answer test 8).  ``bounds=None`` only:
the reference's bounded branch carries a sign bug (``bflow_jax_maf.py:210-212``) that
the torch path (``flow.py:79``) does not have.
"""
from __future__ import annotations

import math
from typing import List

import numpy as np


def sample_mask_indices(input_dim: int, hidden_dim: int) -> np.ndarray:
    """bflow_jax_maf.py:48-50 (simple=True): round-half-to-even of a float32 linspace."""
    return np.round(np.linspace(1, input_dim, hidden_dim, dtype=np.float32))


def create_mask(input_dim: int, context_dim: int, hidden_dims: List[int], permutation: np.ndarray,
                output_dim_multiplier: int):
    """bflow_jax_maf.py:52-72."""
    var_index = np.empty(permutation.shape, dtype=np.float32)
    var_index[permutation] = np.arange(1, input_dim + 1, dtype=np.float32)
    input_indices = np.concatenate([np.zeros(context_dim, dtype=np.float32), var_index])
    if context_dim > 0:
        hidden_indices = [sample_mask_indices(input_dim, h) - 1 for h in hidden_dims]
    else:
        hidden_indices = [sample_mask_indices(input_dim - 1, h) for h in hidden_dims]
    output_indices = np.tile(var_index, output_dim_multiplier)
    masks = [(hidden_indices[0][:, None] >= input_indices[None, :]).astype(np.float64)]
    for i in range(1, len(hidden_dims)):
        masks.append((hidden_indices[i][:, None] >= hidden_indices[i - 1][None, :]).astype(np.float64))
    masks.append((output_indices[:, None] > hidden_indices[-1][None, :]).astype(np.float64))
    return masks


def nn_fn(x: np.ndarray, params, masks, context=None, input_dim: int = None):
    """bflow_jax_maf.py:131-165 (no skip connections, tanh): returns (mean, log_scale)."""
    if context is not None:
        context = np.broadcast_to(context, x.shape[:-1] + (context.shape[-1],))
        h = np.concatenate([context, x], axis=-1)
    else:
        h = x
    for (W, b), m in zip(params[:-1], masks[:-1]):
        h = np.tanh(h @ (W * m).T + b)
    W, b = params[-1]
    out = h @ (W * masks[-1]).T + b
    out = out.reshape(x.shape[:-1] + (2, input_dim))
    return out[..., 0, :], out[..., 1, :]


def inverse_fn(y: np.ndarray, params, masks, perm, context=None):
    """bflow_jax_maf.py:183-193: D sequential passes in permutation order."""
    D = y.shape[-1]
    x = np.zeros_like(y)
    log_scale = None
    for idx in perm:
        mean, log_scale = nn_fn(x, params, masks, context, D)
        inverse_scale = np.exp(-np.clip(log_scale[..., idx], -5.0, 3.0))
        x[..., idx] = (y[..., idx] - mean[..., idx]) * inverse_scale
    return x, np.sum(np.clip(log_scale, -5.0, 3.0), axis=-1)


def cast_layers(layers, dtype):
    """The same layers with weights, biases and masks in ``dtype`` (float32 = the reference's
    own arithmetic precision, the ``ref32`` of tests/parity.py)."""
    return [([(W.astype(dtype), b.astype(dtype)) for (W, b) in params], perm, [m.astype(dtype) for m in masks])
            for params, perm, masks in layers]


def log_prob(x: np.ndarray, layers, context=None, dtype=np.float64):
    """bflow_jax_maf.py:210-212 with bounds=None.  ``layers`` = list of (params, perm) in
    flow order; reversed here as the reference's ``reduce(inv_transform, zip(reversed(...)))``.
    ``dtype`` float32 evaluates at the reference's precision (layers must be cast alike)."""
    D = x.shape[-1]
    z = x.astype(dtype)
    if context is not None:
        context = np.asarray(context).astype(dtype)
    log_det = np.zeros(x.shape[:-1], dtype=dtype)
    for params, perm, masks in reversed(layers):
        z, ld = inverse_fn(z, params, masks, perm, context)
        log_det = log_det + ld
    return -np.sum(0.5 * z ** 2, axis=-1) - 0.5 * D * math.log(2 * math.pi) - log_det


def layers_from_state(spec: dict, state: dict):
    """Canonical state dict (see naz_oracle.build_flow) -> list of (params, perm, masks)."""
    hidden = list(spec["hidden"]) if isinstance(spec["hidden"], (list, tuple)) else [spec["hidden"]]
    out = []
    for l in range(spec["L"]):
        p = f"layers.{l}.nn."
        params = [(np.asarray(state[p + f"layers.{i}.weight"], dtype=np.float64),
                   np.asarray(state[p + f"layers.{i}.bias"], dtype=np.float64)) for i in range(len(hidden) + 1)]
        perm = np.asarray(state[p + "permutation"]).astype(np.int64)
        masks = create_mask(spec["D"], spec["C"], hidden, perm, 2)
        out.append((params, perm, masks))
    return out


def forward_fn(x: np.ndarray, params, masks, context=None):
    """bflow_jax_maf.py:172-178: one MADE pass, y = mean + x * exp(clip(ls, -5, 3))."""
    mean, log_scale = nn_fn(x, params, masks, context, x.shape[-1])
    log_scale = np.clip(log_scale, -5.0, 3.0)
    return mean + x * np.exp(log_scale), np.sum(log_scale, axis=-1)


def sample_from_z(z: np.ndarray, layers, context=None, dtype=np.float64):
    """bflow_jax_maf.py:214-222 (``sampler``) with the base draws ``z`` given (JAX's PRNG is not
    restated) and bounds=None: layers in flow order; returns (y, log_j) with
    log_j = base log-density of z + Σ clip(ls), the sign the reference returns."""
    D = z.shape[-1]
    y = z.astype(dtype)
    if context is not None:
        context = np.asarray(context).astype(dtype)
    log_j = -np.sum(0.5 * y ** 2, axis=-1) - 0.5 * D * math.log(2 * math.pi)
    for params, perm, masks in layers:
        y, ld = forward_fn(y, params, masks, context)
        log_j = log_j + ld
    return y, log_j
