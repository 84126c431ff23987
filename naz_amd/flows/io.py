"""Canonical flow-weight exchange (model I/O).

The canonical state is a flat dict of arrays, one entry per tensor, per layer ``l``:
  layers.{l}.nn.layers.{i}.weight / .bias          conditioner (pyro names, train_flows.py:414)
  layers.{l}.nn.permutation                        MADE variable order (maf / nsa)
  layers.{l}.lower_spline.unnormalized_{widths,heights,derivatives}   coupling lower spline
It is what ``torch_to_jax`` (naz/flows/bflow_jax_maf.py:26-46) extracts from a pyro flow,
so an offline exporter run where pyro exists can feed trained naz flows to naz_amd.
Saved as ``.npz`` (no pickle).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

from ..nn import invalidate_caches
from .transforms import Permute


def _layers(flow):
    return [t for t in flow.transforms if not isinstance(t, Permute)]


def _linears(t):
    """The conditioner's Linear layers: pyro-style ``.nn.layers`` or the CNF vector field's
    ``ConditionalFCNN.nn`` Sequential (naz continuous_transforms.py:41-50)."""
    net = getattr(t, "net", None)
    if net is not None and hasattr(net, "linears"):
        return net.linears()
    return list(t.nn.layers)


def _lower(t):
    inner = getattr(t, "module", None)
    if inner is not None and hasattr(inner, "lower_spline"):
        return inner.lower_spline
    return getattr(t, "lower_spline", None)


def named_state_params(flow) -> Dict[str, torch.nn.Parameter]:
    """Canonical key -> the live trainable tensor (what get_params/set_params in
    naz/trainers/train_flows.py:20-71 walk; gradients are read back by the same keys)."""
    out = {}
    for l, t in enumerate(_layers(flow)):
        p = f"layers.{l}."
        for i, lin in enumerate(_linears(t)):
            out[p + f"nn.layers.{i}.weight"] = lin.weight
            out[p + f"nn.layers.{i}.bias"] = lin.bias
        low = _lower(t)
        if low is not None:
            for n in ("widths", "heights", "derivatives"):
                out[p + "lower_spline.unnormalized_" + n] = getattr(low, "unnormalized_" + n)
    return out


def export_state(flow) -> Dict[str, np.ndarray]:
    out = {}
    for l, t in enumerate(_layers(flow)):
        p = f"layers.{l}."
        for i, lin in enumerate(_linears(t)):
            out[p + f"nn.layers.{i}.weight"] = lin.weight.detach().float().cpu().numpy()
            out[p + f"nn.layers.{i}.bias"] = lin.bias.detach().float().cpu().numpy()
        if hasattr(t, "nn") and hasattr(t.nn, "permutation"):
            out[p + "nn.permutation"] = t.nn.permutation.detach().cpu().numpy().astype(np.int64)
        low = _lower(t)
        if low is not None:
            for n in ("widths", "heights", "derivatives"):
                out[p + "lower_spline.unnormalized_" + n] = getattr(low, "unnormalized_" + n).detach().cpu().numpy()
    return out


@torch.no_grad()
def load_state(flow, state: Dict[str, np.ndarray]) -> None:
    invalidate_caches()
    for l, t in enumerate(_layers(flow)):
        p = f"layers.{l}."
        if hasattr(t, "nn") and hasattr(t.nn, "set_permutation") and (p + "nn.permutation") in state:
            t.nn.set_permutation(torch.as_tensor(np.asarray(state[p + "nn.permutation"])))
        for i, lin in enumerate(_linears(t)):
            lin.weight.copy_(torch.as_tensor(np.asarray(state[p + f"nn.layers.{i}.weight"])))
            lin.bias.copy_(torch.as_tensor(np.asarray(state[p + f"nn.layers.{i}.bias"])))
        low = _lower(t)
        if low is not None:
            for n in ("widths", "heights", "derivatives"):
                getattr(low, "unnormalized_" + n).copy_(
                    torch.as_tensor(np.asarray(state[p + "lower_spline.unnormalized_" + n])))


def save_npz(flow, path) -> None:
    np.savez(path, **export_state(flow))


def load_npz(flow, path) -> None:
    with np.load(path, allow_pickle=False) as z:
        load_state(flow, {k: z[k] for k in z.files})


def _ref_layers(ref_flow):
    """The per-layer transforms of a reference naz flow (pyro objects or any duck-typed
    stand-in): ``flow.flow_dist.transforms`` (naz/flows/flow.py:37-42; bflow_jax_maf.py:30), with a
    ConditionalComposeTransformModule / ComposeTransformModule unwrapped to its parts."""
    ts = list(getattr(getattr(ref_flow, "flow_dist", ref_flow), "transforms", []))
    out = []
    for t in ts:
        parts = getattr(t, "parts", None)
        if parts is None and hasattr(t, "transforms") and not hasattr(t, "nn"):
            parts = t.transforms
        out.extend(list(parts) if parts is not None else [t])
    return [t for t in out if hasattr(t, "nn") or hasattr(t, "net")]


def _np(t):
    t = t.detach() if hasattr(t, "detach") else t
    t = t.cpu() if hasattr(t, "cpu") else t
    return np.asarray(t.numpy() if hasattr(t, "numpy") else t)


def state_from_reference_flow(ref_flow) -> Dict[str, np.ndarray]:
    """Canonical state (this module's docstring) read from a trained reference flow — the
    fields naz's own ``torch_to_jax`` walks (bflow_jax_maf.py:26-46: ``.nn.layers[i].weight /
    .bias``, ``.nn.masks``, ``.nn.permutation``), plus a coupling layer's
    ``lower_spline.unnormalized_*`` and a CNF vector field's ``net.nn`` Linear stack
    (continuous_transforms.py:38-60).  Works on the pickled pyro objects where pyro is installed
    (scripts/export_naz_flow.py) and on any object exposing the same attributes; nothing here
    imports pyro.  Masks are re-derived by naz_amd from the permutation (half-to-even degree
    rounding, as pyro's create_mask), so the exporter stores them only to check that."""
    out: Dict[str, np.ndarray] = {}
    for l, t in enumerate(_ref_layers(ref_flow)):
        p = f"layers.{l}."
        net = getattr(t, "nn", None)
        if net is not None and hasattr(net, "layers"):
            lins = list(net.layers)
        else:  # CNF: ConditionalFCNN.nn Sequential
            seq = getattr(getattr(t, "net", None), "nn", None) or getattr(t, "net", None)
            lins = [m for m in seq if hasattr(m, "weight") and hasattr(m, "bias")]
        for i, lin in enumerate(lins):
            out[p + f"nn.layers.{i}.weight"] = _np(lin.weight).astype(np.float32)
            out[p + f"nn.layers.{i}.bias"] = _np(lin.bias).astype(np.float32)
        if net is not None and getattr(net, "permutation", None) is not None:
            out[p + "nn.permutation"] = _np(net.permutation).astype(np.int64)
        if net is not None and getattr(net, "masks", None) is not None:
            for i, m in enumerate(net.masks):
                out[p + f"nn.masks.{i}"] = _np(m).astype(np.float32)
        low = getattr(t, "lower_spline", None)
        if low is not None:
            for n in ("widths", "heights", "derivatives"):
                out[p + "lower_spline.unnormalized_" + n] = _np(getattr(low, "unnormalized_" + n)).astype(np.float32)
    if not out:
        raise ValueError("no flow layers with .nn.layers / .net found (expected flow.flow_dist.transforms)")
    return out


def check_masks(flow, state: Dict[str, np.ndarray]) -> None:
    """After load_state: the masks naz_amd derived from each permutation equal the exported
    ones (``nn.masks.{i}`` entries), else ValueError (e.g. a flow built with random_mask)."""
    for l, t in enumerate(_layers(flow)):
        masks = getattr(getattr(t, "nn", None), "masks", None)
        if masks is None:
            continue
        for i, m in enumerate(masks):
            k = f"layers.{l}.nn.masks.{i}"
            if k in state and not np.array_equal(np.asarray(state[k]) != 0, m.detach().cpu().numpy() != 0):
                raise ValueError(f"{k}: exported MADE mask differs from the one derived from the permutation")
