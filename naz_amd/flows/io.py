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
