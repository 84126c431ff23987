"""Flow distributions: torch ``TransformedDistribution`` / pyro ``ConditionalTransformedDistribution``
semantics (naz/flows/flow.py:37-42) with every arithmetic step on the HIP kernels.

``log_prob(y)`` walks the transforms in reverse exactly like torch's
TransformedDistribution (``lp -= ladj`` per layer, ``lp += base``), but the per-layer
row log-det is accumulated into ``lp`` inside the spline/affine kernels and the
Normal(0, 1) base density is a kernel too.  When the owning ``NormalizingFlow`` holds
a fused plan (flow_type "nsc" with a compiled shape) the whole walk is ONE launch of
``naz_coupling_log_prob``.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from .. import autograd as ag
from .. import ops


def _rows2d(t: torch.Tensor):
    lead = t.shape[:-1]
    return t.reshape(-1, t.shape[-1]), lead


class TransformedDistribution:
    """Density of T(z), z ~ base (torch.distributions.TransformedDistribution semantics)."""

    def __init__(self, base_dist, transforms, fused=None, context=None):
        self.base_dist = base_dist
        if isinstance(transforms, (list, tuple)):
            self.transforms = list(transforms)
        else:  # a single (compose) transform, as torch does
            self.transforms = [transforms]
        self._fused = fused
        self._context = context

    @property
    def event_dim(self):
        return 1

    def _trainable_modules(self):
        mods = []
        for t in self.transforms:
            for attr in ("module", "arn", "inner", "arn_module"):
                m = getattr(t, attr, None)
                if isinstance(m, torch.nn.Module):
                    mods.append(m)
            if isinstance(t, torch.nn.Module):
                mods.append(t)
        return mods

    def _needs_graph(self, y) -> bool:
        return ag.params_require_grad(self._trainable_modules()) or ag.tensor_requires_grad(y, self._context)

    def _log_prob_graph(self, y: torch.Tensor, bounds=None) -> torch.Tensor:
        """Autograd-recorded walk (training, a10): same order as torch's TransformedDistribution,
        every node a HIP kernel with a HIP backward.  The bounding map (naz/flows/flow.py:52-70)
        acts on the data only and is evaluated outside the graph."""
        acc = None
        if bounds is not None:
            with torch.no_grad():
                y, acc = ops.bounding_fwd(y.detach(), bounds["low"], bounds["high"])
        for t in reversed(self.transforms):
            y, ld = t._inv_ld(y)
            if ld is not None:
                acc = -ld if acc is None else acc - ld
        lp = ag.base_log_prob(y)
        return lp if acc is None else lp + acc

    def _fused_ok(self) -> bool:
        return self._fused is not None and self._fused.usable()

    def _log_prob_into(self, y: torch.Tensor, lp: torch.Tensor, bounds=None) -> torch.Tensor:
        if self._fused_ok() and getattr(self._fused, "log_prob_ready", lambda *a: True)(y, self._context):
            return self._fused.log_prob(y, self._context, bounds=bounds, out=lp)
        if bounds is not None:
            y, lj = ops.bounding_fwd(y, bounds["low"], bounds["high"])
            lp.copy_(lj)
        for t in reversed(self.transforms):
            y = t._inverse_acc(y, lp)
        ops.base_log_prob(y, out=lp, accumulate=True)
        return lp

    def log_prob(self, value: torch.Tensor, bounds=None) -> torch.Tensor:
        y, lead = _rows2d(value)
        if self._needs_graph(y):
            if self._fused_ok() and self._fused.train_ready(y, self._context):
                # the NLL step of an nsc flow: one fused forward + per-layer fused backward
                return self._fused.train_log_prob(y, self._context, bounds).reshape(lead)
            return self._log_prob_graph(y, bounds).reshape(lead)
        lp = torch.zeros(y.shape[0], device=y.device, dtype=torch.float32)
        return self._log_prob_into(y, lp, bounds).reshape(lead)

    def _transform_z(self, z: torch.Tensor, bounds=None) -> torch.Tensor:
        if self._fused_ok() and getattr(self._fused, "can_sample", True) and \
                getattr(self._fused, "sample_ready", lambda *a: True)(z, self._context):
            y, _ = self._fused.sample(z, self._context, bounds=bounds)
            return y
        ld = torch.zeros(z.shape[0], device=z.device, dtype=torch.float32)
        y = z
        for t in self.transforms:
            y = t._call_acc(y, ld)
        if bounds is not None:
            y = ops.bounding_inv(y, bounds["low"], bounds["high"])
        return y

    def rsample(self, sample_shape=torch.Size(), bounds=None) -> torch.Tensor:
        shape = torch.Size(sample_shape)
        loc = self.base_dist.loc
        D = loc.shape[-1]
        z = torch.randn(shape + (D,), device=loc.device, dtype=torch.float32)
        y = self._transform_z(z.reshape(-1, D), bounds)
        return y.reshape(shape + (D,))

    def sample(self, sample_shape=torch.Size(), bounds=None) -> torch.Tensor:
        with torch.no_grad():
            return self.rsample(sample_shape, bounds)

    def clear_cache(self):
        for t in self.transforms:
            if hasattr(t, "_cached_x_y"):
                t._cached_x_y = None, None
            if hasattr(t, "_cache_log_detJ"):
                t._cache_log_detJ = None


class ConditionalTransformedDistribution:
    """[pyro] distributions/conditional.py::ConditionalTransformedDistribution
    (naz/flows/flow.py:40).  ``transforms`` lists the per-layer conditional modules."""

    def __init__(self, base_dist, transforms, fused=None):
        self.base_dist = base_dist
        self.transforms = [t for t in transforms]
        self._fused = fused

    def condition(self, context) -> TransformedDistribution:
        conditioned = [t.condition(context) if hasattr(t, "condition") else t for t in self.transforms]
        return TransformedDistribution(self.base_dist, conditioned, fused=self._fused, context=context)

    def clear_cache(self):
        pass
