"""naz's Monte-Carlo-dropout flow (naz/flows/mcdpflow.py:29-56) on the HIP kernels.

``MCDPNormalizingFlow(flow_type, bounds, *args, dropout_p=p, ...)`` is a NormalizingFlow whose
conditioners carry dropout (naz_dropout after every hidden activation).  ``sample_uncertain``
draws ``niter`` sample sets with dropout active (train mode), each from fresh base draws and
fresh dropout masks, through the flow's forward (sampling) direction — one conditioner pass
per layer per set, as the reference's ``sample_uncached`` does (mcdpflow.py:12-25; its
non-compose branch applies every transform to the base draws instead of chaining them, a bug;
the chained forward of its compose branch is what runs here).  Returns numpy
[niter, *shape, D], as the reference does."""
from __future__ import annotations

import numpy as np
import torch

from .flow import NormalizingFlow

__all__ = ["MCDPNormalizingFlow"]


class MCDPNormalizingFlow(NormalizingFlow):
    """Normalizing flow with Monte-Carlo dropout in its conditioners (mcdpflow.py:29-37)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.flow_maker = args[0]
        assert kwargs.get("dropout_p") not in [None, 0.0], "MCDPNormalizingFlow needs dropout_p > 0"

    def sample_uncertain(self, niter, *args, condition=None, **kwargs):
        """mcdpflow.py:39-56: ``niter`` stochastic forward passes in train mode."""
        self.train()
        pdf = self._pdf(condition)
        bounds = self._bounds_dev(self._base_loc)
        shape = args[0] if args else kwargs.get("sample_shape", ())
        out = []
        with torch.no_grad():
            for _ in range(int(niter)):
                out.append(pdf.sample(shape, bounds=bounds).cpu().numpy())
        return np.array(out)
