"""naz.flows.transforms (src/naz/flows/transforms.py) -> naz_amd.flows.transforms."""
from naz_amd.flows.transforms import *  # noqa: F401,F403
from naz_amd.flows.transforms import (bounding_transform, inverse_bounding_transform, masked_affine_autoregressive,
                                      neural_spline_autoregressive, neural_spline_coupling)

__all__ = ["bounding_transform", "inverse_bounding_transform", "masked_affine_autoregressive",
           "neural_spline_autoregressive", "neural_spline_coupling"]
