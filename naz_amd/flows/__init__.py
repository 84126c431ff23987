"""naz.flows API (naz/flows/__init__.py) on the HIP kernels."""
from .flow import NormalizingFlow, flow_makers  # noqa: F401
from .transforms import (bounding_transform, inverse_bounding_transform, masked_affine_autoregressive,  # noqa: F401
                         neural_spline_autoregressive, neural_spline_coupling)
