"""naz.flows.continuous_transforms (src/naz/flows/continuous_transforms.py) ->
naz_amd.flows.continuous_transforms."""
from naz_amd.flows.continuous_transforms import (ConditionalFCNN, ConditionalFFJORDTransform, FCNN, FFJORDTransform,
                                                 continuous_free_form)

__all__ = ["ConditionalFCNN", "ConditionalFFJORDTransform", "FCNN", "FFJORDTransform", "continuous_free_form"]
